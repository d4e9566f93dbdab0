"""World-size-2 gloo test of the multi-rank sampler path (CPU): the pad=True
batch-count consensus is one all_reduce(MAX); ShardedBatchSampler needs no
exchange and its ranks partition the rows."""
import json
import os
import socket

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_fragment_pad_consensus_world2(tmp_path):
    import _dist_worker

    port = _free_port()
    mp.start_processes(_dist_worker.run, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r0 = json.load(open(tmp_path / "rank0.json"))
    r1 = json.load(open(tmp_path / "rank1.json"))
    # README.md:164-183: 300 vs 294 batches unpadded -> the deadlock; padded: equal
    assert (r0["unpadded"], r1["unpadded"]) == (300, 294)
    assert r0["padded"] == r1["padded"] == 300
    assert r0["max"] == r1["max"] == 13
    # the consensus ran exactly once per plan(): local count, then padded records
    assert r0["calls"][:2] == [-1, 300] and r1["calls"][:2] == [-1, 300]
    rows = sorted(tuple(x) for x in r0["ranges"] + r1["ranges"])
    assert rows[0][0] == 0 and rows[-1][1] == 75750 and len(rows) == 592
    # DistributedSampler: rank/world from the group; the two ranks together
    # cover every index (1001 rows padded to 1002: one repeat), as torch's
    assert (r0["dist_rank"], r1["dist_rank"], r0["dist_world"]) == (0, 1, 2)
    assert len(r0["dist_idx"]) == len(r1["dist_idx"]) == 501
    assert sorted(set(r0["dist_idx"]) | set(r1["dist_idx"])) == list(range(1001))
    from torch.utils.data import DistributedSampler as TorchDS

    for r, got in ((0, r0["dist_idx"]), (1, r1["dist_idx"])):
        t = TorchDS(range(1001), num_replicas=2, rank=r, seed=7)
        t.set_epoch(2)
        assert got == list(t)
