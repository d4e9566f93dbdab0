"""Worker for tests/test_dist_gloo.py (world_size 2, gloo, 127.0.0.1)."""
import os
import sys


def run(rank, world, port, outdir):
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (os.path.join(repo, "lance-distributed-training_amd"), repo, here):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import json

    import torch.distributed as dist

    from ldt_amd import ShardedBatchSampler, ShardedFragmentSampler
    from ldt_amd.sampler import agree_max
    from ldt_amd.synth import FOOD101_FRAGMENTS
    from oracle import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)

    calls = []

    def frag_compute(rows, B, r, W, pad_to):
        calls.append(pad_to)
        local = len(oracle.sharded_fragment_batches(rows, B, r, W))
        if pad_to is None or pad_to < 0:
            return oracle.sharded_fragment_batches(rows, B, r, W), local
        return oracle.sharded_fragment_batches(rows, B, r, W, pad=True)[:pad_to], local

    s = ShardedFragmentSampler(rank, world, pad=True, compute=frag_compute)
    recs = s.plan(FOOD101_FRAGMENTS, 128)
    s2 = ShardedFragmentSampler(rank, world, pad=False, compute=frag_compute)
    recs_nopad = s2.plan(FOOD101_FRAGMENTS, 128)
    b = ShardedBatchSampler(rank, world, compute=oracle.sharded_batch_ranges)
    rng = b.ranges(sum(FOOD101_FRAGMENTS), 128)
    m = agree_max(rank * 10 + 3)
    # map-style DistributedSampler: num_replicas/rank from the process group,
    # as lance_map_style.py:58 constructs it (oracle standing in for the kernel)
    from ldt_amd import DistributedSampler

    def dist_compute(n, W, r, shuffle, seed, drop_last):
        return oracle.distributed_indices(n, W, r, shuffle, seed, 0, drop_last)

    ds = DistributedSampler(range(1001), seed=7, compute=dist_compute)
    ds.set_epoch(2)
    didx = list(ds)
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump({"padded": len(recs), "unpadded": len(recs_nopad), "ranges": rng, "max": m,
                   "calls": calls, "dist_idx": didx, "dist_rank": ds.rank, "dist_world": ds.num_replicas}, f)
    dist.barrier()
    dist.destroy_process_group()
