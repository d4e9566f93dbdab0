"""Full-batch parity at the bench configs' batch sizes (VERDICT r1 item 6,
r5 item 4): the workspace, workgroup map and band geometry of a 256-image c2
batch and a 1024-image c5 batch, and the configs[2] / configs[3] batches of
128 read through LanceDataset + their samplers over FOOD101-shaped uneven
fragments on two ranks, checked image by image against sha256s of the
oracle's output (tests/golden/fullbatch.json, made by make_fullbatch_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fullbatch():
    with open(os.path.join(GOLDEN, "fullbatch.json")) as f:
        return json.load(f)


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _mismatches(img, exp):
    return [k for k in range(len(exp)) if _sha(img[k]) != exp[k]]


def test_c2_full_batch_sync_and_pipelined(fullbatch):
    """256 x 512x512 q90: the synchronous to_tensor_fn on a host RecordBatch
    and the bench's path (resident cells, 3-deep DecodePipeline) both match
    the oracle on every image; labels are copied bit-exactly."""
    import ldt_amd
    from ldt_amd import synth

    g = fullbatch["c2"]
    cells, labels = synth.q90_512(g["n"], seed=fullbatch["seed"])
    assert [int(x) for x in labels] == g["labels"]
    out = ldt_amd.decode_tensor_image(synth.arrow_batch(cells, labels))
    assert out["label"].cpu().numpy().tolist() == g["labels"]
    bad = _mismatches(out["image"].cpu().numpy(), g["sha256"])
    assert not bad, f"sync to_tensor_fn: images {bad[:10]} differ from the oracle"

    rb = ldt_amd.ResidentBatch(cells, labels)
    pipe = ldt_amd.DecodePipeline(depth=3)
    outs = [pipe.decode(rb) for _ in range(4)]  # 4 batches over 3 slots
    pipe.check()
    for k, (img, lbl) in enumerate(outs):
        assert lbl.cpu().numpy().tolist() == g["labels"]
        bad = _mismatches(img.cpu().numpy(), g["sha256"])
        assert not bad, f"pipelined batch {k}: images {bad[:10]} differ from the oracle"


def test_c5_full_batch_raw_resize_normalize(fullbatch):
    """1024 raw 1024x1024 HWC cells resident in HBM (3.2 GB) -> Resize 224 +
    Normalize, every image vs the oracle."""
    import torch

    import ldt_amd
    from ldt_amd import synth

    g = fullbatch["c5"]
    h, w = g["hw"]
    seed = fullbatch["seed"]
    raw = torch.empty((g["n"], h, w, 3), dtype=torch.uint8, device="cuda")
    for i in range(g["n"]):
        raw[i].copy_(torch.from_numpy(synth.raw_hwc_one(h, w, seed * 100003 + i)))
    out = ldt_amd.resize_raw(raw, h, w, normalize=True).cpu().numpy()
    del raw
    bad = _mismatches(out, g["sha256"])
    assert not bad, f"raw c5: images {bad[:10]} differ from the oracle"


# FOOD101's fragments [12500 x 6, 750] (create_datasets/classification.py:16,60)
# scaled to 256 rows: 1551 rows, uneven (the last fragment holds 15)
FRAGS = [256] * 6 + [256 * 750 // 12500]


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("key,kind", [("c3", "batch"), ("c4", "fragment")])
def test_config_batches_through_dataset_two_ranks(fullbatch, tmp_path, key, kind):
    """configs[2] (c3: FOOD101-shaped q75, ShardedBatchSampler) and configs[3]
    (c4: ImageNet-shaped q90 with restart markers, ShardedFragmentSampler(pad=True)
    with its all_reduce(MAX)), batch 128 per rank, W = 2 (gloo, both ranks on
    cuda:0), through LanceDataset and the pipelined copying to_tensor_fn the
    bench's dataset legs run: every decoded image — padding batches included —
    equals the oracle's sha256 of its cell, labels are the rows' own, the ranks'
    rows are disjoint and cover the dataset, and with pad=True both ranks yield
    the same number of batches (rank 1's short fragment list is padded)."""
    import pyarrow as pa
    import torch.multiprocessing as mp

    import ldt_amd
    import _fullbatch_worker
    from ldt_amd import synth

    g = fullbatch[key]
    make = synth.food101_like if key == "c3" else synth.imagenet_like
    cells, labels = make(g["n"], seed=fullbatch["seed"])
    assert [int(x) for x in labels] == g["labels"]
    n = sum(FRAGS)
    uri = str(tmp_path / key)
    ldt_amd.write_dataset(pa.table({"image": pa.array([cells[r % len(cells)] for r in range(n)], pa.binary()),
                                    "label": pa.array(np.arange(n, dtype=np.int64))}), uri,
                          max_rows_per_file=FRAGS[0])
    assert [f.count_rows() for f in ldt_amd.dataset(uri).get_fragments()] == FRAGS
    exp_path = str(tmp_path / "exp.json")
    with open(exp_path, "w") as f:
        json.dump(g["sha256"], f)
    mp.start_processes(_fullbatch_worker.run, args=(2, _free_port(), uri, str(tmp_path), kind, exp_path),
                       nprocs=2, join=True, start_method="spawn")
    r = [json.load(open(tmp_path / f"fb_{kind}_rank{k}.json")) for k in range(2)]
    assert r[0]["bad"] == [] and r[1]["bad"] == [], \
        f"rows {(r[0]['bad'] + r[1]['bad'])[:10]} differ from the oracle"
    if kind == "fragment":
        # rank 0: fragments 0, 2, 4, 6 -> 2 + 2 + 2 + 1 batches; rank 1: 1, 3, 5
        # -> 6, padded to 7 by re-yielding its own batches
        assert r[0]["batches"] == r[1]["batches"] == 7
        own1 = r[1]["labels"][:6]
        assert r[1]["labels"][6] in own1, "pad batch is not one of rank 1's own"
        rows = [set(x for b in r[0]["labels"] for x in b), set(x for b in own1 for x in b)]
    else:
        # 13 global batches of 128 rows (the last 15): rank 0 takes 7, rank 1 six
        assert (r[0]["batches"], r[1]["batches"]) == (7, 6)
        rows = [set(x for b in r[k]["labels"] for x in b) for k in range(2)]
    assert not (rows[0] & rows[1]), "ranks share rows"
    assert sorted(rows[0] | rows[1]) == list(range(n)), "rows missing"
