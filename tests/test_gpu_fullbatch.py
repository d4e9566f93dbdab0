"""Full-batch parity at the bench configs' batch sizes:
the workspace, workgroup map and band geometry of a 256-image c2 batch and a
1024-image c5 batch, checked image by image against sha256s of the oracle's
output (tests/golden/fullbatch.json, made by make_fullbatch_golden.py)."""
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
