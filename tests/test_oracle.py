"""CPU tests: the oracle is pinned against the golden vectors (Pillow/libjpeg-turbo
outputs) and against Pillow directly on seeded inputs; sampler restatement
against the FOOD101 arithmetic of README.md:164-191."""
import hashlib
import io
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, read_golden
from oracle import oracle


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_oracle_matches_golden_decode_resize_tensor(manifest):
    for ent in manifest["images"]:
        b = read_golden(ent["file"])
        rgb = oracle.decode_rgb(b)
        assert rgb.shape == (ent["height"], ent["width"], 3), ent["name"]
        assert sha(rgb) == ent["sha256_rgb"], ent["name"]
        assert sha(oracle.resize_rgb(rgb)) == ent["sha256_resized_u8"], ent["name"]
        assert sha(oracle.jpeg_to_tensor(b)) == ent["sha256_tensor_f32"], ent["name"]
        assert sha(oracle.jpeg_to_tensor(b, normalize=True)) == ent["sha256_tensor_norm_f32"], ent["name"]


def test_oracle_rejects_bad_inputs(manifest):
    for ent in manifest["bad"]:
        b = read_golden(ent["file"])
        with pytest.raises(oracle.OracleError):
            oracle.jpeg_to_tensor(b)


def test_oracle_raw_resize_golden(manifest):
    raw = np.load(f"{__import__('conftest').GOLDEN}/{manifest['raw']['file']}")["hwc"]
    for k, exp in enumerate(manifest["raw"]["expected"]):
        assert sha(oracle.raw_to_tensor(raw[k])) == exp["sha256_tensor_f32"]
        assert sha(oracle.raw_to_tensor(raw[k], normalize=True)) == exp["sha256_tensor_norm_f32"]


@pytest.mark.parametrize("seed", range(6))
def test_oracle_vs_pillow_seeded(seed):
    """Randomised shapes/qualities/subsampling: oracle decode == Pillow decode."""
    from PIL import Image

    from ldt_amd import synth

    r = np.random.RandomState(seed)
    for _ in range(4):
        h, w = int(r.randint(1, 200)), int(r.randint(1, 200))
        kw = dict(quality=int(r.choice([30, 75, 90, 97])),
                  subsampling=str(r.choice(["4:2:0", "4:2:2", "4:4:4"])))
        if r.rand() < 0.3:
            kw["restart_marker_blocks"] = int(r.randint(1, 8))
        if r.rand() < 0.3:
            kw["progressive"] = True  # SOF2: jdphuff.c restatement
        b = synth.encode(synth.field(h, w, int(r.randint(1 << 30)), float(r.choice([0, 5, 30]))), **kw)
        ref = np.asarray(Image.open(io.BytesIO(b)).convert("RGB"))
        assert np.array_equal(oracle.decode_rgb(b), ref), (h, w, kw)
        np.testing.assert_array_equal(oracle.jpeg_to_tensor(b), oracle.pil_image_to_tensor(b))


def test_resample_coeff_shapes():
    # Pillow Resample.c: ksize = ceil(support) * 2 + 1
    for n_in, ks in ((512, 7), (384, 5), (1024, 11), (224, 3), (100, 3)):
        k, bounds, kk = oracle.resample_coeffs(n_in, 224)
        assert k == ks
        assert bounds[:, 0].min() >= 0 and (bounds[:, 0] + bounds[:, 1]).max() <= n_in
        # weights sum to 1<<22 within rounding of each tap
        assert np.all(np.abs(kk.sum(1) - (1 << 22)) <= k)


def test_sampler_oracle_matches_golden(sampler_golden):
    g = sampler_golden
    frags, B, N = g["fragments"], g["batch_size"], g["num_rows"]
    for W, per_rank in g["sharded_batch"].items():
        W = int(W)
        covered = []
        for r, ent in enumerate(per_rank):
            rng = np.asarray(oracle.sharded_batch_ranges(N, B, r, W), np.int64).reshape(-1, 2)
            assert sha(rng) == ent["sha256"] and len(rng) == ent["count"]
            covered += [tuple(x) for x in rng]
        # every row exactly once across ranks
        covered.sort()
        assert covered[0][0] == 0 and covered[-1][1] == N
        assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))
    for W, per_rank in g["sharded_fragment"].items():
        W = int(W)
        for r, ent in enumerate(per_rank):
            rec = np.asarray(oracle.sharded_fragment_batches(frags, B, r, W), np.int64).reshape(-1, 5)
            prec = np.asarray(oracle.sharded_fragment_batches(frags, B, r, W, pad=True), np.int64).reshape(-1, 5)
            assert sha(rec) == ent["sha256"] and sha(prec) == ent["sha256_padded"]


def test_readme_deadlock_arithmetic():
    """README.md:164-191: W=2, B=128 -> rank 0 runs 300 it/epoch, rank 1 294;
    rank 0 hangs on its 2941st all-reduce (Epoch 10/10: 241it)."""
    from ldt_amd.synth import FOOD101_FRAGMENTS as F

    c0 = len(oracle.sharded_fragment_batches(F, 128, 0, 2))
    c1 = len(oracle.sharded_fragment_batches(F, 128, 1, 2))
    assert (c0, c1) == (300, 294)
    assert 10 * c1 + 1 == 9 * c0 + 241
    # with pad=True both ranks yield the same count -> no hang
    assert len(oracle.sharded_fragment_batches(F, 128, 0, 2, pad=True)) == \
        len(oracle.sharded_fragment_batches(F, 128, 1, 2, pad=True)) == 300
    # W=8: rank 7 owns no rows, padded to 98
    assert len(oracle.sharded_fragment_batches(F, 128, 7, 8)) == 0
    assert len(oracle.sharded_fragment_batches(F, 128, 7, 8, pad=True)) == 98


def _distributed_golden():
    return json.load(open(os.path.join(GOLDEN, "distributed.json")))["cases"]


def test_distributed_sampler_oracle_matches_torch_golden():
    """oracle.distributed_indices (MT19937 + Fisher-Yates restatement) vs the
    sha256 of torch's own DistributedSampler output (tests/golden/distributed.json)."""
    for g in _distributed_golden():
        c = g["case"]
        if c["n"] > 100_000:
            continue  # the 1.28M case is checked on the GPU path only (pure-Python loop)
        for r, exp in enumerate(g["ranks"]):
            idx = np.asarray(oracle.distributed_indices(c["n"], c["W"], r, c["shuffle"], c["seed"],
                                                        c["epoch"], c["drop_last"]), np.int64)
            assert len(idx) == exp["count"] == oracle.distributed_num_samples(c["n"], c["W"], c["drop_last"])
            assert hashlib.sha256(idx.tobytes()).hexdigest() == exp["sha256"], c


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (53, 7), (4096, 2**33 + 5), (30000, -9)])
def test_randperm_restatement_vs_torch(n, seed):
    import torch

    g = torch.Generator()
    g.manual_seed(seed)
    assert torch.randperm(n, generator=g).tolist() == oracle.randperm(n, seed % (1 << 64)).tolist()


def test_fullbatch_fixture_matches_oracle():
    """tests/golden/fullbatch.json (full-batch GPU parity) agrees with the
    oracle on its first images of both configs."""
    import hashlib
    import json

    from ldt_amd import synth

    g = json.load(open(os.path.join(GOLDEN, "fullbatch.json")))
    cells, labels = synth.q90_512(3, seed=g["seed"])
    for k, b in enumerate(cells):
        assert hashlib.sha256(oracle.jpeg_to_tensor(b).tobytes()).hexdigest() == g["c2"]["sha256"][k]
    for i in range(2):
        raw = synth.raw_hwc_one(1024, 1024, g["seed"] * 100003 + i)
        assert hashlib.sha256(oracle.raw_to_tensor(raw, normalize=True).tobytes()).hexdigest() == \
            g["c5"]["sha256"][i]
    # c3 / c4: the whole 128-image batches (cells and labels regenerate exactly)
    for key, make in (("c3", synth.food101_like), ("c4", synth.imagenet_like)):
        cells, labels = make(g[key]["n"], seed=g["seed"])
        assert [int(x) for x in labels] == g[key]["labels"]
        got = [hashlib.sha256(oracle.jpeg_to_tensor(b).tobytes()).hexdigest() for b in cells]
        assert got == g[key]["sha256"], key
