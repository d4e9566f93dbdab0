"""Per-image sha256 of the oracle's float32 [3,224,224] output for full
batches at the bench configs' sizes: c2 = 256 synthetic
512x512 q90 4:2:0 JPEGs (synth.q90_512, seed 4242), c5 = 1024 raw 1024x1024
uint8 HWC cells (synth.raw_hwc_one(1024, 1024, 4242 * 100003 + i)) resized
with Normalize. The oracle (oracle/jpeg_oracle.c) is itself pinned to Pillow
12.2 / libjpeg-turbo 3.1.4.1 by tests/golden/make_golden.py.

c3 = 128 FOOD101-shaped PIL-default q75 cells (synth.food101_like, seed 4242)
and c4 = 128 ImageNet-shaped q90 cells with restart markers
(synth.imagenet_like, seed 4242), the configs[2] / configs[3] batch of 128
per rank, read by tests/test_gpu_fullbatch.py through
LanceDataset + the config's sampler.

    python tests/golden/make_fullbatch_golden.py [--all]   # writes fullbatch.json
    (without --all, entries already in fullbatch.json are kept)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lance-distributed-training_amd"))
sys.path.insert(0, REPO)

from ldt_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402

SEED = 4242
C2_N, C5_N, C3_N, C4_N = 256, 1024, 128, 128


def c5_seed(i: int) -> int:
    return SEED * 100003 + i


def _jpeg_entry(cells, labels):
    return {"n": len(cells), "labels": [int(x) for x in labels],
            "sha256": [hashlib.sha256(oracle.jpeg_to_tensor(b).tobytes()).hexdigest() for b in cells]}


def main():
    path = os.path.join(HERE, "fullbatch.json")
    out = {}
    if "--all" not in sys.argv and os.path.exists(path):
        with open(path) as f:
            out = json.load(f)
    out["seed"] = SEED
    if "c2" not in out:
        out["c2"] = _jpeg_entry(*synth.q90_512(C2_N, seed=SEED))
    if "c5" not in out:
        c5 = []
        for i in range(C5_N):
            raw = synth.raw_hwc_one(1024, 1024, c5_seed(i))
            c5.append(hashlib.sha256(oracle.raw_to_tensor(raw, normalize=True).tobytes()).hexdigest())
        out["c5"] = {"n": C5_N, "hw": [1024, 1024], "normalize": True, "sha256": c5}
    if "c3" not in out:
        out["c3"] = _jpeg_entry(*synth.food101_like(C3_N, seed=SEED))
    if "c4" not in out:
        out["c4"] = _jpeg_entry(*synth.imagenet_like(C4_N, seed=SEED))
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print({k: v["n"] for k, v in out.items() if isinstance(v, dict)})


if __name__ == "__main__":
    main()
