"""Per-image sha256 of the oracle's float32 [3,224,224] output for full
batches at the bench configs' sizes: c2 = 256 synthetic
512x512 q90 4:2:0 JPEGs (synth.q90_512, seed 4242), c5 = 1024 raw 1024x1024
uint8 HWC cells (synth.raw_hwc_one(1024, 1024, 4242 * 100003 + i)) resized
with Normalize. The oracle (oracle/jpeg_oracle.c) is itself pinned to Pillow
12.2 / libjpeg-turbo 3.1.4.1 by tests/golden/make_golden.py.

    python tests/golden/make_fullbatch_golden.py   # writes fullbatch.json
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
C2_N, C5_N = 256, 1024


def c5_seed(i: int) -> int:
    return SEED * 100003 + i


def main():
    cells, labels = synth.q90_512(C2_N, seed=SEED)
    c2 = [hashlib.sha256(oracle.jpeg_to_tensor(b).tobytes()).hexdigest() for b in cells]
    c5 = []
    for i in range(C5_N):
        raw = synth.raw_hwc_one(1024, 1024, c5_seed(i))
        c5.append(hashlib.sha256(oracle.raw_to_tensor(raw, normalize=True).tobytes()).hexdigest())
    out = {"seed": SEED, "c2": {"n": C2_N, "labels": [int(x) for x in labels], "sha256": c2},
           "c5": {"n": C5_N, "hw": [1024, 1024], "normalize": True, "sha256": c5}}
    with open(os.path.join(HERE, "fullbatch.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("c2", len(c2), "c5", len(c5))


if __name__ == "__main__":
    main()
