"""PMC probe: c2 batches (256 x 512x512 q90) decoded one at a time (depth 1)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
import torch  # noqa: E402

import ldt_amd  # noqa: E402
from ldt_amd import synth  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
make = {"c2": lambda: synth.q90_512(256, seed=1000), "c1": lambda: synth.food101_like(128, seed=1000),
        "c4": lambda: synth.imagenet_like(128, seed=1000)}[wl]
cells, labels = make()
rb = ldt_amd.ResidentBatch(cells, labels)
for _ in range(6):
    rb.decode()
torch.cuda.synchronize()
print("ok", wl)
