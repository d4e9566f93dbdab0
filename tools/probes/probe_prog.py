"""Decodes one c2p batch (512x512 q90 progressive, 256 images) a few times;
for PMC/kernel-trace runs of k_prog. GPU box only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lance-distributed-training_amd"))
import torch  # noqa: E402

import ldt_amd  # noqa: E402
from ldt_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
cells, labels = synth.q90_512(n, seed=0, progressive=True)
rb = synth.arrow_batch(cells, labels)
for _ in range(2):
    ldt_amd.decode_tensor_image(rb, device="cuda:0")
torch.cuda.synchronize()
print("ok", n, sum(len(c) for c in cells) / n)
