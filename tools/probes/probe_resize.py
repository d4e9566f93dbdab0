"""Diagnostic (not a test): run the resize kernels alone for PMC profiling."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
import torch, ldt_amd
from ldt_amd import synth
which = sys.argv[1] if len(sys.argv) > 1 else "raw"
if which == "raw":
    x = torch.randint(0, 256, (256, 1024, 1024, 3), dtype=torch.uint8, device="cuda")
    for _ in range(5):
        ldt_amd.resize_raw(x, 1024, 1024, normalize=True)
else:
    cells, labels = synth.q90_512(256, seed=1)
    rb = ldt_amd.ResidentBatch(cells, labels)
    for _ in range(5):
        rb.decode()
torch.cuda.synchronize()
print("done", which)
