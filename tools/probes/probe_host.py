"""Diagnostic (not a test): host wall time per DecodePipeline.decode call."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
import numpy as np, torch, ldt_amd
from ldt_amd import synth
dev = torch.device("cuda", 0)
bs = []
for k in range(2):
    cells, labels = synth.q90_512(256, seed=k)
    bs.append(ldt_amd.ResidentBatch(cells, labels, device=dev))
for depth in (1, 2, 3):
    pipe = ldt_amd.DecodePipeline(depth=depth, device=dev)
    for i in range(4):
        pipe.decode(bs[i % 2])
    torch.cuda.synchronize()
    ts = []
    t0 = time.perf_counter()
    for i in range(20):
        a = time.perf_counter()
        pipe.decode(bs[i % 2])
        ts.append((time.perf_counter() - a) * 1e3)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) * 1e3 / 20
    print("depth", depth, "ms/step", round(tot, 3), "host ms per call", [round(x, 2) for x in ts], flush=True)
# planner cost alone: a context with a tiny no-op? time ldt parse via serial calls on CPU side
