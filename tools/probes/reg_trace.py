"""Diagnostic (not a test): one host-input leg (copy or registered) for a
rocprofv3 --kernel-trace --memory-copy-trace run. usage: reg_trace.py c2 registered"""
import os
import sys
import time

R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "lance-distributed-training_amd"))
import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import torch  # noqa: E402

import ldt_amd  # noqa: E402
from bench import WORKLOADS, make_cells  # noqa: E402

w = sys.argv[1]
leg = sys.argv[2]
dev = torch.device("cuda", 0)
B = WORKLOADS[w]["batch"]
bs = []
for k in range(2):
    cells, labels = make_cells(w, B, seed=k)
    bs.append(pa.RecordBatch.from_arrays([pa.array(cells, pa.binary()), pa.array(np.asarray(labels, np.int64))],
                                         names=["image", "label"]))
if leg == "registered":
    for b in bs:
        ldt_amd.register_host(b.column(0), device=dev)
pipe = ldt_amd.DecodePipeline(depth=3, device=dev)
for i in range(6):
    pipe.decode(bs[i % 2])
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(40):
    pipe.decode(bs[i % 2])
torch.cuda.synchronize()
print(f"{leg}: ms/step {(time.perf_counter() - t0) * 1e3 / 40:.3f}", flush=True)
pipe.check()
if leg == "registered":
    for b in bs:
        ldt_amd.unregister_host(b.column(0))
