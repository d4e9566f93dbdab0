"""Diagnostic (not a test): one leg of the c2 bench for a rocprofv3
--kernel-trace --memory-copy-trace run: 'host' = host RecordBatches through the
pipelined to_tensor_fn (the bench's host leg), 'reg' = the same with the
batches' image buffers page-locked in place (register=True), 'resident' = ResidentBatches
through DecodePipeline. usage: host_trace.py host|reg|resident [depth]"""
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
from bench import make_cells  # noqa: E402

leg = sys.argv[1]
depth = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
bs = []
for k in range(2):
    cells, labels = make_cells("c2", 256, seed=k)
    if leg in ("host", "reg"):
        bs.append(pa.RecordBatch.from_arrays([pa.array(cells, pa.binary()), pa.array(np.asarray(labels, np.int64))],
                                             names=["image", "label"]))
    else:
        bs.append(ldt_amd.ResidentBatch(cells, labels, device=dev))
if leg in ("host", "reg"):
    fn = ldt_amd.make_to_tensor_fn(depth=depth, device=dev, register=leg == "reg")
    step = lambda b: fn(b)  # noqa: E731
else:
    pipe = ldt_amd.DecodePipeline(depth=depth, device=dev)
    step = lambda b: pipe.decode(b)  # noqa: E731
for i in range(10):
    step(bs[i % 2])
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(40):
    step(bs[i % 2])
torch.cuda.synchronize()
print(f"{leg}: ms/step {(time.perf_counter() - t0) * 1e3 / 40:.3f}", flush=True)
