"""Diagnostic (not a test): per-call wall time and host phases of the pipelined
to_tensor_fn on host RecordBatches (the bench's host leg), warm-up included, to
see where short runs lose time. usage: python host_calls.py [c2] [depth]"""
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
from ldt_amd import _lib  # noqa: E402
from bench import WORKLOADS, make_cells  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "c2"
depth = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
B = WORKLOADS[w]["batch"]
bs = []
for k in range(2):
    cells, labels = make_cells(w, B, seed=k)
    bs.append(pa.RecordBatch.from_arrays([pa.array(cells, pa.binary()), pa.array(np.asarray(labels, np.int64))],
                                         names=["image", "label"]))
fn = ldt_amd.make_to_tensor_fn(depth=depth, device=dev)
fn.pipeline.set_option(_lib.OPT_HOST_TIMING, 1)
rows = []
t00 = time.perf_counter()
for i in range(60):
    a = time.perf_counter()
    fn(bs[i % 2])
    wall = (time.perf_counter() - a) * 1e6
    us, n = fn.pipeline.host_times(reset=True)
    rows.append((i, wall, us))
torch.cuda.synchronize()
fn.check()
for i, wall, us in rows:
    print(f"call {i:2d} wall {wall:8.1f} us  " + " ".join(f"{k}={v:.0f}" for k, v in us.items()), flush=True)
print(f"total {(time.perf_counter() - t00) * 1e3:.2f} ms for 60 calls")
