"""Diagnostic (not a test): where the host time of the pipelined to_tensor_fn
goes, per call: the ticket check (check_slot), the C decode call
(decode_arrow) and the rest of the Python wrapper, plus the C++ host phases.
usage: python host_calls2.py [c2] [depth] [reg|copy] [copy threads]
env LDT_P_MODE / LDT_P_BIND / LDT_P_NT: LDT_OPT_COPY_MODE / _BIND / _NT."""
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
from ldt_amd import _lib, transforms  # noqa: E402
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
acc = {"check": 0.0, "decode_arrow": 0.0}
orig_check, orig_dec = transforms.DecodePipeline.check_slot, transforms.decode_arrow


def check_slot(self, i):
    a = time.perf_counter()
    orig_check(self, i)
    acc["check"] += time.perf_counter() - a


def decode_arrow(*args, **kw):
    a = time.perf_counter()
    r = orig_dec(*args, **kw)
    acc["decode_arrow"] += time.perf_counter() - a
    return r


transforms.DecodePipeline.check_slot = check_slot
transforms.decode_arrow = decode_arrow
fn = ldt_amd.make_to_tensor_fn(depth=depth, device=dev, register=len(sys.argv) > 3 and sys.argv[3] == "reg")
fn.pipeline.set_option(_lib.OPT_HOST_TIMING, 1)
if len(sys.argv) > 4:
    fn.pipeline.set_option(_lib.OPT_COPY_THREADS, int(sys.argv[4]))
for env, opt in (("LDT_P_MODE", _lib.OPT_COPY_MODE), ("LDT_P_BIND", _lib.OPT_COPY_BIND), ("LDT_P_NT", _lib.OPT_COPY_NT)):
    if os.environ.get(env):
        fn.pipeline.set_option(opt, int(os.environ[env]))
for i in range(12):
    fn(bs[i % 2])
torch.cuda.synchronize()
fn.pipeline.host_times(reset=True)
for k in acc:
    acc[k] = 0.0
N = 60
t0 = time.perf_counter()
walls = []
for i in range(N):
    a = time.perf_counter()
    fn(bs[i % 2])
    walls.append(time.perf_counter() - a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
fn.check()
us, n = fn.pipeline.host_times(reset=True)
print(f"[{' '.join(sys.argv[1:])}] {N} calls: host loop {(t1 - t0) * 1e6 / N:.1f} us/call, until GPU done {(t2 - t0) * 1e6 / N:.1f} us/call")
print(f"  per call: check_slot {acc['check'] * 1e6 / N:.1f}, decode_arrow {acc['decode_arrow'] * 1e6 / N:.1f}, "
      f"rest {(t1 - t0 - acc['check'] - acc['decode_arrow']) * 1e6 / N:.1f} us")
print("  C++ phases us/call " + " ".join(f"{k}={v / max(n, 1):.1f}" for k, v in us.items()))
print("  host_info", fn.pipeline.ctxs[0].host_info())
print("  wall percentiles us", [round(float(np.percentile(walls, q)) * 1e6, 1) for q in (10, 50, 90, 99)])
