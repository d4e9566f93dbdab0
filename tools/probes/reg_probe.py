"""Diagnostic (not a test): host phase times per decode call (LDT_HOST_TIMING)
and ms per step for host RecordBatches, copy path vs registered
(ldt_register_host), on one workload. usage: python reg_probe.py c1"""
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

w = sys.argv[1] if len(sys.argv) > 1 else "c1"
dev = torch.device("cuda", 0)
B = WORKLOADS[w]["batch"]
bs = []
for k in range(2):
    cells, labels = make_cells(w, B, seed=k)
    bs.append(pa.RecordBatch.from_arrays([pa.array(cells, pa.binary()), pa.array(np.asarray(labels, np.int64))],
                                         names=["image", "label"]))


from ldt_amd import _lib  # noqa: E402


def run(tag, threads=-1):
    pipe = ldt_amd.DecodePipeline(depth=3, device=dev)
    pipe.set_option(_lib.OPT_HOST_TIMING, 1)
    pipe.set_option(_lib.OPT_COPY_THREADS, threads)
    for i in range(6):
        pipe.decode(bs[i % 2])
    torch.cuda.synchronize()
    calls = []
    t0 = time.perf_counter()
    for i in range(60):
        a = time.perf_counter()
        pipe.decode(bs[i % 2])
        calls.append((time.perf_counter() - a) * 1e3)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) * 1e3 / 60
    pipe.check()
    us, n = pipe.host_times(reset=True)
    # the first 6 warm-up calls are included in the host phase sums
    print(f"{tag}: ms/step {tot:.3f}  host ms/call median {np.median(calls):.3f} max {max(calls):.3f}  "
          f"phases us/call " + " ".join(f"{k}={v / max(n, 1):.1f}" for k, v in us.items()), flush=True)


run("copy")
for t in (0, 2, 8, 12):
    run(f"copy threads={t}", t)
for b in bs:
    ldt_amd.register_host(b.column(0), device=dev)
run("registered")
for b in bs:
    ldt_amd.unregister_host(b.column(0))
run("copy again")
