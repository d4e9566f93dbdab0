"""Diagnostic: host time per DecodePipeline.decode call (enqueue only) vs the
GPU time per batch, c2 resident batches, depth 3."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
import torch  # noqa: E402

import ldt_amd  # noqa: E402
from ldt_amd import synth  # noqa: E402

batches = []
for k in range(2):
    cells, labels = synth.q90_512(256, seed=1000 + k)
    batches.append(ldt_amd.ResidentBatch(cells, labels))
for prof in (False, True):
    pipe = ldt_amd.DecodePipeline(depth=3, profile=prof)
    for k in range(10):
        pipe.decode(batches[k % 2])
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for k in range(100):
        a = time.perf_counter()
        pipe.decode(batches[k % 2])
        host.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.sort()
    print(f"profile={prof}: host per call median {host[50]*1e3:.3f} ms p90 {host[90]*1e3:.3f} ms; "
          f"enqueue loop {(t1-t0)*10:.3f} ms/step; total {(t2-t0)*10:.3f} ms/step", flush=True)
# host planner alone: ldt_decode_batch on a resident batch with sync off, no stream waits
ctx = ldt_amd._lib.get_context(0)
