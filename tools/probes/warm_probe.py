"""Diagnostic (not a test): where a short driver-style bench run (5 warm-up +
20 timed c2 steps) loses time against a long one. Prints host ms per decode
call of each timed step, torch allocator segment counts and the timed total,
for a fresh pipeline, twice in one process."""
import os
import sys
import time

R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "lance-distributed-training_amd"))
import torch  # noqa: E402

import ldt_amd  # noqa: E402
from bench import make_cells  # noqa: E402

dev = torch.device("cuda", 0)
batches = []
for k in range(2):
    cells, labels = make_cells("c2", 256, seed=k)
    batches.append(ldt_amd.ResidentBatch(cells, labels, device=dev))

for trial in range(3):
    pipe = ldt_amd.DecodePipeline(depth=3, device=dev)
    it = [0]

    def step():
        b = batches[it[0] % 2]
        it[0] += 1
        return pipe.decode(b)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    seg0 = torch.cuda.memory_stats(dev).get("segment.all.allocated", 0)
    ts = []
    t0 = time.perf_counter()
    for _ in range(20):
        a = time.perf_counter()
        step()
        ts.append((time.perf_counter() - a) * 1e3)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    seg1 = torch.cuda.memory_stats(dev).get("segment.all.allocated", 0)
    print(f"trial {trial}: total {(t2 - t0) * 1e3:.3f} ms (enqueue {(t1 - t0) * 1e3:.3f}, drain {(t2 - t1) * 1e3:.3f}), "
          f"new segments {seg1 - seg0}; host ms per call: {[round(x, 2) for x in ts]}", flush=True)
