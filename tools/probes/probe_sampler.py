"""Times the DistributedSampler index kernels (ldt_distributed_indices) against
torch's CPU DistributedSampler for FOOD101 (75,750) and ImageNet (1,281,167)
rows, W=8. Prints one JSON line per size. GPU box only."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lance-distributed-training_amd"))

import torch  # noqa: E402
from torch.utils.data import DistributedSampler as TorchDS  # noqa: E402

from ldt_amd.sampler import device_distributed_indices  # noqa: E402

for n in (75750, 1281167):
    W = 8
    for _ in range(2):
        device_distributed_indices(n, W, 3, True, 7, False)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 10
    ev[0].record()
    for k in range(reps):
        t = device_distributed_indices(n, W, 3, True, 7 + k, False)
    ev[1].record()
    torch.cuda.synchronize()
    gpu_ms = ev[0].elapsed_time(ev[1]) / reps
    s = TorchDS(range(n), num_replicas=W, rank=3, seed=7)
    t0 = time.perf_counter()
    for k in range(3):
        s.set_epoch(k)
        list(s)
    cpu_ms = (time.perf_counter() - t0) / 3 * 1e3
    print(json.dumps({"n": n, "W": W, "gpu_ms": round(gpu_ms, 3), "torch_cpu_ms": round(cpu_ms, 3)}))
