"""Diagnostic: does hipMemcpyAsync (pinned host -> device) block the host while
the stream is busy? Times the enqueue call behind a long kernel."""
import time

import torch

torch.cuda.init()
big = torch.empty(1 << 28, device="cuda")
for stream_kind in ("default", "side"):
    st = torch.cuda.current_stream() if stream_kind == "default" else torch.cuda.Stream()
    with torch.cuda.stream(st):
        for nbytes in (4096, 65536, 262144, 1 << 20, 4 << 20):
            src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
            dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
            res = []
            for rep in range(5):
                torch.cuda.synchronize()
                for _ in range(20):
                    big.mul_(1.0001)  # ~20 x 2 GB of HBM traffic queued
                a = time.perf_counter()
                dst.copy_(src, non_blocking=True)
                b = time.perf_counter()
                torch.cuda.synchronize()
                c = time.perf_counter()
                res.append(((b - a) * 1e6, (c - a) * 1e6))
            res.sort()
            print(f"{stream_kind:7s} {nbytes:8d} B: enqueue {res[2][0]:9.1f} us (queue drain {res[2][1]:9.1f} us)", flush=True)
