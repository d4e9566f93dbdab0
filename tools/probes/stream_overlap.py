"""Diagnostic: how many of torch's pool streams run kernels concurrently on
this process's HIP hardware queues (GPU_MAX_HW_QUEUES)? Launches one
torch.cuda._sleep kernel (one wave) per stream and times the lot; also
tries streams from the high-priority pool and ExternalStreams."""
import time

import torch

dev = torch.device("cuda:0")
cyc = 20_000_000  # ~8-10 ms per sleep kernel


def run(streams, label):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for s in streams:
        with torch.cuda.stream(s):
            torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


with torch.cuda.stream(torch.cuda.Stream(dev)):
    torch.cuda._sleep(1000)
torch.cuda.synchronize()
one = run([torch.cuda.current_stream(dev)], "one")
print(f"one sleep kernel: {one:.1f} ms", flush=True)
for n in (2, 3, 4, 5, 6, 8):
    ss = [torch.cuda.Stream(dev) for _ in range(n)]
    run(ss, "warm")
    t = run(ss, "pool")
    hp = [torch.cuda.Stream(dev, priority=-1 if k % 2 else 0) for k in range(n)]
    run(hp, "warm")
    t2 = run(hp, "mixed")
    print(f"{n} pool streams: {t:.1f} ms ({t / one:.2f} x one); alternating priority: {t2:.1f} ms ({t2 / one:.2f} x)",
          flush=True)
