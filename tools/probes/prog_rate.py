"""c2p resident decode rate (img/s) of the loaded libldt (LDT_LIBRARY) at
several pipeline depths: 256 progressive 512x512 q90 cells per batch, as
bench.py's c2p leg. usage: python tools/probes/prog_rate.py [depth ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import ldt_amd  # noqa: E402
from ldt_amd import _lib  # noqa: E402


def main():
    depths = [int(x) for x in sys.argv[1:]] or [7]
    dev = torch.device("cuda:0")
    cells, labels = bench.make_cells("c2p", 256, seed=0)
    rb = ldt_amd.ResidentBatch(cells, labels, device=dev)
    for d in depths:
        pipe = ldt_amd.DecodePipeline(depth=d, device=dev)
        for c in pipe.ctxs:
            c.set_option(_lib.OPT_PROFILE, 1)
        for _ in range(3 * d + 5):
            pipe.decode(rb)
        torch.cuda.synchronize(dev)
        pipe.stage_times(reset=True)
        K = 80
        t0 = time.perf_counter()
        for _ in range(K):
            pipe.decode(rb)
        torch.cuda.synchronize(dev)
        t = time.perf_counter() - t0
        st = pipe.stage_times(reset=True)
        pipe.check()
        huff = st["huffman"][0] / max(st["huffman"][1], 1)
        print(f"depth {d}: {256 * K / t:.0f} img/s, huffman {huff:.2f} ms per launch, "
              f"in flight {huff / (t / K * 1e3):.2f}", flush=True)
        del pipe


if __name__ == "__main__":
    main()
