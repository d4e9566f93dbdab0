"""Diagnostic (not a test): parallel Huffman sync statistics per workload."""
import sys, os, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
import torch, ldt_amd
from ldt_amd import _lib, synth
ctx = _lib.get_context(0)
ctx.set_option(_lib.OPT_DEBUG_COUNTERS, 1)
# ldt_debug_counters layout (ldt_abi.cpp)
names = ["unused0", "wgs", "rounds_sum", "rounds_max", "memo_hits", "write_syms", "write_wave_max", "unused7",
         "t_setup", "t_phase1", "t_rounds", "t_scan", "t_write", "need_lanes", "need_waves"]
for wl, fn, n in (("c2", synth.q90_512, 64), ("c1", synth.food101_like, 64), ("c4", synth.imagenet_like, 64)):
    cells, labels = fn(n, seed=1)
    for S in (512, 1024, 2048):
        ctx.set_option(_lib.OPT_SUBSEQ_BITS, S)
        rb = ldt_amd.ResidentBatch(cells, labels)
        rb.decode()
        out = np.zeros(16, np.int32)
        ctx.check(ctx.lib.ldt_debug_counters(ctx.handle, out.ctypes.data, None), "dbg")
        print(wl, S, dict(zip(names, out[:15].tolist())), flush=True)
