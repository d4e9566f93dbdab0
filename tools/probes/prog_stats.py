"""Diagnostic (library built with -DLDT_PROG_STATS, e.g. LDT_LIBRARY=
ldt_amd/libldt_pstats.so): the luma AC chain's time split in k_prog for one
c2p batch (512x512 q90 progressive), in microseconds per image."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
import ldt_amd  # noqa: E402
from ldt_amd import _lib, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ctx = _lib.get_context(0)
ctx.set_option(_lib.OPT_DEBUG_COUNTERS, 1)
cells, labels = synth.q90_512(n, seed=0, progressive=True)
rb = ldt_amd.ResidentBatch(cells, labels)
for rep in range(2):
    rb.decode()
    out = np.zeros(16, np.int32)
    ctx.check(ctx.lib.ldt_debug_counters(ctx.handle, out.ctypes.data, None), "dbg")
    nimg = max(int(out[15]), 1)
    us = lambda i: round(float(out[i]) / nimg / 100.0, 1)  # noqa: E731
    print({"images": nimg,
           "scan_us": [us(i) for i in range(4)], "wait_us": [us(4 + i) for i in range(4)],
           "decode_us": [us(8 + i) for i in range(4)],
           "last_scan_per_image": {"symbols": int(out[12]) // nimg, "corr_bits": int(out[13]) // nimg,
                                   "fills": int(out[14]) // nimg}}, flush=True)

if os.environ.get("LDT_PROG_STATS_MODE") == "2":
    # library built with -DLDT_PROG_STATS=2: every chain's scan times
    print("per image (us): chain 0 = DC scans, 1 = luma AC, 2/3 = chroma AC; scan order within the chain")
    for ch in range(4):
        print(ch, [round(float(out[4 * ch + j]) / n / 100.0, 1) for j in range(4)])
