"""Diagnostic: parallel Huffman sync counters (rounds per workgroup, boundary
walks) for the c2/c1/c4 workloads at the default subsequence length."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lance-distributed-training_amd"))
import ldt_amd  # noqa: E402
from ldt_amd import _lib, synth  # noqa: E402

ctx = _lib.get_context(0)
ctx.set_option(_lib.OPT_DEBUG_COUNTERS, 1)
if os.environ.get("LDT_HUFF_WINDOW"):  # study: cap the LDS stream window (bytes)
    ctx.set_option(_lib.OPT_HUFF_WINDOW, int(os.environ["LDT_HUFF_WINDOW"]))
if os.environ.get("LDT_RESIZE_WG"):  # study: waves per k_resize4 workgroup
    ctx.set_option(_lib.OPT_RESIZE_WG_WAVES, int(os.environ["LDT_RESIZE_WG"]))
if os.environ.get("LDT_RESIZE_PCT"):  # study: resize bands (LDT_OPT_RESIZE_WAVES_PCT)
    ctx.set_option(_lib.OPT_RESIZE_WAVES_PCT, int(os.environ["LDT_RESIZE_PCT"]))
names = ["redo", "wgs", "rounds_sum", "rounds_max", "memo_hits", "write_syms", "write_wave_max", "fallbacks",
         "t_setup", "t_phase1", "t_rounds", "t_scan", "t_write", "need_lanes", "need_waves", "t_dc_idct"]
want = sys.argv[1:] or ["c2", "c1", "c4"]
ctx.set_option(_lib.OPT_PROFILE, 1)
for wl, fn, n in (("c2", synth.q90_512, 256), ("c1", synth.food101_like, 128), ("c4", synth.imagenet_like, 128)):
    if wl not in want:
        continue
    cells, labels = fn(n, seed=1000)
    rb = ldt_amd.ResidentBatch(cells, labels)

    def dec():
        try:
            rb.decode()
        except _lib.ImageDecodeError:
            # timing-only study builds (LDT_PROBE_TOLERATE=1) decode nothing valid
            if os.environ.get("LDT_PROBE_TOLERATE") != "1":
                raise

    dec()
    # standalone stage times (one batch in flight): 4 batches after a warm one
    ctx.stage_times(reset=True)
    for _ in range(4):
        dec()
    st = {k: round(v[0] / max(v[1], 1), 4) for k, v in ctx.stage_times(reset=True).items()}
    out = np.zeros(16, np.int32)
    ctx.check(ctx.lib.ldt_debug_counters(ctx.handle, out.ctypes.data, None), "dbg")
    d = dict(zip(names, out[:16].tolist()))
    w = max(d["wgs"], 1)
    d["rounds_avg"] = round(d["rounds_sum"] / w, 2)
    for k in ("t_setup", "t_phase1", "t_rounds", "t_scan", "t_write", "t_dc_idct"):
        d[k + "_us"] = round(d.pop(k) / w / 100.0, 2)  # 10 ns ticks per image
    d["need_lanes_per_round"] = round(d["need_lanes"] / max(d["rounds_sum"], 1), 1)
    d["need_waves_per_round"] = round(d["need_waves"] / max(d["rounds_sum"], 1), 2)
    # write pass: symbols per image, per lane, and the slowest lane of each wave
    d["write_syms_per_img"] = round(d["write_syms"] / w, 1)
    d["write_syms_per_lane"] = round(d["write_syms"] / w / 1024, 2)
    d["write_wave_max_per_lane"] = round(d["write_wave_max"] / w / 16, 2)
    d["stage_ms"] = st
    print(wl, d, flush=True)
