"""Pipeline overlap from a rocprofv3 --kernel-trace CSV directory: over the
last `ms` milliseconds of the trace, the time each kernel family has at least
one dispatch running, and the time families run together (e.g. k_idct beside
k_huff_image). usage: python tools/overlap_kernels.py <trace dir> [ms]"""
import csv
import glob
import sys

d = sys.argv[1]
ms = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
fams = ("k_huff_image", "k_idct", "k_resize4", "copyBuffer")
ev = []
for r in csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])):
    n = r["Kernel_Name"]
    f = next((x for x in fams if x in n), None)
    if f:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f))
t1 = max(e for _, e, f in ev if f != "copyBuffer")  # end of the last decode step
t0 = t1 - int(ms * 1e6)
pts = sorted({t for s, e, _ in ev for t in (s, e) if t0 <= t <= t1} | {t0, t1})
busy = {f: 0 for f in fams}
combo = {}
for a, b in zip(pts, pts[1:]):
    act = tuple(f for f in fams if any(s <= a and e >= b for s, e, g in ev if g == f))
    for f in act:
        busy[f] += b - a
    combo[act] = combo.get(act, 0) + b - a
span = t1 - t0
print(f"window {ms} ms")
for f in fams:
    print(f"  {f:14s} running {busy[f] / span:6.1%} of the window")
for act, t in sorted(combo.items(), key=lambda x: -x[1])[:8]:
    print(f"  {' + '.join(act) or '(idle)':45s} {t / span:6.1%}")
