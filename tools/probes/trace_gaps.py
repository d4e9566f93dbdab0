"""Diagnostic: from a rocprofv3 kernel (+ memory-copy) trace directory, the
steady-state period between k_huff_image launches, the fraction of that time
some kernel runs, the H2D copies (count, duration, bytes/s) and how much of
their time overlaps kernels. usage: trace_gaps.py <dir> [steps]"""
import csv
import glob
import sys

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-22:], r["Stream_Id"])
      for r in csv.DictReader(open(glob.glob(f"{d}/*kernel_trace.csv")[0]))]
cp = []
for f in glob.glob(f"{d}/*memory_copy_trace.csv"):
    for r in csv.DictReader(open(f)):
        cp.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", ""), r.get("Stream_Id", "")))
ks.sort()
huff = [s for s, e, n, _ in ks if "huff_image" in n]
lo, hi = huff[-steps - 1], huff[-1]
print(f"period between Huffman launches over the last {steps}: {(hi - lo) / steps / 1e3:.1f} us")


def busy(intervals):
    ev = sorted([(max(s, lo), 1) for s, e in intervals if e > lo and s < hi] +
                [(min(e, hi), -1) for s, e in intervals if e > lo and s < hi])
    tot, cur, last = 0, 0, lo
    for t, dd in ev:
        if cur > 0:
            tot += t - last
        cur += dd
        last = t
    return tot / (hi - lo)


print(f"kernel-busy fraction {busy([(s, e) for s, e, _, _ in ks]):.3f}")
h2d = [(s, e) for s, e, dirn, _ in cp if "HOST_TO_DEVICE" in dirn and e > lo and s < hi]
if h2d:
    durs = sorted(e - s for s, e in h2d)
    print(f"H2D copies in window: {len(h2d)}, median {durs[len(durs) // 2] / 1e3:.1f} us, "
          f"busy fraction {busy(h2d):.3f}")
# per-kernel mean durations in the window
agg = {}
for s, e, n, _ in ks:
    if s >= lo and s < hi:
        a = agg.setdefault(n, [0, 0])
        a[0] += e - s
        a[1] += 1
for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0]):
    print(f"  {n:24s} n={c:3d} mean {t / c / 1e3:7.1f} us")
