"""Concurrency of pipelined batches from a rocprofv3 --kernel-trace CSV
directory: per kernel name, its mean duration and the share of its time that
overlaps another stream's dispatch; the union of busy time per step."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
ev = []
for r in csv.DictReader(open(glob.glob(f"{d}/*kernel_trace.csv")[0])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"],
               r["Kernel_Name"].split("(")[0].replace("void ", "")[-24:]))
ev.sort()
ev = ev[len(ev) // 3:]  # steady state
t0, t1 = ev[0][0], max(e for _, e, _, _ in ev)
dur = collections.defaultdict(list)
ovl = collections.defaultdict(int)
for i, (s, e, st, n) in enumerate(ev):
    dur[n].append(e - s)
    cover = []
    for s2, e2, st2, n2 in ev:
        if st2 != st and s2 < e and e2 > s:
            cover.append((max(s, s2), min(e, e2)))
    cover.sort()
    tot, cur_s, cur_e = 0, None, None
    for a, b in cover:
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        tot += cur_e - cur_s
    ovl[n] += tot
busy = 0
cs, ce = None, None
for s, e, _, _ in ev:
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"window {(t1 - t0) / 1e3:.1f} us, busy (any kernel) {busy / 1e3:.1f} us ({busy / (t1 - t0):.2%})")
for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n:26s} n={len(v):4d} mean {sum(v) / len(v) / 1e3:8.1f} us  overlapped {ovl[n] / max(sum(v), 1):.0%}")
