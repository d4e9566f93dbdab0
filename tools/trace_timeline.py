"""Print a kernel/memcpy timeline (µs from the first event) from a rocprofv3
--kernel-trace [--memory-copy-trace] CSV directory: one line per dispatch
with its queue/stream, so overlap between pipelined batches is visible."""
import csv, glob, sys
d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
ev = []
for r in csv.DictReader(open(glob.glob(f"{d}/*kernel_trace.csv")[0])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Stream_Id"], r["Queue_Id"], r["Kernel_Name"].split("(")[0][-28:]))
for f in glob.glob(f"{d}/*memory_copy_trace.csv"):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M", r.get("Stream_Id", "?"), r.get("Queue_Id", "?"), r.get("Direction", "") + " " + r.get("Bytes", r.get("Size", ""))))
ev.sort()
ev = ev[-last:]
t0 = ev[0][0]
for s, e, k, st, q, n in ev:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {k} s{st} q{q} {n}")
