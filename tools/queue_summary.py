"""Per (queue, stream): k_prog dispatches and their busy time, from
rocprofv3 --kernel-trace CSVs (tools/history/c2p_queue_trace.sh)."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "k_prog" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = collections.defaultdict(list)
    for r in rows:
        by[(r["Queue_Id"], r["Stream_Id"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
    t1 = max(int(r["End_Timestamp"]) for r in rows) if rows else 0
    print(d, "k_prog dispatches", len(rows), "span ms", round((t1 - t0) / 1e6, 1))
    for k, v in sorted(by.items()):
        print("  queue", k[0], "stream", k[1], "n", len(v), "avg ms", round(sum(v) / len(v) / 1e6, 2))
