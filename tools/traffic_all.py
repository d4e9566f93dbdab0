"""Per-kernel mean HBM traffic from tools/traffic.sh output (all kernels).
usage: python tools/traffic_all.py gpurun_out/traffic_<tag>"""
import collections, csv, glob, sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{d}/{c}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                acc[r["Kernel_Name"][:40]][c].append(float(r["Counter_Value"]) * 1024)
print("%-40s %6s %12s %12s %12s" % ("kernel", "n", "fetch x2 MB", "write MB", "total MB"))
for k, v in sorted(acc.items()):
    f = 2 * sum(v["FETCH_SIZE"]) / max(len(v["FETCH_SIZE"]), 1)
    w = sum(v["WRITE_SIZE"]) / max(len(v["WRITE_SIZE"]), 1)
    print("%-40s %6d %12.1f %12.1f %12.1f" % (k, len(v["FETCH_SIZE"]), f / 1e6, w / 1e6, (f + w) / 1e6))
