"""Mean PMC counter values per kernel from tools/pmc.sh passes, one line per
counter (A/B of builds: diff two of these).
usage: python tools/pmc_raw.py <pmc dir> [kernel substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ldt::", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(acc.items()):
    if want not in k:
        continue
    for n, v in sorted(c.items()):
        print(f"{k:24s} {n:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
