"""Summarise tools/pmc.sh output: mean counter value per kernel."""
import collections, csv, glob, sys
tag = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        res[r["Kernel_Name"][:28]][r["Counter_Name"]].append(float(r["Counter_Value"]))
want = sys.argv[2:] or None
for k, d in sorted(res.items()):
    if want and not any(w in k for w in want):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print("   %-24s %14.4g" % (c, sum(v) / len(v)))
