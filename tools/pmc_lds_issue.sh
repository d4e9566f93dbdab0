#!/bin/bash
# LDS and VALU issue counters per kernel of the c2 decode (tools/probes/pmc_c2.py,
# one batch at a time), one rocprofv3 --pmc pass (8 SQ counters).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmclds
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_ANY --output-format csv -d $O -o run -- python3 $R/tools/probes/pmc_c2.py c2 > $O/out.txt 2>&1 || { tail -5 $O/out.txt; exit 1; }
python3 - $O <<'PY'
import collections, csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][-40:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    wc = c["SQ_WAVE_CYCLES"] or 1
    print(k, {n: round(v / wc, 3) for n, v in sorted(c.items()) if n.startswith(("SQ_WAIT", "SQ_ACTIVE"))},
          "LDS insts per VALU inst", round(c["SQ_INSTS_LDS"] / max(c["SQ_INSTS_VALU"], 1), 3))
PY
