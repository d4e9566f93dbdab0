#!/bin/bash
# WRITE_SIZE per kernel (one rocprofv3 --pmc pass each) of the current build and
# of experiment builds. usage: bash tools/r3_wsize.sh <tag> v1 [v2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in cur "$@"; do
  if [ $v = cur ]; then unset LDT_LIBRARY; else export LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_$v.so; fi
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/ws_$v -o run -- python3 $R/bench.py --steps 4 --warmup 1 --depth 1 --no-cpu-baseline --dataset-batches 0 > $O/ws_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/ws_$v.log; exit 1; }
  python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("$O/ws_$v/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "WRITE_SIZE":
            acc[r["Kernel_Name"][:24]].append(float(r["Counter_Value"]) * 1024)
print("$v", {k: round(sum(x) / len(x) / 1e6, 1) for k, x in acc.items() if "ldt" in k})
PY
done
unset LDT_LIBRARY
echo wsize done
