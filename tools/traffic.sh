#!/bin/bash
# HBM traffic of the roofline kernel from PMC counters, one rocprofv3 --pmc
# pass per counter (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot
# share a pass), over the bench command itself at depth 1.
# usage: bash tools/traffic.sh <workload> <tag>   (run on the GPU box)
R=$GRAFT_REPO_ROOT
W=$1
T=$2
OUT=$R/gpurun_out/traffic_$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 $R/bench.py --workload $W --steps 4 --warmup 1 --depth 1 --no-cpu-baseline > $OUT/$c.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc $c failed rc=$rc"; tail -5 $OUT/$c.log; exit $rc; fi
done
python3 $R/tools/traffic_summary.py $OUT $W > $OUT/summary.json && cat $OUT/summary.json
