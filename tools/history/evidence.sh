#!/bin/bash
# Round evidence on the GPU box: GPU tests, benches with CPU baselines for
# every workload, rocprofv3 kernel-trace stats of the default (c2) bench, PMC
# HBM traffic of the resize kernel (c2, c5). Stops at the first failure.
# usage: bash tools/evidence.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/ev_$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for w in c2 c1 c4 c5 c2p; do
  timeout -k 10 300 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  echo "$w: $(head -c 200 $O/bench_$w.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
for w in c2 c5; do
  bash $R/tools/traffic.sh $w ${T}_$w > /dev/null || exit 1
  cp $R/gpurun_out/traffic_${T}_$w/summary.json $O/traffic_$w.json
done
echo evidence done
