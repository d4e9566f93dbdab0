#!/bin/bash
# Round-2 evidence on the GPU box: GPU tests, benches (CPU baselines) for every
# workload, rocprofv3 kernel stats of the default bench, PMC HBM traffic of the
# resize kernel (c2, c5), PMC decode-efficiency counters (VALU, LDS bank
# conflicts) per kernel at c2. Stops at the first failure.
# usage: bash tools/evidence_r2.sh <tag> [steps]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/ev_$T
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for w in c2 c1 c4 c5 c2p; do
  timeout -k 10 400 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  echo "$w: $(head -c 160 $O/bench_$w.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
python3 $R/tools/overlap.py $O/prof_c2 > $O/overlap_c2.txt
for w in c2 c5; do
  bash $R/tools/traffic.sh $w ${T}_$w > /dev/null || exit 1
  cp $R/gpurun_out/traffic_${T}_$w/summary.json $O/traffic_$w.json
done
PROBE=../tools/probes/pmc_c2.py bash $R/tools/pmc.sh ${T}_dec c2 1 2 3 > /dev/null || exit 1
python3 $R/tools/decode_eff.py $R/gpurun_out/pmc_${T}_dec c2 > $O/pmc_c2_decode.json
timeout -k 10 120 python3 $R/tools/probes/huff_rounds.py > $O/huff_rounds.txt 2>&1
echo evidence done
