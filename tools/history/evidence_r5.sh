#!/bin/bash
# Round-5 evidence on the GPU box (each part within one gpurun call; stops at
# the first failure).
#   A: GPU tests; the driver-shaped bench line (20 timed steps) and a 100-step
#      line; Huffman phase times; rocprofv3 kernel stats of the c2 resident
#      leg alone and of the c5 workload alone (the launches the lines'
#      rooflines are timed over).
#   B: per-kernel HBM traffic at c2 (FETCH_SIZE / WRITE_SIZE passes, depth 1);
#      PMC decode efficiency of the shipped kernels (tools/pmc.sh passes 1-3);
#      bench lines of c1 and c4.
# usage: bash tools/evidence_r5.sh <tag> A|B
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/ev_$T
mkdir -p $O
cd $R
if [ "$2" = "A" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_c2_k20.json 2> $O/bench_c2_k20.err || { tail -5 $O/bench_c2_k20.err; exit 1; }
  echo "c2 K=20: $(head -c 200 $O/bench_c2_k20.json)"
  timeout -k 10 600 python bench.py --no-workload-legs > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
  echo "c2 K=100: $(head -c 200 $O/bench_c2.json)"
  timeout -k 10 120 python3 tools/probes/huff_rounds.py > $O/huff_rounds.txt 2>&1 || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --only-resident --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --workload c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { tail -5 $O/prof_c5.log; exit 1; }
  echo A done
else
  cd /tmp && export TMPDIR=/tmp
  mkdir -p $O/traffic
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/traffic/$c -o run -- python3 $R/bench.py --steps 4 --warmup 1 --depth 1 --only-resident --no-cpu-baseline > $O/traffic/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $O/traffic/$c.log; exit 1; }
  done
  python3 $R/tools/traffic_all.py $O/traffic > $O/traffic_c2_perkernel.txt && cat $O/traffic_c2_perkernel.txt
  python3 $R/tools/traffic_summary.py $O/traffic c2 > $O/traffic_c2.json
  cd $R
  PROBE=pmc_c2.py bash $R/tools/pmc.sh ${T}_dec c2 1 2 3 > /dev/null || exit 1
  python3 $R/tools/decode_eff.py $R/gpurun_out/pmc_${T}_dec c2 > $O/pmc_c2_decode.json
  for w in c1 c4; do
    timeout -k 10 400 python bench.py --workload $w --cpu-workers 8,16 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
    echo "$w: $(head -c 200 $O/bench_$w.json)"
  done
  echo B done
fi
