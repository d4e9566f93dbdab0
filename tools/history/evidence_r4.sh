#!/bin/bash
# Round-4 evidence on the GPU box (each part within one gpurun call; stops at
# the first failure).
#   A: GPU tests; the default bench line (c2, CPU legs); Huffman phase times;
#      rocprofv3 kernel stats of the c2 resident leg alone (the launches the
#      line's roofline is timed over: --only-resident); per-kernel HBM traffic
#      (FETCH_SIZE / WRITE_SIZE passes, depth 1).
#   B: PMC decode efficiency of the shipped kernels at c2 (VALU, LDS bank
#      conflicts; tools/pmc.sh passes 1-3, one batch at a time); bench lines of
#      c1, c4, c5, c2p with their CPU legs.
# usage: bash tools/evidence_r4.sh <tag> A|B
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/ev_$T
mkdir -p $O
cd $R
if [ "$2" = "A" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 500 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
  echo "c2: $(head -c 300 $O/bench_c2.json)"
  timeout -k 10 120 python3 tools/probes/huff_rounds.py > $O/huff_rounds.txt 2>&1 || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --only-resident --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
  mkdir -p $O/traffic
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/traffic/$c -o run -- python3 $R/bench.py --steps 4 --warmup 1 --depth 1 --only-resident --no-cpu-baseline > $O/traffic/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $O/traffic/$c.log; exit 1; }
  done
  python3 $R/tools/traffic_all.py $O/traffic > $O/traffic_c2_perkernel.txt && cat $O/traffic_c2_perkernel.txt
  python3 $R/tools/traffic_summary.py $O/traffic c2 > $O/traffic_c2.json
else
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -x -q --timeout 120 --timeout-method thread -k "fused or corrupt or golden or config_batches or fullbatch or huffman or restart or marker or progressive" > $O/pytest_b.log 2>&1 || { tail -30 $O/pytest_b.log; exit 1; }
  tail -1 $O/pytest_b.log
  PROBE=../tools/probes/pmc_c2.py bash $R/tools/pmc.sh ${T}_dec c2 1 2 3 > /dev/null || exit 1
  python3 $R/tools/decode_eff.py $R/gpurun_out/pmc_${T}_dec c2 > $O/pmc_c2_decode.json
  for w in c1 c4 c5 c2p; do
    timeout -k 10 400 python bench.py --workload $w --cpu-workers 8,16 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
    echo "$w: $(head -c 200 $O/bench_$w.json)"
  done
fi
echo evidence $2 done
