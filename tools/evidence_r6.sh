#!/bin/bash
# Round-6 evidence on the GPU box, of the shipped kernels (each part within
# one gpurun call; stops at the first failure). The PMC summaries it writes
# carry the kernel sources' digest (bench.csrc_digest), which bench.py checks
# before it quotes them.
#   A: GPU tests; the driver-shaped bench line (20 timed steps) and a
#      100-step line; Huffman phase times; rocprofv3 kernel stats of the c2
#      resident leg alone and of the c5 workload alone.
#   B: HBM traffic: FETCH_SIZE / WRITE_SIZE passes over the c2 resident leg and
#      the c5 workload at depth 1 (per kernel, and the resize's summaries
#      traffic_c2.json / traffic_c5.json); PMC decode efficiency (tools/pmc.sh
#      passes 1-3, one c2 batch at a time).
# usage: bash tools/evidence_r6.sh <tag> A|B
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/ev_$T
mkdir -p $O
cd $R
if [ "$2" = "A" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_c2_k20.json 2> $O/bench_c2_k20.err || { tail -5 $O/bench_c2_k20.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c2_k20.json'));print('K=20', json.dumps(d['summary']))"
  timeout -k 10 600 python bench.py --no-workload-legs > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('K=100', json.dumps(d['summary']))"
  timeout -k 10 120 python3 tools/probes/huff_rounds.py > $O/huff_rounds.txt 2>&1 || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --only-resident --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --workload c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { tail -5 $O/prof_c5.log; exit 1; }
  echo A done
else
  cd /tmp && export TMPDIR=/tmp
  for w in c2 c5; do
    mkdir -p $O/traffic_$w
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/traffic_$w/$c -o run -- python3 $R/bench.py --workload $w --steps 4 --warmup 1 --depth 1 --only-resident --no-cpu-baseline > $O/traffic_$w/$c.log 2>&1 || { echo "pmc $w $c failed"; tail -5 $O/traffic_$w/$c.log; exit 1; }
    done
    python3 $R/tools/traffic_summary.py $O/traffic_$w $w > $O/traffic_$w.json || exit 1
  done
  python3 $R/tools/traffic_all.py $O/traffic_c2 > $O/traffic_c2_perkernel.txt && cat $O/traffic_c2_perkernel.txt
  cd $R
  PROBE=pmc_c2.py bash $R/tools/pmc.sh ${T}_dec c2 1 2 3 > /dev/null || exit 1
  python3 $R/tools/decode_eff.py $R/gpurun_out/pmc_${T}_dec c2 > $O/pmc_c2_decode.json
  echo B done
fi
