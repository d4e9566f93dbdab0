#!/bin/bash
# Quick GPU cycle: GPU tests, c2 bench, sync-round counters, depth-1 kernel
# stats. Stops at the first failure. usage: bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
K=${2:+-k "$2"}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $K > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python tools/probes/huff_rounds.py > $O/rounds.txt 2>&1 || { tail -5 $O/rounds.txt; exit 1; }
cat $O/rounds.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
head -c 400 $O/bench_c2.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --depth 1 --steps 30 --warmup 5 > $O/prof1.log 2>&1 || { tail -5 $O/prof1.log; exit 1; }
echo quick done
