#!/bin/bash
# Full default bench (with CPU baseline) + depth-3 kernel trace of the same
# command. usage: bash tools/gpu_bench.sh <tag> [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 3000 $O/bench.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof3 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/prof3.log 2>&1 || { tail -5 $O/prof3.log; exit 1; }
python3 $R/tools/overlap.py $O/prof3 > $O/overlap.txt && cat $O/overlap.txt
echo bench done
