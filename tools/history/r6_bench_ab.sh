#!/bin/bash
# Resident c2 bench lines (K=100) of libldt builds, alternated on one box.
# usage: bash tools/history/r6_bench_ab.sh <tag> <reps> <lib.so>...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
REPS=$2
shift 2
mkdir -p $O
cd $R
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$lib timeout -k 10 200 python bench.py --only-resident --no-cpu-baseline --steps 100 > $O/bench_${lib}_$rep.json 2> $O/bench_${lib}_$rep.err || { tail -5 $O/bench_${lib}_$rep.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/bench_${lib}_$rep.json').read().strip().splitlines()[-1]);print('$lib', $rep, d['value'])"
  done
done
