#!/bin/bash
# Resident c2 bench A/B of (libldt build, extra bench args) pairs, alternated.
# usage: bash tools/ab_bench.sh <tag> <reps> "<lib.so>|<bench args>[|VAR=val ...]" ...
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
REPS=$2
shift 2
mkdir -p $O
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    lib=${spec%%|*}
    rest=${spec#*|}
    args=${rest%%|*}
    envs=""
    [ "$rest" != "$args" ] && envs=${rest#*|}
    f=$O/bench_${rep}_$(echo "$spec" | tr -c 'A-Za-z0-9._-' '_').json
    env $envs LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$lib timeout -k 10 200 python $R/bench.py --only-resident --no-cpu-baseline --steps 100 $args > $f 2> $f.err || { echo "FAIL $spec"; tail -3 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['stages_ms_per_step'])" $f "$spec" $rep
  done
done
