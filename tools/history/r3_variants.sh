#!/bin/bash
# A/B of experiment builds (ldt_amd/libldt_<v>.so via LDT_LIBRARY) against the
# current build on one box: c2 bench lines (no CPU legs, no dataset leg),
# alternated twice. usage: bash tools/r3_variants.sh <tag> "<bench flags>" v1 [v2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; F=$2; shift 2
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
for rep in ${REPS:-1 2}; do
  for v in cur "$@"; do
    if [ $v = cur ]; then unset LDT_LIBRARY; else export LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --dataset-batches 0 $F > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -20 $O/${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1])
print('$v $rep', d['value'], d.get('value_host_input'), 'standalone', d.get('stages_standalone_ms'), 'pipe', d.get('stages_ms_per_step'))"
  done
done
unset LDT_LIBRARY
echo variants done
