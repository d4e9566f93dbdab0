#!/bin/bash
# A/B of the resize wave target (LDT_RESIZE_WAVES_PCT, % of one full wave of
# waves on the GPU) per workload. usage on the GPU box: bash tools/resize_waves_ab.sh "c2 c4" "100 150 200" [reps]
set -o pipefail
mkdir -p gpurun_out/rw
for w in $1; do
for rep in ${3:-1 2}; do
  for p in $2; do
    LDT_RESIZE_WAVES_PCT=$p timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/rw/${w}_p${p}_$rep.json 2> gpurun_out/rw/${w}_p${p}_$rep.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/rw/${w}_p${p}_$rep.json')); print('$w pct $p $rep', d['value'], d['stages_standalone_ms']['resize'], d['stages_ms_per_step']['resize'])"
  done
done
done
