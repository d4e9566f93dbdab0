#!/bin/bash
# Diagnostic: bench value against warm-up and step counts (short, driver-style
# runs vs the default). usage on the GPU box: bash tools/ceil_first_ab.sh
set -o pipefail
mkdir -p gpurun_out/cf
for rep in 1 2; do
  for ws in "5 20" "20 20" "5 100" "50 20"; do
    set -- $ws
    timeout -k 10 200 python bench.py --warmup $1 --steps $2 --no-cpu-baseline > gpurun_out/cf/w$1_s$2_$rep.json 2> gpurun_out/cf/w$1_s$2_$rep.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/cf/w$1_s$2_$rep.json')); print('w$1 s$2 $rep', d['value'], d['ms_per_step'])"
  done
done
