#!/bin/bash
# A/B on one GPU box: gpu tests on the current build, then each workload with
# the current libldt.so and with ldt_amd/libldt_prev.so (LDT_LIBRARY), twice,
# interleaved. usage: bash tools/ab.sh "c2 c5" [extra bench args]
set -o pipefail
R=$PWD
mkdir -p gpurun_out/ab
[ -n "$NOTEST" ] || timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
PREV=$R/lance-distributed-training_amd/ldt_amd/libldt_prev.so
for w in $1; do
  for rep in ${REPS:-1 2}; do
    for v in new prev; do
      if [ $v = prev ]; then export LDT_LIBRARY=$PREV; else unset LDT_LIBRARY; fi
      timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline ${*:2} > gpurun_out/ab/${w}_${v}_$rep.json 2> gpurun_out/ab/${w}_${v}_$rep.err || exit 1
      python -c "
import json
d=json.load(open('gpurun_out/ab/${w}_${v}_$rep.json')); print('$w $v $rep', d['value'], d['ms_per_step'], d.get('stages_standalone_ms'), d['roofline'].get('standalone', {}).get('frac', d['roofline']['frac']))
"
    done
  done
done
unset LDT_LIBRARY
