#!/bin/bash
# Dev loop on the GPU box: gpu tests, then benches for the given workloads,
# then (optional) a rocprofv3 kernel-trace of the c2 bench.
# usage: bash tools/gpu_cycle.sh "c2 c1 c4" [prof_tag]
set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for w in $1; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['roofline']['frac'])
"
done
if [ -n "$2" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$2 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$2.log 2>&1 || exit 1
  python3 -c "
import csv
r=list(csv.DictReader(open('$R/gpurun_out/prof_$2/run_kernel_stats.csv')))
for x in r: print('%-40s %5s %10.1f us %6.2f%%' % (x['Name'][:40], x['Calls'], float(x['AverageNs'])/1e3, float(x['Percentage'])))
"
fi
