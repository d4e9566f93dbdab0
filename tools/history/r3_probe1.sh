#!/bin/bash
# Round-3 probe: host-input copy vs registered legs (phase times, copy-thread
# sweep, rocprofv3 kernel + memory-copy traces), then the c2 pipeline at more
# hardware queues per process and deeper pipelines.
# usage: bash tools/r3_probe1.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
bash tools/r3_reg_probe.sh $T c2 || exit 1
cd $R
for q in 4 8; do
  for d in 3 4 6; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --steps 100 --warmup 20 --depth $d --no-cpu-baseline --dataset-batches 0 --no-stage-events > $O/bench_q${q}_d${d}.json 2> $O/bench_q${q}_d${d}.err || { tail -20 $O/bench_q${q}_d${d}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/bench_q${q}_d${d}.json').read().strip().splitlines()[-1])
print('q=$q d=$d', d['value'], d.get('value_host_input'), d.get('host_us_per_call'))"
  done
done
echo probe1 done
