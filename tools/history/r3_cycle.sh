#!/bin/bash
# Round-3 GPU cycle: GPU tests (optionally -k), then the default bench (c2),
# then a 2-rank gloo rehearsal of the multi-rank path on configs[2] (c3).
# Stops at the first failure. usage: bash tools/r3_cycle.sh <tag> [pytest -k expr] [skip-tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ "$3" != "skip-tests" ]; then
  K=${2:+-k "$2"}
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','value_host_input','value_dataset','ms_per_step','host_us_per_call','stages_standalone_ms')})
print(d.get('dataset_leg'))"
LDT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload c3 --steps 20 --warmup 5 > $O/bench_c3_gloo2.json 2> $O/bench_c3_gloo2.err || { tail -20 $O/bench_c3_gloo2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c3_gloo2.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','value_per_gpu','value_host_input','value_dataset','value_dataset_per_gpu')})
print(d['config']['workload']); print(d.get('dataset_leg'))"
echo cycle done
