#!/bin/bash
# Round-3 GPU step: GPU tests (unless "skip"), then bench c2 lines with the
# given extra flag sets (one JSON per set), printing the key fields.
# usage: bash tools/r3_ab.sh <tag> <skip|test> "<flags A>" ["<flags B>" ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ "$1" != "skip" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
shift
i=0
for f in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $f > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1])
print('[$f]', {k: d.get(k) for k in ('value','value_host_input','value_dataset','ms_per_step')})
print('   host', d.get('host_us_per_call'))
print('   standalone', d.get('stages_standalone_ms'))
print('   pipelined', d.get('stages_ms_per_step'))"
done
echo ab done
