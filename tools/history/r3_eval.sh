#!/bin/bash
# Round-3 evaluation on the GPU box: GPU tests, the default c2 bench line,
# Huffman phase times, rocprofv3 kernel stats of a c2 bench, per-kernel HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes at depth 1). Stops at the first failure.
# usage: bash tools/r3_eval.sh <tag> [skip-tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','value_host_input','value_dataset','ms_per_step')})
print('standalone', d.get('stages_standalone_ms')); print('pipelined', d.get('stages_ms_per_step'))"
timeout -k 10 120 python3 tools/probes/huff_rounds.py > $O/huff_rounds.txt 2>&1 || { tail -5 $O/huff_rounds.txt; exit 1; }
head -1 $O/huff_rounds.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 --dataset-batches 0 > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/traffic/$c -o run -- python3 $R/bench.py --steps 4 --warmup 1 --depth 1 --no-cpu-baseline --dataset-batches 0 > $O/traffic_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $O/traffic_$c.log; exit 1; }
done
python3 $R/tools/traffic_all.py $O/traffic > $O/traffic_perkernel.txt && cat $O/traffic_perkernel.txt
echo eval done
