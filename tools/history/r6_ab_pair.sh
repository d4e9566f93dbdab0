#!/bin/bash
# Write-pass unit pairing A/B: parity of the paired build, phase times and
# bench (tools/ab_libs.sh), then a WRITE_SIZE pass per build (per-kernel HBM
# writes at depth 1). usage: bash tools/history/r6_ab_pair.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_pair.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_pair.log 2>&1 || { tail -30 $O/pytest_pair.log; exit 1; }
tail -1 $O/pytest_pair.log
bash tools/ab_libs.sh r6_$1/ab 2 libldt_pair.so libldt.so || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in libldt.so libldt_pair.so; do
  LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$lib timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$lib/WRITE_SIZE -o run -- python3 $R/bench.py --steps 4 --warmup 1 --depth 1 --only-resident --no-cpu-baseline > $O/w_$lib.log 2>&1 || { tail -5 $O/w_$lib.log; exit 1; }
  echo $lib; python3 $R/tools/traffic_all.py $O/w_$lib
done
