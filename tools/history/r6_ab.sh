#!/bin/bash
# GPU parity of the current libldt.so, then an A/B of libldt builds
# (tools/ab_libs.sh). usage: bash tools/history/r6_ab.sh <tag> <reps> <lib.so>...
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/r6_$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
shift
bash tools/ab_libs.sh r6_$T/ab "$@"
