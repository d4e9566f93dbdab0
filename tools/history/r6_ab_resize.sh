#!/bin/bash
# Resize variant: parity of a libldt build on the resize tests, then the A/B
# (tools/ab_libs.sh). usage: bash tools/history/r6_ab_resize.sh <tag> <reps> <variant lib> <base lib>
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
O=$R/gpurun_out/r6_$T
mkdir -p $O
cd $R
LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or config or resize or edge or c2_full or tall or raw" > $O/pytest_$3.log 2>&1 || { tail -40 $O/pytest_$3.log; exit 1; }
tail -1 $O/pytest_$3.log
bash tools/ab_libs.sh r6_$T/ab $2 $3 $4
