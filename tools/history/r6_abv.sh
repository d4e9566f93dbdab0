#!/bin/bash
# Parity of a variant build (LDT_LIBRARY), then an A/B against the shipped
# libldt.so (tools/ab_libs.sh). usage: bash tools/history/r6_abv.sh <tag> <variant.so> [reps]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_variant.log 2>&1 || { tail -30 $O/pytest_variant.log; exit 1; }
tail -1 $O/pytest_variant.log
bash tools/ab_libs.sh r6_$1/ab ${3:-2} $2 libldt.so
