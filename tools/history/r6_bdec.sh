#!/bin/bash
# Block-parallel AC decode (LDT_OPT_BLOCK_DECODE): the option tests on the
# default build, the parity suite on the build that defaults to it, then an
# A/B against the write pass (tools/ab_libs.sh). usage: bash tools/history/r6_bdec.sh <tag> [reps]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_options.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_opts.log 2>&1 || { tail -30 $O/pytest_opts.log; exit 1; }
tail -1 $O/pytest_opts.log
LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_bdec.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_bdec.log 2>&1 || { tail -30 $O/pytest_bdec.log; exit 1; }
tail -1 $O/pytest_bdec.log
bash tools/ab_libs.sh r6_$1/ab ${2:-2} libldt_bdec.so libldt.so
