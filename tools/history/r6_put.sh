#!/bin/bash
# Fused-destuff byte stores: a timing-only build without them (setup phase
# only: its output is not a decode), then the skewed-store build's parity and
# an A/B against the shipped build. usage: bash tools/history/r6_put.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
L=$R/lance-distributed-training_amd/ldt_amd
mkdir -p $O
cd $R
LDT_PROBE_TOLERATE=1 LDT_LIBRARY=$L/libldt_noput.so timeout -k 10 120 python tools/probes/huff_rounds.py c2 > $O/noput.txt 2>&1 || { tail -5 $O/noput.txt; exit 1; }
grep "^c2" $O/noput.txt | cut -c1-420
LDT_LIBRARY=$L/libldt_skew.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_skew.log 2>&1 || { tail -30 $O/pytest_skew.log; exit 1; }
tail -1 $O/pytest_skew.log
bash tools/ab_libs.sh r6_$1/ab 2 libldt_skew.so libldt.so
