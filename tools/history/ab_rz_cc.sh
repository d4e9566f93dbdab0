#!/bin/bash
# (Cb, Cr)-interleaved 4:2:0 staging (LDT_RZ_CC build) vs the shipped one:
# GPU parity tests on the variant, then standalone resize and resident c2.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_cc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/ab_resize_wg.sh $1 libldt.so:4 libldt_cc.so:4 libldt.so:4 libldt_cc.so:4
