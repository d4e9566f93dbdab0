#!/bin/bash
# Round-4 probe 2: HIP API host costs (tools/probes/hip_api_cost), the fused
# destuff parity tests after the end-marker fix, Huffman phase times.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4p2}
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/probes/hip_api_cost > $O/hip_api_cost.txt 2>&1 || { cat $O/hip_api_cost.txt; exit 1; }
cat $O/hip_api_cost.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "fused or corrupt or golden or config_batches" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python3 tools/probes/huff_rounds.py > $O/huff_rounds.txt 2>&1 || { tail -5 $O/huff_rounds.txt; exit 1; }
cat $O/huff_rounds.txt
