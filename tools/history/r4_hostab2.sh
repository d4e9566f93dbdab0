#!/bin/bash
# Round-4 host-path A/B 2: NT copies; the cells' DMA on the slot's stream
# (mode 1) vs on a copy stream (mode 0) with 4 or 8 HW queues per process, and
# depth 2 vs 3. host_calls2 per variant twice, then traces of the best guess.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4ab2}
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in "1 3 4" "0 3 4" "0 3 8" "1 3 8" "0 2 4"; do
    set -- $v
    tag="m$1d$2q$3"
    GPU_MAX_HW_QUEUES=$3 LDT_P_MODE=$1 timeout -k 10 120 python3 tools/probes/host_calls2.py c2 $2 copy > $O/hc_${tag}_$rep.txt 2>&1 || { tail -5 $O/hc_${tag}_$rep.txt; exit 1; }
    echo "== $tag rep $rep"; grep -v amdgpu.ids $O/hc_${tag}_$rep.txt | grep -v host_info
  done
done
