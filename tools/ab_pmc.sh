#!/bin/bash
# PMC passes 1-3 (tools/pmc.sh) of the c2 decode probe for each libldt build
# named (LDT_LIBRARY), then the raw per-kernel means of each.
# usage: bash tools/ab_pmc.sh <tag> <lib.so under ldt_amd/>...
R=$GRAFT_REPO_ROOT
T=$1
shift
for lib in "$@"; do
  LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$lib PROBE=pmc_c2.py bash $R/tools/pmc.sh ${T}_$lib c2 1 2 3 || exit 1
  python3 $R/tools/pmc_raw.py $R/gpurun_out/pmc_${T}_$lib k_huff_image > $R/gpurun_out/pmc_${T}_$lib.txt
done
paste $R/gpurun_out/pmc_${T}_$1.txt $R/gpurun_out/pmc_${T}_$2.txt | awk '{print $2, $3, $8}'
