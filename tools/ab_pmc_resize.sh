#!/bin/bash
# Resize-only A/B of libldt builds: standalone stage times of a c2 batch
# (huff_rounds.py prints them) and PMC passes 1-3 of the c2 decode probe,
# raw k_resize4 counter means per build.
# usage: bash tools/ab_pmc_resize.sh <tag> <lib.so>...
R=$GRAFT_REPO_ROOT
T=$1
shift
mkdir -p $R/gpurun_out/$T
for lib in "$@"; do
  LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$lib timeout -k 10 120 python $R/tools/probes/huff_rounds.py c2 > $R/gpurun_out/$T/huff_$lib.txt 2>&1 || exit 1
  echo "$lib $(grep -o "'stage_ms'.*" $R/gpurun_out/$T/huff_$lib.txt)"
done
for lib in "$@"; do
  LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$lib PROBE=pmc_c2.py bash $R/tools/pmc.sh ${T}_$lib c2 1 2 3 > /dev/null || exit 1
  python3 $R/tools/pmc_raw.py $R/gpurun_out/pmc_${T}_$lib k_resize4 > $R/gpurun_out/$T/pmc_$lib.txt
  echo "== $lib"; cat $R/gpurun_out/$T/pmc_$lib.txt
done
