#!/bin/bash
# Parallel-Huffman phase times of a c2 batch (tools/probes/huff_rounds.py)
# for each libldt build named (LDT_LIBRARY), alternated <reps> times.
# usage: bash tools/ab_huff.sh <tag> <reps> <lib.so under ldt_amd/>...
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
REPS=$2
shift 2
mkdir -p $O
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    f=$O/${lib}_$rep.txt
    LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$lib timeout -k 10 120 python $R/tools/probes/huff_rounds.py ${AB_WL:-c2} > $f 2>&1 || { echo "FAIL $lib"; tail -3 $f; exit 1; }
    echo "$lib $rep $(grep -o "t_phase1_us.: [0-9.]*" $f) $(grep -o "t_rounds_us.: [0-9.]*" $f) $(grep -o "t_write_us.: [0-9.]*" $f) $(grep -o "huffman.: [0-9.]*" $f)"
  done
done
