#!/bin/bash
# k_prog variants: progressive parity of each (LDT_LIBRARY), then the c2p
# resident rate at several depths, interleaved with the shipped libldt.so.
# usage: bash tools/history/r6_prog_ab.sh <tag> "<variant.so ...>" "<depths>"
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
L=$R/lance-distributed-training_amd/ldt_amd
for v in $2; do
  LDT_LIBRARY=$L/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "progressive" -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2; do
  for v in libldt.so $2; do
    LDT_LIBRARY=$L/$v timeout -k 10 300 python -u tools/probes/prog_rate.py $3 > $O/rate_${v}_$rep.txt 2>&1 || { tail -20 $O/rate_${v}_$rep.txt; exit 1; }
    echo "== $v rep $rep"; grep depth $O/rate_${v}_$rep.txt
  done
done
