#!/bin/bash
# A/B diagnostics on one GPU box: Huffman phase timers (huff_rounds probe) and
# depth-1 rocprofv3 kernel stats of the c2 bench, current build vs
# ldt_amd/libldt_prev.so. usage: bash tools/ab_prof.sh <tag>
set -o pipefail
R=$PWD
O=$R/gpurun_out/abp_$1
mkdir -p $O
PREV=$R/lance-distributed-training_amd/ldt_amd/libldt_prev.so
for v in new prev; do
  if [ $v = prev ]; then export LDT_LIBRARY=$PREV; else unset LDT_LIBRARY; fi
  timeout -k 10 120 python tools/probes/huff_rounds.py > $O/rounds_$v.txt 2>&1 || { tail -5 $O/rounds_$v.txt; exit 1; }
  grep -E "^c2|^c4" $O/rounds_$v.txt | sed "s/^/$v /" | cut -c1-400
done
cd /tmp && export TMPDIR=/tmp
for v in new prev; do
  if [ $v = prev ]; then export LDT_LIBRARY=$PREV; else unset LDT_LIBRARY; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --depth 1 --steps 30 --warmup 5 > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  python3 -c "
import csv
r=list(csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')))
for x in r[:7]: print('$v %-28s %5s %8.1f us' % (x['Name'][:28], x['Calls'], float(x['AverageNs'])/1e3))
"
done
unset LDT_LIBRARY
