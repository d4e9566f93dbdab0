#!/bin/bash
# c2p pipeline-depth sweep on the GPU box: the resident leg (--only-resident)
# at each depth for each library (ldt_amd/libldt_<name>.so; "cur" = libldt.so).
# usage: [QUEUES="4 8"] [PRIOS="0 1"] [WL=c2p] bash tools/r4_progdepth.sh <tag> "<depths>" <lib>...
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; D=$2; shift 2
O=$R/gpurun_out/pdepth_$T
mkdir -p $O
cd $R
for v in "$@"; do
  if [ "$v" = cur ]; then L=$R/lance-distributed-training_amd/ldt_amd/libldt.so; else L=$R/lance-distributed-training_amd/ldt_amd/libldt_$v.so; fi
  for q in ${QUEUES:-4}; do
  for p in ${PRIOS:-0}; do
  for d in $D; do
    f=$O/${WL:-c2p}_${v}_q${q}_p${p}_d$d
    if [ "$p" = auto ]; then unset LDT_SLOT_PRIORITY; else export LDT_SLOT_PRIORITY=$p; fi; GPU_MAX_HW_QUEUES=$q LDT_LIBRARY=$L timeout -k 10 300 python bench.py --workload ${WL:-c2p} --no-cpu-baseline --only-resident --depth $d --steps 60 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f.json'));print('${WL:-c2p} $v queues $q prio $p depth $d', d['value'], d['ms_per_step'])"
  done
  done
  done
done
