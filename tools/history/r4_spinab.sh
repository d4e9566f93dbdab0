#!/bin/bash
# Copy-pool spin A/B on the GPU box: the c2 line's resident and host legs with
# LDT_COPY_SPIN_US=0 (sleep at once) and the default, alternated.
# usage: bash tools/r4_spinab.sh <tag> [workload]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/spin_$1
W=${2:-c2}
mkdir -p $O
cd $R
for rep in 1 2; do
  for sp in 0 400; do
    LDT_COPY_SPIN_US=$sp timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --dataset-batches 0 > $O/${W}_s${sp}_$rep.json 2> $O/${W}_s${sp}_$rep.err || { tail -5 $O/${W}_s${sp}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${W}_s${sp}_$rep.json'));h=d.get('host_us_per_call',{});print('$W spin $sp rep $rep', d['value'], d.get('value_host_input_reps'), d.get('value_host_registered'), 'wake', h.get('copy_wake'), 'slot', h.get('slot'))"
  done
done
