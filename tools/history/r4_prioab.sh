#!/bin/bash
# Slot-stream priority A/B on the GPU box (LDT_SLOT_PRIORITY 0/1): the full
# default c2 bench line (resident + host legs) and the c2p line at depth 4
# (resident and host legs) for a k_prog library variant.
# usage: bash tools/r4_prioab.sh <tag> <c2p lib>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prio_$1
mkdir -p $O
cd $R
for p in 0 1; do
  LDT_SLOT_PRIORITY=$p timeout -k 10 400 python bench.py --no-cpu-baseline --dataset-batches 0 > $O/c2_p$p.json 2> $O/c2_p$p.err || { tail -5 $O/c2_p$p.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c2_p$p.json'));print('c2 prio $p', d['value'], d.get('value_host_input'), d.get('value_host_input_reps'), d.get('value_host_registered'))"
done
L=$R/lance-distributed-training_amd/ldt_amd/libldt_$2.so
for p in 0 1; do
  LDT_SLOT_PRIORITY=$p LDT_LIBRARY=$L timeout -k 10 400 python bench.py --workload c2p --no-cpu-baseline --dataset-batches 0 --depth 4 --host-depth 4 --host-reps 2 > $O/c2p_p$p.json 2> $O/c2p_p$p.err || { tail -5 $O/c2p_p$p.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c2p_p$p.json'));print('c2p prio $p', d['value'], d.get('value_host_input'), d.get('value_host_input_reps'), d.get('value_host_registered'))"
done
