#!/bin/bash
# Slot streams from torch's pool vs the pipeline's own (ldt_stream_create),
# high priority, c2 adaptive host leg and c2p depth 4: clean / DDP-before /
# DDP-after / after an earlier pipeline. usage: bash tools/history/r6_streams4.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
run() {
  local name=$1 mode=$2 wl=$3; shift 3
  env "$@" timeout -k 10 240 python tools/probes/stream_env.py $mode $wl > $O/st4_$name.json 2> $O/st4_$name.err || { tail -5 $O/st4_$name.err; exit 1; }
  echo "$name $(grep '^{' $O/st4_$name.json)"
}
for m in clean after before; do
  run c2_pool_$m $m c2 LDT_SLOT_PRIORITY=1
  run c2_own_$m $m c2 LDT_SLOT_PRIORITY=1 LDT_SLOT_OWN_QUEUE=2
  run c2p_d4own_$m $m c2p LDT_SLOT_PRIORITY=1 LDT_SLOT_OWN_QUEUE=2 LDT_PROBE_DEPTH=4
done
run c2_pool_prev clean c2 LDT_SLOT_PRIORITY=1 LDT_PROBE_PREV=1
run c2_own_prev clean c2 LDT_SLOT_PRIORITY=1 LDT_SLOT_OWN_QUEUE=2 LDT_PROBE_PREV=1
run c2p_d7_prev clean c2p LDT_PROBE_PREV=1
run c2p_d4own_prev clean c2p LDT_SLOT_PRIORITY=1 LDT_SLOT_OWN_QUEUE=2 LDT_PROBE_DEPTH=4 LDT_PROBE_PREV=1
run c2p_d4pool_prev clean c2p LDT_SLOT_PRIORITY=1 LDT_PROBE_DEPTH=4 LDT_PROBE_PREV=1
echo done
