#!/bin/bash
# Stream-environment matrix (tools/probes/stream_env.py): slot priority
# policies under clean / DDP-before / DDP-after processes. usage: bash tools/history/r6_streams.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
run() { # name env... -- args
  local name=$1; shift
  env "$@" timeout -k 10 240 python tools/probes/stream_env.py $MODE $WL > $O/st_$name.json 2> $O/st_$name.err || { tail -5 $O/st_$name.err; exit 1; }
  echo "$name $(cat $O/st_$name.json)"
}
for MODE in clean after before; do
  WL=c2 run c2_hp_$MODE LDT_SLOT_PRIORITY=1
  WL=c2 run c2_res_norm_$MODE LDT_SLOT_PRIORITY=0 LDT_PROBE_RESIDENT=1 LDT_PROBE_DEPTH=3
  WL=c2 run c2_res_hp_$MODE LDT_SLOT_PRIORITY=1 LDT_PROBE_RESIDENT=1 LDT_PROBE_DEPTH=3
  WL=c2p run c2p_d4hp_$MODE LDT_SLOT_PRIORITY=1 LDT_PROBE_DEPTH=4
  WL=c2p run c2p_d5hp_$MODE LDT_SLOT_PRIORITY=1 LDT_PROBE_DEPTH=5
done
echo done
