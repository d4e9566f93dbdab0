#!/bin/bash
# Own-queue slot streams (LDT_SLOT_OWN_QUEUE=1, ldt_stream_create with a CU
# mask of every CU) against the shipped streams, clean and DDP-after, c2 and
# c2p host legs. usage: bash tools/history/r6_streams3.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
run() {
  local name=$1 mode=$2 wl=$3; shift 3
  env "$@" timeout -k 10 240 python tools/probes/stream_env.py $mode $wl > $O/st3_$name.json 2> $O/st3_$name.err || { tail -5 $O/st3_$name.err; exit 1; }
  echo "$name $(grep '^{' $O/st3_$name.json)"
}
for wl in c2 c2p; do
  for m in clean after before; do
    run ${wl}_own_$m $m $wl LDT_SLOT_OWN_QUEUE=1
    run ${wl}_res_own_$m $m $wl LDT_SLOT_OWN_QUEUE=1 LDT_PROBE_RESIDENT=1
  done
done
echo done
