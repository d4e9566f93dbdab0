#!/bin/bash
# Which part of a DDP-like environment created after the pipeline costs the
# c2 host leg (tools/probes/stream_env.py after c2). usage: bash tools/history/r6_streams2.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python tools/probes/stream_env.py after c2 > $O/st2_$name.json 2> $O/st2_$name.err || { tail -5 $O/st2_$name.err; exit 1; }
  echo "$name $(grep '^{' $O/st2_$name.json)"
}
for pr in 0 1; do
  run pg_only_p$pr LDT_SLOT_PRIORITY=$pr LDT_ENV_SIDE=0 LDT_ENV_COMM=0
  run side_only_p$pr LDT_SLOT_PRIORITY=$pr LDT_ENV_PG=0 LDT_ENV_COMM=0
  run comm_only_p$pr LDT_SLOT_PRIORITY=$pr LDT_ENV_PG=0 LDT_ENV_SIDE=0
  run side_comm_p$pr LDT_SLOT_PRIORITY=$pr LDT_ENV_PG=0
  run all_p$pr LDT_SLOT_PRIORITY=$pr
done
echo done
