#!/bin/bash
# Process-wide slot streams taken at the first decode (DecodePipeline
# default) vs per-pipeline pool streams taken at construction (round 5,
# LDT_SLOT_OWN_QUEUE=3), across stream orders; then the default bench line.
# usage: bash tools/history/r6_streams6.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
run() {
  local name=$1 mode=$2 wl=$3; shift 3
  env "$@" timeout -k 10 240 python tools/probes/stream_env.py $mode $wl > $O/st6_$name.json 2> $O/st6_$name.err || { tail -5 $O/st6_$name.err; exit 1; }
  echo "$name $(grep '^{' $O/st6_$name.json)"
}
for wl in c2 c2p; do
  for m in clean ref before after; do
    run ${wl}_$m $m $wl
  done
  run ${wl}_prev clean $wl LDT_PROBE_PREV=1
  run ${wl}_old_ref ref $wl LDT_SLOT_OWN_QUEUE=3
done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', json.dumps(d['summary']))"
echo done
