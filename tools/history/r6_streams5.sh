#!/bin/bash
# The reference's stream order (probe mode ref) for c2/c2p, normal vs
# high-priority c2 slots, and the default bench line with and without
# LDT_SLOT_PRIORITY=1 (every later leg's pipeline draws new pool streams).
# usage: bash tools/history/r6_streams5.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
run() {
  local name=$1 mode=$2 wl=$3; shift 3
  env "$@" timeout -k 10 240 python tools/probes/stream_env.py $mode $wl > $O/st5_$name.json 2> $O/st5_$name.err || { tail -5 $O/st5_$name.err; exit 1; }
  echo "$name $(grep '^{' $O/st5_$name.json)"
}
run c2_norm_ref ref c2 LDT_SLOT_PRIORITY=0
run c2_high_ref ref c2 LDT_SLOT_PRIORITY=1
run c2p_ref ref c2p
run c2_norm_clean clean c2 LDT_SLOT_PRIORITY=0
run c2_high_clean clean c2 LDT_SLOT_PRIORITY=1
for pr in 1 0; do
  LDT_SLOT_PRIORITY=$pr timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_p$pr.json 2> $O/bench_p$pr.err || { tail -5 $O/bench_p$pr.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_p$pr.json'));print('bench p$pr', json.dumps(d['summary']))"
done
echo done
