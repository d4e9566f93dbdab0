#!/bin/bash
# Round-4 host-path A/B on one box: host_calls2 (60 pipelined to_tensor_fn
# calls, c2) per copy variant (LDT_OPT_COPY_MODE / _BIND / _NT), twice,
# then one short bench line. usage: bash tools/r4_hostab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4ab}
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in "0 1 0" "1 1 0" "0 0 0" "0 1 1"; do
    set -- $v
    tag="m$1b$2n$3"
    LDT_P_MODE=$1 LDT_P_BIND=$2 LDT_P_NT=$3 timeout -k 10 120 python3 tools/probes/host_calls2.py c2 3 copy > $O/hc_${tag}_$rep.txt 2>&1 || { tail -5 $O/hc_${tag}_$rep.txt; exit 1; }
    echo "== $tag rep $rep"; grep -v amdgpu.ids $O/hc_${tag}_$rep.txt
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 60 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().splitlines()[-1])
print({k: d.get(k) for k in ("value", "value_host_input", "value_host_registered", "value_dataset", "host_us_per_call")})
print({k: v["value"] for k, v in d.get("config_legs", {}).items()})
PY
