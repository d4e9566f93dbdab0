#!/bin/bash
# Standalone k_resize4 time (huff_rounds probe, c2) and the resident c2 line
# per LDT_OPT_RESIZE_WAVES_PCT value (bands per image = 12 * pct / 100 at c2).
# usage: bash tools/ab_resize_pct.sh <tag> <pct> ...
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
for pct in "$@"; do
  LDT_RESIZE_PCT=$pct timeout -k 10 150 python tools/probes/huff_rounds.py c2 > $O/huff_$pct.txt 2>&1 || { tail -5 $O/huff_$pct.txt; exit 1; }
  timeout -k 10 200 python bench.py --only-resident --no-cpu-baseline --steps 100 --resize-waves-pct $pct > $O/bench_$pct.json 2> $O/bench_$pct.err || { tail -5 $O/bench_$pct.err; exit 1; }
  python3 - "$O/huff_$pct.txt" "$O/bench_$pct.json" "$pct" <<'PY'
import ast, json, sys
h = [l for l in open(sys.argv[1]).read().splitlines() if l.startswith("c2 ")]
d = ast.literal_eval(h[0][3:])
b = json.load(open(sys.argv[2]))
print("pct", sys.argv[3], "standalone resize ms", d["stage_ms"]["resize"], "bench", b["value"], "pipeline resize", b["stages_ms_per_step"]["resize"])
PY
done
