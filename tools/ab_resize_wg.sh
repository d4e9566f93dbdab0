#!/bin/bash
# Standalone k_resize4 time (huff_rounds probe, c2) and the resident c2 line
# for (libldt build, waves per resize workgroup) pairs, one box.
# usage: bash tools/ab_resize_wg.sh <tag> "<lib.so>:<wg waves>" ...
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
for spec in "$@"; do
  lib=${spec%%:*}
  wg=${spec#*:}
  L=$R/lance-distributed-training_amd/ldt_amd/$lib
  LDT_RESIZE_WG=$wg LDT_LIBRARY=$L timeout -k 10 150 python tools/probes/huff_rounds.py c2 > $O/huff_${lib}_$wg.txt 2>&1 || { tail -5 $O/huff_${lib}_$wg.txt; exit 1; }
  LDT_LIBRARY=$L timeout -k 10 200 python bench.py --only-resident --no-cpu-baseline --steps 100 --resize-wg-waves $wg > $O/bench_${lib}_$wg.json 2> $O/bench_${lib}_$wg.err || { tail -5 $O/bench_${lib}_$wg.err; exit 1; }
  python3 - "$O/huff_${lib}_$wg.txt" "$O/bench_${lib}_$wg.json" "$spec" <<'PY'
import ast, json, sys
h = [l for l in open(sys.argv[1]).read().splitlines() if l.startswith("c2 ")]
d = ast.literal_eval(h[0][3:])
b = json.load(open(sys.argv[2]))
print(sys.argv[3], "standalone resize ms", d["stage_ms"]["resize"], "bench", b["value"], "pipeline resize", b["stages_ms_per_step"]["resize"])
PY
done
