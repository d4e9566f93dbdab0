#!/bin/bash
# Hiding capacity beside the decoder: k_idct timing builds with extra VALU
# work per block (LDT_IDCT_EXTRA), their standalone stage times
# (huff_rounds probe, c2) and the resident c2 line.
# usage: bash tools/ab_idct_extra.sh <tag> <lib.so> ...
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
for lib in "$@"; do
  L=$R/lance-distributed-training_amd/ldt_amd/$lib
  LDT_LIBRARY=$L timeout -k 10 150 python tools/probes/huff_rounds.py c2 > $O/huff_$lib.txt 2>&1 || { tail -5 $O/huff_$lib.txt; exit 1; }
  LDT_LIBRARY=$L timeout -k 10 200 python bench.py --only-resident --no-cpu-baseline --steps 100 > $O/bench_$lib.json 2> $O/bench_$lib.err || { tail -5 $O/bench_$lib.err; exit 1; }
  python3 - "$O/huff_$lib.txt" "$O/bench_$lib.json" "$lib" <<'PY'
import ast, json, sys
h = [l for l in open(sys.argv[1]).read().splitlines() if l.startswith("c2 ")]
d = ast.literal_eval(h[0][3:])
b = json.load(open(sys.argv[2]))
print(sys.argv[3], "standalone ms", {k: round(v, 4) for k, v in d["stage_ms"].items()}, "bench", b["value"])
PY
done
