#!/bin/bash
# A/B of libldt builds on one box (LDT_LIBRARY), alternated: per build, the
# parallel Huffman decoder's phase times + standalone stage times of a c2
# batch (tools/probes/huff_rounds.py) and the resident c2 bench line.
# usage: bash tools/ab_libs.sh <tag> <reps> <lib.so under ldt_amd/>...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
REPS=$2
shift 2
mkdir -p $O
cd $R
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    L=$R/lance-distributed-training_amd/ldt_amd/$lib
    LDT_LIBRARY=$L timeout -k 10 150 python tools/probes/huff_rounds.py ${AB_WL:-c2} > $O/huff_${lib}_$rep.txt 2>&1 || { tail -5 $O/huff_${lib}_$rep.txt; exit 1; }
    LDT_LIBRARY=$L timeout -k 10 200 python bench.py --only-resident --no-cpu-baseline --steps 100 ${AB_BENCH_ARGS} > $O/bench_${lib}_$rep.json 2> $O/bench_${lib}_$rep.err || { tail -5 $O/bench_${lib}_$rep.err; exit 1; }
    python3 - "$O/huff_${lib}_$rep.txt" "$O/bench_${lib}_$rep.json" "$lib" "$rep" <<'PY'
import ast, json, sys
h = open(sys.argv[1]).read().strip().splitlines()
b = json.load(open(sys.argv[2]))
for line in h:
    if line[:3] in ("c2 ", "c1 ", "c4 "):
        d = ast.literal_eval(line[3:])
        print(sys.argv[3], sys.argv[4], line[:2], "setup/ph1/rounds/write us:", d["t_setup_us"], d["t_phase1_us"],
              d["t_rounds_us"], d["t_write_us"], "stages:", d.get("stage_ms"))
print(sys.argv[3], sys.argv[4], "bench value", b["value"], "stages", b["stages_ms_per_step"])
PY
  done
done
