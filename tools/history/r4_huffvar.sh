#!/bin/bash
# Round-4 A/B of Huffman builds (libldt_<v>.so via LDT_LIBRARY; "cur" = the
# default libldt.so): the fused-destuff parity tests on the default build,
# then per build the in-kernel phase times (tools/probes/huff_rounds.py) and a
# resident-only c2 bench line, alternated twice.
# usage: bash tools/r4_huffvar.sh <tag> v1 [v2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -x -q --timeout 120 --timeout-method thread -k "fused or corrupt or golden or config_batches or fullbatch or huffman or restart or marker" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in cur "$@"; do
    if [ $v = cur ]; then unset LDT_LIBRARY; else export LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_$v.so; fi
    timeout -k 10 120 python3 tools/probes/huff_rounds.py > $O/huff_${v}_$rep.txt 2>&1 || { tail -5 $O/huff_${v}_$rep.txt; exit 1; }
    timeout -k 10 300 python bench.py --only-resident --no-cpu-baseline --steps 100 --warmup 20 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -20 $O/${v}_$rep.err; exit 1; }
    python3 - $O $v $rep <<'PY'
import ast, json, sys
o, v, rep = sys.argv[1:4]
for l in open(f"{o}/huff_{v}_{rep}.txt"):
    if l.startswith("c2 "):
        d = ast.literal_eval(l[3:])
        h = {k: d[k] for k in ("t_setup_us", "t_phase1_us", "t_rounds_us", "t_write_us")}
b = json.loads(open(f"{o}/{v}_{rep}.json").read().strip().splitlines()[-1])
print(v, rep, "c2", b["value"], "huff(pipe) ms", b["stages_ms_per_step"]["huffman"], h)
PY
  done
done
unset LDT_LIBRARY
echo huffvar done
