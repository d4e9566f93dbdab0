#!/bin/bash
# Round-4 A/B of resize kernels on one build: LDT_OPT_RESIZE_IMPL 0
# (k_resize4, two staged rows per step, 3 waves/SIMD) vs 4 (k_resize4r, one
# staged row per step, 4 waves/SIMD): parity tests, then c2 and c1 bench lines
# (pipelined + standalone resize times), alternated twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4ri}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -x -q --timeout 120 --timeout-method thread -k "golden or config_batches or fullbatch or resize or large_image or tall" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for impl in 0 4; do
    for w in c2 c1; do
      timeout -k 10 300 python bench.py --resize-impl $impl --workload $w --no-cpu-baseline --dataset-batches 0 --no-registered --host-reps 1 --steps 100 --warmup 20 > $O/i${impl}_${w}_$rep.json 2> $O/i${impl}_${w}_$rep.err || { tail -20 $O/i${impl}_${w}_$rep.err; exit 1; }
      python3 - $O/i${impl}_${w}_$rep.json $impl $w $rep <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sa = b.get("stages_standalone_ms", {})
print("impl", sys.argv[2], sys.argv[3], sys.argv[4], "value", b["value"], "host", b.get("value_host_input"), "resize pipe/solo ms",
      b["stages_ms_per_step"]["resize"], sa.get("resize"), "frac", b["roofline"]["frac"], b["roofline"].get("standalone", {}).get("frac"))
PY
    done
  done
done
echo resizeimpl done
