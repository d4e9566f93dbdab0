#!/bin/bash
# Round-4 A/B: LDT_OPT_RESIZE_IMPL 1 (k_resize4<0>: 4:2:0 fancy upsampling on
# 32-bit lanes) vs 0 (default since r4pk; k_resize4<5>: packed 16-bit pairs, v_perm
# context pairs with per-lane edge selectors): resize parity tests (impl 0
# bit-identical to impl 1 on goldens, c2-like and FOOD101-like batches), then
# c2 and c1 lines alternated twice; then the headline command (K=20, W=5)
# with and without the 0.25 s warm-up floor.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4pk}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -x -q --timeout 120 --timeout-method thread -k "golden or config_batches or fullbatch or resize or large_image or tall" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 tools/probes/resize_pk_eq.py > $O/eq.log 2>&1 || { tail -20 $O/eq.log; exit 1; }
cat $O/eq.log
for rep in 1 2; do
  for impl in 1 0; do
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
for mw in 0 0.25 0 0.25; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --min-warm-s $mw --no-cpu-baseline --dataset-batches 0 --no-registered --host-reps 1 > $O/warm_$mw.json 2> $O/warm_$mw.err || { tail -20 $O/warm_$mw.err; exit 1; }
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('min_warm_s', sys.argv[2], 'K=20 value', b['value'], 'warm', b['warmup_run'], 'host', b.get('value_host_input'))" $O/warm_$mw.json $mw
done
echo resizepk done
