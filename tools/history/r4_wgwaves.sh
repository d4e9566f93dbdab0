#!/bin/bash
# Round-4 A/B: k_resize4 workgroups of 2 waves (default; ~25 KB of LDS at
# 512 px, cannot share a CU with a k_huff_image workgroup of another batch)
# vs 1 wave (~14 KB, fits beside it) vs 4; resize parity tests first; c2 and
# c1 resident lines alternated twice (20 warm-up + 100 timed steps).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4wg}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "resize_impls" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for wg in 2 1 4; do
    for w in c2 c1; do
      timeout -k 10 200 python bench.py --workload $w --only-resident --no-cpu-baseline --resize-wg-waves $wg > $O/wg${wg}_${w}_$rep.json 2> $O/wg${wg}_${w}_$rep.err || { tail -20 $O/wg${wg}_${w}_$rep.err; exit 1; }
      python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('wg', sys.argv[2], sys.argv[3], 'rep', sys.argv[4], 'value', b['value'], 'stages', b['stages_ms_per_step'])" $O/wg${wg}_${w}_$rep.json $wg $w $rep
    done
  done
done
echo wgwaves done
