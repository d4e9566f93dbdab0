#!/bin/bash
# Round-4 A/B of the parallel Huffman decoder's phase-1 warm start
# (LDT_OPT_SYNC_WARM = 7: each lane starts decoding this % of S before its
# range, so more lanes enter their range in sync and fewer rounds follow):
# 0 (default), 15, 35, 60; resident c2 and c1, alternated twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4sw}
mkdir -p $O
cd $R
for rep in 1 2; do
  for wm in 0 15 35 60; do
    for w in c2 c1; do
      timeout -k 10 200 python bench.py --workload $w --only-resident --no-cpu-baseline --opt 7=$wm > $O/sw${wm}_${w}_$rep.json 2> $O/sw${wm}_${w}_$rep.err || { tail -20 $O/sw${wm}_${w}_$rep.err; exit 1; }
      python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('warm', sys.argv[2], sys.argv[3], 'rep', sys.argv[4], 'value', b['value'], 'huffman ms', b['stages_ms_per_step']['huffman'], 'solo', b.get('stages_standalone_ms',{}).get('huffman'))" $O/sw${wm}_${w}_$rep.json $wm $w $rep
    done
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -x -q --timeout 120 --timeout-method thread -k "fullbatch or sync" > $O/pytest.log 2>&1; tail -1 $O/pytest.log
echo syncwarm done
