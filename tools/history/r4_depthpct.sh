#!/bin/bash
# Round-4 A/B of the resident c2 leg after the packed resize: pipeline depth
# (3 default, 4) x resize bands (LDT_OPT_RESIZE_WAVES_PCT 100 default, 70, 150),
# alternated twice; 20 warm-up + 100 timed steps, --only-resident.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4dp}
mkdir -p $O
cd $R
for rep in 1 2; do
  for d in 3 4; do
    for pct in 100 70 150; do
      timeout -k 10 200 python bench.py --only-resident --no-cpu-baseline --depth $d --resize-waves-pct $pct > $O/d${d}_p${pct}_$rep.json 2> $O/d${d}_p${pct}_$rep.err || { tail -20 $O/d${d}_p${pct}_$rep.err; exit 1; }
      python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('depth', sys.argv[2], 'pct', sys.argv[3], 'rep', sys.argv[4], 'value', b['value'], 'stages', b['stages_ms_per_step'])" $O/d${d}_p${pct}_$rep.json $d $pct $rep
    done
  done
done
echo depthpct done
