#!/bin/bash
# Round-4 A/B (final tree): make_to_tensor_fn depth 2 (default: the copy
# stream keeps its own hardware queue) vs 3 (DMA on the slot streams), host
# input legs of c2 and c1 (3 reps each), alternated twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4hd}
mkdir -p $O
cd $R
for rep in 1 2; do
  for hd in 2 3; do
    for w in c2 c1; do
      timeout -k 10 200 python bench.py --workload $w --host-depth $hd --no-cpu-baseline --dataset-batches 0 --no-registered --no-config-legs --host-reps 3 > $O/hd${hd}_${w}_$rep.json 2> $O/hd${hd}_${w}_$rep.err || { tail -20 $O/hd${hd}_${w}_$rep.err; exit 1; }
      python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('host depth', sys.argv[2], sys.argv[3], 'rep', sys.argv[4], 'resident', b['value'], 'host', b['value_host_input'], b['value_host_input_reps'])" $O/hd${hd}_${w}_$rep.json $hd $w $rep
    done
  done
done
echo hostdepth done
