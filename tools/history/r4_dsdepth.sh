#!/bin/bash
# Round-4 A/B: dataset legs (LanceDataset + sampler + registered mapped
# fragments; c2 value_dataset, c3 and c4 config legs) at depth 3 (default)
# vs make_to_tensor_fn's own choice (--dataset-depth 0: 2 for batches of
# >= 8 MB of cells), alternated twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4dd}
mkdir -p $O
cd $R
for rep in 1 2; do
  for dd in 3 0; do
    timeout -k 10 300 python bench.py --dataset-depth $dd --no-cpu-baseline --no-registered --host-reps 1 > $O/dd${dd}_$rep.json 2> $O/dd${dd}_$rep.err || { tail -20 $O/dd${dd}_$rep.err; exit 1; }
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('dataset depth', sys.argv[2], 'rep', sys.argv[3], 'value_dataset', b['value_dataset'], b['dataset_leg']['harness'][-40:], 'c3', b['config_legs']['c3']['value'], 'c4', b['config_legs']['c4']['value'])" $O/dd${dd}_$rep.json $dd $rep
  done
done
echo dsdepth done
