#!/bin/bash
# c2p host-input legs at pipeline depth 6 and 7 (resident + host + registered).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hostd
mkdir -p $O
cd $R
for d in ${DEPTHS:-6 7}; do
  timeout -k 10 400 python bench.py --workload c2p --no-cpu-baseline --dataset-batches 0 --depth $d --host-depth $d --host-reps 3 > $O/c2p_d$d.json 2> $O/c2p_d$d.err || { tail -5 $O/c2p_d$d.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c2p_d$d.json'));print('c2p depth $d', d['value'], d.get('value_host_input'), d.get('value_host_input_reps'), d.get('value_host_registered'))"
done
