#!/bin/bash
# Progressive (c2p) resident and host-input rates by pipeline depth and the
# process's HIP hardware queues (GPU_MAX_HW_QUEUES), one box.
# usage: bash tools/c2p_depth_ab.sh <tag> "depth:queues" ...
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
for spec in "$@"; do
  d=${spec%%:*}
  q=${spec#*:}
  f=$O/c2p_d${d}_q${q}.json
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --workload c2p --depth $d --host-depth $d --steps 40 \
    --no-cpu-baseline --no-registered --dataset-batches 0 --host-reps 1 > $f 2> $f.err || { echo "FAIL $spec"; tail -3 $f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('depth', sys.argv[2], 'queues', sys.argv[3], 'resident', d['value'], 'host', d.get('value_host_input'))" $f $d $q
done
