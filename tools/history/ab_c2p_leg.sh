#!/bin/bash
# The default line twice (its c2p leg: resident and host legs on one pipeline)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 600 python bench.py --no-cpu-baseline > $O/default$i.json 2> $O/default$i.err || { tail -5 $O/default$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); w=d['workload_legs']
print('default', d['value'], 'host', d['value_host_input'], 'dataset', d.get('value_dataset'), 'copy', d.get('value_dataset_copy'), 'c2p', w['c2p']['value'], w['c2p']['value_host_input'], w['c2p']['stages_ms_per_launch'], 'c5', w['c5']['value'])" $O/default$i.json
done
