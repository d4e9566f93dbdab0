#!/bin/bash
# Deep (progressive) pipelines on high-priority streams only, with 8 hardware
# queues per priority (bench.py --hw-queues 8) so that all 7 c2p slots get
# queues of their own away from the consumer's normal-priority queue; against
# the shipped 4 queues (4 high-priority + 3 shared slots).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "progressive or pipeline or prefetch or async or adaptive" > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for q in 8 4; do
  timeout -k 10 300 python bench.py --workload c2p --steps 40 --no-cpu-baseline --hw-queues $q > $O/c2p_q$q.json 2> $O/c2p_q$q.err || { tail -5 $O/c2p_q$q.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2p line q=$q resident', d['value'], 'host', d.get('value_host_input'))" $O/c2p_q$q.json
done
for q in 8 4 8; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --hw-queues $q > $O/default_q$q.json 2> $O/default_q$q.err || { tail -5 $O/default_q$q.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); w=d['workload_legs']
print('default q=$q', d['value'], 'host', d['value_host_input'], 'dataset', d.get('value_dataset'), 'copy', d.get('value_dataset_copy'), 'c2p', w['c2p']['value'], w['c2p']['value_host_input'], 'c5', w['c5']['value'], {k: v.get('value') for k, v in (d.get('config_legs') or {}).items()})" $O/default_q$q.json
done
