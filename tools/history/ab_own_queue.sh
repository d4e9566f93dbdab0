#!/bin/bash
# Own-queue slot streams for deep (progressive) pipelines: GPU tests that use
# them, the c2p line with and without (LDT_SLOT_OWN_QUEUE=0: 4 high-priority
# + 3 shared-queue slots), then the default c2 line whose c2p leg runs after
# the c2 legs. usage: bash tools/ab_own_queue.sh <tag>
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "progressive or pipeline or prefetch or async or adaptive" > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for v in 1 0 1; do
  LDT_SLOT_OWN_QUEUE=$v timeout -k 10 300 python bench.py --workload c2p --steps 40 --no-cpu-baseline > $O/c2p_own$v.json 2> $O/c2p_own$v.err || { tail -5 $O/c2p_own$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2p line own_queue=$v resident', d['value'], 'host', d.get('value_host_input'))" $O/c2p_own$v.json
done
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/default.json 2> $O/default.err || { tail -5 $O/default.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); w=d['workload_legs']['c2p']; print('default line', d['value'], 'host', d['value_host_input'], 'c2p leg resident', w['value'], 'host', w['value_host_input'])" $O/default.json
