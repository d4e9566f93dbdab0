#!/bin/bash
# Queues of the resident c2p pipeline's k_prog dispatches with the slot
# queue probe on and off (LDT_SLOT_QUEUE_PROBE).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c2pp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  LDT_SLOT_QUEUE_PROBE=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p$v -o run -- python3 $R/bench.py --workload c2p --steps 40 --no-cpu-baseline --only-resident > $O/p$v.json 2> $O/p$v.err || { tail -5 $O/p$v.err; exit 1; }
  grep -h '"value"' $O/p$v.json | head -1 | cut -c1-120
done
python3 $R/tools/queue_summary.py $O/p1 $O/p0
