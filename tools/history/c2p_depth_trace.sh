#!/bin/bash
# Kernel traces of the c2p line at depth 6 and 7 (resident and host-input
# legs), to see which HIP queues the slots' k_prog dispatches land on.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c2pd
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for d in 6 7; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/d$d -o run -- python3 $R/bench.py --workload c2p --depth $d --host-depth $d --steps 40 --no-cpu-baseline --dataset-batches 0 --host-reps 1 --no-registered > $O/d$d.json 2> $O/d$d.err || { tail -5 $O/d$d.err; exit 1; }
done
python3 $R/tools/queue_summary.py $O/d6 $O/d7
