#!/bin/bash
# Kernel traces (queue and stream of every dispatch) of the progressive c2p
# path: inside the default c2 line (workload leg) and in its own line, to
# compare the HIP hardware queues its pipeline's slots land on.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c2pq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/line -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --dataset-batches 0 --host-reps 1 --no-registered --no-config-legs > $O/line.json 2> $O/line.err || { tail -5 $O/line.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/own -o run -- python3 $R/bench.py --workload c2p --steps 40 --no-cpu-baseline --dataset-batches 0 --host-reps 1 --no-registered > $O/own.json 2> $O/own.err || { tail -5 $O/own.err; exit 1; }
python3 $R/tools/queue_summary.py $O/line $O/own
