#!/bin/bash
# Multi-rank rehearsal of bench.py on the one-GPU box (gloo, ranks share the
# GPU), output kept under gpurun_out/reh; then the Huffman symbol-record
# timing experiment beside the shipped build (huff_rounds probe).
# usage: bash tools/rehearse_r5.sh <ranks>
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/reh
N=${1:-2}
LDT_BENCH_BACKEND=gloo timeout -k 10 800 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $N --steps 3 --warmup 1 --no-cpu-baseline --dataset-batches 2 --dataset-epochs 1 --host-reps 1 > gpurun_out/reh/out_$N.txt 2> gpurun_out/reh/err_$N.txt
rc=$?
echo "rehearsal $N ranks rc $rc"
grep "^\[rank" gpurun_out/reh/err_$N.txt | tail -20
head -c 300 gpurun_out/reh/out_$N.txt
exit $rc
