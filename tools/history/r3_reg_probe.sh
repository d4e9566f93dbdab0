#!/bin/bash
# Round-3 probe of the host-input paths on the GPU box: host phase times of
# the copy vs registered legs, then a rocprofv3 kernel + memory-copy trace of
# each leg (which engine moves the cells, what runs on the compute queue).
# usage: bash tools/r3_reg_probe.sh <tag> [workload]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
W=${2:-c2}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 200 python tools/probes/reg_probe.py $W > $O/reg_probe.txt 2>&1 || { tail -20 $O/reg_probe.txt; exit 1; }
grep -v "^ldt host" $O/reg_probe.txt
grep "^ldt host" $O/reg_probe.txt | tail -6
cd /tmp && export TMPDIR=/tmp
for leg in copy registered; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace_$leg -o run --output-format csv -- python3 $R/tools/probes/reg_trace.py $W $leg > $O/trace_$leg.log 2>&1 || { tail -5 $O/trace_$leg.log; exit 1; }
done
echo probe done
