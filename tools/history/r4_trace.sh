#!/bin/bash
# Round-4 host-path timelines: rocprofv3 kernel + memory-copy traces of the
# c2 host (copy) / reg / resident legs (tools/probes/host_trace.py), with the
# gap summary (tools/probes/trace_gaps.py). usage: bash tools/r4_trace.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for leg in ${LEGS:-host reg resident}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace_$leg -o run --output-format csv -- python3 $R/tools/probes/host_trace.py $leg > $O/trace_$leg.log 2>&1 || { tail -5 $O/trace_$leg.log; exit 1; }
  grep "ms/step" $O/trace_$leg.log
  python3 $R/tools/probes/trace_gaps.py $O/trace_$leg 30
done
echo trace done
