#!/bin/bash
# rocprofv3 kernel + memory-copy traces of the c2 host-input leg (pipelined
# to_tensor_fn on host RecordBatches) and of the resident leg, for the
# timeline analysis in tools/trace_timeline.py. usage: bash tools/r3_hosttrace.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for leg in ${LEGS:-host resident}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace_$leg -o run --output-format csv -- python3 $R/tools/probes/host_trace.py $leg > $O/trace_$leg.log 2>&1 || { tail -5 $O/trace_$leg.log; exit 1; }
  grep "ms/step" $O/trace_$leg.log
done
echo hosttrace done
