#!/bin/bash
# Instruction-cache check of the c2 pipeline (3 batches in flight, the kernels
# co-resident): the SQC counters this ROCm lists, then one --pmc pass of the
# I-cache counters and one of the wait/issue counters over a short resident
# bench. usage: bash tools/history/r6_icache.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1
grep -o "SQC_[A-Z0-9_]*\|SQ_IFETCH[A-Z0-9_]*\|SQ_INST_LEVEL[A-Z0-9_]*\|SQ_WAIT_INST[A-Z0-9_]*" $O/avail.txt | sort -u > $O/avail_sq.txt || true
echo "counters: $(wc -l < $O/avail_sq.txt)"
B="python3 $R/bench.py --steps 10 --warmup 3 --only-resident --no-cpu-baseline --no-stage-events"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- $B > $O/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $O/$name.log; return 1; }
  python3 $R/tools/pmc_raw.py $O/$name > $O/$name.txt && echo "== $name" && cat $O/$name.txt
}
pass ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH && \
pass wait SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAVES
