#!/bin/bash
# k_prog instruction mix of one build (LDT_LIBRARY): SALU / VALU / LDS /
# branch instructions and wave cycles per launch (tools/probes/prog_rate.py
# at depth 7 under one rocprofv3 --pmc pass).
# usage: bash tools/history/r6_prog_pmc.sh <tag> <lib.so>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1/pmc_${2%.so}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$2 timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O -o run -- python3 $R/tools/probes/prog_rate.py 7 > $O.log 2>&1 || { tail -5 $O.log; exit 1; }
cd $R && python3 tools/pmc_raw.py $O k_prog
