#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) of tools/probes/probe_resize.py <mode> (PROBE=<file in tools/probes>).
# Stops at the first failed pass. usage: bash tools/pmc.sh <tag> <mode> [pass numbers]
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_$1
cd /tmp && export TMPDIR=/tmp
GROUPS_=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
 "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
 "SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_IFETCH"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
PASSES=${*:3}
PASSES=${PASSES:-"1 2 3 4 5"}
for i in $PASSES; do
  ctrs=${GROUPS_[$((i-1))]}
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/pmc_$1/p$i -o run -- python3 $R/tools/probes/${PROBE:-probe_resize.py} $2 > $R/gpurun_out/pmc_$1/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 $R/gpurun_out/pmc_$1/p$i.log; exit $rc; fi
done
echo pmc done $1
