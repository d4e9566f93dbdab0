R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  for w in raw jpeg; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/tests/probe_resize.py $w > $R/gpurun_out/pmc/p$i.log 2>&1 || exit 1
  done
done
echo pmc done
