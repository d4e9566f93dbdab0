set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4c; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -x -v --timeout 120 --timeout-method thread -k "copy or pipelined or registered or fused or fullbatch or prefetch or status_tickets or golden" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/r4_hostab.sh r4c
