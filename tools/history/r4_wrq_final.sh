set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_wq.log 2>&1 || { tail -30 gpurun_out/pytest_wq.log; exit 1; }
tail -1 gpurun_out/pytest_wq.log
bash tools/r4_wrq.sh c q1 cur
