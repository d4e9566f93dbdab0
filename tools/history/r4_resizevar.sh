#!/bin/bash
# Round-4 A/B of resize builds (libldt_<v>.so via LDT_LIBRARY; "cur" = the
# default libldt.so): resize/golden parity tests on the default build, then
# per build a c2 bench line without host/dataset/CPU legs (pipelined and
# standalone stage times), alternated twice. usage: bash tools/r4_resizevar.sh <tag> v1 [v2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py -x -q --timeout 120 --timeout-method thread -k "golden or config_batches or fullbatch or resize or large_image or tall or progressive or raw" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in cur "$@"; do
    if [ $v = cur ]; then unset LDT_LIBRARY; else export LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_$v.so; fi
    for w in ${WORKLOADS:-c2}; do
      timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --dataset-batches 0 --no-registered --host-reps 1 --steps 100 --warmup 20 > $O/${v}_${w}_$rep.json 2> $O/${v}_${w}_$rep.err || { tail -20 $O/${v}_${w}_$rep.err; exit 1; }
      python3 - $O/${v}_${w}_$rep.json $v $w $rep <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sa = b.get("stages_standalone_ms", {})
print(sys.argv[2], sys.argv[3], sys.argv[4], "value", b["value"], "host", b.get("value_host_input"), "resize pipe/solo ms",
      b["stages_ms_per_step"]["resize"], sa.get("resize"), "frac", b["roofline"]["frac"], b["roofline"].get("standalone", {}).get("frac"))
PY
    done
  done
done
unset LDT_LIBRARY
echo resizevar done
