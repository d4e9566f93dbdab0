#!/bin/bash
# Round-4 host-path A/B 3: the bench's host legs (3 back-to-back copying legs,
# registered leg) at host depth 2 and 3, NUMA-bound rank, alternated 3 times.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4ab3}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py tests/test_gpu_loaders.py -x -q --timeout 120 --timeout-method thread -k "copy or pipelined or registered or status or golden or fullbatch or prefetch or loader or register or huffman_decoder" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 ./tools/probes/hip_api_cost > $O/hip_api_cost.txt 2>&1 && grep "waiting for a busy" $O/hip_api_cost.txt
for rep in 1 2 3; do
  for hd in 2 3; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --dataset-batches 0 --steps 60 --warmup 10 --host-depth $hd > $O/b_d${hd}_$rep.json 2> $O/b_d${hd}_$rep.err || { tail -5 $O/b_d${hd}_$rep.err; exit 1; }
    python3 - $O/b_d${hd}_$rep.json $hd $rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
print("depth", sys.argv[2], "rep", sys.argv[3], {k: d.get(k) for k in ("value", "value_host_input", "value_host_input_reps", "value_host_registered")})
print("   ", d["host_us_per_call"], {k: d["host_placement"][k] for k in ("gpu_numa", "copy_cpus", "numa_bound_cpus")})
PY
  done
done
