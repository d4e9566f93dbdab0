#!/bin/bash
# Round-4 host-path probe on the GPU box: topology + host copy/DMA bandwidth
# (tools/probes/host_bw), then the host-call split of the copying
# to_tensor_fn with cgroup throttling deltas, then a default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4p1}
mkdir -p $O
cd $R
cat /sys/fs/cgroup/cpu.stat > $O/cpustat0.txt 2>&1
timeout -k 10 120 ./tools/probes/host_bw 17.2 20 > $O/host_bw.txt 2>&1 || { tail -5 $O/host_bw.txt; exit 1; }
cat $O/host_bw.txt
cat /sys/fs/cgroup/cpu.stat > $O/cpustat1.txt 2>&1
timeout -k 10 180 python3 tools/probes/host_calls2.py c2 3 copy > $O/host_calls.txt 2>&1 || { tail -5 $O/host_calls.txt; exit 1; }
cat /sys/fs/cgroup/cpu.stat > $O/cpustat2.txt 2>&1
cat $O/host_calls.txt
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat /sys/fs/cgroup/cpu.stat > $O/cpustat3.txt 2>&1
python3 - $O <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().splitlines()[-1])
print({k: d.get(k) for k in ("value", "value_host_input", "value_host_registered", "value_dataset", "host_us_per_call")})
EOF
for f in $O/cpustat*.txt; do echo "$f: $(tr '\n' ' ' < $f)"; done
