#!/bin/bash
# Round-end evidence on the GPU box: default benches with CPU baselines, the
# rocprofv3 kernel-trace summary of the default bench command, PMC traffic of
# the resize kernel (c2, c5) and decode-efficiency counters (c2).
# usage: bash tools/round_profiles.sh <tag>
set -o pipefail
T=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round_$T
mkdir -p $O
for w in c2 c1 c4 c5; do
  timeout -k 10 300 python $R/bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
  echo "$w $(python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print(d['value'], d.get('cpu_baseline',{}).get('value'), d['roofline']['frac'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
bash $R/tools/traffic.sh c2 c2_$T > /dev/null && bash $R/tools/traffic.sh c5 c5_$T > /dev/null || exit 1
bash $R/tools/pmc.sh eff_$T jpeg 1 2 3 > /dev/null || exit 1
python3 $R/tools/decode_eff.py $R/gpurun_out/pmc_eff_$T c2 > $O/pmc_c2_decode.json
echo done
