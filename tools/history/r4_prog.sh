#!/bin/bash
# k_prog A/B on the GPU box: progressive parity tests with the in-tree
# library, then k_prog kernel times (rocprofv3 kernel stats of
# tests/probe_prog.py, one c2p batch) for each library named on the command
# line (ldt_amd/libldt_<name>.so; "cur" = libldt.so), then the c2p bench line.
# usage: bash tools/r4_prog.sh <tag> <lib>...
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; shift
O=$R/gpurun_out/prog_$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "progressive or golden or corrupt" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = cur ]; then export LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt.so; else export LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 $R/tests/probe_prog.py 256 > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/$v/**/run_kernel_stats.csv', recursive=True)[0])):
    if 'k_prog' in r['Name']: print('$v k_prog avg ms', float(r['AverageNs'])/1e6, 'calls', r['Calls'])
"
done
unset LDT_LIBRARY
cd $R
timeout -k 10 400 python bench.py --workload c2p --no-cpu-baseline > $O/bench_c2p.json 2> $O/bench_c2p.err || { tail -5 $O/bench_c2p.err; exit 1; }
echo "c2p: $(head -c 300 $O/bench_c2p.json)"
