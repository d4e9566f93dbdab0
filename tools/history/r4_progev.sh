#!/bin/bash
# Round-4 progressive evidence on the GPU box: the GPU test suite, the c2p
# bench line (defaults: depth 4, host depth 4, CPU legs 8/16 workers),
# rocprofv3 kernel stats of the c2p resident leg, and the k_prog time split
# of the stats build (tools/probes/prog_stats.py).
# usage: bash tools/r4_progev.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/progev_$1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 500 python bench.py --workload c2p --cpu-workers 8,16 > $O/bench_c2p.json 2> $O/bench_c2p.err || { tail -5 $O/bench_c2p.err; exit 1; }
echo "c2p: $(head -c 400 $O/bench_c2p.json)"
LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_pstats.so timeout -k 10 120 python3 tools/probes/prog_stats.py 64 > $O/prog_stats.txt 2>&1 || exit 1
tail -1 $O/prog_stats.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2p -o run --output-format csv -- python3 $R/bench.py --workload c2p --only-resident --no-cpu-baseline > $O/prof_c2p.log 2>&1 || { tail -5 $O/prof_c2p.log; exit 1; }
echo progev done
