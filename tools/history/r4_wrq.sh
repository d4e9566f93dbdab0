#!/bin/bash
# Huffman write-queue A/B on the GPU box: for each library (libldt_<name>.so;
# "cur" = libldt.so) the c2 resident rate (bench --only-resident) and the
# per-kernel WRITE_SIZE at depth 1 (rocprofv3 --pmc, tools/traffic_all.py).
# usage: bash tools/r4_wrq.sh <tag> <lib>...
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; shift
O=$R/gpurun_out/wrq_$T
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or config_batches or fused or marker" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
for v in "$@"; do
  if [ "$v" = cur ]; then L=$R/lance-distributed-training_amd/ldt_amd/libldt.so; else L=$R/lance-distributed-training_amd/ldt_amd/libldt_$v.so; fi
  LDT_LIBRARY=$L timeout -k 10 300 pytest -x -q tests/test_gpu_parity.py -k "golden or config_batches" > $O/pt_$v.log 2>&1 || { tail -20 $O/pt_$v.log; exit 1; }
  LDT_LIBRARY=$L timeout -k 10 300 python bench.py --only-resident --no-cpu-baseline > $O/c2_$v.json 2> $O/c2_$v.err || { tail -5 $O/c2_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$v.json'));print('$v c2', d['value'], 'parity', open('$O/pt_$v.log').read().strip().splitlines()[-1])"
  ( cd /tmp && export TMPDIR=/tmp && LDT_LIBRARY=$L timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/t_$v/WRITE_SIZE -o run -- python3 $R/bench.py --steps 4 --warmup 1 --depth 1 --only-resident --no-cpu-baseline > $O/t_$v.log 2>&1 ) || { echo "pmc failed"; tail -5 $O/t_$v.log; exit 1; }
  python3 $R/tools/traffic_all.py $O/t_$v | grep -E "huff|kernel"
done
