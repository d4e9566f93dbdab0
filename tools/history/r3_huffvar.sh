#!/bin/bash
# A/B of Huffman write-pass variants (libldt_<v>.so via LDT_LIBRARY): the
# in-kernel phase times (tools/probes/huff_rounds.py) and a short c2 bench
# line per build, alternated twice. usage: bash tools/r3_huffvar.sh <tag> v1 [v2 ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in cur "$@"; do
    if [ $v = cur ]; then unset LDT_LIBRARY; else export LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/libldt_$v.so; fi
    timeout -k 10 120 python3 tools/probes/huff_rounds.py > $O/huff_${v}_$rep.txt 2>&1 || { tail -5 $O/huff_${v}_$rep.txt; exit 1; }
    python3 -c "
import ast
for l in open('$O/huff_${v}_$rep.txt'):
    if l.startswith('c2 '):
        d=ast.literal_eval(l[3:]); print('$v $rep', {k: d[k] for k in ('t_phase1_us','t_rounds_us','t_write_us')})"
    timeout -k 10 300 python bench.py --no-cpu-baseline --dataset-batches 0 --steps 60 --warmup 10 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -20 $O/${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1])
print('   ', d['value'], d.get('value_host_input'), 'huff standalone', d['stages_standalone_ms']['huffman'])"
  done
done
unset LDT_LIBRARY
echo huffvar done
