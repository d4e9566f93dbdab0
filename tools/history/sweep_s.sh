#!/bin/bash
# Subsequence-length sweep: c2/c1 throughput (depth 3) and standalone Huffman ms.
for w in c2 c1; do
for cfg in "1024 1" "1024 0" "768 0" "512 0" "512 1" "1536 0" "2048 0"; do
  set -- $cfg
  LDT_SUBSEQ_BITS=$1 LDT_SUBSEQ_FIT=$2 timeout -k 10 100 python bench.py --workload $w --no-cpu-baseline --steps 30 > gpurun_out/s.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s.json')); print('$w S=$1 fit=$2', d['value'], d['stages_standalone_ms']['huffman'], d['stages_standalone_ms']['resize'])"
done
done
