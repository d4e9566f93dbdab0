#!/bin/bash
# Sync warm-up sweep (same box): throughput at depth 3 and standalone Huffman ms.
for w in c2 c1; do
for warm in 0 50 100 0 50 100; do
  LDT_SYNC_WARM=$warm timeout -k 10 100 python bench.py --workload $w --no-cpu-baseline --steps 30 > gpurun_out/s.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s.json')); print('$w warm=$warm', d['value'], d['stages_standalone_ms']['huffman'])"
done
done
