#!/bin/bash
# Round-4 A/B of the parallel Huffman decoder's minimum subsequence length
# (LDT_OPT_SUBSEQ_BITS = 3; default 256; each image uses the smallest S >= it
# that fits its slots in 1024 lanes, so only images under ~32 KB of entropy
# data are affected): 160 / 256 / 384 / 512 bits, resident c1, c4 and c2,
# alternated twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4ss}
mkdir -p $O
cd $R
for rep in 1 2; do
  for sb in 256 160 384 512; do
    for w in c1 c4 c2; do
      timeout -k 10 200 python bench.py --workload $w --only-resident --no-cpu-baseline --opt 3=$sb > $O/ss${sb}_${w}_$rep.json 2> $O/ss${sb}_${w}_$rep.err || { tail -20 $O/ss${sb}_${w}_$rep.err; exit 1; }
      python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('subseq', sys.argv[2], sys.argv[3], 'rep', sys.argv[4], 'value', b['value'], 'huffman ms', b['stages_ms_per_step']['huffman'])" $O/ss${sb}_${w}_$rep.json $sb $w $rep
    done
  done
done
echo subseq done
