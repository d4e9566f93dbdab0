#!/bin/bash
# Spread of the resident c2 line on one box: the driver's shape (20 timed
# steps after 5 warm-up) five times, then 100 timed steps twice.
# usage: bash tools/history/r6_spread.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_$1
mkdir -p $O
cd $R
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --only-resident --no-cpu-baseline > $O/k20_$i.json 2> $O/k20_$i.err || { tail -5 $O/k20_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/k20_$i.json'));print('K=20', d['value'], d['ms_per_step'])"
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 100 --only-resident --no-cpu-baseline > $O/k100_$i.json 2> $O/k100_$i.err || { tail -5 $O/k100_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/k100_$i.json'));print('K=100', d['value'], d['ms_per_step'])"
done
