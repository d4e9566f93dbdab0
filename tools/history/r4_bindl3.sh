#!/bin/bash
# Round-4 A/B of the host-input leg's copy-pool binding: LDT_OPT_COPY_BIND 1
# (default: each pool thread pinned to one GPU-local core, one per L3 domain)
# vs 2 (each thread free within its core's L3 domain). The slow mode seen in
# some processes (pool wake and slot wait ~200 us per call instead of ~5 us,
# profiles/r4/warm_ab_r4w.txt) comes and goes per process, so the legs run
# in 6 alternating processes per mode, 3 reps each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4bl}
mkdir -p $O
cd $R
for rep in 1 2 3 4 5 6; do
  for b in 1 2; do
    timeout -k 10 200 python bench.py --copy-bind $b --no-cpu-baseline --dataset-batches 0 --no-registered --no-config-legs --host-reps 3 > $O/b${b}_$rep.json 2> $O/b${b}_$rep.err || { tail -20 $O/b${b}_$rep.err; exit 1; }
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=b['host_us_per_call']; print('bind', sys.argv[2], 'rep', sys.argv[3], 'resident', b['value'], 'host reps', b['value_host_input_reps'], 'slot', h['slot'], 'wake', h['copy_wake'], 'span', h['copy_span'])" $O/b${b}_$rep.json $b $rep
  done
done
echo bindl3 done
