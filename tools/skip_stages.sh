for k in 0 1 2 3; do LDT_DEBUG_SKIP=$k timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline > gpurun_out/skip_$k.json 2>gpurun_out/skip_$k.err || exit 1; python -c "
import json; d=json.load(open('gpurun_out/skip_$k.json')); print('skip $k', d['value'], d['ms_per_step'], d['stages_standalone_ms'])"; done
