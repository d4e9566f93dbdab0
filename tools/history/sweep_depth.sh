set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/sweep1; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/probes/host_cost.py > $O/host.txt 2>&1 || { tail -5 $O/host.txt; exit 1; }
cat $O/host.txt
for q in 4 8; do for d in 2 3 4 6; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --depth $d > $O/b_${q}_${d}.json 2>$O/b_${q}_${d}.err || { tail -3 $O/b_${q}_${d}.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b_${q}_${d}.json').readline());print('q=$q d=$d',d['value'],d['ms_per_step'])"
done; done
