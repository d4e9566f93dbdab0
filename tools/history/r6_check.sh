#!/bin/bash
# Round-6 GPU call: GPU test suite, the driver-shaped bench line and the
# stream-environment probe (tools/probes/stream_env.py). Stops at the first
# failure. usage: bash tools/history/r6_check.sh <tag> [tests|bench|streams]...
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1
shift
O=$R/gpurun_out/r6_$T
mkdir -p $O
cd $R
for part in "$@"; do
  case $part in
  tests)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
    tail -1 $O/pytest_gpu.log ;;
  bench)
    timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_c2_k20.json 2> $O/bench_c2_k20.err || { tail -5 $O/bench_c2_k20.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_c2_k20.json'));print(json.dumps(d['summary']));print(d.get('stages_standalone_ms'))" ;;
  streams)
    for wl in c2 c2p; do
      for m in clean before after; do
        timeout -k 10 240 python tools/probes/stream_env.py $m $wl > $O/streams_${wl}_$m.json 2> $O/streams_${wl}_$m.err || { tail -5 $O/streams_${wl}_$m.err; exit 1; }
        cat $O/streams_${wl}_$m.json
        LDT_SLOT_PRIORITY=1 timeout -k 10 240 python tools/probes/stream_env.py $m $wl > $O/streams_${wl}_${m}_hp.json 2> $O/streams_${wl}_${m}_hp.err || { tail -5 $O/streams_${wl}_${m}_hp.err; exit 1; }
        cat $O/streams_${wl}_${m}_hp.json
      done
    done ;;
  esac
done
echo done $T
