set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/progprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in 256 64 8; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/n$n -o run --output-format csv -- python3 $R/tests/probe_prog.py $n > $O/n$n.log 2>&1 || { tail -5 $O/n$n.log; exit 1; }
  f=$(find $O/n$n -name '*kernel_stats.csv' | head -1); echo "n=$n"; cut -c1-60,200- $f | head -6
done
