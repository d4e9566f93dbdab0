set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6_x
cd $R
for lib in libldt_nozero.so libldt.so libldt_nozero.so libldt.so; do
  LDT_PROBE_TOLERATE=1 LDT_LIBRARY=$R/lance-distributed-training_amd/ldt_amd/$lib timeout -k 10 120 python tools/probes/huff_rounds.py c2 > $R/gpurun_out/r6_x/$lib.txt 2>&1 || exit 1
  echo $lib $(grep "^c2" $R/gpurun_out/r6_x/$lib.txt | grep -o "'t_write_us': [0-9.]*\|'huffman': [0-9.]*")
done
