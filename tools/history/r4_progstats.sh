#!/bin/bash
# k_prog diagnostics on the GPU box: the stats build's luma-chain time split
# (tools/probes/prog_stats.py), then the A/B of tools/r4_prog.sh.
# usage: bash tools/r4_progstats.sh <tag> <lib>...
set -o pipefail
cd $GRAFT_REPO_ROOT
LDT_LIBRARY=$GRAFT_REPO_ROOT/lance-distributed-training_amd/ldt_amd/libldt_pstats.so timeout -k 10 120 python3 tools/probes/prog_stats.py 64 > gpurun_out/prog_stats_$1.txt 2>&1 || { tail -5 gpurun_out/prog_stats_$1.txt; exit 1; }
tail -1 gpurun_out/prog_stats_$1.txt
bash tools/r4_prog.sh "$@"
