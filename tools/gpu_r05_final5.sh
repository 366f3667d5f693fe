#!/bin/bash
# Round 5's closing measurements, part A: the GPU suite, smoke, the default bench line, the cfg3
# kernel trace + PMC passes (tools/profile.sh), the k_combined block schedule.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash tools/gpu_check.sh r05final5 || exit 1
bash tools/profile.sh r05final5 || { echo "profile failed"; ls gpurun_out/prof_r05final5; exit 1; }
BT_UNIT=256 BT_TICKS=4 GWAOI_LIB=$R/goworld_amd/lib/variants/bt.so timeout -k 10 200 python -u tools/blocktime.py > gpurun_out/r05final5_blocktime.txt 2>&1 || { cat gpurun_out/r05final5_blocktime.txt; exit 1; }
head -14 gpurun_out/r05final5_blocktime.txt
