#!/bin/bash
# k_combined persistent-wave A/B: static one-unit-per-wave, the old block kernel, unit schedules
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
BT_TICKS=4 GWAOI_LIB=$R/goworld_amd/lib/variants/stbt.so timeout -k 10 200 python -u tools/blocktime.py > gpurun_out/r05_blocktime_st.txt 2>&1 || { cat gpurun_out/r05_blocktime_st.txt; exit 1; }
head -14 gpurun_out/r05_blocktime_st.txt
bash tools/trace_variants.sh r05c base st cq0 > gpurun_out/r05c_variants.log 2>&1 || { tail -20 gpurun_out/r05c_variants.log; exit 1; }
cat gpurun_out/r05c_variants.log
