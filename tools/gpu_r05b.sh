#!/bin/bash
# round 5: GPU suite on the persistent-wave k_combined, unit schedules, kernel-trace A/B of the variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05b.log 2>&1 || { tail -40 gpurun_out/pytest_r05b.log; exit 1; }
tail -3 gpurun_out/pytest_r05b.log
BT_TICKS=4 GWAOI_LIB=$R/goworld_amd/lib/variants/bt.so timeout -k 10 200 python -u tools/blocktime.py > gpurun_out/r05_blocktime_cq.txt 2>&1 || { cat gpurun_out/r05_blocktime_cq.txt; exit 1; }
BT_TICKS=4 GWAOI_LIB=$R/goworld_amd/lib/variants/b1bt.so timeout -k 10 200 python -u tools/blocktime.py > gpurun_out/r05_blocktime_cq_b1.txt 2>&1 || exit 1
BT_UNIT=256 BT_TICKS=4 GWAOI_LIB=$R/goworld_amd/lib/variants/cq0bt.so timeout -k 10 200 python -u tools/blocktime.py > gpurun_out/r05_blocktime_cq0.txt 2>&1 || exit 1
head -12 gpurun_out/r05_blocktime_cq.txt
bash tools/trace_variants.sh r05b base cq0 b1 b2 pf wpe6 > gpurun_out/r05b_variants.log 2>&1 || { tail -20 gpurun_out/r05b_variants.log; exit 1; }
cat gpurun_out/r05b_variants.log
