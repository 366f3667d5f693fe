#!/bin/bash
# round 5, first call: counter list, k_combined block schedule at HEAD, stall-breakdown PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/r05_counters.txt 2>&1 || true
cd $R
BT_TICKS=4 GWAOI_LIB=$R/goworld_amd/lib/variants/bt.so timeout -k 10 200 python -u tools/blocktime.py > gpurun_out/r05_blocktime_base.txt 2>&1 || exit 1
cat gpurun_out/r05_blocktime_base.txt | head -20
bash tools/pmc.sh r05a "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" || { echo pmc failed; ls gpurun_out/pmc_r05a; tail -5 gpurun_out/pmc_r05a/*.err; exit 1; }
ls gpurun_out/pmc_r05a
