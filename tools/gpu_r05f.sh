#!/bin/bash
# k_combined: the block kernel with the XCD ranges cut by measured time (pb), by candidates (pbc),
# the round-4 schedule (cq0); the premarked claims on and off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
BT_UNIT=256 BT_TICKS=4 GWAOI_LIB=$R/goworld_amd/lib/variants/pbbt.so timeout -k 10 200 python -u tools/blocktime.py > gpurun_out/r05_blocktime_pb.txt 2>&1 || { cat gpurun_out/r05_blocktime_pb.txt; exit 1; }
head -14 gpurun_out/r05_blocktime_pb.txt
bash tools/trace_variants.sh r05f pb pbc cq0 > gpurun_out/r05f_variants.log 2>&1 || { tail -20 gpurun_out/r05f_variants.log; exit 1; }
GWAOI_BATCH_READY=0 bash tools/trace_variants.sh r05f0 pb >> gpurun_out/r05f_variants.log 2>&1 || { tail -20 gpurun_out/r05f_variants.log; exit 1; }
cat gpurun_out/r05f_variants.log
