#!/bin/bash
# the cfg5 strip job alone, 4 gloo ranks on one GPU, with per-tick input-generation times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
GWAOI_INPUT_TRACE=1 timeout -k 10 170 python -u bench.py --workload cfg5 --gpus 4 --dist-backend gloo --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/r05q_cfg5_gloo4.json 2> gpurun_out/r05q_cfg5_gloo4.err
rc=$?
grep -E "strip_ops rank 0|cfg5 rank 0" gpurun_out/r05q_cfg5_gloo4.err | head -40
exit $rc
