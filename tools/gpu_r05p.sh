#!/bin/bash
# cfg5 input generation op by op, 1 process then 4 sharing the GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/cfg5_inputs_probe.py 1 2>&1 | tee gpurun_out/r05p_inputs_1.txt | grep procs
timeout -k 10 400 python -u tools/cfg5_inputs_probe.py 4 2>&1 | tee gpurun_out/r05p_inputs_4.txt | grep procs
