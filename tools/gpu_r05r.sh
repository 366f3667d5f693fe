#!/bin/bash
# strip_ops alone: 1 process, 4 processes, 4 processes in a gloo group
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/cfg5_inputs_probe2.py 1 8 0 > gpurun_out/r05r_1.txt 2>&1; tail -3 gpurun_out/r05r_1.txt
timeout -k 10 150 python -u tools/cfg5_inputs_probe2.py 4 8 0 > gpurun_out/r05r_4.txt 2>&1; grep -E "procs|tick" gpurun_out/r05r_4.txt | tail -12
timeout -k 10 150 python -u tools/cfg5_inputs_probe2.py 4 8 1 > gpurun_out/r05r_4g.txt 2>&1; grep -E "procs|tick" gpurun_out/r05r_4g.txt | tail -12
exit 0
