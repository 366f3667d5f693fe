#!/bin/bash
# the cfg5 input ops one by one, 4 processes in a gloo group (the slow case), then 2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 170 python -u tools/cfg5_inputs_probe.py 4 16777216 1 > gpurun_out/r05s_4g.txt 2>&1; grep procs gpurun_out/r05s_4g.txt
timeout -k 10 170 python -u tools/cfg5_inputs_probe.py 2 16777216 1 > gpurun_out/r05s_2g.txt 2>&1; grep procs gpurun_out/r05s_2g.txt
exit 0
