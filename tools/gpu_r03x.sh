#!/bin/bash
# r03x: timing experiment -- k_combined without its per-block atomic on the event counter
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/variants.py run base noatomic base noatomic > gpurun_out/variants_r03x.log 2>&1 || { tail -20 gpurun_out/variants_r03x.log; exit 1; }
cat gpurun_out/variants_r03x.log
