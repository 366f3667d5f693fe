#!/bin/bash
# the split fan-out write A/B, the 8-waves-per-SIMD k_combined variants, then the 4-rank gloo
# rehearsal of the default line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r05o.sh || exit 1
bash tools/gpu_r05m.sh || exit 1
bash tools/gpu_r05g.sh
