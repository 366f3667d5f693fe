#!/bin/bash
# cfg5 inputs before the process group: the 4-rank strip job alone, the default line's 4-rank
# rehearsal, then the op-by-op probe of GPU work after a gloo init
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash tools/gpu_r05q.sh || exit 1
bash tools/gpu_r05g.sh || exit 1
bash tools/gpu_r05s.sh
