#!/bin/bash
# cfg5 inputs before the process group: the 4-rank strip job alone, the default line's 4-rank
# rehearsal, then the op-by-op probe of GPU work after a gloo init
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash tools/gpu_r05q.sh || exit 1
bash tools/gpu_r05g.sh || exit 1

timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sparse or tick_finish" > gpurun_out/pytest_r05t_sparse.log 2>&1; tail -3 gpurun_out/pytest_r05t_sparse.log
