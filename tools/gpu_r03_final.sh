#!/bin/bash
# Round-3 final check at HEAD: every GPU test, smoke, the driver's bench command, then the cfg3 rocprof trace + PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { tail -30 gpurun_out/pytest_final.log; exit 1; }
tail -2 gpurun_out/pytest_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
bash tools/gpu_r03_prof.sh ${1:-r03final}
