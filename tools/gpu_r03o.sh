#!/bin/bash
# r03o: keygen counting only the cell changers (GWAOI_DELTA_COUNTS): GPU tests, bench A/B, trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/pytest_r03o.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_r03o.log | head; tail -40 gpurun_out/pytest_r03o.log; exit 1; }
tail -1 gpurun_out/pytest_r03o.log
timeout -k 10 600 python -u tools/variants.py run base counts_old base counts_old > gpurun_out/variants_r03o.log 2>&1 || { tail -20 gpurun_out/variants_r03o.log; exit 1; }
cat gpurun_out/variants_r03o.log
bash tools/trace_variants.sh r03o base
