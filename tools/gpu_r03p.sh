#!/bin/bash
# r03p: apply with 2 / 4 ops per thread, finish with 4 tiles per block (bench A/B), parity of ap4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/variants.py run base ap2 ap4 ft4 base ap2 ap4 ft4 > gpurun_out/variants_r03p.log 2>&1 || { tail -20 gpurun_out/variants_r03p.log; exit 1; }
cat gpurun_out/variants_r03p.log
GWAOI_LIB=$R/goworld_amd/lib/variants/ap4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r03p.log 2>&1; echo "ap4 parity rc=$?"; tail -1 gpurun_out/pytest_r03p.log
