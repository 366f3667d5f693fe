#!/bin/bash
# r03l: X' row-grouping and finish-tile variants (bench A/B), parity of the grouped build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/variants.py run base xpair2 xpair3 xpair2u3 ft8 base xpair2 xpair3 > gpurun_out/variants_r03l.log 2>&1 || { tail -20 gpurun_out/variants_r03l.log; exit 1; }
cat gpurun_out/variants_r03l.log
for v in xpair2 xpair3; do
GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r03l_$v.log 2>&1; echo "$v parity rc=$?"; tail -1 gpurun_out/pytest_r03l_$v.log
done
