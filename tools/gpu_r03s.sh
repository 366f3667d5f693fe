#!/bin/bash
# r03s: k_combined knob variants with the row pairs, Z row pairs, arrival-side re-zeroing; parity of zpair / arz
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/variants.py run base zpair u3 u6 q512 wpe7 arz base zpair arz > gpurun_out/variants_r03s.log 2>&1 || { tail -20 gpurun_out/variants_r03s.log; exit 1; }
cat gpurun_out/variants_r03s.log
for v in zpair arz; do
GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_strips_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r03s_$v.log 2>&1; echo "$v parity rc=$?"; tail -1 gpurun_out/pytest_r03s_$v.log
done
