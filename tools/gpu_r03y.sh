# flat sweep: parity with the variant library, then A/B timing
export GWAOI_LIB=goworld_amd/lib/variants/flat7.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py tests/test_golden.py > gpurun_out/pytest_r03y_flat7.log 2>&1 || { tail -30 gpurun_out/pytest_r03y_flat7.log; exit 1; }
tail -3 gpurun_out/pytest_r03y_flat7.log
unset GWAOI_LIB
timeout -k 10 600 python -u tools/variants.py run base flat flat7 flat7u1 flat7u4 base flat7 > gpurun_out/variants_r03y.log 2>&1 || { tail -20 gpurun_out/variants_r03y.log; exit 1; }
cat gpurun_out/variants_r03y.log
