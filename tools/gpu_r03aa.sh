# flat sweep: where the time goes (timing-only EXP variants drop work; events wrong) + no-regroup parity
GWAOI_LIB=goworld_amd/lib/variants/fnp.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py > gpurun_out/pytest_r03aa_fnp.log 2>&1 || { tail -30 gpurun_out/pytest_r03aa_fnp.log; exit 1; }
tail -1 gpurun_out/pytest_r03aa_fnp.log
timeout -k 10 700 python -u tools/variants.py run base f fnp fnd fnx fnz fnxz f fnp > gpurun_out/variants_r03aa.log 2>&1 || { tail -20 gpurun_out/variants_r03aa.log; exit 1; }
cat gpurun_out/variants_r03aa.log
