# flat sweep default + heaviest-first tile order: parity, then A/B (order on/off, lock-step)
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py tests/test_golden.py tests/test_strips_gpu.py > gpurun_out/pytest_r03ac.log 2>&1 || { tail -30 gpurun_out/pytest_r03ac.log; exit 1; }
tail -1 gpurun_out/pytest_r03ac.log
timeout -k 10 300 python -u tools/variants.py run base base > gpurun_out/variants_r03ac.log 2>&1 || { tail -20 gpurun_out/variants_r03ac.log; exit 1; }
GWAOI_TILE_ORDER=0 timeout -k 10 300 python -u tools/variants.py run base lockstep >> gpurun_out/variants_r03ac.log 2>&1 || { tail -20 gpurun_out/variants_r03ac.log; exit 1; }
timeout -k 10 300 python -u tools/variants.py run base >> gpurun_out/variants_r03ac.log 2>&1 || { tail -20 gpurun_out/variants_r03ac.log; exit 1; }
cat gpurun_out/variants_r03ac.log
