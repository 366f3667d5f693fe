# waves dealt work-ranked entries (GWAOI_DEAL): parity, then A/B timing
GWAOI_LIB=goworld_amd/lib/variants/deal.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py tests/test_strips_gpu.py > gpurun_out/pytest_r03af_deal.log 2>&1 || { tail -30 gpurun_out/pytest_r03af_deal.log; exit 1; }
tail -1 gpurun_out/pytest_r03af_deal.log
timeout -k 10 500 python -u tools/variants.py run base deal base deal > gpurun_out/variants_r03af.log 2>&1 || { tail -20 gpurun_out/variants_r03af.log; exit 1; }
cat gpurun_out/variants_r03af.log
