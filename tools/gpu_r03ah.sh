# cell scan tile (cells per thread 16 / 8 / 4) and XCD ranges split by work: parity, then A/B timing
for v in s4 xb; do
  GWAOI_LIB=goworld_amd/lib/variants/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py tests/test_strips_gpu.py > gpurun_out/pytest_r03ah_$v.log 2>&1 || { tail -30 gpurun_out/pytest_r03ah_$v.log; exit 1; }
  tail -1 gpurun_out/pytest_r03ah_$v.log
done
timeout -k 10 700 python -u tools/variants.py run base s8 s4 xb base s8 s4 xb > gpurun_out/variants_r03ah.log 2>&1 || { tail -20 gpurun_out/variants_r03ah.log; exit 1; }
cat gpurun_out/variants_r03ah.log
