# merged strips default; tile size 256 / 128 / 64: parity, then A/B timing
for v in ct64 ct128; do
  GWAOI_LIB=goworld_amd/lib/variants/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py tests/test_strips_gpu.py > gpurun_out/pytest_r03ae_$v.log 2>&1 || { tail -30 gpurun_out/pytest_r03ae_$v.log; exit 1; }
  tail -1 gpurun_out/pytest_r03ae_$v.log
done
timeout -k 10 700 python -u tools/variants.py run base nomerge ct128 ct64 ct64w8 base ct128 ct64 ct64w8 > gpurun_out/variants_r03ae.log 2>&1 || { tail -20 gpurun_out/variants_r03ae.log; exit 1; }
cat gpurun_out/variants_r03ae.log
