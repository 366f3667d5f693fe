# flat sweep sub-variants: parity of the new code paths, then A/B timing
for v in flat7x4a flat7x3; do
  GWAOI_LIB=goworld_amd/lib/variants/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py > gpurun_out/pytest_r03z_$v.log 2>&1 || { tail -30 gpurun_out/pytest_r03z_$v.log; exit 1; }
  tail -1 gpurun_out/pytest_r03z_$v.log
done
timeout -k 10 700 python -u tools/variants.py run base flat7 flat7a flat7x4 flat7x3 flat7x4a flat7 flat7a flat7x4 > gpurun_out/variants_r03z.log 2>&1 || { tail -20 gpurun_out/variants_r03z.log; exit 1; }
cat gpurun_out/variants_r03z.log
