# k_combined block schedule (diagnostics build), tile order on and off
export GWAOI_LIB=$PWD/goworld_amd/lib/variants/bt.so
timeout -k 10 300 python -u tools/blocktime.py > gpurun_out/blocktime_r03ad.txt 2>&1 || { tail -20 gpurun_out/blocktime_r03ad.txt; exit 1; }
echo "== order off" >> gpurun_out/blocktime_r03ad.txt
GWAOI_TILE_ORDER=0 timeout -k 10 300 python -u tools/blocktime.py >> gpurun_out/blocktime_r03ad.txt 2>&1 || { tail -20 gpurun_out/blocktime_r03ad.txt; exit 1; }
cat gpurun_out/blocktime_r03ad.txt
unset GWAOI_LIB
for v in m2 m4; do
  GWAOI_LIB=goworld_amd/lib/variants/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py > gpurun_out/pytest_r03ad_$v.log 2>&1 || { tail -30 gpurun_out/pytest_r03ad_$v.log; exit 1; }
  tail -1 gpurun_out/pytest_r03ad_$v.log
done
timeout -k 10 600 python -u tools/variants.py run base m2 m3 m4 base m2 m3 m4 > gpurun_out/variants_r03ad.log 2>&1 || { tail -20 gpurun_out/variants_r03ad.log; exit 1; }
cat gpurun_out/variants_r03ad.log
