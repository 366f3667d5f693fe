# k_combined block schedule (diagnostics build), tile order on and off
export GWAOI_LIB=$PWD/goworld_amd/lib/variants/bt.so
timeout -k 10 300 python -u tools/blocktime.py > gpurun_out/blocktime_r03ad.txt 2>&1 || { tail -20 gpurun_out/blocktime_r03ad.txt; exit 1; }
echo "== order off" >> gpurun_out/blocktime_r03ad.txt
GWAOI_TILE_ORDER=0 timeout -k 10 300 python -u tools/blocktime.py >> gpurun_out/blocktime_r03ad.txt 2>&1 || { tail -20 gpurun_out/blocktime_r03ad.txt; exit 1; }
cat gpurun_out/blocktime_r03ad.txt
