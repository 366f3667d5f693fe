# tile order folded into k_finish: parity, A/B order on/off, k_combined HBM bytes on/off
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py tests/test_strips_gpu.py tests/test_golden.py > gpurun_out/pytest_r03ag.log 2>&1 || { tail -30 gpurun_out/pytest_r03ag.log; exit 1; }
tail -1 gpurun_out/pytest_r03ag.log
timeout -k 10 300 python -u tools/variants.py run base base > gpurun_out/variants_r03ag.log 2>&1 && \
GWAOI_TILE_ORDER=0 timeout -k 10 300 python -u tools/variants.py run base base >> gpurun_out/variants_r03ag.log 2>&1 || { tail -20 gpurun_out/variants_r03ag.log; exit 1; }
cat gpurun_out/variants_r03ag.log
bash tools/pmc.sh r03ag_on FETCH_SIZE WRITE_SIZE && GWAOI_TILE_ORDER=0 bash tools/pmc.sh r03ag_off FETCH_SIZE WRITE_SIZE && \
for t in on off; do echo "== order $t"; python3 tools/pmc_median.py gpurun_out/pmc_r03ag_$t k_combined; done > gpurun_out/pmc_r03ag.txt
cat gpurun_out/pmc_r03ag.txt
