set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_strips_gpu.py tests/test_sync.py tests/test_aoi_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03d.log 2>&1 || { tail -30 gpurun_out/pytest_r03d.log; exit 1; }
tail -2 gpurun_out/pytest_r03d.log
timeout -k 10 600 python -u tools/variants.py run base old nozero base old > gpurun_out/variants_r03d.log 2>&1 || { tail -20 gpurun_out/variants_r03d.log; exit 1; }
cat gpurun_out/variants_r03d.log
bash tools/trace_variants.sh r03d base
