set -o pipefail
mkdir -p gpurun_out
GWAOI_CHECK_STAGES=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "poisons or device_enter_leave or zero_copy or incremental_sort" > gpurun_out/pytest_r04d0.log 2>&1 || { tail -30 gpurun_out/pytest_r04d0.log; exit 1; }
tail -2 gpurun_out/pytest_r04d0.log
bash tools/gpu_run.sh r04d "" --steps 20 --warmup 5 || exit 1
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 --cpu-seconds 3 --host-tick-steps 0 --wire-steps 0 > gpurun_out/bench_r04d_gloo2.json 2> gpurun_out/bench_r04d_gloo2.err || { tail -20 gpurun_out/bench_r04d_gloo2.err; exit 1; }
tail -c 600 gpurun_out/bench_r04d_gloo2.json
