set -o pipefail
bash tools/gpu_run.sh r04d "" --steps 20 --warmup 5 || exit 1
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 --cpu-seconds 3 --host-tick-steps 0 --wire-steps 0 > gpurun_out/bench_r04d_gloo2.json 2> gpurun_out/bench_r04d_gloo2.err || { tail -20 gpurun_out/bench_r04d_gloo2.err; exit 1; }
tail -c 600 gpurun_out/bench_r04d_gloo2.json
