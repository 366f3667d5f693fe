set -o pipefail
# round-4 final code: GPU suite, the default bench line, and the two-rank gloo rehearsal of the multi-GPU line
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
bash tools/gpu_run.sh r04p "" || exit 1
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 --cpu-seconds 3 --host-tick-steps 0 --wire-steps 0 > gpurun_out/bench_r04p_gloo2.json 2> gpurun_out/bench_r04p_gloo2.err || { tail -20 gpurun_out/bench_r04p_gloo2.err; exit 1; }
tail -c 300 gpurun_out/bench_r04p_gloo2.json
