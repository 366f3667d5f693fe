#!/bin/bash
# Round 5's closing measurements, part B: the default line's multi-rank rehearsals on one GPU over
# gloo (2 ranks: the whole line; 4 ranks: the cfg3 headline and the cfg5 child job)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 --cpu-seconds 3 --host-tick-steps 0 --wire-steps 0 > gpurun_out/bench_r05final_gloo2.json 2> gpurun_out/bench_r05final_gloo2.err || { tail -20 gpurun_out/bench_r05final_gloo2.err; exit 1; }
tail -c 400 gpurun_out/bench_r05final_gloo2.json
bash tools/gpu_r05g.sh
