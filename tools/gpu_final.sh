#!/bin/bash
# A round's closing GPU call: the -m gpu suite, smoke, the default bench line (tools/gpu_check.sh),
# the cfg3 kernel trace + PMC passes (tools/profile.sh), and the two-rank gloo rehearsal of the
# multi-GPU bench line.  usage: bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_check.sh $TAG && bash tools/profile.sh $TAG || exit 1
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 --cpu-seconds 3 --host-tick-steps 0 --wire-steps 0 > gpurun_out/bench_${TAG}_gloo2.json 2> gpurun_out/bench_${TAG}_gloo2.err || { tail -20 gpurun_out/bench_${TAG}_gloo2.err; exit 1; }
tail -c 300 gpurun_out/bench_${TAG}_gloo2.json
