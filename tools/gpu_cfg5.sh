#!/bin/bash
# cfg5 bench legs on the 1-GPU box: small single strip, (FULL=1) the full 2^24
# single strip, and a 2-rank gloo rehearsal of the multi-strip path (both
# ranks on cuda:0; RCCL allows one rank per device).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 240 python -u bench.py --workload cfg5 --entities 1000000 --steps 10 --warmup 2 > gpurun_out/cfg5_1m.json 2> gpurun_out/cfg5_1m.err || { echo "cfg5 1m failed"; tail -20 gpurun_out/cfg5_1m.err; exit 1; }
cat gpurun_out/cfg5_1m.json
if [ -n "$FULL" ]; then
  timeout -k 10 400 python -u bench.py --workload cfg5 --steps 10 --warmup 2 > gpurun_out/cfg5_full.json 2> gpurun_out/cfg5_full.err || { echo "cfg5 full failed"; tail -20 gpurun_out/cfg5_full.err; exit 1; }
  cat gpurun_out/cfg5_full.json
fi
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --workload cfg5 --entities 4000000 --steps 8 --warmup 2 --dist-backend gloo > gpurun_out/cfg5_r2.json 2> gpurun_out/cfg5_r2.err || { echo "cfg5 2-rank failed"; tail -30 gpurun_out/cfg5_r2.err; exit 1; }
cat gpurun_out/cfg5_r2.json
