#!/bin/bash
# r03k: default bench (host_tick replay with one table per entity), gloo rehearsals of --gpus 2 (cfg3, cfg5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r03k_default.json 2> gpurun_out/bench_r03k_default.err || { tail -20 gpurun_out/bench_r03k_default.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r03k_default.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['p99_tick_ms']); print(json.dumps(d['host_tick']))"
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --workload cfg5 --entities 2000000 --steps 10 --warmup 2 > gpurun_out/bench_r03k_cfg5_gloo2.json 2> gpurun_out/bench_r03k_cfg5_gloo2.err || { tail -20 gpurun_out/bench_r03k_cfg5_gloo2.err; exit 1; }
tail -c 1500 gpurun_out/bench_r03k_cfg5_gloo2.json
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 --sync-steps 0 --host-tick-steps 0 --wire-steps 0 --cfg4-steps 3 > gpurun_out/bench_r03k_cfg3_gloo2.json 2> gpurun_out/bench_r03k_cfg3_gloo2.err || { tail -20 gpurun_out/bench_r03k_cfg3_gloo2.err; exit 1; }
tail -c 600 gpurun_out/bench_r03k_cfg3_gloo2.json
