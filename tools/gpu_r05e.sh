#!/bin/bash
# k_combined static work-balanced unit schedule: unit schedule, kernel-trace A/B, then the GPU suite
# (sparse flush parity) and a bench line with the small-flush leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
BT_TICKS=4 GWAOI_LIB=$R/goworld_amd/lib/variants/bt.so timeout -k 10 200 python -u tools/blocktime.py > gpurun_out/r05_blocktime_jobs.txt 2>&1 || { cat gpurun_out/r05_blocktime_jobs.txt; exit 1; }
head -14 gpurun_out/r05_blocktime_jobs.txt
bash tools/trace_variants.sh r05e base th16 th28 nosplit cq0 > gpurun_out/r05e_variants.log 2>&1 || { tail -20 gpurun_out/r05e_variants.log; exit 1; }
cat gpurun_out/r05e_variants.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05e.log 2>&1 || { tail -40 gpurun_out/pytest_r05e.log; exit 1; }
tail -3 gpurun_out/pytest_r05e.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 > gpurun_out/bench_r05e.json 2> gpurun_out/bench_r05e.err || { tail -20 gpurun_out/bench_r05e.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_r05e.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']); print(json.dumps(d.get('small_flush')))"
