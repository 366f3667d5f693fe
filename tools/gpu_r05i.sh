#!/bin/bash
# GPU suite on the round-5 code (sparse flush, premarked claims, time-balanced XCD ranges), the
# premark A/B, the block schedule, and a bench line with the small-flush leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05i.log 2>&1 || { tail -40 gpurun_out/pytest_r05i.log; exit 1; }
tail -3 gpurun_out/pytest_r05i.log
BT_UNIT=256 BT_TICKS=4 GWAOI_LIB=$R/goworld_amd/lib/variants/bt.so timeout -k 10 200 python -u tools/blocktime.py > gpurun_out/r05_blocktime_h.txt 2>&1 || { cat gpurun_out/r05_blocktime_h.txt; exit 1; }
head -14 gpurun_out/r05_blocktime_h.txt
bash tools/trace_variants.sh r05i base > gpurun_out/r05i_variants.log 2>&1 || { tail -20 gpurun_out/r05i_variants.log; exit 1; }
GWAOI_PREMARK_LATE=1 bash tools/trace_variants.sh r05il base >> gpurun_out/r05i_variants.log 2>&1 || exit 1
GWAOI_SPECIAL_SIDE=0 bash tools/trace_variants.sh r05is base >> gpurun_out/r05i_variants.log 2>&1 || exit 1
cat gpurun_out/r05i_variants.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 > gpurun_out/bench_r05i.json 2> gpurun_out/bench_r05i.err || { tail -20 gpurun_out/bench_r05i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_r05i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['p99_tick_ms'], d['roofline']); print(json.dumps(d.get('small_flush')))"
