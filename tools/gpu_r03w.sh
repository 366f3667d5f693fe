#!/bin/bash
# r03w: the special pass skips tiles keygen saw no special entity in: all GPU tests, bench, trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/pytest_r03w.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_r03w.log | head; tail -40 gpurun_out/pytest_r03w.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_r03w.log | tail -1
B="--no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0"
for r in 1 2; do
timeout -k 10 300 python -u bench.py $B > gpurun_out/bench_r03w_$r.json 2> gpurun_out/bench_r03w_$r.err || { tail -20 gpurun_out/bench_r03w_$r.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r03w_$r.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['p99_tick_ms'],4), d.get('stages_ms_per_tick'))"
done
bash tools/trace_variants.sh r03w base
