#!/bin/bash
# r03v: adaptive cell size: all GPU tests (incl. at-size), cfg3 / cfg4 / cfg5 benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/pytest_r03v.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_r03v.log | head; tail -40 gpurun_out/pytest_r03v.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_r03v.log | tail -1
B="--no-cpu-baseline --host-io-steps 0 --sync-steps 0 --host-tick-steps 0 --wire-steps 0"
for w in cfg3 cfg4 cfg5; do
  A=""; [ $w != cfg3 ] && A="--steps 10 --warmup 3 --cfg4-steps 0"
  timeout -k 10 300 python -u bench.py $B --workload $w $A > gpurun_out/bench_r03v_$w.json 2> gpurun_out/bench_r03v_$w.err || { tail -20 gpurun_out/bench_r03v_$w.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r03v_$w.json').read().strip().splitlines()[-1]);print('$w', round(d['ms_per_step'],4), round(d['p99_tick_ms'],4), d['config'].get('total_cells'), d.get('stages_ms_per_tick'), json.dumps(d.get('cfg4_strong') or {})[:200])"
done
