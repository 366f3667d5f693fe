#!/bin/bash
# r03m: full GPU check at HEAD (every -m gpu test incl. the at-size files), smoke, default bench, profile passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread > gpurun_out/pytest_r03m.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_r03m.log | head -20; tail -30 gpurun_out/pytest_r03m.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_r03m.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r03m.log 2>&1 || { tail -20 gpurun_out/smoke_r03m.log; exit 1; }
tail -1 gpurun_out/smoke_r03m.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r03m_default.json 2> gpurun_out/bench_r03m_default.err || { tail -20 gpurun_out/bench_r03m_default.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r03m_default.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['p99_tick_ms'], d['roofline'], d['stages_ms_per_tick'])"
timeout -k 10 700 bash tools/profile.sh r03v2 > /dev/null || exit 1
echo profile ok
