#!/bin/bash
# r03e: GPU tests (speculative flush pipeline), bench speculative vs not, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_r03e.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r03e.log; exit 1; }
tail -2 gpurun_out/pytest_r03e.log
B="--no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0"
for k in 1 2; do
  timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_r03e_spec$k.json 2> gpurun_out/bench_r03e_spec$k.err || { tail -20 gpurun_out/bench_r03e_spec$k.err; exit 1; }
  timeout -k 10 200 python -u bench.py $B --no-speculative > gpurun_out/bench_r03e_nospec$k.json 2> gpurun_out/bench_r03e_nospec$k.err || { tail -20 gpurun_out/bench_r03e_nospec$k.err; exit 1; }
done
python3 - <<'PY'
import json
for f in ["spec1","nospec1","spec2","nospec2"]:
    d=json.loads(open(f"gpurun_out/bench_r03e_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"],4), round(d["p99_tick_ms"],4), d["roofline"]["avg_launch_ms"], d["tick_loop"][:60])
PY
bash tools/trace_variants.sh r03e base
