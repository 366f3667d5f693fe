#!/bin/bash
# r03n: side-stream claims of the speculative launch: GPU tests, bench A/B (GWAOI_SIDE_CLAIMS), kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --ignore=tests/test_configs_full.py --ignore=tests/test_cfg3_full.py > gpurun_out/pytest_r03n.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_r03n.log | head; tail -40 gpurun_out/pytest_r03n.log; exit 1; }
tail -1 gpurun_out/pytest_r03n.log
B="--no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0"
run() {  # name, env, args
  env $2 timeout -k 10 300 python -u bench.py $B $3 > gpurun_out/bench_r03n_$1.json 2> gpurun_out/bench_r03n_$1.err || { tail -20 gpurun_out/bench_r03n_$1.err; exit 1; }
}
run side "GWAOI_SIDE_CLAIMS=1" "" && run noside "GWAOI_SIDE_CLAIMS=0" "" && run side2 "GWAOI_SIDE_CLAIMS=1" "" && run noside2 "GWAOI_SIDE_CLAIMS=0" "" || exit 1
python3 - <<'PY'
import json
for f in ["side","noside","side2","noside2"]:
    d=json.loads(open(f"gpurun_out/bench_r03n_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"],4), round(d["p99_tick_ms"],4), d["roofline"]["avg_launch_ms"])
PY
bash tools/trace_variants.sh r03n base
