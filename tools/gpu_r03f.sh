#!/bin/bash
# r03f: GPU tests without the at-size files, bench A/B (bucketed vs legacy apply, speculative vs not), kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --ignore=tests/test_configs_full.py --ignore=tests/test_cfg3_full.py > gpurun_out/pytest_r03f.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_r03f.log; exit 1; }
tail -2 gpurun_out/pytest_r03f.log
B="--no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0"
run() {  # name, env, args
  env $2 timeout -k 10 200 python -u bench.py $B $3 > gpurun_out/bench_r03f_$1.json 2> gpurun_out/bench_r03f_$1.err || { tail -20 gpurun_out/bench_r03f_$1.err; exit 1; }
}
run bkt "GWAOI_MOVES_LEGACY=0" "" && run legacy "GWAOI_MOVES_LEGACY=1" "" && run nospec "GWAOI_MOVES_LEGACY=0" "--no-speculative" && run bkt2 "GWAOI_MOVES_LEGACY=0" "" && run legacy2 "GWAOI_MOVES_LEGACY=1" "" || exit 1
python3 - <<'PY'
import json
for f in ["bkt","legacy","nospec","bkt2","legacy2"]:
    d=json.loads(open(f"gpurun_out/bench_r03f_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"],4), round(d["p99_tick_ms"],4), d["roofline"]["avg_launch_ms"], d.get("stages_ms_per_tick"))
PY
bash tools/trace_variants.sh r03f base
