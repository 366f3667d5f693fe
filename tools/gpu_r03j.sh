#!/bin/bash
# r03j: GPU tests (no at-size files), cfg3 bench, cfg5 strip bench (bucketed apply by default at 2^24)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --ignore=tests/test_configs_full.py --ignore=tests/test_cfg3_full.py > gpurun_out/pytest_r03j.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_r03j.log; exit 1; }
tail -2 gpurun_out/pytest_r03j.log
B="--no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0"
run() {  # name, env, args
  env $2 timeout -k 10 300 python -u bench.py $B $3 > gpurun_out/bench_r03j_$1.json 2> gpurun_out/bench_r03j_$1.err || { tail -20 gpurun_out/bench_r03j_$1.err; exit 1; }
}
run cfg3 "GWAOI_X=0" "" && run cfg5 "GWAOI_X=0" "--workload cfg5 --steps 10 --warmup 2" && run cfg5_legacy "GWAOI_MOVES_BUCKETED=0" "--workload cfg5 --steps 10 --warmup 2" && run cfg4 "GWAOI_X=0" "--workload cfg4 --steps 10 --warmup 2" || exit 1
python3 - <<'PY'
import json
for f in ["cfg3","cfg5","cfg5_legacy","cfg4"]:
    d=json.loads(open(f"gpurun_out/bench_r03j_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"],4), round(d["p99_tick_ms"],4), (d.get("roofline") or {}).get("avg_launch_ms"), d.get("stages_ms_per_tick"), d.get("rank0_phase_ms_per_tick"))
PY
timeout -k 10 600 python -u tools/variants.py run base zlds192 zlds128 zlds256q448 base zlds192 > gpurun_out/variants_r03j.log 2>&1 || { tail -20 gpurun_out/variants_r03j.log; exit 1; }
cat gpurun_out/variants_r03j.log
GWAOI_LIB=$R/goworld_amd/lib/variants/zlds192.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "cfg or churn or boundary" > gpurun_out/pytest_r03j_zlds.log 2>&1; echo "zlds parity rc=$?"; tail -2 gpurun_out/pytest_r03j_zlds.log
