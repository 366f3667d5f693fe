#!/bin/bash
# r03r: sync id table in 64-B three-way buckets: all GPU tests, sync leg, decode kernel times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --ignore=tests/test_configs_full.py --ignore=tests/test_cfg3_full.py > gpurun_out/pytest_r03r.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_r03r.log | head; tail -40 gpurun_out/pytest_r03r.log; exit 1; }
tail -1 gpurun_out/pytest_r03r.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 8 > gpurun_out/bench_r03r_$r.json 2> gpurun_out/bench_r03r_$r.err || { tail -20 gpurun_out/bench_r03r_$r.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r03r_$r.json').read().strip().splitlines()[-1]);s=d['sync_leg'];print('run $r', round(d['ms_per_step'],4), round(s['decode_flush_ms'],4), round(s['collect_ms'],4))"
done
OUT=$R/gpurun_out/prof_sync_r
mkdir -p $OUT
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --host-io-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 4 > $OUT/bench.json 2> $OUT/err.log) || { tail -5 $OUT/err.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_sync_r/run_kernel_stats.csv")):
    n=r["Name"]
    if any(k in n for k in ("k_decode","k_fan","k_moves_apply","k_scatter")):
        print(n[:60], r["Calls"], round(float(r["AverageNs"])/1e3,1))
PY
