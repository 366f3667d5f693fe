#!/bin/bash
# r03q: decode with 2 / 4 records per thread: sync tests per variant, sync leg A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for v in base dec2 dec4; do
  if [ $v = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_sync.py tests/test_wire.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r03q_$v.log 2>&1 || { echo "$v tests failed"; tail -30 gpurun_out/pytest_r03q_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/pytest_r03q_$v.log)"
done
for r in 1 2; do for v in base dec2 dec4; do
  if [ $v = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 8 > gpurun_out/bench_r03q_$v.json 2> gpurun_out/bench_r03q_$v.err || { tail -20 gpurun_out/bench_r03q_$v.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r03q_$v.json').read().strip().splitlines()[-1]);s=d['sync_leg'];print('$v', round(d['ms_per_step'],4), round(s['decode_flush_ms'],4), round(s['collect_ms'],4))"
done; done
unset GWAOI_LIB
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_sync_q
mkdir -p $OUT
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --host-io-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 4 > $OUT/bench.json 2> $OUT/err.log) || { tail -5 $OUT/err.log; exit 1; }
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/prof_sync_q/run_kernel_stats.csv")))
for r in rows:
    n=r["Name"]
    if any(k in n for k in ("k_decode","k_fan","k_moves_apply","k_prologue","k_route")):
        print(n[:60], r["Calls"], round(float(r["AverageNs"])/1e3,1))
PY
