#!/bin/bash
# k_fan_write with the walk twice, no hits scratch (GWAOI_FAN_FUSED): sync parity, then the sync leg A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
GWAOI_LIB=$R/goworld_amd/lib/variants/ff.so timeout -k 10 400 python -u -m pytest tests/test_sync.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05u_ff.log 2>&1 || { tail -30 gpurun_out/pytest_r05u_ff.log; exit 1; }
tail -2 gpurun_out/pytest_r05u_ff.log
A="--steps 3 --warmup 1 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --host-io-steps 0 --small-flush-reps 0 --sync-steps 10"
for rep in 1 2; do
  for v in base ff; do
    if [ $v = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
    timeout -k 10 300 python -u bench.py $A > gpurun_out/r05u_$v.json 2> gpurun_out/r05u_$v.err || { tail -5 gpurun_out/r05u_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r05u_$v.json').read().strip().splitlines()[-1]); s=d.get('sync_leg') or {}; print('$rep $v', {k: s.get(k) for k in ('decode_flush_ms','collect_ms','records_per_tick')})"
  done
done
unset GWAOI_LIB
