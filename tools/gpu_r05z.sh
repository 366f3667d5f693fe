#!/bin/bash
# the tile-order skew gate by candidate count (default 8 classes) against off (sk0) and 4 / 12;
# cfg3 and cfg5 twice, cfg4 once; a parity subset on the default first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cfg3_full.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "cfg3 or incremental or speculative or tile or regrow" > gpurun_out/pytest_r05z.log 2>&1 || { tail -30 gpurun_out/pytest_r05z.log; exit 1; }
tail -2 gpurun_out/pytest_r05z.log
: > gpurun_out/r05z_ab.txt
run() {
  local rep=$1 v=$2 wl=$3
  unset GWAOI_LIB GWAOI_TILE_ORDER
  case $v in base) ;; noorder) export GWAOI_TILE_ORDER=0;; *) export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so;; esac
  timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0 > gpurun_out/r05z_${v}_${wl}.json 2> gpurun_out/r05z_${v}_${wl}.err || { tail -5 gpurun_out/r05z_${v}_${wl}.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05z_${v}_${wl}.json').read().strip().splitlines()[-1]); print('$rep $v $wl', round(d['ms_per_step'],4), (d.get('roofline') or {}).get('avg_launch_ms'))" >> gpurun_out/r05z_ab.txt
}
for rep in 1 2; do
  for v in base sk0 sk4 sk12; do
    run $rep $v cfg5 || exit 1
    run $rep $v cfg3 || exit 1
  done
done
for v in base sk0; do run 1 $v cfg4 || exit 1; done
unset GWAOI_LIB GWAOI_TILE_ORDER
cat gpurun_out/r05z_ab.txt
bash tools/gpu_r05aa.sh
