#!/bin/bash
# skew-gated tile order (sk6 / sk10: even ranges keep frame order) against base and no order;
# cfg3, cfg5 twice, cfg4 once
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
: > gpurun_out/r05x_ab.txt
run() {
  local rep=$1 v=$2 wl=$3
  unset GWAOI_LIB GWAOI_TILE_ORDER
  case $v in base) ;; noorder) export GWAOI_TILE_ORDER=0;; *) export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so;; esac
  timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0 > gpurun_out/r05x_${v}_${wl}.json 2> gpurun_out/r05x_${v}_${wl}.err || { tail -5 gpurun_out/r05x_${v}_${wl}.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05x_${v}_${wl}.json').read().strip().splitlines()[-1]); print('$rep $v $wl', round(d['ms_per_step'],4), (d.get('roofline') or {}).get('avg_launch_ms'))" >> gpurun_out/r05x_ab.txt
}
for rep in 1 2; do
  for v in base sk6 sk10; do
    run $rep $v cfg5 || exit 1
    run $rep $v cfg3 || exit 1
  done
done
for v in base sk6 sk10 noorder; do run 1 $v cfg4 || exit 1; done
bash tools/gpu_r05y.sh
unset GWAOI_LIB GWAOI_TILE_ORDER
cat gpurun_out/r05x_ab.txt
