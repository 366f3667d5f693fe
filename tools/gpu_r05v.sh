#!/bin/bash
# cfg5 / cfg4 / cfg3 against the tile schedule: measured-time classes (base), candidate-count
# classes (tt0), no order (GWAOI_TILE_ORDER=0); then the fused fan-out A/B (tools/gpu_r05u.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
: > gpurun_out/r05v_ab.txt
for rep in 1 2; do
  for v in base tt0 noorder; do
    unset GWAOI_LIB GWAOI_TILE_ORDER
    [ $v = tt0 ] && export GWAOI_LIB=$R/goworld_amd/lib/variants/tt0.so
    [ $v = noorder ] && export GWAOI_TILE_ORDER=0
    for wl in cfg5 cfg3; do
      timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0 > gpurun_out/r05v_${v}_${wl}.json 2> gpurun_out/r05v_${v}_${wl}.err || { tail -5 gpurun_out/r05v_${v}_${wl}.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/r05v_${v}_${wl}.json').read().strip().splitlines()[-1]); print('$rep $v $wl', round(d['ms_per_step'],4), (d.get('roofline') or {}).get('avg_launch_ms'))" >> gpurun_out/r05v_ab.txt
    done
  done
done
unset GWAOI_LIB GWAOI_TILE_ORDER
cat gpurun_out/r05v_ab.txt
bash tools/gpu_r05u.sh
