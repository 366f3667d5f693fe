#!/bin/bash
# tile order inside each XCD range: stable counting sort (st1), the same with candidate-count
# classes (st1tt0), 4 bands (b4), against base and no order; cfg3 and cfg5; then cfg5 kernel traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
: > gpurun_out/r05w_ab.txt
for rep in 1 2; do
  for v in base st1 st1tt0 b4 noorder; do
    unset GWAOI_LIB GWAOI_TILE_ORDER
    case $v in base) ;; noorder) export GWAOI_TILE_ORDER=0;; *) export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so;; esac
    for wl in cfg5 cfg3; do
      timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0 > gpurun_out/r05w_${v}_${wl}.json 2> gpurun_out/r05w_${v}_${wl}.err || { tail -5 gpurun_out/r05w_${v}_${wl}.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/r05w_${v}_${wl}.json').read().strip().splitlines()[-1]); print('$rep $v $wl', round(d['ms_per_step'],4), (d.get('roofline') or {}).get('avg_launch_ms'))" >> gpurun_out/r05w_ab.txt
    done
  done
done
unset GWAOI_LIB GWAOI_TILE_ORDER
cat gpurun_out/r05w_ab.txt
export TMPDIR=/tmp
for v in base noorder; do
  unset GWAOI_TILE_ORDER
  [ $v = noorder ] && export GWAOI_TILE_ORDER=0
  OUT=$R/gpurun_out/tv_r05w_cfg5_$v
  mkdir -p $OUT
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --workload cfg5 --steps 8 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/err.log) || { echo "trace $v failed"; tail -5 $OUT/err.log; exit 1; }
  python3 tools/tick_kernels.py $OUT/run_kernel_trace.csv cfg5_$v
done
