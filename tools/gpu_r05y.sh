#!/bin/bash
# round 4's tree (r04tree/, a git worktree of 5d26e4b built here) against HEAD on cfg5 and cfg4:
# bench lines and cfg5 kernel traces, to place the round-5 slowdown of the big worlds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r05y_ab.txt
for rep in 1; do
  for t in r04 head; do
    D=$R; [ $t = r04 ] && D=$R/r04tree
    for wl in cfg5 cfg4; do
      (cd $D && timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 > $R/gpurun_out/r05y_${t}_${wl}.json 2> $R/gpurun_out/r05y_${t}_${wl}.err) || { tail -5 gpurun_out/r05y_${t}_${wl}.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/r05y_${t}_${wl}.json').read().strip().splitlines()[-1]); print('$rep $t $wl', round(d['ms_per_step'],4), (d.get('roofline') or {}).get('avg_launch_ms'))" >> gpurun_out/r05y_ab.txt
    done
  done
done
cat gpurun_out/r05y_ab.txt
for t in r04 head; do
  D=$R; [ $t = r04 ] && D=$R/r04tree
  OUT=$R/gpurun_out/tv_r05y_cfg5_$t
  mkdir -p $OUT
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $D/bench.py --workload cfg5 --steps 8 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/err.log) || { echo "trace $t failed"; tail -5 $OUT/err.log; exit 1; }
  python3 tools/tick_kernels.py $OUT/run_kernel_trace.csv cfg5_$t
done
