#!/bin/bash
# GWAOI_F_UNIQUE_MOVES: its parity tests + the speculative/cfg3 subset, then the cfg3 bench with the
# flag (default) against --claims, interleaved twice, and one kernel trace of each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_unique_moves_gpu.py tests/test_cfg3_full.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "unique or cfg3 or speculative or incremental" > gpurun_out/pytest_r05u1.log 2>&1 || { tail -40 gpurun_out/pytest_r05u1.log; exit 1; }
tail -2 gpurun_out/pytest_r05u1.log
A="--steps 50 --warmup 5 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0"
: > gpurun_out/r05u1_ab.txt
for rep in 1 2; do
  for v in uniq claims; do
    X=""; [ $v = claims ] && X="--claims"
    timeout -k 10 200 python -u bench.py $A $X > gpurun_out/r05u1_${v}_${rep}.json 2> gpurun_out/r05u1_${v}_${rep}.err || { tail -5 gpurun_out/r05u1_${v}_${rep}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r05u1_${v}_${rep}.json').read().strip().splitlines()[-1]); print('$rep $v', round(d['ms_per_step'],4), round(d['p99_tick_ms'],4), d['roofline']['avg_launch_ms'], d['debug_counters'])" >> gpurun_out/r05u1_ab.txt
  done
done
cat gpurun_out/r05u1_ab.txt
for v in uniq claims; do
  X=""; [ $v = claims ] && X="--claims"
  O=$R/gpurun_out/kt_r05u1_$v
  mkdir -p $O
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0 --breakdown-steps 0 $X > $O/b.json 2> $O/b.err) || { echo "trace $v failed"; tail -5 $O/b.err; exit 1; }
  python3 tools/tick_kernels.py $(find $O -name '*kernel_trace.csv' | head -1) $v
done
