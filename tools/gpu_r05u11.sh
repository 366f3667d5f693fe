#!/bin/bash
# (the GWAOI_DEFER_DONE deferral was removed after this run: profiles/r05_ab_defer_done.txt)
# Deferred done events (the next flush signals a flush's end): the whole GPU suite, the cfg3 bench
# with GWAOI_DEFER_DONE=1 (default) / 0 interleaved twice, a kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r05u11.log 2>&1 || { tail -40 gpurun_out/pytest_r05u11.log; exit 1; }
tail -2 gpurun_out/pytest_r05u11.log
A="--steps 50 --warmup 5 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0"
for rep in 1 2; do
  for v in 1 0; do
    GWAOI_DEFER_DONE=$v timeout -k 10 200 python -u bench.py $A > gpurun_out/r05u11_${v}_$rep.json 2> gpurun_out/r05u11_${v}_$rep.err || { tail -5 gpurun_out/r05u11_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r05u11_${v}_$rep.json').read().strip().splitlines()[-1]); print('defer=$v rep $rep', round(d['ms_per_step'],4), round(d['p99_tick_ms'],4), d['roofline']['avg_launch_ms'], d['stages_ms_per_tick'])"
  done
done
O=$R/gpurun_out/kt_r05u11
mkdir -p $O
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0 --breakdown-steps 0 > $O/b.json 2> $O/b.err) || { echo "trace failed"; tail -5 $O/b.err; exit 1; }
python3 tools/tick_kernels.py $O/run_kernel_trace.csv defer_done
