#!/bin/bash
# (the GWAOI_EXTRA_MARKERS probe hook was removed after this run: profiles/r05_probe_markers.txt)
# Probe: the price of a marker packet between two flushes (GWAOI_EXTRA_MARKERS=0/2/4 more event
# records after each flush's done event), from the kernel trace's gap between ticks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 0 2 4; do
  O=$R/gpurun_out/kt_r05u10_$k
  mkdir -p $O
  (cd /tmp && GWAOI_EXTRA_MARKERS=$k timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0 --breakdown-steps 0 > $O/b.json 2> $O/b.err) || { echo "trace $k failed"; tail -5 $O/b.err; exit 1; }
  python3 tools/tick_kernels.py $O/run_kernel_trace.csv markers_$k | head -1
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('  bench under trace ms_per_step', round(d['ms_per_step'],4))"
done
