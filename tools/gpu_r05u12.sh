#!/bin/bash
# (the GWAOI_PROBE_HOSTWRITE hook was removed after this run: profiles/r05_probe_hostwrite.txt)
# Probe: does a kernel that stores to mapped host memory end late?  keygen's last block stores 4 B
# there (GWAOI_PROBE_HOSTWRITE=1) or not; kernel-trace gaps after keygen and between ticks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 0 1; do
  O=$R/gpurun_out/kt_r05u12_$k
  mkdir -p $O
  (cd /tmp && GWAOI_PROBE_HOSTWRITE=$k timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0 --breakdown-steps 0 > $O/b.json 2> $O/b.err) || { echo "trace $k failed"; tail -5 $O/b.err; exit 1; }
  python3 tools/tick_kernels.py $O/run_kernel_trace.csv hostwrite_$k | head -1
  python3 tools/kernel_gaps.py $O/run_kernel_trace.csv
done
