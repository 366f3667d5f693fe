#!/bin/bash
# keygen with two S' entries per thread (base) against one (kg1): the whole GPU suite on the default,
# then the cfg3 bench interleaved twice and a kernel trace of each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r05u15.log 2>&1 || { tail -40 gpurun_out/pytest_r05u15.log; exit 1; }
tail -2 gpurun_out/pytest_r05u15.log
timeout -k 10 600 python -u tools/variants.py run base kg1 base kg1 -- --steps 50 --warmup 5 > gpurun_out/r05u15_ab.txt 2>&1 || { tail -5 gpurun_out/r05u15_ab.txt; exit 1; }
cat gpurun_out/r05u15_ab.txt
for v in base kg1; do
  O=$R/gpurun_out/kt_r05u15_$v
  mkdir -p $O
  unset GWAOI_LIB; [ $v = kg1 ] && export GWAOI_LIB=$R/goworld_amd/lib/variants/kg1.so
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0 --breakdown-steps 0 > $O/b.json 2> $O/b.err) || { echo "trace $v failed"; tail -5 $O/b.err; exit 1; }
  python3 tools/tick_kernels.py $O/run_kernel_trace.csv $v | head -4
done
unset GWAOI_LIB
