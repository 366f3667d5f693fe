#!/bin/bash
# Kernel trace of the cfg3 bench for each variant lib: bash tools/trace_variants.sh TAG base NAME...
# (base = goworld_amd/lib/libgwaoi.so; NAME = goworld_amd/lib/variants/NAME.so)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --cfg5-steps 0 --small-flush-reps 0 --host-tick-steps 0 --wire-steps 0 --claims-steps 0"
for v in "$@"; do
  OUT=$R/gpurun_out/tv_${TAG}_$v
  mkdir -p $OUT
  if [ "$v" = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py $ARGS > $OUT/bench.json 2> $OUT/err.log) || { echo "trace $v failed"; tail -5 $OUT/err.log; exit 1; }
  python3 $R/tools/tick_kernels.py $OUT/run_kernel_trace.csv $v
done
