#!/bin/bash
# Extra PMC passes on the cfg3 bench: bash tools/pmc.sh <tag> "<counters pass1>" "<counters pass2>" ...
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp
ARGS="--steps 6 --warmup 1 --no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --cfg5-steps 0 --small-flush-reps 0 --wire-steps 0 --host-tick-steps 0 --claims-steps 0"
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/p$i.err
done
