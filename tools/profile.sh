#!/bin/bash
# Profile the cfg3 bench on the GPU box: kernel trace + stats, then PMC passes.
# usage: bash tools/profile.sh <tag> [bench args...]
set -e
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp
ARGS="--steps 8 --warmup 2 --no-cpu-baseline --cfg4-steps 0 --host-tick-steps 0 $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_sq.err
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_fetch.err
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_write.err
ls -R $OUT | head -50
