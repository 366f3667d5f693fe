#!/bin/bash
# Kernel trace + PMC passes (SQ block, HBM bytes) of the bench's entity-sync leg
# (decode / fan-out / route kernels).
# usage: bash tools/prof_sync.sh <tag>     (summary: gpurun_out/prof_<tag>/summary.{md,json})
TAG=${1:-sync}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp
ARGS="--steps 4 --warmup 2 --no-cpu-baseline --cfg4-steps 0 --host-tick-steps 0 --host-io-steps 0 --breakdown-steps 0"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_sq.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_write.err || exit 1
cd $R
python3 tools/prof_summary.py $OUT $OUT/summary > /dev/null
grep -E "k_fan|k_decode|k_route|k_side" $OUT/summary.md
python3 tools/prof_sync_pmc.py $OUT/summary.json
python3 -c "import json;d=json.load(open('$OUT/trace_bench.json'));print(d['sync_leg'])"
