#!/bin/bash
# Profile the cfg3 tick on the GPU box: kernel trace + stats, then separate PMC passes
# (rocprofv3 does not split counters over passes; each pass stays within the gfx950 slots).
# usage: bash tools/profile.sh <tag> [bench args...]
set -e
TAG=${1:-r04}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp
ARGS="--steps 8 --warmup 2 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --host-io-steps 0 --sync-steps 0 --wire-steps 0 --small-flush-reps 0 --claims-steps 0 $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_sq.err
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_tcp -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_tcp.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_fetch.err
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d $OUT/pmc_rdreq -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_rdreq.err
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum --output-format csv -d $OUT/pmc_dram -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_dram.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc_write.err
ls $OUT
