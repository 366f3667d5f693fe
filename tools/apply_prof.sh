#!/bin/bash
# Kernel-trace the bench's headline and claims ticks for libgwaoi variants (GPU box):
#   bash tools/apply_prof.sh base br ...   -> gpurun_out/apply_prof_<v>/ (rocprofv3 databases)
# then (here) python3 tools/apply_prof.py gpurun_out/apply_prof_*
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
    if [ "$v" = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/apply_prof_$v -o p -- python3 $R/bench.py --no-cpu-baseline \
        --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --sync-steps 0 --wire-steps 0 --small-flush-reps 0 \
        > $R/gpurun_out/apply_prof_$v.json 2> $R/gpurun_out/apply_prof_$v.err || { echo "$v failed"; exit 1; }
done
