#!/bin/bash
# Round-3 artefacts at HEAD: the default bench line (the driver's command), then the cfg3 rocprof trace + PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
( time timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err ) 2> gpurun_out/bench_default.time || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.time
timeout -k 10 700 bash tools/profile.sh $1 || exit 1
