#!/bin/bash
# Round 5 closing, part C: smoke + the default bench line (every leg, tick bench built) at HEAD, then
# part B's multi-rank gloo rehearsals on one GPU (2 ranks: the whole line; 4 ranks: cfg3 + cfg5 child)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05final3.log 2>&1 || { cat gpurun_out/smoke_r05final3.log; exit 1; }
tail -1 gpurun_out/smoke_r05final3.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r05final3.json 2> gpurun_out/bench_r05final3.err || { tail -20 gpurun_out/bench_r05final3.err; exit 1; }
tail -c 300 gpurun_out/bench_r05final3.json
bash tools/gpu_r05_final_b.sh
