#!/bin/bash
# A/B of an env switch on the cfg3 bench: bash tools/ab_env.sh VAR [reps]   (VAR=0 vs VAR=1, interleaved)
# Runs the GPU tests first; prints ms/tick, p99 and the per-stage times of each run.
set -o pipefail
VAR=$1; REPS=${2:-2}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
for r in $(seq $REPS); do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --sync-steps 0 > gpurun_out/ab_${v}_${r}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_${v}_${r}.json')); print('$VAR=$v', round(d['ms_per_step'],4), 'p99', round(d['p99_tick_ms'],4), 'pcie', round(d['pcie_inclusive']['ms_per_step'],3), d['stages_ms_per_tick'])"
  done
done
