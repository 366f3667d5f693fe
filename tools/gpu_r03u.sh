#!/bin/bash
# r03u: cell size at config 3 (clustered): cells_per_dist 4, 3, 2, 5
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
B="--no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0"
for c in 4 3 2 5 4 2; do
  timeout -k 10 300 python -u bench.py $B --cells-per-dist $c > gpurun_out/bench_r03u_$c.json 2> gpurun_out/bench_r03u_$c.err || { tail -20 gpurun_out/bench_r03u_$c.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r03u_$c.json').read().strip().splitlines()[-1]);print('cfg3 cells D/$c', round(d['ms_per_step'],4), d.get('stages_ms_per_tick'))"
done
