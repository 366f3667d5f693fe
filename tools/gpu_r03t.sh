#!/bin/bash
# r03t: cell size at config 5 / config 4 density (one GPU): cells_per_dist 2, 3, 4; kernel trace of cfg5
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
B="--no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0 --steps 10 --warmup 2"
for w in cfg5 cfg4; do for c in 4 3 2; do
  timeout -k 10 300 python -u bench.py $B --workload $w --cells-per-dist $c > gpurun_out/bench_r03t_${w}_$c.json 2> gpurun_out/bench_r03t_${w}_$c.err || { tail -20 gpurun_out/bench_r03t_${w}_$c.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r03t_${w}_$c.json').read().strip().splitlines()[-1]);print('$w cells D/$c', round(d['ms_per_step'],4), d.get('stages_ms_per_tick'), d.get('rank0_phase_ms_per_tick'), (d.get('roofline') or {}).get('avg_launch_ms'))"
done; done
export TMPDIR=/tmp
OUT=$R/gpurun_out/tv_cfg5
mkdir -p $OUT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py $B --workload cfg5 > $OUT/bench.json 2> $OUT/err.log) || { tail -5 $OUT/err.log; exit 1; }
python3 - <<'PY'
import csv
rows=sorted(csv.DictReader(open("gpurun_out/tv_cfg5/run_kernel_stats.csv")), key=lambda r:-float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"])/1e3,1), round(float(r["Percentage"]),1))
PY
