#!/bin/bash
# r03g: which combination fails: speculative x bucketed apply (Python errors continue; a signal/timeout stops)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
B="--no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --host-tick-steps 0 --wire-steps 0"
for cfg in "legacy_spec:GWAOI_MOVES_LEGACY=1:" "bkt_nospec:GWAOI_MOVES_LEGACY=0:--no-speculative" "legacy_nospec:GWAOI_MOVES_LEGACY=1:--no-speculative" "bkt_spec_notime:GWAOI_MOVES_LEGACY=0:--no-timing"; do
  IFS=: read name envv args <<< "$cfg"
  env $envv timeout -k 10 200 python -u bench.py $B $args > gpurun_out/bench_r03g_$name.json 2> gpurun_out/bench_r03g_$name.err
  rc=$?
  echo "$name rc=$rc"; tail -3 gpurun_out/bench_r03g_$name.err | grep -v amdgpu.ids
  if [ $rc -ge 124 ]; then exit 1; fi
  if [ $rc -eq 0 ]; then python3 -c "
import json;d=json.loads(open('gpurun_out/bench_r03g_$name.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4),round(d['p99_tick_ms'],4),d['roofline']['avg_launch_ms'],d.get('stages_ms_per_tick'))"; fi
done
