#!/bin/bash
# cfg5 child job rehearsal: the default line at --gpus 4 over gloo on one GPU (four ranks share it),
# only the cfg3 headline and the cfg5 sub-record; the child's phase lines go to stderr
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --gpus 4 --dist-backend gloo --steps 5 --warmup 2 --no-cpu-baseline \
  --host-io-steps 0 --host-tick-steps 0 --sync-steps 0 --wire-steps 0 --cfg4-steps 0 --small-flush-reps 0 \
  --cfg5-timeout 400 > gpurun_out/bench_gloo4_r05.json 2> gpurun_out/bench_gloo4_r05.err
rc=$?
grep "cfg5 rank" gpurun_out/bench_gloo4_r05.err | head -60
python -c "import json; d=json.loads(open('gpurun_out/bench_gloo4_r05.json').read().strip().splitlines()[-1]); c=d.get('cfg5_strips') or {}; print(json.dumps({k: c.get(k) for k in ('ms_per_step','setup_s','phases_s','job','error','strip_counts','rank0_phase_ms_per_tick','host_waits_per_tick')}))"
exit $rc
