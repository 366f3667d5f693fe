#!/bin/bash
# k_combined at 8 waves per SIMD: LDS cut to 8 blocks per CU (event buffer / queue), VGPRs to 64
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash tools/trace_variants.sh r05m base w8e w8e2 w7e base > gpurun_out/r05m_variants.log 2>&1 || { tail -20 gpurun_out/r05m_variants.log; exit 1; }
grep -E "==|k_combined" gpurun_out/r05m_variants.log
for v in base w8e w8e2 w7e; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/tv_r05m_$v/bench.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('debug_counters'))" || true; done
