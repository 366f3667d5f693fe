#!/bin/bash
# software-pipelined flat sweep (GWAOI_FLAT_PIPE) at three VGPR budgets against the base
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05k.log 2>&1 || { tail -40 gpurun_out/pytest_r05k.log; exit 1; }
tail -3 gpurun_out/pytest_r05k.log
bash tools/trace_variants.sh r05k base fp fpw6 fpw0 > gpurun_out/r05k_variants.log 2>&1 || { tail -20 gpurun_out/r05k_variants.log; exit 1; }
cat gpurun_out/r05k_variants.log
GWAOI_LIB=$R/goworld_amd/lib/variants/fpw0.so timeout -k 10 300 python -u -m pytest tests/test_cfg3_full.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "cfg3 or speculative or incremental" > gpurun_out/pytest_r05k_fp.log 2>&1 || { tail -30 gpurun_out/pytest_r05k_fp.log; exit 1; }
tail -2 gpurun_out/pytest_r05k_fp.log
mkdir -p gpurun_out/sf_r05k
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sf_r05k -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --small-flush-reps 30 > $R/gpurun_out/sf_r05k/bench.json 2> $R/gpurun_out/sf_r05k/err.log) || { tail -5 gpurun_out/sf_r05k/err.log; exit 1; }
python3 tools/sparse_trace.py gpurun_out/sf_r05k/run_kernel_trace.csv small_flush
python3 -c "import json; d=json.loads(open('gpurun_out/sf_r05k/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d.get('small_flush')))"
