#!/bin/bash
# fused sparse flush: its parity tests, the GPU suite, the small-flush kernel trace and bench leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "sparse" > gpurun_out/pytest_r05l_sparse.log 2>&1 || { tail -40 gpurun_out/pytest_r05l_sparse.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pytest_r05l_sparse.log | tail -6
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05l.log 2>&1 || { tail -40 gpurun_out/pytest_r05l.log; exit 1; }
tail -2 gpurun_out/pytest_r05l.log
mkdir -p gpurun_out/sf_r05l
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sf_r05l -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --small-flush-reps 30 > $R/gpurun_out/sf_r05l/bench.json 2> $R/gpurun_out/sf_r05l/err.log) || { tail -5 gpurun_out/sf_r05l/err.log; exit 1; }
python3 tools/sparse_trace.py gpurun_out/sf_r05l/run_kernel_trace.csv small_flush_trace || true
grep -c k_sp_fused gpurun_out/sf_r05l/run_kernel_trace.csv || true
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 40 > gpurun_out/bench_r05l.json 2> gpurun_out/bench_r05l.err || { tail -20 gpurun_out/bench_r05l.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r05l.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['p99_tick_ms']); print(json.dumps(d.get('small_flush')))"
