#!/bin/bash
# One GPU call: the -m gpu suite (or a subset: $1 = pytest -k expression), then a default bench line.
# Usage (from the repo root on the box): bash tools/gpu_run.sh TAG [pytest -k expr] [bench args...]
set -o pipefail
tag=${1:-run}; kexpr=${2:-}; shift 2 2>/dev/null
mkdir -p gpurun_out
if [ -n "$kexpr" ] && [ "$kexpr" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$kexpr" > gpurun_out/pytest_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_$tag.log; exit 1; }
elif [ "$kexpr" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_$tag.log; exit 1; }
fi
tail -3 gpurun_out/pytest_$tag.log 2>/dev/null
if [ "$#" -gt 0 ] || [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
  tail -c 1500 gpurun_out/bench_$tag.json
fi
