#!/bin/bash
# BASELINE configs at their own sizes (tests/test_cfg3_full.py, tests/test_configs_full.py), progress printed
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_cfg3_full.py tests/test_configs_full.py -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/pytest_atsize.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_atsize.log; exit $rc
