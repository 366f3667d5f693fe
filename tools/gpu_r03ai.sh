# HEAD sanity after the knob commit: parity subset + smoke with the default library
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cfg3_full.py > gpurun_out/pytest_r03ai.log 2>&1 || { tail -30 gpurun_out/pytest_r03ai.log; exit 1; }
tail -1 gpurun_out/pytest_r03ai.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
