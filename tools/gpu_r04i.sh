set -o pipefail
# round-4: the event copy-out by a kernel (GWAOI_COPYOUT_KERNEL=1) against the DMA copy, host->host leg only
mkdir -p gpurun_out
GWAOI_COPYOUT_KERNEL=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "zero_copy" > gpurun_out/pytest_r04i.log 2>&1 || { tail -30 gpurun_out/pytest_r04i.log; exit 1; }
tail -1 gpurun_out/pytest_r04i.log
A="--steps 5 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --sync-steps 0 --wire-steps 0"
for k in 0 1 0 1; do
  GWAOI_COPYOUT_KERNEL=$k timeout -k 10 300 python -u bench.py $A > gpurun_out/bench_r04i_k$k.json 2> gpurun_out/bench_r04i_k$k.err || { tail -20 gpurun_out/bench_r04i_k$k.err; exit 1; }
  python3 -c "import json,sys; b=json.loads(open('gpurun_out/bench_r04i_k$k.json').read().strip().splitlines()[-1]); h=b['host_to_host_tick']; print('kernel=$k', round(b['ms_per_step'],4), 'h2h pipelined', round(h['ms_per_step'],4), 'p50', round(h['p50_tick_ms'],3), 'p99', round(h['p99_tick_ms'],3), 'serial p99', round(h['serial_p99_tick_ms'],3))"
done
