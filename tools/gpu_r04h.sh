set -o pipefail
# round-4: async copy-out parity + the default bench line, cell size D/3 against D/4 (kernel traces),
# then the rocprofv3 profile of the cfg3 tick and the FETCH_SIZE calibration
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
bash tools/gpu_run.sh r04h "zero_copy or speculative or device_enter" || exit 1
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0"
for c in 4 3; do
  OUT=$R/gpurun_out/tv_r04h_c$c
  mkdir -p $OUT
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py $ARGS --cells-per-dist $c > $OUT/bench.json 2> $OUT/err.log) || { echo "trace c=$c failed"; tail -5 $OUT/err.log; exit 1; }
  python3 $R/tools/tick_kernels.py $OUT/run_kernel_trace.csv c$c
done
bash tools/profile.sh r04 && bash tools/calib_fetch.sh
