set -o pipefail
# round-4: PCIe copy rates, then a kernel + memory-copy trace of the pipelined host->host leg
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/pcie_probe.py > gpurun_out/pcie_probe.txt 2>&1 || { cat gpurun_out/pcie_probe.txt; exit 1; }
cat gpurun_out/pcie_probe.txt
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/tr_hio
mkdir -p $OUT
A="--steps 5 --warmup 3 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --sync-steps 0 --wire-steps 0 --host-io-steps 12"
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o run -- python3 $R/bench.py $A > $OUT/bench.json 2> $OUT/err.log) || { tail -5 $OUT/err.log; exit 1; }
ls $OUT | head -3
# round-4 A/B: the cell scan without look-back (tile totals from keygen), 32 cells per thread, a one-block
# fixup; then the cell size D/3 against D/4 again
bash tools/gpu_variants.sh r04k base scanbt s64i32 scanbt32 fix1 || exit 1
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0"
for c in 3 4; do
  OUT=$R/gpurun_out/tv_r04k_c$c
  mkdir -p $OUT
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py $ARGS --cells-per-dist $c > $OUT/bench.json 2> $OUT/err.log) || { echo "trace c=$c failed"; tail -5 $OUT/err.log; exit 1; }
  python3 $R/tools/tick_kernels.py $OUT/run_kernel_trace.csv c$c
done
