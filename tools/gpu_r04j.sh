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
ls $OUT
