#!/bin/bash
# k_combined's HBM traffic against the tile order: default (skew gate), sk0 (always reorder), no order
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
A="--steps 6 --warmup 1 --no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --cfg5-steps 0 --small-flush-reps 0 --wire-steps 0 --host-tick-steps 0"
for v in base sk0 noorder; do
  unset GWAOI_LIB GWAOI_TILE_ORDER
  case $v in base) ;; noorder) export GWAOI_TILE_ORDER=0;; *) export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so;; esac
  O=$R/gpurun_out/pmc_r05aa_$v
  mkdir -p $O
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/rd -o run -- python3 $R/bench.py $A > /dev/null 2> $O/rd.err) || { echo "pmc rd $v failed"; tail -3 $O/rd.err; exit 1; }
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wr -o run -- python3 $R/bench.py $A > /dev/null 2> $O/wr.err) || { echo "pmc wr $v failed"; tail -3 $O/wr.err; exit 1; }
  echo -n "$v: "; python3 tools/pmc_kernel.py k_combined $O/rd $O/wr
done
unset GWAOI_LIB GWAOI_TILE_ORDER
