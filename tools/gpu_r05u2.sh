#!/bin/bash
# After the single-pass keygen fold (block 0 of k_scan64): the whole GPU suite, then the apply's
# moves per thread under GWAOI_F_UNIQUE_MOVES (4 = base, 2, 8) interleaved, then the apply stage's
# counted bytes (PMC read-request sizes + WRITE_SIZE) for the unique and the claims path
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r05u2.log 2>&1 || { tail -40 gpurun_out/pytest_r05u2.log; exit 1; }
tail -2 gpurun_out/pytest_r05u2.log
timeout -k 10 600 python -u tools/variants.py run base ap2 ap8 base ap2 ap8 -- --steps 50 --warmup 5 > gpurun_out/r05u2_ab.txt 2>&1 || { tail -5 gpurun_out/r05u2_ab.txt; exit 1; }
cat gpurun_out/r05u2_ab.txt
A="--steps 6 --warmup 1 --no-cpu-baseline --host-io-steps 0 --sync-steps 0 --cfg4-steps 0 --cfg5-steps 0 --small-flush-reps 0 --wire-steps 0 --host-tick-steps 0"
for v in uniq claims; do
  X=""; [ $v = claims ] && X="--claims"
  O=$R/gpurun_out/pmc_r05u2_$v
  mkdir -p $O
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/rd -o run -- python3 $R/bench.py $A $X > /dev/null 2> $O/rd.err) || { echo "pmc rd $v failed"; tail -3 $O/rd.err; exit 1; }
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wr -o run -- python3 $R/bench.py $A $X > /dev/null 2> $O/wr.err) || { echo "pmc wr $v failed"; tail -3 $O/wr.err; exit 1; }
  for k in k_prologue k_moves_apply_n k_moves_fixup k_keygen k_scan64 k_gather; do echo -n "$v $k: "; python3 tools/pmc_kernel.py $k $O/rd $O/wr || true; done
done
