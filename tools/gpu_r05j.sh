#!/bin/bash
# A/B of the side-stream special pass and the premarked claims, bench lines only, interleaved twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
A="--steps 50 --warmup 5 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --wire-steps 0 --sync-steps 0 --host-io-steps 0 --small-flush-reps 0"
: > gpurun_out/r05j_ab.txt
for rep in 1 2; do
  for v in def side0 side0_nbr nbr; do
    case $v in
      def) E=""; X="";;
      side0) E="GWAOI_SPECIAL_SIDE=0"; X="";;
      side0_nbr) E="GWAOI_SPECIAL_SIDE=0"; X="--no-batch-ready";;
      nbr) E=""; X="--no-batch-ready";;
    esac
    env $E timeout -k 10 200 python -u bench.py $A $X > gpurun_out/r05j_$v.json 2> gpurun_out/r05j_$v.err || { tail -5 gpurun_out/r05j_$v.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/r05j_$v.json').read().strip().splitlines()[-1]); print('$rep $v', round(d['ms_per_step'],4), round(d['p99_tick_ms'],4), d['roofline']['avg_launch_ms'])" >> gpurun_out/r05j_ab.txt
  done
done
cat gpurun_out/r05j_ab.txt
