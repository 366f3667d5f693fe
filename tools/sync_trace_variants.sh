#!/bin/bash
# Kernel-trace medians (us) of the entity-sync kernels for libgwaoi variants (tools/variants.py build ...).
# usage: bash tools/sync_trace_variants.sh TAG base name ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
A="--steps 3 --warmup 2 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --host-io-steps 0 --wire-steps 0 --breakdown-steps 0 --sync-steps 5"
for v in "$@"; do
  if [ $v = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
  OUT=$R/gpurun_out/st_${TAG}_$v
  mkdir -p $OUT
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $R/bench.py $A > $OUT/bench.json 2> $OUT/err.log) || { tail -5 $OUT/err.log; exit 1; }
  python3 - $OUT $v <<'PY'
import csv, glob, json, statistics, sys
d, v = sys.argv[1], sys.argv[2]
t = {}
for r in csv.DictReader(open(glob.glob(d + "/run_kernel_trace.csv")[0])):
    n = r["Kernel_Name"]
    for k in ("k_decode<", "k_decode_apply", "k_fan_hits", "k_fan_write", "k_fan_prep", "k_route"):
        if k in n:
            t.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
b = json.loads(open(d + "/bench.json").read().strip().splitlines()[-1])["sync_leg"]
print(v, "decode_flush_ms", round(b["decode_flush_ms"], 4), "collect_ms", round(b["collect_ms"], 4),
      {k: round(statistics.median(x), 1) for k, x in sorted(t.items())})
PY
done
