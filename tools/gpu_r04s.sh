set -o pipefail
# round-4: k_decode records per thread (1 = base, 2, 4) and k_fan_write record groups in flight (4 = base, 8, 2):
# sync parity, then the sync leg's decode + flush and collect times
# and the k_decode kernel time
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
for v in dec2 dec4 fw8 fw2; do
  GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sync" > $R/gpurun_out/pytest_r04s_$v.log 2>&1 || { tail -30 $R/gpurun_out/pytest_r04s_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $R/gpurun_out/pytest_r04s_$v.log)"
done
A="--steps 3 --warmup 2 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --host-io-steps 0 --wire-steps 0 --breakdown-steps 0 --sync-steps 5"
for v in base dec2 dec4 fw8 fw2 base dec2 dec4 fw8 fw2; do
  if [ $v = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
  OUT=$R/gpurun_out/ts_r04s_$v
  mkdir -p $OUT
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $R/bench.py $A > $OUT/bench.json 2> $OUT/err.log) || { tail -5 $OUT/err.log; exit 1; }
  python3 - $OUT $v <<'PY'
import csv, glob, json, statistics, sys
d, v = sys.argv[1], sys.argv[2]
t = {}
for r in csv.DictReader(open(glob.glob(d + "/run_kernel_trace.csv")[0])):
    n = r["Kernel_Name"]
    for k in ("k_decode<", "k_decode_apply", "k_fan_hits", "k_fan_write", "k_fan_prep"):
        if k in n:
            t.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
b = json.loads(open(d + "/bench.json").read().strip().splitlines()[-1])["sync_leg"]
print(v, "decode_flush_ms", round(b["decode_flush_ms"], 4), "collect_ms", round(b["collect_ms"], 4),
      {k: round(statistics.median(x), 1) for k, x in sorted(t.items())})
PY
done
