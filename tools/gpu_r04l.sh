set -o pipefail
# round-4 A/B: k_fan_hits storing 64 B of hits per lane at a time (hits64) against 16 B (base):
# sync parity, the sync leg's collect time, and k_fan_hits' counted writes
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
GWAOI_LIB=$R/goworld_amd/lib/variants/hits64.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sync" > $R/gpurun_out/pytest_r04l.log 2>&1 || { tail -30 $R/gpurun_out/pytest_r04l.log; exit 1; }
tail -1 $R/gpurun_out/pytest_r04l.log
export TMPDIR=/tmp
A="--steps 3 --warmup 2 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 --host-io-steps 0 --wire-steps 0 --breakdown-steps 0 --sync-steps 5"
for v in base hits64 base hits64; do
  if [ $v = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python -u bench.py $A > $R/gpurun_out/bench_r04l_$v.json 2> $R/gpurun_out/bench_r04l_$v.err || { tail -5 $R/gpurun_out/bench_r04l_$v.err; exit 1; }
  python3 -c "import json; b=json.loads(open('$R/gpurun_out/bench_r04l_$v.json').read().strip().splitlines()[-1]); s=b['sync_leg']; print('$v', 'decode_flush_ms', round(s['decode_flush_ms'],4), 'collect_ms', round(s['collect_ms'],4))"
done
for v in base hits64; do
  if [ $v = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
  OUT=$R/gpurun_out/pw_r04l_$v
  mkdir -p $OUT
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o run -- python3 $R/bench.py $A > /dev/null 2> $OUT/err.log) || { tail -5 $OUT/err.log; exit 1; }
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $A > /dev/null 2> $OUT/trace.err) || { tail -5 $OUT/trace.err; exit 1; }
  python3 - $OUT <<'PY'
import csv, statistics, sys, glob
d = sys.argv[1]
w = {}
for r in csv.DictReader(open(glob.glob(d + "/run_counter_collection.csv")[0])):
    if "k_fan" in r["Kernel_Name"] or "k_decode" in r["Kernel_Name"]:
        w.setdefault(r["Kernel_Name"].split("(")[0], []).append(float(r["Counter_Value"]))
t = {}
for r in csv.DictReader(open(glob.glob(d + "/trace/run_kernel_trace.csv")[0])):
    if "k_fan" in r["Kernel_Name"] or "k_decode" in r["Kernel_Name"]:
        t.setdefault(r["Kernel_Name"].split("(")[0], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in sorted(set(w) | set(t)):
    print(d.split("_")[-1], k, "WRITE_SIZE MB", round(statistics.median(w.get(k, [0])) * 1024 / 1e6, 1), "us", round(statistics.median(t.get(k, [0])), 1))
PY
done
