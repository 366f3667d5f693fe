#!/bin/bash
# Entity-sync leg of the bench for several libgwaoi variants (tools/variants.py build ...).
# usage: bash tools/sync_variants.sh base name ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L=$R/goworld_amd/lib/variants/$v.so; fi
  GWAOI_LIB=$L timeout -k 10 200 python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --cfg4-steps 0 --host-tick-steps 0 --host-io-steps 0 --breakdown-steps 0 --sync-steps 8 > /tmp/sv.json 2>/tmp/sv.err || { echo "$v failed"; tail -5 /tmp/sv.err; exit 1; }
  python3 -c "import json;d=json.load(open('/tmp/sv.json'));s=d['sync_leg'];print('$v', round(d['ms_per_step'],4), 'decode_flush', round(s['decode_flush_ms'],4), 'collect', round(s['collect_ms'],4))"
done
