#!/bin/bash
# A/B of libgwaoi variants on the bench's entity-sync leg only (GPU box):
#   bash tools/sync_ab.sh base fw2 fw8 ...   (variants from tools/variants.py build; base = the in-tree library)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
    if [ "$v" = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
    timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 \
        --host-tick-steps 0 --host-io-steps 0 --wire-steps 0 --small-flush-reps 0 --claims-steps 0 > /tmp/sync_ab.json 2> /tmp/sync_ab.err || { echo "$v failed"; tail -5 /tmp/sync_ab.err; exit 1; }
    python3 -c "import json,sys;b=json.loads(open('/tmp/sync_ab.json').read().strip().splitlines()[-1]);s=b['sync_leg'];print(sys.argv[1], 'decode+flush', round(s['decode_flush_ms'],4), 'collect', round(s['collect_ms'],4))" $v
done
