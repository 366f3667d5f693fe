#!/bin/bash
# A/B of the overlapped flushes (GPU box): the headline tick and the host -> host leg, in-tree library
# against the GWAOI_EXP_NO_OVERLAP variant (tools/variants.py build noovl=GWAOI_EXP_NO_OVERLAP).
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
    if [ "$v" = base ]; then unset GWAOI_LIB; else export GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so; fi
    timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --cfg4-steps 0 --cfg5-steps 0 --host-tick-steps 0 \
        --sync-steps 0 --wire-steps 0 --small-flush-reps 0 --claims-steps 0 > /tmp/ovl_ab.json 2> /tmp/ovl_ab.err || { echo "$v failed"; tail -5 /tmp/ovl_ab.err; exit 1; }
    python3 -c "import json,sys;b=json.loads(open('/tmp/ovl_ab.json').read().strip().splitlines()[-1]);h=b.get('host_to_host_tick') or {};print(sys.argv[1], 'tick', round(b['ms_per_step'],4), 'p99', round(b['p99_tick_ms'],4), 'h2h', h.get('ms_per_step'), 'h2h p50/p99', h.get('p50_tick_ms'), h.get('p99_tick_ms'))" $v
done
