#!/usr/bin/env python3
"""Mean durations (us) of the move-apply kernels per template form in rocprofv3 databases (tools/apply_prof.sh),
with the bench line's headline and claims ticks."""
import collections
import glob
import json
import os
import sqlite3
import sys

for d in sys.argv[1:]:
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(db)
        t = collections.defaultdict(list)
        for n, dt in c.execute("select name, end - start from kernels"):
            if "k_moves_apply_n" in n or "k_moves_mark" in n:
                t[n[n.index("k_moves"):][:60]].append(dt / 1e3)
        line = ""
        js = d.rstrip("/") + ".json"
        if os.path.exists(js):
            b = json.loads(open(js).read().strip().splitlines()[-1])
            line = f"tick {b['ms_per_step']:.4f} claims {(b.get('claims_tick') or {}).get('ms_per_step')}"
        print(os.path.basename(d.rstrip("/")), line)
        for k, v in sorted(t.items()):
            print(f"   {k} n={len(v)} mean {sum(v) / len(v):.1f}")
