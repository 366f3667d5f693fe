#!/usr/bin/env python3
"""Per-kernel mean durations (us) of the collect kernels in rocprofv3 databases (tools/sync_prof.sh)."""
import glob
import os
import sqlite3
import sys

KERNELS = ("k_decode<", "k_decode_apply", "k_fan_prep", "k_fan_hits", "k_fan_write")

for d in sys.argv[1:]:
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(db)
        rows = c.execute("select name, end - start from kernels").fetchall()
        out = []
        for k in KERNELS:
            t = [dt / 1e3 for n, dt in rows if k in n]
            t = t[2:] if len(t) > 3 else t  # (the untimed first collects)
            if t:
                out.append(f"{k} {sum(t) / len(t):.1f}")
        print(os.path.basename(d.rstrip("/")), " ".join(out))
