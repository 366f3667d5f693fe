#!/usr/bin/env python3
"""Median per dispatch of each PMC counter for one kernel: pmc_median.py <dir> <kernel-substring>.
Reads every run_counter_collection.csv under <dir> (tools/pmc.sh output, one pass per subdir)."""
import csv
import glob
import os
import statistics
import sys

root, kname = sys.argv[1], sys.argv[2]
vals = {}
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    per = {}
    for r in csv.DictReader(open(f)):
        if kname not in r.get("Kernel_Name", ""):
            continue
        key = (r["Counter_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (c, _), v in per.items():
        vals.setdefault(c, []).append(v)
for c in sorted(vals):
    v = sorted(vals[c])
    steady = v[1:] if len(v) > 2 else v
    print(f"{c:40s} {statistics.median(steady):.4g}  (n={len(v)})")
