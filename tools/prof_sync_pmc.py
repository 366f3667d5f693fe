#!/usr/bin/env python3
"""Print the PMC medians of the entity-sync kernels from a prof_summary JSON.

    python tools/prof_sync_pmc.py gpurun_out/prof_<tag>/summary.json
"""
import json
import sys

d = json.load(open(sys.argv[1]))["kernels"]
for k in ("k_fan_write", "k_fan_hits", "k_fan_prep", "k_decode", "k_decode_fix", "k_decode_yaw"):
    if k in d:
        print(k, {c: round(v) for c, v in d[k]["pmc"].items()})
