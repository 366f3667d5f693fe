#!/usr/bin/env python3
"""Median idle gap before each kernel (its start minus the previous kernel's end) over a
rocprofv3 kernel trace's steady part: which kernel boundaries of the flush cost time.

    python tools/kernel_gaps.py run_kernel_trace.csv
"""
import csv
import re
import statistics
import sys


def short(n):
    m = re.search(r"(k_[a-z_0-9]+(?:<[^>]*>)?|__amd_[a-zA-Z_]+)", n)
    return m.group(1) if m else n[:30]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[len(rows) // 4: -len(rows) // 4] if len(rows) > 40 else rows
    gaps = {}
    for a, b in zip(rows, rows[1:]):
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        gaps.setdefault(f"{short(a['Kernel_Name'])} -> {short(b['Kernel_Name'])}", []).append(g)
    for k, v in sorted(gaps.items(), key=lambda kv: -statistics.median(kv[1])):
        if len(v) >= 3:
            print(f"   {k:50s} {statistics.median(v):6.2f} us  (n={len(v)})")


if __name__ == "__main__":
    main()
