#!/usr/bin/env python3
"""Sparse flushes in a rocprofv3 kernel trace: per-kernel duration, the gaps between them, and
the span from the first kernel (k_ops_claim) to the last (k_sp_apply), medians.

    python tools/sparse_trace.py run_kernel_trace.csv [label]
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
    flushes, cur = [], None
    for r in rows:
        k = short(r["Kernel_Name"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if k == "k_ops_claim":
            cur = [(k, s, e)]
        elif cur is not None and k.startswith("k_sp_"):
            cur.append((k, s, e))
            if k == "k_sp_apply":
                flushes.append(cur)
                cur = None
        else:
            cur = None
    label = sys.argv[2] if len(sys.argv) > 2 else ""
    if not flushes:
        print(f"== {label}: no sparse flush in the trace")
        return
    span = statistics.median([(f[-1][2] - f[0][1]) / 1e3 for f in flushes])
    busy = statistics.median([sum(e - s for _, s, e in f) / 1e3 for f in flushes])
    between = [(b[0][1] - a[-1][2]) / 1e3 for a, b in zip(flushes, flushes[1:])]
    print(f"== {label}: {len(flushes)} sparse flushes, median span {span:.1f} us (kernels {busy:.1f}), "
          f"median gap to the next {statistics.median(between) if between else 0:.1f} us")
    names = [k for k, _, _ in flushes[0]]
    for i, k in enumerate(names):
        d = statistics.median([(f[i][2] - f[i][1]) / 1e3 for f in flushes if len(f) == len(names)])
        g = statistics.median([(f[i][1] - f[i - 1][2]) / 1e3 for f in flushes if len(f) == len(names)]) if i else 0.0
        print(f"   {k:24s} {d:7.1f} us  (gap before {g:5.1f})")


if __name__ == "__main__":
    main()
