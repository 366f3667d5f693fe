#!/usr/bin/env python3
"""Median per-kernel duration over the steady cfg3 ticks of a rocprofv3 kernel trace.

    python tools/tick_kernels.py run_kernel_trace.csv [label]
A tick starts at k_prologue, or at the apply when no prologue precedes it (a unique-moves flush
on the previous grid); the first 3 ticks and the stage-timed tail are skipped.
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
    ticks, cur, prev = [], None, None
    for r in rows:
        k = short(r["Kernel_Name"])
        if k == "k_prologue" or (k.startswith("k_moves_apply_n") and prev != "k_prologue"):
            cur = []
            ticks.append(cur)
        prev = k
        if cur is not None:
            cur.append((k, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    steady = ticks[3:-12] if len(ticks) > 16 else ticks[1:]
    per = {}
    for t in steady:
        seen = {}
        for k, s, e in t:
            seen[k] = seen.get(k, 0) + (e - s)
        for k, v in seen.items():
            per.setdefault(k, []).append(v / 1e3)
    span = statistics.median([(t[-1][2] - t[0][1]) / 1e3 for t in steady])
    busy = statistics.median([sum(e - s for _, s, e in t) / 1e3 for t in steady])
    inner = statistics.median([sum(max(0, b[1] - a[2]) for a, b in zip(t, t[1:])) / 1e3 for t in steady])
    gaps = statistics.median([(b[0][1] - a[-1][2]) / 1e3 for a, b in zip(steady, steady[1:])])
    label = sys.argv[2] if len(sys.argv) > 2 else ""
    print(f"== {label}: {len(steady)} ticks, median span {span:.1f} us (kernels {busy:.1f}, gaps between them "
          f"{inner:.1f}), gap to next tick {gaps:.1f} us")
    for k, v in per.items():
        print(f"   {k:28s} {statistics.median(v):7.1f}")


if __name__ == "__main__":
    main()
