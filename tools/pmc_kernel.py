#!/usr/bin/env python3
"""Median per-dispatch value of each counter for one kernel in rocprofv3 --pmc outputs (the first
dispatch dropped), and the read/write bytes when the request-size / WRITE_SIZE counters are there.

    python tools/pmc_kernel.py KERNEL DIR [DIR ...]   (DIR: a -d output holding run_counter_collection.csv)
"""
import csv
import glob
import os
import statistics
import sys


def main():
    kern, dirs = sys.argv[1], sys.argv[2:]
    per = {}
    for d in dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                if kern not in r["Kernel_Name"]:
                    continue
                per.setdefault(r["Counter_Name"], {}).setdefault(int(r["Dispatch_Id"]), 0.0)
                per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    med = {c: statistics.median([v[i] for i in sorted(v)][1:] or list(v.values())) for c, v in per.items()}
    out = dict(med)
    if all(c in med for c in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
        out["read_MB"] = round((32 * med["TCC_EA0_RDREQ_32B_sum"] + 64 * med["TCC_EA0_RDREQ_64B_sum"] +
                                128 * med["TCC_EA0_RDREQ_128B_sum"]) / 1e6, 2)
    if "WRITE_SIZE" in med:
        out["write_MB"] = round(med["WRITE_SIZE"] * 1024 / 1e6, 2)
    print(kern, {k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()})


if __name__ == "__main__":
    main()
