#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory into profiles/<name>.md + .json.

    python tools/prof_summary.py gpurun_out/prof_<tag> profiles/r01_<name>

Kernel table: rocprofv3 --kernel-trace --stats (run_kernel_stats.csv).
Per-kernel PMC: median over the steady-state dispatches (the first dispatch
of each kernel -- the populate flush -- is dropped).  HBM bytes follow
MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are KiB; on
gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads,
so it is doubled.
"""
import csv
import json
import os
import re
import statistics
import sys


def short(name):
    """Kernel name without namespace and parameters, template arguments kept:
    k_keygen<true> (steady flush) and k_keygen<false> (populate) are different kernels."""
    m = re.search(r"(k_[a-z_0-9]+(?:<[^<>()]*>)?|__amd_[a-zA-Z_]+)", name)
    return m.group(1).replace(" ", "") if m else name[:40]


def kernel_stats(d):
    p = os.path.join(d, "trace", "run_kernel_stats.csv")
    rows = []
    for r in csv.DictReader(open(p)):
        rows.append({"kernel": short(r["Name"]), "calls": int(r["Calls"]),
                     "avg_us": float(r["AverageNs"]) / 1e3, "min_us": float(r["MinNs"]) / 1e3,
                     "max_us": float(r["MaxNs"]) / 1e3, "pct": float(r["Percentage"])})
    return rows


def trace_steady(d):
    """median duration per kernel over dispatches after the first (kernel trace)"""
    p = os.path.join(d, "trace", "run_kernel_trace.csv")
    per = {}
    for r in csv.DictReader(open(p)):
        k = short(r["Kernel_Name"])
        per.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: statistics.median(v[1:] if len(v) > 1 else v) for k, v in per.items()}


def pmc(d, sub):
    p = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}
    per = {}
    for r in csv.DictReader(open(p)):
        k = short(r["Kernel_Name"])
        per.setdefault(k, {}).setdefault(r["Counter_Name"], {}).setdefault(int(r["Dispatch_Id"]), 0.0)
        per[k][r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for k, cs in per.items():
        out[k] = {}
        for c, disp in cs.items():
            vals = [disp[i] for i in sorted(disp)]
            out[k][c] = statistics.median(vals[1:] if len(vals) > 1 else vals)
    return out


def main():
    d, dst = sys.argv[1], sys.argv[2]
    bench = None
    bp = os.path.join(d, "trace_bench.json")
    if os.path.exists(bp):
        try:
            bench = json.loads(open(bp).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            bench = None
    ks = kernel_stats(d)
    steady = trace_steady(d)
    sq = pmc(d, "pmc_sq")
    tc = pmc(d, "pmc_tcp")
    fe = pmc(d, "pmc_fetch")
    wr = pmc(d, "pmc_write")
    rq = pmc(d, "pmc_rdreq")  # L2 -> fabric read requests by size (exact read bytes, no FETCH_SIZE factor)
    dr = pmc(d, "pmc_dram")   # ... of them, the ones that went to DRAM (the rest hit the Infinity Cache)
    kern = {}
    for r in ks:
        k = r["kernel"]
        e = dict(r)
        e["steady_median_us"] = steady.get(k)
        e["pmc"] = dict(sq.get(k, {}))
        e["pmc"].update(tc.get(k, {}))
        p = e["pmc"]
        if p.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
                if c in p:
                    e.setdefault("derived", {})[c + "_frac"] = p[c] / p["SQ_WAVE_CYCLES"]
        if p.get("TCP_TOTAL_CACHE_ACCESSES_sum") and "TCP_TCC_READ_REQ_sum" in p:
            e.setdefault("derived", {})["tcp_hit_rate"] = 1.0 - p["TCP_TCC_READ_REQ_sum"] / p["TCP_TOTAL_CACHE_ACCESSES_sum"]
        if p.get("TCC_HIT_sum") is not None and p.get("TCC_MISS_sum") is not None and p["TCC_HIT_sum"] + p["TCC_MISS_sum"]:
            e.setdefault("derived", {})["l2_hit_rate"] = p["TCC_HIT_sum"] / (p["TCC_HIT_sum"] + p["TCC_MISS_sum"])
        f = fe.get(k, {}).get("FETCH_SIZE")
        w = wr.get(k, {}).get("WRITE_SIZE")
        r = rq.get(k, {})
        e["pmc"].update(r)
        e["pmc"].update(dr.get(k, {}))
        if f is not None:
            e["pmc"]["FETCH_SIZE_KiB"] = f
            e["hbm_read_bytes"] = 2.0 * f * 1024.0
        if all(c in r for c in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
            # requests by size: the read bytes without FETCH_SIZE's factor (which holds for 128-B requests only)
            e["read_bytes_by_request_size"] = (32.0 * r["TCC_EA0_RDREQ_32B_sum"] + 64.0 * r["TCC_EA0_RDREQ_64B_sum"] +
                                               128.0 * r["TCC_EA0_RDREQ_128B_sum"])
            e["hbm_read_bytes"] = e["read_bytes_by_request_size"]
        if w is not None:
            e["pmc"]["WRITE_SIZE_KiB"] = w
            e["hbm_write_bytes"] = w * 1024.0
        if f is not None and w is not None:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        kern[k] = e
    js = {"source": d, "bench": bench, "kernels": kern}
    with open(dst + ".json", "w") as fh:
        json.dump(js, fh, indent=1)
    lines = [f"# rocprofv3 summary ({os.path.basename(dst)})", "",
             "Command: `tools/profile.sh` = `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 8 --warmup 2`, "
             "then separate `--pmc` passes (SQ block with SQ_WAIT_ANY / SQ_ACTIVE_INST_ANY, TCP/TCC hit counters, FETCH_SIZE, WRITE_SIZE). "
             "PMC values are medians over steady-state dispatches; read bytes = 32/64/128 B x TCC_EA0_RDREQ_{32B,64B,128B} "
             "when that pass ran (else 2 x FETCH_SIZE, the gfx950 factor for 128-B streaming requests).", ""]
    if bench:
        lines += [f"bench under trace: ms_per_step {bench.get('ms_per_step'):.4f}, value {bench.get('value'):.4g} "
                  f"{bench.get('unit')}", ""]
    lines += ["| kernel | calls | avg us | steady median us | % | HBM read MB | HBM write MB |",
              "|---|---|---|---|---|---|---|"]
    for k, e in kern.items():
        rd = e.get("hbm_read_bytes")
        wrb = e.get("hbm_write_bytes")
        lines.append(f"| {k} | {e['calls']} | {e['avg_us']:.2f} | "
                     f"{e['steady_median_us'] if e['steady_median_us'] is None else round(e['steady_median_us'], 2)} | "
                     f"{e['pct']:.2f} | {'' if rd is None else round(rd / 1e6, 3)} | "
                     f"{'' if wrb is None else round(wrb / 1e6, 3)} |")
    # the dominant hot-path kernel (rocclr copies are bench setup, outside the timed region)
    top = "k_combined" if "k_combined" in kern else (ks[0]["kernel"] if ks else None)
    if top and kern[top]["pmc"]:
        lines += ["", f"## PMC, {top} (steady-state median per dispatch)", ""]
        for c, v in sorted(kern[top]["pmc"].items()):
            lines.append(f"- {c}: {v:.6g}")
        for c, v in sorted(kern[top].get("derived", {}).items()):
            lines.append(f"- {c}: {v:.4f}")
    open(dst + ".md", "w").write("\n".join(lines) + "\n")
    kc = kern.get("k_combined")
    if kc and "hbm_bytes" in kc:
        # per-launch HBM traffic of the dominant kernel, read by bench.py (roofline.traffic)
        pm = {"workload": (bench or {}).get("config", {}).get("workload", "cfg3").split(":")[0],
              "kernel": "k_combined", "source": os.path.basename(dst),
              "hbm_read_bytes_per_launch": kc["hbm_read_bytes"], "hbm_write_bytes_per_launch": kc["hbm_write_bytes"],
              "hbm_bytes_per_launch": kc["hbm_bytes"], "steady_median_us": kc.get("steady_median_us"),
              "note": "median over steady-state dispatches; read = L2->fabric read requests x their size "
                      "(TCC_EA0_RDREQ_32B/64B/128B; 2 x FETCH_SIZE without that pass), write = WRITE_SIZE"}
        rnd = os.path.basename(dst).split("_")[0]  # profiles/<round>_pmc_k_combined.json
        with open(os.path.join(os.path.dirname(dst), f"{rnd}_pmc_k_combined.json"), "w") as fh:
            json.dump(pm, fh, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
