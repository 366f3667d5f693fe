#!/usr/bin/env python3
"""Build / run A/B tuning variants of libgwaoi (-D overrides of the kernel tunables).

    python tools/variants.py build NAME=DEF,DEF ...     # here (CPU): goworld_amd/lib/variants/NAME.so
    python tools/variants.py run NAME ... [-- bench args]  # GPU box: one bench line per variant
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "goworld_amd", "lib", "variants")
sys.path.insert(0, ROOT)


def main():
    cmd, rest = sys.argv[1], sys.argv[2:]
    if cmd == "build":
        from goworld_amd import build
        for spec in rest:
            name, _, defs = spec.partition("=")
            out = build.build(out=os.path.join(VDIR, name + ".so"), defines=[d for d in defs.split(",") if d])
            print(out)
    elif cmd == "run":
        names, bargs = (rest[:rest.index("--")], rest[rest.index("--") + 1:]) if "--" in rest else (rest, [])
        for name in names:
            env = dict(os.environ)
            if name != "base":
                env["GWAOI_LIB"] = os.path.join(VDIR, name + ".so")
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline",
                                "--host-io-steps", "0", "--sync-steps", "0", "--cfg4-steps", "0",
                                "--host-tick-steps", "0", "--wire-steps", "0", "--cfg5-steps", "0", "--small-flush-reps", "0",
                                "--claims-steps", "0", *bargs],
                               env=env, capture_output=True, text=True, timeout=400)
            try:
                b = json.loads(r.stdout.strip().splitlines()[-1])
                print(json.dumps({"variant": name, "ms_per_step": round(b["ms_per_step"], 4),
                                  "p99": round(b["p99_tick_ms"], 4), "stages": b["stages_ms_per_tick"]}), flush=True)
            except Exception:
                print(json.dumps({"variant": name, "error": r.stderr[-2000:]}), flush=True)
                sys.exit(1)


if __name__ == "__main__":
    main()
