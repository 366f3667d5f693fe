"""Build libgwaoi.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m goworld_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "lib", "libgwaoi.so")
SOURCES = ["gwaoi_kernels.hip", "gwaoi_world.cpp", "gwaoi_strips.hip", "gwaoi_sync.hip", "gwaoi_wire.hip",
           "gwaoi_sparse.hip"]
HEADERS = ["gwaoi_internal.h", "gwaoi_device.h", os.path.join("..", "..", "include", "gwaoi.h"),
           os.path.join("..", "..", "include", "gwaoi_sync.h"),
           os.path.join("..", "..", "include", "gwaoi_strips.h"), os.path.join("..", "..", "include", "gwaoi_wire.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: the go-aoi window bounds are plain float32 sums and must
# not be fused or re-associated (no fast-math anywhere).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-fast-math", "-Wall"]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=()) -> str:
    """Compile libgwaoi.so (or a tuning variant: `out` + -D `defines`)."""
    if out == OUT and not defines and not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in defines], "-o", tmp, *[os.path.join(CSRC, s) for s in SOURCES]]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


CPP_TEST_SRC = os.path.join(ROOT, "tests", "cpp", "aoi_manager_test.cpp")
CPP_TEST_OUT = os.path.join(HERE, "lib", "aoi_manager_test")


def build_cpp_tests(force: bool = False, verbose: bool = False) -> str:
    """Host C++ test of include/gwaoi_aoi.hpp, linked against the in-tree libgwaoi.so."""
    lib = build(force=force, verbose=verbose)
    deps = [CPP_TEST_SRC, lib, os.path.join(ROOT, "include", "gwaoi_aoi.hpp"), os.path.join(ROOT, "include", "gwaoi.h")]
    if (not force and os.path.exists(CPP_TEST_OUT)
            and all(os.path.getmtime(d) <= os.path.getmtime(CPP_TEST_OUT) for d in deps)):
        return CPP_TEST_OUT
    tmp = CPP_TEST_OUT + ".tmp"
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"), CPP_TEST_SRC, "-o", tmp,
           "-L", os.path.dirname(lib), "-lgwaoi", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath-link,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, CPP_TEST_OUT)
    return CPP_TEST_OUT


TICK_BENCH_SRC = os.path.join(ROOT, "tools", "tick_bench.cpp")
TICK_BENCH_OUT = os.path.join(HERE, "lib", "gwaoi_tick_bench")


def build_tick_bench(force: bool = False, verbose: bool = False) -> str:
    """C++ host tick bench (tools/tick_bench.cpp): the cgo-like end-to-end tick + callback replay."""
    lib = build(force=force, verbose=verbose)
    deps = [TICK_BENCH_SRC, lib, os.path.join(ROOT, "include", "gwaoi.h"), os.path.join(ROOT, "tools", "interest_sets.hpp")]
    if (not force and os.path.exists(TICK_BENCH_OUT)
            and all(os.path.getmtime(d) <= os.path.getmtime(TICK_BENCH_OUT) for d in deps)):
        return TICK_BENCH_OUT
    tmp = TICK_BENCH_OUT + ".tmp"
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-pthread", "-I", os.path.join(ROOT, "include"), "-I",
           os.path.join(ROOT, "tools"), TICK_BENCH_SRC,
           "-o", tmp, "-L", os.path.dirname(lib), "-lgwaoi", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath-link,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, TICK_BENCH_OUT)
    return TICK_BENCH_OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_cpp_tests(verbose=True))
    print(build_tick_bench(verbose=True))
