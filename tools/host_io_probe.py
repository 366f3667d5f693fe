"""Split the PCIe-inclusive tick (host move arrays in, host event arrays out) into its host-side
phases on the GPU box: moved_batch (validate + stage + H2D issue), gwaoi_tick (flush + event D2H),
and the numpy copy of the events.  usage: python tools/host_io_probe.py [n] [ticks]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import ctypes as C  # noqa: E402

from goworld_amd import World  # noqa: E402
from goworld_amd._lib import Events  # noqa: E402
from goworld_amd.workload import make_workload  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    wl = make_workload("cfg3", n=n)
    slots, x0, z0, _ = wl.initial()
    batches = [wl.tick(t) for t in range(ticks)]
    with World(n) as w:
        s = w.space_create(wl.D)
        w.enter_batch(s, slots, x0, z0)
        w.tick_device()
        tm = {"moved_batch": [], "gwaoi_tick (flush + D2H)": [], "numpy copy": []}
        for sl, nx, nz in batches:
            a = time.perf_counter()
            w.moved_batch(sl, nx, nz)
            b = time.perf_counter()
            ev = Events()
            assert w._L.gwaoi_tick(w._w, C.byref(ev)) == 0
            c = time.perf_counter()
            ne, nl = ev.n_enter, ev.n_leave
            np.ctypeslib.as_array(ev.enter, shape=(2 * ne,)).copy()
            np.ctypeslib.as_array(ev.leave, shape=(2 * nl,)).copy()
            d = time.perf_counter()
            tm["moved_batch"].append(b - a)
            tm["gwaoi_tick (flush + D2H)"].append(c - b)
            tm["numpy copy"].append(d - c)
        for k, v in tm.items():
            print(f"{k:26s} median {np.median(v[1:]) * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
