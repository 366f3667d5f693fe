#!/usr/bin/env python3
"""Block schedule of k_combined at config 3 (diagnostics; GPU box, variant library built with
-DGWAOI_EXP_BLOCKTIME, path in GWAOI_LIB): per-block start/end on the wall clock (100 MHz),
how many blocks run at once over the launch, and how long the tail is."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from goworld_amd import World  # noqa: E402
from goworld_amd.workload import make_workload  # noqa: E402


def main():
    import torch
    wl = make_workload("cfg3")
    n = wl.n
    lib = ctypes.CDLL(os.environ["GWAOI_LIB"])
    unit = int(os.environ.get("BT_UNIT", "64"))  # entries per k_combined unit (64: one wave's, GWAOI_CQ; 256: a block's)
    nb = (n + unit - 1) // unit
    buf = np.zeros(3 * 65536, np.uint64)
    with World(n, device=0) as w:
        s = w.space_create(wl.D)
        slots, x0, z0, _ = wl.initial()
        w.enter_batch(s, slots, x0, z0)
        w.tick()
        for t in range(int(os.environ.get("BT_TICKS", "4"))):
            sl, nx, nz = wl.tick(t)
            ds = torch.from_numpy(sl.astype(np.int32)).to("cuda:0")
            dx = torch.from_numpy(nx).to("cuda:0")
            dz = torch.from_numpy(nz).to("cuda:0")
            torch.cuda.synchronize()
            w.moved_batch_device(ds.data_ptr(), dx.data_ptr(), dz.data_ptr(), sl.size)
            w.tick()
        assert lib.gwaoi_debug_blocktime(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.size)) == 0
    b = buf[:3 * nb].reshape(nb, 3)
    t0, t1, hw = b[:, 0].astype(np.int64), b[:, 1].astype(np.int64), b[:, 2]
    t0 -= t0.min()
    t1 -= b[:, 0].astype(np.int64).min()
    us = 0.01  # 100 MHz wall clock
    dur = (t1 - t0) * us
    span = t1.max() * us
    print(f"blocks {nb}  span {span:.1f} us  block duration us: mean {dur.mean():.1f} p50 {np.median(dur):.1f} "
          f"p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}")
    print(f"sum of block durations / span = {dur.sum() / span:.0f} blocks in flight on average")
    grid = np.arange(0, span, span / 40)
    act = [int(((t0 * us <= g) & (t1 * us > g)).sum()) for g in grid]
    print("blocks running, 40 steps over the span:", act)
    starts = np.sort(t0 * us)
    print("start time of block k (us): k=0 %.1f, k=nb/2 %.1f, k=3nb/4 %.1f, last %.1f" %
          (starts[0], starts[nb // 2], starts[3 * nb // 4], starts[-1]))
    xcc = (hw >> np.uint64(32)) & np.uint64(0xFF)
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"xcc {x}: blocks {int(m.sum())} end {t1[m].max() * us:.1f} us, mean dur {dur[m].mean():.1f}")
    bid = (hw >> np.uint64(40)).astype(np.int64)
    order = np.argsort(bid)
    q = len(order) // 8
    print("mean duration by dispatch octile:", [round(float(dur[order[i * q:(i + 1) * q]].mean()), 1) for i in range(8)])


if __name__ == "__main__":
    main()
