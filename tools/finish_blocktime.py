#!/usr/bin/env python3
"""Block schedule of k_finish at config 3 (diagnostics; GPU box, variant library built with
-DGWAOI_EXP_BLOCKTIME, path in GWAOI_LIB): thread 0's start / return per block on the wall clock
(100 MHz), by block kind (tile order, summary + bbox fold, copy)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from goworld_amd import World  # noqa: E402
from goworld_amd.workload import make_workload  # noqa: E402

BT_FIN = 40000


def main():
    import torch
    wl = make_workload("cfg3")
    lib = ctypes.CDLL(os.environ["GWAOI_LIB"])
    buf = np.zeros(3 * 65536, np.uint64)
    with World(wl.n, device=0) as w:
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
    b = buf.reshape(-1, 3)[BT_FIN:BT_FIN + 2000]
    nb = int((b[:, 0] != 0).sum())
    b = b[:nb]
    t0 = b[:, 0].astype(np.int64)
    t1 = b[:, 1].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) * 0.01, (t1 - base) * 0.01
    print(f"blocks {nb}  span {e.max():.1f} us")
    kinds = {"tile order": slice(0, 8), "summary+fold": slice(nb - 1, nb), "copy": slice(8, nb - 1)}
    for k, sl in kinds.items():
        print(f"  {k:13s} start {s[sl].min():6.1f}..{s[sl].max():6.1f}  end max {e[sl].max():6.1f}  "
              f"dur mean {(e[sl] - s[sl]).mean():6.1f} max {(e[sl] - s[sl]).max():6.1f}")
    r = buf.reshape(-1, 3)
    st = [int(r[BT_FIN + 2000][0]), int(r[BT_FIN + 2000][1]), int(r[BT_FIN + 2000][2]), int(r[BT_FIN + 2001][1])]
    print("  fold block stamps (us from its start): summary %.1f, fold loop %.1f, bbox_block + barrier %.1f, end %.1f" %
          tuple((x - int(t0[nb - 1])) * 0.01 for x in st))
    o = [int(x) for x in r[BT_FIN + 2004:BT_FIN + 2006].reshape(-1)[:4]]
    print("  tile order block 0 stamps (us from its start): LDS staged %.1f, segment scan %.1f, cuts %.1f, order_range %.1f"
          % tuple((x - int(t0[0])) * 0.01 for x in o))
    order = np.argsort(e)[-5:]
    print("  last 5 to end (block, start, end):", [(int(i), round(float(s[i]), 1), round(float(e[i]), 1)) for i in order])


if __name__ == "__main__":
    main()
