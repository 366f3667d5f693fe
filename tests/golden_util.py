"""Load and replay the golden fixtures of tests/golden/ (see make_golden.py)."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MOVED, ENTER, LEAVE = 0, 1, 2


def names():
    return sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def expected(fx, i):
    """Sorted (enter keys, leave keys) of flush i."""
    eo, lo = fx["enter_off"].astype(np.int64), fx["leave_off"].astype(np.int64)
    return fx["enter_keys"][eo[i]:eo[i + 1]], fx["leave_keys"][lo[i]:lo[i + 1]]


def final_state(fx):
    """(x, z, seq, space-or-DEAD) per slot after the whole stream; seq = call order."""
    n = int(fx["max_slots"])
    x = np.zeros(n, np.float32)
    z = np.zeros(n, np.float32)
    seq = np.zeros(n, np.uint64)
    sp = np.full(n, 0xFFFFFFFF, np.uint32)
    for j, (k, s) in enumerate(zip(fx["op_kind"].tolist(), fx["op_slot"].tolist())):
        if k == LEAVE:
            sp[s] = 0xFFFFFFFF
            continue
        if k == ENTER:
            sp[s] = fx["op_space"][j]
        x[s], z[s] = fx["op_x"][j], fx["op_z"][j]
        seq[s] = j + 1
    return x, z, seq, sp


def replay(fx, apply_op, flush):
    """Drive apply_op(kind, slot, x, z, space) in order and yield
    (flush index, flush()) at every flush point."""
    kind, slot = fx["op_kind"].tolist(), fx["op_slot"].tolist()
    xs, zs, sps = fx["op_x"], fx["op_z"], fx["op_space"].tolist()
    k0 = 0
    for i, k1 in enumerate(fx["flush_at"].tolist()):
        for j in range(k0, k1):
            apply_op(kind[j], slot[j], xs[j], zs[j], sps[j])
        k0 = k1
        yield i, flush()
