#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (SURVEY.md §8c).

go-aoi v0.2.0 (the module the reference's AOI path lives in, go.mod:29) is
not vendored and Go is absent here, and the reference holds no AOI tests or
vectors, so the expected outputs come from the sequential XZ-list
restatement in oracle/ (oracle/xzlist.c) -- the
fixtures pin the GPU path to that restatement and the restatement to
itself across rounds ("parity unpinned" against go-aoi itself; the KAT
fixtures are additionally checked against the hand-derived expectations of
Appendix C in tests/test_golden.py).

Every fixture is one op stream in call (= seq) order with flush points, and
per flush the sorted net directed enter / leave keys (a << 32 | b) computed
per space manager (a pair that changes spaces is a leave in one manager and
an enter in the other).  Format: numpy .npz, no pickles.

    python tests/golden/make_golden.py      # rewrites the .npz files
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402  (test infrastructure)
from goworld_amd.workload import make_workload  # noqa: E402

MOVED, ENTER, LEAVE = 0, 1, 2
D100 = np.float32(100.0)


def f32(bits):
    return np.frombuffer(np.uint32(bits).tobytes(), np.float32)[0]


def nudge(v, k):
    v = np.float32(v)
    for _ in range(abs(k)):
        v = np.nextafter(v, np.float32(np.inf) if k > 0 else np.float32(-np.inf))
    return np.float32(v)


class Stream:
    def __init__(self, max_slots, space_D):
        self.max_slots = max_slots
        self.space_D = [np.float32(d) for d in space_D]
        self.kind, self.slot, self.x, self.z, self.space = [], [], [], [], []
        self.flush_at = []

    def op(self, kind, slot, x=0.0, z=0.0, space=0):
        self.kind.append(kind)
        self.slot.append(slot)
        self.x.append(np.float32(x))
        self.z.append(np.float32(z))
        self.space.append(space)

    def enter(self, slot, x, z, space=0):
        self.op(ENTER, slot, x, z, space)

    def moved(self, slot, x, z):
        self.op(MOVED, slot, x, z)

    def leave(self, slot):
        self.op(LEAVE, slot)

    def flush(self):
        self.flush_at.append(len(self.kind))


def run_oracle(st: Stream):
    """Replay through one sequential XZList per space; per-flush net events."""
    orc = oracle.SpacesOracle({i: d for i, d in enumerate(st.space_D)}, st.max_slots)
    ent_keys, lev_keys, ent_off, lev_off = [], [], [0], [0]
    k0 = 0
    for k1 in st.flush_at:
        for i in range(k0, k1):
            kd, s = st.kind[i], st.slot[i]
            if kd == ENTER:
                orc.enter(st.space[i], s, st.x[i], st.z[i])
            elif kd == LEAVE:
                orc.leave(s)
            else:
                orc.moved(s, st.x[i], st.z[i])
        k0 = k1
        es, ls = [], []
        for m in orc.mgr.values():
            e, l = oracle.net_events(*m.take_events())
            es.append(e)
            ls.append(l)
        e = np.sort(np.concatenate(es)) if es else np.empty(0, np.uint64)
        l = np.sort(np.concatenate(ls)) if ls else np.empty(0, np.uint64)
        ent_keys.append(e)
        lev_keys.append(l)
        ent_off.append(ent_off[-1] + e.size)
        lev_off.append(lev_off[-1] + l.size)
    return (np.concatenate(ent_keys).astype(np.uint64), np.array(ent_off, np.uint64),
            np.concatenate(lev_keys).astype(np.uint64), np.array(lev_off, np.uint64), orc.pairs())


def save(name, st: Stream, note: str):
    ek, eo, lk, lo, pairs = run_oracle(st)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(
        path, max_slots=np.uint32(st.max_slots), space_D=np.array(st.space_D, np.float32),
        op_kind=np.array(st.kind, np.uint8), op_slot=np.array(st.slot, np.uint32),
        op_x=np.array(st.x, np.float32), op_z=np.array(st.z, np.float32),
        op_space=np.array(st.space, np.uint32), flush_at=np.array(st.flush_at, np.uint64),
        enter_keys=ek, enter_off=eo, leave_keys=lk, leave_off=lo, final_pairs=pairs,
        note=np.array(note))
    print(f"{name}: {len(st.kind)} ops, {len(st.flush_at)} flushes, {ek.size} enters, {lk.size} leaves, "
          f"{pairs.size} final pairs, {os.path.getsize(path)} B")


def kats():
    a, b = f32(0xC57CC1A7), f32(0xC58180D4)  # R1
    st = Stream(4, [D100])
    st.enter(1, b, 0)
    st.enter(0, a, 0)
    st.flush()  # A last: P_A(B) -> neighbours
    st.moved(1, b, 0)
    st.flush()  # B last: P_B(A) false -> leave
    save("kat_r1", st, "Appendix C R1: A=0xc57cc1a7 B=0xc58180d4, ownership decides")

    a, b = f32(0x43978D94), f32(0x434B1B27)  # R2
    st = Stream(4, [D100])
    st.enter(0, a, 0)
    st.enter(1, b, 0)
    st.flush()  # B last: P_B(A) true -> neighbours
    st.moved(0, a, 0)
    st.flush()  # A last: P_A(B) false -> leave
    save("kat_r2", st, "Appendix C R2 (mirror of R1): A=0x43978d94 B=0x434b1b27")

    st = Stream(16, [D100])
    for i in range(10):
        st.enter(i, 0.0, 0.0)
    st.flush()
    save("kat_t1", st, "Appendix C T1: 10 co-located entities -> 45 pairs, 90 directed enters")

    st = Stream(8, [D100])
    st.enter(0, 0.0, 0.0)
    st.enter(1, 100.0, 0.0)
    st.enter(2, -100.0, 0.0)
    st.enter(3, 0.0, 100.0)
    st.enter(4, np.nextafter(np.float32(100.0), np.float32(np.inf)), 0.0)
    st.enter(5, 0.0, np.nextafter(np.float32(-100.0), np.float32(-np.inf)))
    st.flush()
    save("kat_t2_t3", st, "Appendix C T2/T3: |d| == D inclusive, nextafter(D) excluded")

    st = Stream(16, [D100])
    for i in range(8):
        st.enter(i, 10.0 * i, 5.0 * (i % 3))
    st.flush()
    st.leave(3)
    st.flush()
    save("kat_l1", st, "Appendix C L1: leave of an entity with k neighbours -> 2k directed leaves")


def cfg1():
    wl = make_workload("cfg1")
    st = Stream(wl.n, [wl.D])
    slots, x0, z0, _ = wl.initial()
    for i in range(wl.n):
        st.enter(int(slots[i]), x0[i], z0[i])
    st.flush()
    for t in range(50):
        sl, nx, nz = wl.tick(t)
        for s, x, z in zip(sl.tolist(), nx, nz):
            st.moved(int(s), x, z)
        st.flush()
    save("cfg1_1k_50t", st, "config 1: 1000 Avatars in [-400,400)^2, bot walk p=0.5, 50 ticks, seed 0x5EED0001")


def lattice():
    """64 entities on a 100-spaced lattice, every coordinate k*100 +- a few
    ulps; Enter/Moved/Leave churn; forces asymmetric (ownership) pairs."""
    rng = np.random.default_rng(0x1A77)
    n = 64
    st = Stream(n, [D100])
    live = np.zeros(n, bool)
    for step in range(3000):
        i = int(rng.integers(n))
        x = nudge(np.float32(100.0 * rng.integers(-4, 5)) + np.float32(rng.choice([0.0, 0.5, 3e-5])),
                  int(rng.integers(-3, 4)))
        z = nudge(np.float32(100.0 * rng.integers(-4, 5)), int(rng.integers(-3, 4)))
        if not live[i]:
            st.enter(i, x, z)
            live[i] = True
        elif rng.random() < 0.06:
            st.leave(i)
            live[i] = False
        else:
            st.moved(i, x, z)
        if step % 7 == 6:
            st.flush()
    st.flush()
    save("lattice64", st, "64-entity boundary lattice, coords k*100 +- ulps, flush every 7 ops")


def multispace():
    """16 spaces x 128 entities, per-space D, moves + teleports + leaves +
    re-enters + space changes."""
    rng = np.random.default_rng(0x5BACE)
    ns, per = 16, 128
    n = ns * per
    Ds = [np.float32(100.0 if s % 4 else 37.5 + s) for s in range(ns)]
    st = Stream(n + 64, Ds)
    L = 400.0
    sp = np.repeat(np.arange(ns), per)
    x = rng.uniform(-L, L, n).astype(np.float32)
    z = rng.uniform(-L, L, n).astype(np.float32)
    live = np.ones(n, bool)
    for i in rng.permutation(n):
        st.enter(int(i), x[i], z[i], int(sp[i]))
    st.flush()
    for t in range(12):
        for i in rng.permutation(n):
            r = rng.random()
            if not live[i]:
                if r < 0.5:
                    sp[i] = int(rng.integers(ns))
                    x[i] = np.float32(rng.uniform(-L, L))
                    z[i] = np.float32(rng.uniform(-L, L))
                    st.enter(int(i), x[i], z[i], int(sp[i]))
                    live[i] = True
            elif r < 0.03:
                st.leave(int(i))
                live[i] = False
            elif r < 0.05:  # teleport
                x[i] = np.float32(rng.uniform(-L, L))
                z[i] = np.float32(rng.uniform(-L, L))
                st.moved(int(i), x[i], z[i])
            elif r < 0.06:  # change space within the flush
                st.leave(int(i))
                sp[i] = int(rng.integers(ns))
                st.enter(int(i), x[i], z[i], int(sp[i]))
            elif r < 0.8:
                x[i] = np.float32(x[i] + np.float32(rng.uniform(-3, 3)))
                z[i] = np.float32(z[i] + np.float32(rng.uniform(-3, 3)))
                st.moved(int(i), x[i], z[i])
        st.flush()
    save("multispace16x128", st, "16 spaces x 128 entities, per-space D, churn incl. space changes, 12 ticks")


if __name__ == "__main__":
    oracle.build()
    kats()
    cfg1()
    lattice()
    multispace()
