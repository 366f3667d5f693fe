"""The CPU oracle against the known-answer tests of SURVEY.md Appendix C and
against itself (sequential XZ-list vs the closed-form batch relation).

The reference (go-aoi v0.2.0, go.mod:29) ships no AOI fixtures and cannot be
built here, so these KATs plus the sequential/closed-form cross-check are the
oracle's only pins ("parity unpinned").
"""
import numpy as np
import pytest

D = np.float32(100.0)


def f32(bits):
    return np.frombuffer(np.uint32(bits).tobytes(), np.float32)[0]


def test_kat_float_bits():
    # Appendix C bit patterns
    assert D.view(np.uint32) == 0x42C80000
    assert f32(0xC57CC1A7) == np.float32(-4044.103271484375)
    assert f32(0xC58180D4) == np.float32(-4144.103515625)


def test_kat_r1_asymmetric(oracle_mod):
    a, b = f32(0xC57CC1A7), f32(0xC58180D4)
    assert oracle_mod.pred(a, 0, b, 0, D) is True   # P_A(B)
    assert oracle_mod.pred(b, 0, a, 0, D) is False  # P_B(A)
    assert not abs(np.float32(b - a)) <= D
    # A moved last -> neighbours
    m = oracle_mod.XZList(D, 2)
    m.enter(1, b, 0)
    m.enter(0, a, 0)
    assert list(m.neighbors(0)) == [1] and list(m.neighbors(1)) == [0]
    # B moves last (same position) -> no longer neighbours
    m.moved(1, b, 0)
    assert m.neighbors(0).size == 0 and m.neighbors(1).size == 0
    t, ea, eb = m.take_events()
    ent, lev = oracle_mod.events_to_keys(t, ea, eb)
    assert ent.size == 2 and lev.size == 2


def test_kat_r2_mirror(oracle_mod):
    a, b = f32(0x43978D94), f32(0x434B1B27)
    assert a == np.float32(303.1060791015625) and b == np.float32(203.10606384277344)
    assert oracle_mod.pred(a, 0, b, 0, D) is False
    assert oracle_mod.pred(b, 0, a, 0, D) is True
    m = oracle_mod.XZList(D, 2)
    m.enter(0, a, 0)
    m.enter(1, b, 0)  # B last -> neighbours
    assert list(m.neighbors(0)) == [1]
    m.moved(0, a, 0)  # A last -> not
    assert m.neighbors(0).size == 0


def test_kat_t1_colocated(oracle_mod):
    # 10 monsters at the origin (examples/test_game/MySpace.go:61-64)
    m = oracle_mod.XZList(D, 10)
    for i in range(10):
        m.enter(i, 0, 0)
    t, a, b = m.take_events()
    ent, lev = oracle_mod.events_to_keys(t, a, b)
    assert ent.size == 90 and lev.size == 0
    assert m.pairs().size == 90


@pytest.mark.parametrize("dx,expect", [(100.0, True), (-100.0, True),
                                       (float(np.nextafter(np.float32(100), np.float32(np.inf))), False)])
def test_kat_t2_t3_inclusive_bounds(oracle_mod, dx, expect):
    m = oracle_mod.XZList(D, 2)
    m.enter(0, 0, 0)
    m.enter(1, np.float32(dx), 0)
    assert (m.neighbors(0).size == 1) == expect
    m2 = oracle_mod.XZList(D, 2)
    m2.enter(0, 0, 0)
    m2.enter(1, 0, np.float32(dx))
    assert (m2.neighbors(0).size == 1) == expect


def test_kat_l1_leave(oracle_mod):
    m = oracle_mod.XZList(D, 8)
    for i in range(8):
        m.enter(i, np.float32(i * 10), 0)
    m.take_events()
    k = m.neighbors(3).size
    assert k == 7
    m.leave(3)
    t, a, b = m.take_events()
    ent, lev = oracle_mod.events_to_keys(t, a, b)
    assert ent.size == 0 and lev.size == 2 * k
    assert m.neighbors(3).size == 0
    for i in range(8):
        assert 3 not in set(m.neighbors(i).tolist())


def test_errors_mirror_panics(oracle_mod):
    m = oracle_mod.XZList(D, 2)
    with pytest.raises(RuntimeError):
        m.moved(0, 1, 1)
    with pytest.raises(RuntimeError):
        m.leave(0)
    m.enter(0, 0, 0)
    with pytest.raises(RuntimeError):
        m.enter(0, 0, 0)


def _nudge(v, k):
    v = np.float32(v)
    for _ in range(abs(k)):
        v = np.nextafter(v, np.float32(np.inf) if k > 0 else np.float32(-np.inf))
    return np.float32(v)


def boundary_ops(rng, n, steps, span=5000.0):
    """Random Enter/Moved/Leave stream whose positions sit on other entities'
    window edges: x = fl32(anchor +- D) nudged by a few ulps.  Spans several
    binades so that fl32(x+-D) rounds and P_A(B) != P_B(A) occurs."""
    live = np.zeros(n, bool)
    px = np.zeros(n, np.float32)
    pz = np.zeros(n, np.float32)
    ops = []
    for _ in range(steps):
        i = int(rng.integers(n))
        cand = np.nonzero(live)[0]
        if cand.size and rng.random() < 0.8:
            j = int(rng.choice(cand))
            x = _nudge(px[j] + np.float32(rng.choice([-1, 0, 1])) * D, int(rng.integers(-2, 3)))
            z = _nudge(pz[j] + np.float32(rng.choice([-1, 0, 1])) * D, int(rng.integers(-2, 3)))
        else:
            x = np.float32(rng.uniform(-span, span))
            z = np.float32(rng.uniform(-span, span))
        if not live[i]:
            ops.append((1, i, x, z))
            live[i] = True
        elif rng.random() < 0.08:
            ops.append((2, i, np.float32(0), np.float32(0)))
            live[i] = False
            continue
        else:
            ops.append((0, i, x, z))
        px[i], pz[i] = x, z
    return ops


def count_asymmetric(oracle_mod, x, z, live):
    c = 0
    for a in live:
        for b in live:
            if a < b and oracle_mod.pred(x[a], z[a], x[b], z[b], D) != oracle_mod.pred(x[b], z[b], x[a], z[a], D):
                c += 1
    return c


@pytest.mark.parametrize("seed,span", [(1, 5000.0), (2, 5000.0), (3, 300.0), (4, 70000.0)])
def test_sequential_matches_closed_form(oracle_mod, seed, span):
    """Appendix B: the sequential manager's relation == P_W(L) with W = last mover,
    and the net events between checkpoints == the diff of the two relations."""
    rng = np.random.default_rng(seed)
    n = 48
    m = oracle_mod.XZList(D, n)
    x = np.zeros(n, np.float32)
    z = np.zeros(n, np.float32)
    seq = np.zeros(n, np.uint64)
    sp = np.full(n, oracle_mod.DEAD, np.uint32)
    s = 0
    asym = 0
    ops = boundary_ops(rng, n, 1500, span)
    prev = np.empty(0, np.uint64)
    for k, (op, i, xi, zi) in enumerate(ops):
        if op == 1:
            m.enter(i, xi, zi)
        elif op == 0:
            m.moved(i, xi, zi)
        else:
            m.leave(i)
        if op == 2:
            sp[i] = oracle_mod.DEAD
        else:
            x[i], z[i] = xi, zi
            s += 1
            seq[i] = s
            sp[i] = 0
        if k % 25 == 24 or k == len(ops) - 1:
            assert m.check() == 0
            got = m.pairs()
            want = oracle_mod.closed_form_pairs(x, z, seq, sp, {0: D})
            np.testing.assert_array_equal(got, want)
            t, ea, eb = m.take_events()
            ent, lev = oracle_mod.net_events(t, ea, eb)
            np.testing.assert_array_equal(ent, np.setdiff1d(want, prev))
            np.testing.assert_array_equal(lev, np.setdiff1d(prev, want))
            prev = want
            if k % 100 == 99:
                asym += count_asymmetric(oracle_mod, x, z, np.nonzero(sp != oracle_mod.DEAD)[0])
    if span >= 5000:
        assert asym > 0, "boundary stream never exercised an asymmetric pair"


def test_workload_cfg1_sequential_vs_closed_form(oracle_mod):
    from goworld_amd.workload import make_workload
    w = make_workload("cfg1")
    m = oracle_mod.XZList(w.D, w.n)
    slots, x0, z0, _sp = w.initial()
    seq = np.zeros(w.n, np.uint64)
    s = 0
    for i in range(w.n):
        m.enter(int(slots[i]), x0[i], z0[i])
        s += 1
        seq[slots[i]] = s
    for t in range(5):
        sl, nx, nz = w.tick(t)
        m.moved_batch(sl, nx, nz)
        seq[sl] = s + 1 + np.arange(sl.size, dtype=np.uint64)
        s += sl.size
    want = oracle_mod.closed_form_pairs(w.x, w.z, seq, np.zeros(w.n, np.uint32), {0: w.D})
    np.testing.assert_array_equal(m.pairs(), want)
    assert want.size > 1000


def test_bulk_enter_equals_sequential_enters(oracle_mod):
    """xz_bulk_enter (used to populate the 1M-entity cpu_baseline) == Enter in order."""
    from goworld_amd.workload import make_workload
    w = make_workload("cfg3", n=3000)
    a = oracle_mod.XZList(w.D, w.n)
    b = oracle_mod.XZList(w.D, w.n, record=False)
    order = np.random.default_rng(5).permutation(w.n).astype(np.int32)
    for i in order:
        a.enter(int(i), w.x[i], w.z[i])
    b.bulk_enter(order, w.x[order], w.z[order])
    assert b.check() == 0
    np.testing.assert_array_equal(a.pairs(), b.pairs())
    sl, nx, nz = w.tick(0)
    a.take_events()
    a.moved_batch(sl, nx, nz)
    b.moved_batch(sl, nx, nz)
    np.testing.assert_array_equal(a.pairs(), b.pairs())


def test_closed_form_diff_matches_setdiff(oracle_mod):
    """cf_diff (the multithreaded tick diff used at full cfg3 size) == set
    difference of two cf_pairs relations, with leaves, enters and space changes."""
    rng = np.random.default_rng(17)
    n = 4000
    x0 = rng.uniform(-1500, 1500, n).astype(np.float32)
    z0 = rng.uniform(-1500, 1500, n).astype(np.float32)
    sp0 = rng.integers(0, 2, n).astype(np.uint32)
    s0 = rng.permutation(n).astype(np.uint64) + 1
    sp0[rng.random(n) < 0.05] = oracle_mod.DEAD
    x1 = (x0 + rng.uniform(-30, 30, n)).astype(np.float32)
    z1 = (z0 + rng.uniform(-30, 30, n)).astype(np.float32)
    sp1 = sp0.copy()
    ch = rng.random(n) < 0.05
    sp1[ch] = rng.integers(0, 2, ch.sum()).astype(np.uint32)
    sp1[rng.random(n) < 0.05] = oracle_mod.DEAD
    s1 = s0.copy()
    mv = rng.random(n) < 0.7
    s1[mv] = n + 1 + rng.permutation(mv.sum()).astype(np.uint64)
    Ds = {0: np.float32(100.0), 1: np.float32(60.0)}
    ent, lev = oracle_mod.closed_form_diff((x0, z0, s0, sp0), (x1, z1, s1, sp1), Ds, threads=3)

    def rel(x, z, s, sp):  # space-qualified keys (each space its own manager)
        k = oracle_mod.closed_form_pairs(x, z, s, sp, Ds)
        a = (k >> np.uint64(32)).astype(np.int64)
        return set(zip(sp[a].tolist(), k.tolist()))

    r0, r1 = rel(x0, z0, s0, sp0), rel(x1, z1, s1, sp1)
    want_e = np.array(sorted(k for _, k in r1 - r0), np.uint64)
    want_l = np.array(sorted(k for _, k in r0 - r1), np.uint64)
    np.testing.assert_array_equal(ent, want_e)
    np.testing.assert_array_equal(lev, want_l)
    assert ent.size > 100 and lev.size > 100
    rows = oracle_mod.closed_form_rows(x1, z1, s1, sp1, Ds, [0, 5, 17])
    k1 = oracle_mod.closed_form_pairs(x1, z1, s1, sp1, Ds)
    for q, r in zip([0, 5, 17], rows):
        np.testing.assert_array_equal(r, (k1[(k1 >> np.uint64(32)) == q] & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    assert oracle_mod.key_checksum(ent) == oracle_mod.key_checksum(ent[::-1].copy())


def test_cpu_grid_comparator_counts(oracle_mod):
    """The CPU-grid comparator of bench.py (oracle/cpu_grid.c) reports, tick by tick,
    the enter/leave counts of the closed-form diff (it computes the same relation)."""
    from goworld_amd.workload import make_workload
    wl = make_workload("cfg3", n=20000)
    n = wl.n
    seq = 1 + np.arange(n, dtype=np.uint64)
    sp = np.zeros(n, np.uint32)
    g = oracle_mod.CpuGrid(wl.x, wl.z, wl.D, threads=3)
    want = oracle_mod.closed_form_pairs(wl.x, wl.z, seq, sp, {0: wl.D})
    assert g.pairs == want.size
    nxt = n + 1
    for t in range(3):
        before = (wl.x.copy(), wl.z.copy(), seq.copy(), sp)
        sl, nx, nz = wl.tick(t)
        seq[sl] = nxt + np.arange(sl.size, dtype=np.uint64)
        nxt += sl.size
        ne, nl = g.tick(sl, nx, nz)
        e, l = oracle_mod.closed_form_diff(before, (wl.x, wl.z, seq, sp), {0: wl.D}, threads=3)
        assert (ne, nl) == (e.size, l.size) and ne > 0
