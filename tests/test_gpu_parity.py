"""HIP path (through the C ABI) vs the CPU oracle: bit-exact event sets.

Every test drives libgwaoi.so exactly as GoWorld's Space drives go-aoi
(Enter/Leave/Moved in call order, Space.go:211,243,259), flushes, and
compares the sorted enter/leave sets with the oracle's net events and the
neighbour relation with the oracle's sets.  Integer/index outputs: bit-exact,
no tolerance.
"""
import numpy as np
import pytest

from goworld_amd import World, GwaoiError, pair_keys
from goworld_amd._lib import (GWAOI_F_TEST_BUCKETED, GWAOI_F_TEST_FORCE_COPY, GWAOI_F_TEST_FORCE_RADIX,
                              GWAOI_F_TEST_REGROW_FAIL, GWAOI_F_TEST_SPARSE_SCR2, GWAOI_F_TEST_SPARSE_SEQUENCE)
from goworld_amd.workload import make_workload

pytestmark = pytest.mark.gpu

D = np.float32(100.0)


def f32(bits):
    return np.frombuffer(np.uint32(bits).tobytes(), np.float32)[0]


def flush(w):
    ent, lev = w.tick()
    return pair_keys(ent), pair_keys(lev)


def test_kat_r1_ownership_gpu():
    a, b = f32(0xC57CC1A7), f32(0xC58180D4)
    with World(4) as w:
        s = w.space_create(D)
        w.enter(s, 1, b, 0)
        w.enter(s, 0, a, 0)  # A last: P_A(B) true -> neighbours
        ent, lev = flush(w)
        assert ent.tolist() == [(0 << 32) | 1, (1 << 32) | 0] and lev.size == 0
        w.moved(1, b, 0)  # B last at the same position: P_B(A) false -> leave
        ent, lev = flush(w)
        assert ent.size == 0 and lev.tolist() == [(0 << 32) | 1, (1 << 32) | 0]
        assert w.neighbors(0).size == 0


def test_kat_r2_mirror_gpu():
    a, b = f32(0x43978D94), f32(0x434B1B27)
    with World(4) as w:
        s = w.space_create(D)
        w.enter(s, 0, a, 0)
        w.enter(s, 1, b, 0)
        ent, _ = flush(w)
        assert ent.size == 2
        w.moved(0, a, 0)
        _, lev = flush(w)
        assert lev.size == 2


def test_kat_t1_colocated_gpu():
    with World(16) as w:
        s = w.space_create(D)
        for i in range(10):
            w.enter(s, i, 0.0, 0.0)
        ent, lev = flush(w)
        assert ent.size == 90 and lev.size == 0
        assert w.neighbors(3).tolist() == [i for i in range(10) if i != 3]


@pytest.mark.parametrize("dx,expect", [(100.0, True), (-100.0, True),
                                       (float(np.nextafter(np.float32(100), np.float32(np.inf))), False)])
def test_kat_t2_t3_bounds_gpu(dx, expect):
    with World(4) as w:
        s = w.space_create(D)
        w.enter(s, 0, 0.0, 0.0)
        w.enter(s, 1, np.float32(dx), 0.0)
        w.enter(s, 2, 7000.0, 0.0)
        w.enter(s, 3, 7000.0, np.float32(dx))
        ent, _ = flush(w)
        keys = set(ent.tolist())
        assert ((0 << 32 | 1) in keys) == expect
        assert ((2 << 32 | 3) in keys) == expect


def test_kat_l1_leave_gpu():
    with World(8) as w:
        s = w.space_create(D)
        for i in range(8):
            w.enter(s, i, np.float32(i * 10), 0.0)
        flush(w)
        w.leave(3)
        ent, lev = flush(w)
        assert ent.size == 0 and lev.size == 14
        assert all(3 not in w.neighbors(i).tolist() for i in range(8) if i != 3)


def test_error_paths_gpu():
    with World(8) as w:
        s = w.space_create(D)
        with pytest.raises(GwaoiError):
            w.moved(0, 1, 1)
        with pytest.raises(GwaoiError):
            w.leave(0)
        with pytest.raises(GwaoiError):
            w.enter(s, 8, 0, 0)
        with pytest.raises(GwaoiError):
            w.enter(s, 0, float("nan"), 0)
        with pytest.raises(GwaoiError):
            w.space_create(0.0)
        w.enter(s, 0, 0, 0)
        with pytest.raises(GwaoiError):
            w.enter(s, 0, 0, 0)
        with pytest.raises(GwaoiError):
            w.space_destroy(s)


def run_stream_vs_oracle(oracle_mod, ops, n, flush_every, D_by_space=None, check_neighbors=True):
    """Apply one op stream to the GPU world and to one sequential manager per
    space; after every `flush_every` ops compare net events and relations."""
    D_by_space = D_by_space or {0: D}
    orc = oracle_mod.SpacesOracle(D_by_space, n)
    with World(n, max_spaces=max(D_by_space) + 1) as w:
        ids = {}
        for sp in sorted(D_by_space):
            ids[sp] = w.space_create(D_by_space[sp])
        for k, op in enumerate(ops):
            kind = op[0]
            if kind == 1:
                _, i, x, z, sp = op
                w.enter(ids[sp], i, x, z)
                orc.enter(sp, i, x, z)
            elif kind == 0:
                _, i, x, z = op[:4]
                w.moved(i, x, z)
                orc.moved(i, x, z)
            else:
                w.leave(op[1])
                orc.leave(op[1])
            if k % flush_every == flush_every - 1 or k == len(ops) - 1:
                ge, gl = flush(w)
                oe, ol = oracle_mod.net_events(*orc.take_events(with_space=True))
                np.testing.assert_array_equal(ge, oe)
                np.testing.assert_array_equal(gl, ol)
                if check_neighbors:
                    for i in range(0, n, max(1, n // 16)):
                        if i in orc.local:
                            np.testing.assert_array_equal(w.neighbors(i), orc.neighbors(i).astype(np.uint32))


def boundary_ops(rng, n, steps, span=5000.0, spaces=(0,)):
    """Enter/Moved/Leave stream on other entities' window edges (+- a few ulps)."""
    live = np.zeros(n, bool)
    spc = np.zeros(n, np.int64)
    px = np.zeros(n, np.float32)
    pz = np.zeros(n, np.float32)
    ops = []

    def nudge(v, k):
        v = np.float32(v)
        for _ in range(abs(k)):
            v = np.nextafter(v, np.float32(np.inf) if k > 0 else np.float32(-np.inf))
        return np.float32(v)

    for _ in range(steps):
        i = int(rng.integers(n))
        cand = np.nonzero(live)[0]
        if cand.size and rng.random() < 0.8:
            j = int(rng.choice(cand))
            x = nudge(px[j] + np.float32(rng.choice([-1, 0, 1])) * D, int(rng.integers(-2, 3)))
            z = nudge(pz[j] + np.float32(rng.choice([-1, 0, 1])) * D, int(rng.integers(-2, 3)))
        else:
            x = np.float32(rng.uniform(-span, span))
            z = np.float32(rng.uniform(-span, span))
        if not live[i]:
            sp = int(rng.choice(spaces))
            ops.append((1, i, x, z, sp))
            live[i] = True
            spc[i] = sp
        elif rng.random() < 0.08:
            ops.append((2, i))
            live[i] = False
            continue
        else:
            ops.append((0, i, x, z))
        px[i], pz[i] = x, z
    return ops


@pytest.mark.parametrize("seed,flush_every", [(11, 1), (12, 7), (13, 50), (14, 400)])
def test_boundary_stream_gpu(oracle_mod, seed, flush_every):
    rng = np.random.default_rng(seed)
    ops = boundary_ops(rng, 64, 1200)
    run_stream_vs_oracle(oracle_mod, ops, 64, flush_every)


@pytest.mark.parametrize("seed", [15, 16])
def test_boundary_stream_1m_background_gpu(oracle_mod, seed):
    """The flush_every=1 boundary stream inside a 1M-entity world: the stream's 64 entities move
    on each other's window edges (+- a few ulps) near the origin, flushed after every op -- a
    Moved flush is a sparse flush of one call against the 1M-entry frame, an Enter / Leave flush
    a full one -- while 2^20 background entities of the same space sit far to the side (same
    grid rows, so a stream entity that changes row shifts background entries of the frame).  No
    background entity is ever within reach, so the events and relations are exactly the
    sequential oracle's over the stream alone."""
    rng = np.random.default_rng(seed)
    n_s, n_bg = 64, 1 << 20
    ops = boundary_ops(rng, n_s, 700)
    orc = oracle_mod.SpacesOracle({0: D}, n_s)
    L = float(np.sqrt(n_bg * 1250.0))
    bx = rng.uniform(100000.0, 100000.0 + L, n_bg).astype(np.float32)
    bz = rng.uniform(-L / 2, L / 2, n_bg).astype(np.float32)
    with World(n_s + n_bg) as w:
        s = w.space_create(D)
        w.enter_batch(s, np.arange(n_s, n_s + n_bg, dtype=np.uint32), bx, bz)
        w.tick_device()  # the background's own relation (not part of the comparison)
        sparse0 = w.debug_counters()["sparse_flushes"]
        for k, op in enumerate(ops):
            if op[0] == 1:
                _, i, x, z, _sp = op
                w.enter(s, i, x, z)
                orc.enter(0, i, x, z)
            elif op[0] == 0:
                _, i, x, z = op[:4]
                w.moved(i, x, z)
                orc.moved(i, x, z)
            else:
                w.leave(op[1])
                orc.leave(op[1])
            ge, gl = flush(w)
            oe, ol = oracle_mod.net_events(*orc.take_events(with_space=True))
            np.testing.assert_array_equal(ge, oe, err_msg=f"op {k}: enters")
            np.testing.assert_array_equal(gl, ol, err_msg=f"op {k}: leaves")
            if k % 100 == 99:
                for i in range(0, n_s, 4):
                    if i in orc.local:
                        np.testing.assert_array_equal(w.neighbors(i), orc.neighbors(i).astype(np.uint32))
        assert w.debug_counters()["sparse_flushes"] - sparse0 > 200


def test_boundary_stream_multispace_gpu(oracle_mod):
    rng = np.random.default_rng(21)
    ops = boundary_ops(rng, 96, 1500, span=800.0, spaces=(0, 1, 2))
    run_stream_vs_oracle(oracle_mod, ops, 96, 37, {0: D, 1: np.float32(50.0), 2: np.float32(100.0)})


def test_empty_and_ragged_flushes_gpu():
    with World(32) as w:
        s = w.space_create(D)
        assert flush(w)[0].size == 0  # empty world
        assert flush(w)[0].size == 0
        w.enter(s, 5, 1.0, 1.0)
        ent, lev = flush(w)
        assert ent.size == 0 and lev.size == 0  # a lone entity has no neighbours
        w.leave(5)
        assert flush(w)[1].size == 0
        w.enter(s, 5, 1.0, 1.0)  # slot reuse after a flush
        w.enter(s, 6, 2.0, 2.0)
        w.leave(6)  # enter + leave inside one flush: no net event
        ent, lev = flush(w)
        assert ent.size == 0 and lev.size == 0


def test_cfg1_vs_sequential_oracle_gpu(oracle_mod):
    """examples/test_game-style space, 1000 Avatars, bot random walk (cfg1)."""
    wl = make_workload("cfg1")
    m = oracle_mod.XZList(wl.D, wl.n)
    with World(wl.n) as w:
        s = w.space_create(wl.D)
        slots, x0, z0, _ = wl.initial()
        w.enter_batch(s, slots, x0, z0)
        for i in range(wl.n):
            m.enter(int(slots[i]), x0[i], z0[i])
        ge, gl = flush(w)
        oe, ol = oracle_mod.net_events(*m.take_events())
        np.testing.assert_array_equal(ge, oe)
        assert gl.size == 0 and ge.size > 10000
        for t in range(30):
            sl, nx, nz = wl.tick(t)
            w.moved_batch(sl, nx, nz)
            m.moved_batch(sl, nx, nz)
            ge, gl = flush(w)
            oe, ol = oracle_mod.net_events(*m.take_events())
            np.testing.assert_array_equal(ge, oe)
            np.testing.assert_array_equal(gl, ol)


@pytest.mark.parametrize("cfg,n,ticks", [("cfg2", 20000, 4), ("cfg2", 100000, 4), ("cfg3", 40000, 3)])
def test_scaled_configs_vs_closed_form_gpu(oracle_mod, cfg, n, ticks):
    """cfg2 at its own size (100k) and reduced, cfg3 reduced (same density): GPU
    events == diff of the closed-form relation, and the GPU relation == the
    closed form."""
    wl = make_workload(cfg, n=n)
    seq = np.zeros(wl.n, np.uint64)
    sp = np.zeros(wl.n, np.uint32)
    with World(wl.n) as w:
        s = w.space_create(wl.D)
        slots, x0, z0, _ = wl.initial()
        w.enter_batch(s, slots, x0, z0)
        seq[slots] = 1 + np.arange(wl.n, dtype=np.uint64)
        nxt = wl.n + 1
        ge, _ = flush(w)
        prev = oracle_mod.closed_form_pairs(wl.x, wl.z, seq, sp, {0: wl.D})
        np.testing.assert_array_equal(ge, prev)
        for t in range(ticks):
            sl, nx, nz = wl.tick(t)
            w.moved_batch(sl, nx, nz)
            seq[sl] = nxt + np.arange(sl.size, dtype=np.uint64)
            nxt += sl.size
            ge, gl = flush(w)
            cur = oracle_mod.closed_form_pairs(wl.x, wl.z, seq, sp, {0: wl.D})
            np.testing.assert_array_equal(ge, np.setdiff1d(cur, prev))
            np.testing.assert_array_equal(gl, np.setdiff1d(prev, cur))
            prev = cur
        for i in range(0, wl.n, wl.n // 7):
            want = (prev[(prev >> np.uint64(32)) == np.uint64(i)] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            np.testing.assert_array_equal(w.neighbors(i), want)


def test_staged_host_batches_mixed_with_calls_gpu(oracle_mod):
    """Host move batches go through pinned staging + one H2D each (>= 64 moves) and run as
    device batches.  Interleave them in one flush with single Moved/Enter/Leave calls, small
    batches (host ops), a batch past the staging capacity (falls back to host ops) and repeated
    slots; the sequential XZ-list oracle decides every event."""
    rng = np.random.default_rng(11)
    n = 90000
    wl = make_workload("cfg2", n=n)
    slots, x0, z0, _ = wl.initial()
    live = np.zeros(n, bool)
    m = oracle_mod.XZList(wl.D, n)
    with World(n) as w:
        s = w.space_create(wl.D)
        k0 = n - 2000  # the last 2000 slots enter and leave along the way
        w.enter_batch(s, slots[:k0], x0[:k0], z0[:k0])
        m.bulk_enter(slots[:k0], x0[:k0], z0[:k0])
        live[slots[:k0]] = True
        flush(w)
        m.take_events()
        x, z = x0.copy(), z0.copy()

        def batch(k, span=None):
            pool = np.nonzero(live)[0] if span is None else np.nonzero(live)[0][:span]
            sl = rng.choice(pool, k).astype(np.uint32)  # with repeats
            nx = (x[sl] + rng.uniform(-40, 40, k)).astype(np.float32)
            nz = (z[sl] + rng.uniform(-40, 40, k)).astype(np.float32)
            w.moved_batch(sl, nx, nz)
            m.moved_batch(sl, nx, nz)
            x[sl], z[sl] = nx, nz

        for t in range(3):
            batch(5000)
            for i in rng.choice(np.nonzero(~live)[0], 300, replace=False):  # Enter between batches
                w.enter(s, int(i), x[i], z[i])
                m.enter(int(i), x[i], z[i])
                live[i] = True
            batch(70)
            batch(40)  # below the staging threshold: host ops
            for i in rng.choice(np.nonzero(live)[0], 200, replace=False):
                w.leave(int(i))
                m.leave(int(i))
                live[i] = False
            j = int(np.nonzero(live)[0][0])
            w.moved(j, x[j] + np.float32(3), z[j])
            m.moved(j, x[j] + np.float32(3), z[j])
            x[j] += np.float32(3)
            batch(64000 if t == 1 else 3000, span=500 if t == 2 else None)  # t=1: past capacity
            ge, gl = flush(w)
            oe, ol = oracle_mod.net_events(*m.take_events())
            np.testing.assert_array_equal(ge, oe)
            np.testing.assert_array_equal(gl, ol)
        for i in np.nonzero(live)[0][::997]:
            np.testing.assert_array_equal(w.neighbors(int(i)), np.asarray(m.neighbors(int(i)), np.uint32))


def test_staged_batch_many_spaces_gpu(oracle_mod):
    """cfg4-style world (160 spaces x 2000): each tick is one host batch of 320k moves interleaved
    over all spaces, staged on two host threads with per-space boxes.  Events == the diff of the
    closed-form relation, tick by tick."""
    nsp = 160
    wl = make_workload("cfg4", n_spaces=nsp)
    slots, x0, z0, sp = wl.initial()
    seq = np.zeros(wl.n, np.uint64)
    dmap = {s: wl.D for s in range(nsp)}
    with World(wl.n, max_spaces=nsp) as w:
        ids = [w.space_create(wl.D) for _ in range(nsp)]
        nxt = 1
        for s in range(nsp):
            sel = np.nonzero(sp == s)[0]
            w.enter_batch(ids[s], slots[sel], x0[sel], z0[sel])
            seq[slots[sel]] = nxt + np.arange(sel.size, dtype=np.uint64)
            nxt += sel.size
        flush(w)
        prev = oracle_mod.closed_form_pairs(wl.x, wl.z, seq, sp, dmap)
        for t in range(2):
            sl, nx, nz = wl.tick(t)
            assert sl.size >= 2 * (1 << 17)  # two staging threads
            w.moved_batch(sl, nx, nz)
            seq[sl] = nxt + np.arange(sl.size, dtype=np.uint64)
            nxt += sl.size
            ge, gl = flush(w)
            cur = oracle_mod.closed_form_pairs(wl.x, wl.z, seq, sp, dmap)
            np.testing.assert_array_equal(ge, np.setdiff1d(cur, prev))
            np.testing.assert_array_equal(gl, np.setdiff1d(prev, cur))
            prev = cur


@pytest.mark.parametrize("bad", ["slot", "dead", "nan"])
def test_staged_host_batch_rejects_whole_batch_gpu(bad):
    """A staged host batch (>= 64 moves, validated on several host threads when large) with one bad
    move is rejected as a whole with the same status as per-call Moved, and queues nothing."""
    n = 300000
    rng = np.random.default_rng(3)
    with World(n + 1) as w:
        s = w.space_create(D)
        x0 = rng.uniform(-3000, 3000, n).astype(np.float32)
        z0 = rng.uniform(-3000, 3000, n).astype(np.float32)
        w.enter_batch(s, np.arange(n, dtype=np.uint32), x0, z0)
        flush(w)
        sl = np.arange(n, dtype=np.uint32)
        nx = (x0 + np.float32(500)).astype(np.float32)  # would change most relations
        k = n - 12345  # in the last host thread's chunk
        if bad == "slot":
            sl[k] = n + 7
        elif bad == "dead":
            sl[k] = n  # never entered
        else:
            nx[k] = np.float32("nan")
        with pytest.raises(GwaoiError):
            w.moved_batch(sl, nx, z0)
        ent, lev = flush(w)
        assert ent.size == 0 and lev.size == 0


def test_device_batch_matches_host_batch_gpu():
    torch = pytest.importorskip("torch")
    wl_a = make_workload("cfg2", n=8000)
    wl_b = make_workload("cfg2", n=8000)
    with World(wl_a.n) as wa, World(wl_b.n) as wb:
        for w, wl in ((wa, wl_a), (wb, wl_b)):
            s = w.space_create(wl.D)
            slots, x0, z0, _ = wl.initial()
            w.enter_batch(s, slots, x0, z0)
            w.tick()
        for t in range(3):
            sl, nx, nz = wl_a.tick(t)
            wa.moved_batch(sl, nx, nz)
            ea, la = wa.tick()
            sl2, nx2, nz2 = wl_b.tick(t)
            ds = torch.from_numpy(sl2.astype(np.int32)).cuda()
            dx = torch.from_numpy(nx2).cuda()
            dz = torch.from_numpy(nz2).cuda()
            torch.cuda.synchronize()
            wb.moved_batch_device(ds.data_ptr(), dx.data_ptr(), dz.data_ptr(), sl2.size)
            eb, lb = wb.tick()
            np.testing.assert_array_equal(pair_keys(ea), pair_keys(eb))
            np.testing.assert_array_equal(pair_keys(la), pair_keys(lb))


def test_device_batch_repeated_slots_gpu():
    """Slots moved several times in one flush, inside one device batch and
    across two (the single-pass apply's collision fixup): the last call wins,
    exactly as with host calls."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    wl = make_workload("cfg2", n=6000)
    slots, x0, z0, _ = wl.initial()
    with World(wl.n) as wa, World(wl.n) as wb:
        for w in (wa, wb):
            s = w.space_create(wl.D)
            w.enter_batch(s, slots, x0, z0)
            w.tick()
        x, z = x0.copy(), z0.copy()
        for t in range(4):
            runs = []
            for r in range(2):
                sl = rng.integers(0, 300 if r else wl.n, 5000).astype(np.uint32)  # many repeats
                nx = (x[sl] + rng.uniform(-30, 30, sl.size)).astype(np.float32)
                nz = (z[sl] + rng.uniform(-30, 30, sl.size)).astype(np.float32)
                runs.append((sl, nx, nz))
            dev = []
            for sl, nx, nz in runs:
                wa.moved_batch(sl, nx, nz)
                d = [torch.from_numpy(v).cuda() for v in (sl.astype(np.int32), nx, nz)]
                dev.append(d)
                wb.moved_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), sl.size)
            torch.cuda.synchronize()
            ea, la = wa.tick()
            eb, lb = wb.tick()
            np.testing.assert_array_equal(pair_keys(ea), pair_keys(eb))
            np.testing.assert_array_equal(pair_keys(la), pair_keys(lb))
            for sl, nx, nz in runs:  # last write wins
                x[sl], z[sl] = nx, nz
        for i in (0, 1, 7, 299, 5999):
            np.testing.assert_array_equal(wa.neighbors(i), wb.neighbors(i))


@pytest.mark.parametrize("bucketed", [False, True])
def test_device_batches_many_buckets_vs_closed_form_gpu(oracle_mod, bucketed):
    """Moves-only flushes through the global-claim apply and (GWAOI_F_TEST_BUCKETED)
    the bucketed one (slots regrouped by 4096-slot bucket, last op per slot by LDS
    claim): live slots scattered over 14 buckets, three device batches per flush
    with slots repeated inside a batch and across batches, one batch with
    explicit seqs.  Last call wins (Space.go:259 in call order); events vs the
    closed form."""
    torch = pytest.importorskip("torch")
    O = oracle_mod
    rng = np.random.default_rng(77)
    N = 57000
    live = np.sort(rng.choice(N, 20000, replace=False)).astype(np.uint32)
    L = float(np.sqrt(live.size * 1250.0))
    x = np.zeros(N, np.float32)
    z = np.zeros(N, np.float32)
    seq = np.zeros(N, np.uint64)
    sp = np.full(N, O.DEAD, np.uint32)
    x[live] = rng.uniform(-L / 2, L / 2, live.size).astype(np.float32)
    z[live] = rng.uniform(-L / 2, L / 2, live.size).astype(np.float32)
    with World(N, test_flags=GWAOI_F_TEST_BUCKETED if bucketed else 0) as w:
        s = w.space_create(D)
        w.enter_batch(s, live, x[live], z[live])
        seq[live] = 1 + np.arange(live.size, dtype=np.uint64)
        sp[live] = s
        nxt = live.size + 1
        w.tick()
        for t in range(4):
            before = (x.copy(), z.copy(), seq.copy(), sp.copy())
            keep = []
            for r in range(3):
                k = 9000 if r != 1 else 3000
                sl = (live[rng.integers(0, live.size, k)] if r != 1 else
                      live[rng.integers(0, 50, k)]).astype(np.uint32)  # run 1: 50 slots, ~60 moves each
                nx = (x[sl] + rng.uniform(-40, 40, k)).astype(np.float32)
                nz = (z[sl] + rng.uniform(-40, 40, k)).astype(np.float32)
                d = [torch.from_numpy(v).cuda() for v in (sl.astype(np.int32), nx, nz)]
                if r == 2 and t % 2:  # explicit seqs, above every earlier one
                    q = nxt + np.arange(k, dtype=np.uint64)
                    d.append(torch.from_numpy(q.astype(np.int64)).cuda())
                    torch.cuda.synchronize()
                    w.moved_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), k, d_seq=d[3].data_ptr())
                else:
                    torch.cuda.synchronize()
                    w.moved_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), k)
                keep.append(d)
                u, first_rev = np.unique(sl[::-1], return_index=True)
                lastpos = k - 1 - first_rev  # each slot's last call in the batch
                x[u], z[u] = nx[lastpos], nz[lastpos]
                seq[u] = nxt + lastpos.astype(np.uint64)
                nxt += k
            ge, gl = w.tick()
            want_e, want_l = O.closed_form_diff(before, (x, z, seq, sp), {s: D})
            assert want_e.size > 1000 and want_l.size > 1000
            np.testing.assert_array_equal(pair_keys(ge), want_e, err_msg=f"flush {t}: enters")
            np.testing.assert_array_equal(pair_keys(gl), want_l, err_msg=f"flush {t}: leaves")
        for i in live[rng.integers(0, live.size, 200)]:
            np.testing.assert_array_equal(
                w.neighbors(int(i)), O.closed_form_rows(x, z, seq, sp, {s: D}, np.array([i]))[0])


def test_device_batch_errors_reported_gpu():
    torch = pytest.importorskip("torch")
    with World(8) as w:
        s = w.space_create(D)
        w.enter(s, 0, 0, 0)
        w.tick()
        ds = torch.tensor([0, 5], dtype=torch.int32, device="cuda")  # slot 5 is not live
        dx = torch.tensor([1.0, 1.0], device="cuda")
        dz = torch.tensor([1.0, 1.0], device="cuda")
        torch.cuda.synchronize()
        w.moved_batch_device(ds.data_ptr(), dx.data_ptr(), dz.data_ptr(), 2)
        with pytest.raises(GwaoiError):
            w.tick()
        assert w.neighbors(0).size == 0


@pytest.mark.parametrize("seed,spaces", [(31, 1), (32, 3)])
def test_mixed_churn_vs_closed_form_gpu(oracle_mod, seed, spaces):
    """Steps, teleports (far movers), leaves, re-enters and space changes in
    one flush: exercises the combined pass and the special-entity pass.  The
    reference is the closed form evaluated on the queued state (seq = call order)."""
    rng = np.random.default_rng(seed)
    n = 12000
    L = float(np.sqrt(n / spaces * 1250.0))
    Ds = {s: np.float32(100.0 if s != 1 else 60.0) for s in range(spaces)}
    x = (rng.uniform(-L / 2, L / 2, n)).astype(np.float32)
    z = (rng.uniform(-L / 2, L / 2, n)).astype(np.float32)
    sp = rng.integers(0, spaces, n).astype(np.uint32)
    seq = np.zeros(n, np.uint64)
    live = np.ones(n, bool)
    nxt = 1
    with World(n, max_spaces=spaces) as w:
        ids = [w.space_create(Ds[s]) for s in range(spaces)]
        order = rng.permutation(n)
        for i in order:
            w.enter(ids[sp[i]], int(i), x[i], z[i])
            seq[i] = nxt
            nxt += 1
        w.tick()

        def cf():
            # relation keyed by (space, a, b): every space is its own go-aoi manager, so a
            # pair related in space 0 before and in space 2 after is a leave AND an enter
            spv = np.where(live, sp, oracle_mod.DEAD).astype(np.uint32)
            k = oracle_mod.closed_form_pairs(x, z, seq, spv, Ds)
            a = (k >> np.uint64(32)).astype(np.int64)
            return np.sort((spv[a].astype(np.uint64) << np.uint64(56)) | ((k >> np.uint64(32)) << np.uint64(28))
                           | (k & np.uint64(0xFFFFFFF)))

        def ab(keys):
            return np.sort(((keys >> np.uint64(28)) & np.uint64(0xFFFFFFF)) << np.uint64(32)
                           | (keys & np.uint64(0xFFFFFFF)))

        prev = cf()
        for t in range(6):
            ops = []
            for i in rng.permutation(n):
                r = rng.random()
                if live[i]:
                    if r < 0.01:
                        ops.append(("leave", i))
                    elif r < 0.02:  # leave + enter another (or the same) space: space change
                        ops.append(("leave", i))
                        ops.append(("enter", i, int(rng.integers(spaces)), rng.uniform(-L / 2, L / 2),
                                    rng.uniform(-L / 2, L / 2)))
                    elif r < 0.05:  # teleport
                        ops.append(("move", i, rng.uniform(-L / 2, L / 2), rng.uniform(-L / 2, L / 2)))
                    elif r < 0.95:
                        ops.append(("move", i, x[i] + rng.uniform(-1, 1), z[i] + rng.uniform(-1, 1)))
                elif r < 0.3:
                    ops.append(("enter", i, int(rng.integers(spaces)), rng.uniform(-L / 2, L / 2),
                                rng.uniform(-L / 2, L / 2)))
            for op in ops:
                if op[0] == "leave":
                    w.leave(int(op[1]))
                    live[op[1]] = False
                elif op[0] == "enter":
                    i, s_, xi, zi = op[1], op[2], np.float32(op[3]), np.float32(op[4])
                    w.enter(ids[s_], int(i), xi, zi)
                    live[i], sp[i], x[i], z[i], seq[i] = True, s_, xi, zi, nxt
                    nxt += 1
                else:
                    i, xi, zi = op[1], np.float32(op[2]), np.float32(op[3])
                    w.moved(int(i), xi, zi)
                    x[i], z[i], seq[i] = xi, zi, nxt
                    nxt += 1
            ge, gl = flush(w)
            cur = cf()
            np.testing.assert_array_equal(ge, ab(np.setdiff1d(cur, prev)))
            np.testing.assert_array_equal(gl, ab(np.setdiff1d(prev, cur)))
            prev = cur


@pytest.mark.parametrize("cfg,n", [("cfg3", 60000), ("cfg2", 30000)])
def test_incremental_sort_equals_radix_gpu(cfg, n):
    """The incremental frame sort (grid unchanged) is the stable sort by cell
    key: the flush's event arrays -- order included -- equal those of the
    full radix-sort path (GWAOI_FORCE_RADIX=1), with churn in every flush."""
    rng = np.random.default_rng(9)
    wl = make_workload(cfg, n=n)
    slots, x0, z0, _ = wl.initial()
    wr = World(n + 500, test_flags=GWAOI_F_TEST_FORCE_RADIX)
    wi = World(n + 500)
    try:
        for w in (wr, wi):
            s = w.space_create(wl.D)
            w.enter_batch(s, slots, x0, z0)
            w.tick()
        live = set(range(n))
        spare = list(range(n, n + 500))
        for t in range(5):
            sl, nx, nz = wl.tick(t)
            keep = np.array([int(v) in live for v in sl])
            sl, nx, nz = sl[keep], nx[keep], nz[keep]
            jump = rng.choice(sl.size, 200, replace=False)
            nx[jump] += rng.uniform(-300, 300, 200).astype(np.float32)
            leavers = rng.choice(sorted(live), 50, replace=False)
            enter = [spare.pop() for _ in range(40)]
            ex = rng.uniform(-wl.L / 2, wl.L / 2, 40).astype(np.float32)
            ez = rng.uniform(-wl.L / 2, wl.L / 2, 40).astype(np.float32)
            mv = ~np.isin(sl, leavers)
            outs = []
            for w in (wr, wi):
                w.moved_batch(sl[mv], nx[mv], nz[mv])
                w.leave_batch(leavers)
                w.enter_batch(0, np.array(enter, np.uint32), ex, ez)
                outs.append(w.tick())
            live -= set(int(v) for v in leavers)
            live |= set(enter)
            spare.extend(int(v) for v in leavers)
            (er, lr), (ei, li) = outs
            np.testing.assert_array_equal(er, ei)
            np.testing.assert_array_equal(lr, li)
            assert er.size + lr.size > 0
    finally:
        wr.close()
        wi.close()


@pytest.mark.parametrize("n", [255, 257, 4095, 4097, 16383, 16385, 32769])
def test_chain_free_offsets_at_tile_boundaries_gpu(oracle_mod, n):
    """Frame sizes either side of the block boundaries of the chain-free offsets (the cell scan's
    tiles, k_finish's groups of 256 tile entries, the combined pass's tiles): three churned
    flushes, incremental and radix paths equal (order included) and equal to the oracle."""
    rng = np.random.default_rng(n)
    wl = make_workload("cfg2", n=n)
    slots, x0, z0, _ = wl.initial()
    wr = World(n, cells_per_dist=3.0, sparse=False,  # full flushes only: the sort paths are the subject
               test_flags=GWAOI_F_TEST_FORCE_RADIX)
    wi = World(n, cells_per_dist=3.0, sparse=False)
    ref = oracle_mod.SpacesOracle({0: wl.D}, n)
    try:
        for w in (wr, wi):
            sp = w.space_create(wl.D)
            w.enter_batch(sp, slots, x0, z0)
            w.tick()
        for i in range(n):
            ref.enter(0, int(slots[i]), x0[i], z0[i])
        ref.take_events(with_space=True)
        for t in range(3):
            sl, nx, nz = wl.tick(t)
            jump = rng.choice(sl.size, max(1, sl.size // 50), replace=False)
            nx[jump] += rng.uniform(-400, 400, jump.size).astype(np.float32)
            outs = []
            for w in (wr, wi):
                w.moved_batch(sl, nx, nz)
                outs.append(w.tick())
            for i, a, b in zip(sl, nx, nz):
                ref.moved(int(i), a, b)
            oe, ol = oracle_mod.net_events(*ref.take_events(with_space=True))
            (er, lr), (ei, li) = outs
            np.testing.assert_array_equal(er, ei)
            np.testing.assert_array_equal(lr, li)
            np.testing.assert_array_equal(pair_keys(ei), oe)
            np.testing.assert_array_equal(pair_keys(li), ol)
        assert wi.debug_counters()["incremental_sorts"] >= 1
    finally:
        wr.close()
        wi.close()


def test_incremental_sort_pileup_gpu(oracle_mod):
    """Crowds piling into and draining out of a few cells, grid unchanged: hot cells
    get hundreds of arrivals a flush -- from below and above their previous run in S'
    order, and appended entries -- while others lose most of their run.  k_cell_merge's
    three-part layout and its per-tile changed-cell lists must still give the stable sort:
    event arrays, order included, equal those of the radix-sort path, and the oracle's."""
    rng = np.random.default_rng(21)
    n, D, L = 4000, 100.0, 3000.0
    x = rng.uniform(-L / 2, L / 2, n).astype(np.float32)
    z = rng.uniform(-L / 2, L / 2, n).astype(np.float32)
    x[:4], z[:4] = [-L / 2, L / 2, -L / 2, L / 2], [-L / 2, -L / 2, L / 2, L / 2]  # fixed corners: same grid
    hot = np.array([[-700.0, 300.0], [0.0, 0.0], [650.0, -420.0]], np.float32)
    wr = World(n + 400, cells_per_dist=3.0,  # a fixed cell size: the grid stays the same all along
               test_flags=GWAOI_F_TEST_FORCE_RADIX)
    wi = World(n + 400, cells_per_dist=3.0)
    ref = oracle_mod.SpacesOracle({0: D}, n + 400)
    try:
        slots = np.arange(n, dtype=np.uint32)
        for w in (wr, wi):
            sp = w.space_create(D)
            w.enter_batch(sp, slots, x, z)
            w.tick()
        for i in range(n):
            ref.enter(0, i, x[i], z[i])
        ref.take_events(with_space=True)
        live, spare = set(range(4, n)), list(range(n, n + 400))
        for t in range(6):
            mv = rng.choice(sorted(live), 500, replace=False).astype(np.uint32)
            h = hot[rng.integers(0, 3, mv.size)] if t < 4 else rng.uniform(-L / 2, L / 2, (mv.size, 2)).astype(np.float32)
            nx = (h[:, 0] + rng.uniform(-6, 6, mv.size)).astype(np.float32)  # into one or two cells
            nz = (h[:, 1] + rng.uniform(-6, 6, mv.size)).astype(np.float32)
            leavers = rng.choice(sorted(set(live) - set(int(v) for v in mv)), 30, replace=False)
            enter = np.array([spare.pop() for _ in range(40)], np.uint32)
            eh = hot[rng.integers(0, 3, enter.size)]
            ex = (eh[:, 0] + rng.uniform(-6, 6, enter.size)).astype(np.float32)
            ez = (eh[:, 1] + rng.uniform(-6, 6, enter.size)).astype(np.float32)
            outs = []
            for w in (wr, wi):
                w.moved_batch(mv, nx, nz)
                w.leave_batch(leavers)
                w.enter_batch(0, enter, ex, ez)
                outs.append(w.tick())
            for i, a, b in zip(mv, nx, nz):
                ref.moved(int(i), a, b)
            for i in leavers:
                ref.leave(int(i))
            for i, a, b in zip(enter, ex, ez):
                ref.enter(0, int(i), a, b)
            oe, ol = oracle_mod.net_events(*ref.take_events(with_space=True))
            live = (live - set(int(v) for v in leavers)) | set(int(v) for v in enter)
            spare.extend(int(v) for v in leavers)
            (er, lr), (ei, li) = outs
            np.testing.assert_array_equal(er, ei)
            np.testing.assert_array_equal(lr, li)
            np.testing.assert_array_equal(pair_keys(ei), oe)
            np.testing.assert_array_equal(pair_keys(li), ol)
        assert wi.debug_counters()["incremental_sorts"] == 6
        assert wr.debug_counters()["incremental_sorts"] == 0
    finally:
        wr.close()
        wi.close()


def test_virtual_sprime_equals_copied_sprime_gpu():
    """A flush of Moved batches only skips the prologue's copy of the previous
    frame (k_keygen takes the records no op wrote from the previous frame, by
    their seq).  Its event arrays -- order included -- and neighbour rows equal
    those of the copying path (GWAOI_FORCE_COPY=1) over: partial batches (most
    entities unmoved), repeated slots across two batches (fixup), an empty
    flush, a batch with a stale explicit seq (op dropped, flush reports it),
    and host Enter/Leave flushes (which copy) between moves-only ones."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(77)
    wl = make_workload("cfg3", n=30000)
    slots, x0, z0, _ = wl.initial()
    n = wl.n
    wc = World(n + 200, test_flags=GWAOI_F_TEST_FORCE_COPY)
    wv = World(n + 200)

    def both(fn):
        outs = []
        for w in (wc, wv):
            fn(w)
            try:
                outs.append((w.tick(), None))
            except GwaoiError as e:
                outs.append((e.events, e.code))
        ((ec, lc), cc), ((ev, lv), cv) = outs
        assert cc == cv
        np.testing.assert_array_equal(ec, ev)
        np.testing.assert_array_equal(lc, lv)
        return ec.shape[0] + lc.shape[0]

    def dev(*arrs):
        t = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]
        torch.cuda.synchronize()
        keep.append(t)
        return t

    keep = []
    try:
        for w in (wc, wv):
            s = w.space_create(wl.D)
            w.enter_batch(s, slots, x0, z0)
            w.tick()
        x = np.concatenate([x0, np.zeros(200, np.float32)])
        z = np.concatenate([z0, np.zeros(200, np.float32)])
        live = np.ones(n + 200, bool)
        live[n:] = False
        total = 0
        for t in range(8):
            kind = t % 4
            if kind == 0:  # a third of the live entities move, in a device batch
                sl = rng.choice(np.nonzero(live)[0], int(live.sum()) // 3, replace=False).astype(np.uint32)
                nx = (x[sl] + rng.uniform(-1, 1, sl.size)).astype(np.float32)
                nz = (z[sl] + rng.uniform(-1, 1, sl.size)).astype(np.float32)
                d = dev(sl.astype(np.int32), nx, nz)
                total += both(lambda w: w.moved_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                                             sl.size))
                x[sl], z[sl] = nx, nz
            elif kind == 1:  # two batches with repeated slots (collision fixup), then an empty flush
                pool = np.nonzero(live)[0]
                runs = []
                for r in range(2):
                    sl = rng.choice(pool[:400] if r else pool, 3000).astype(np.uint32)
                    nx = (x[sl] + rng.uniform(-40, 40, sl.size)).astype(np.float32)
                    nz = (z[sl] + rng.uniform(-40, 40, sl.size)).astype(np.float32)
                    runs.append((sl, dev(sl.astype(np.int32), nx, nz)))
                    x[sl], z[sl] = nx, nz

                def issue(w):
                    for sl, d in runs:
                        w.moved_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), sl.size)
                total += both(issue)
                assert both(lambda w: None) == 0
            elif kind == 2:  # explicit seqs, one of them stale: that op is dropped, the flush reports it
                floors = {wc.info()["next_seq"], wv.info()["next_seq"]}
                assert len(floors) == 1
                floor = floors.pop()
                sl = rng.choice(np.nonzero(live)[0], 2000, replace=False).astype(np.uint32)
                nx = (x[sl] + rng.uniform(-2, 2, sl.size)).astype(np.float32)
                nz = (z[sl] + rng.uniform(-2, 2, sl.size)).astype(np.float32)
                sq = (floor + np.arange(sl.size)).astype(np.int64)
                sq[7] = floor - 1
                d = dev(sl.astype(np.int32), nx, nz, sq)
                total += both(lambda w: w.moved_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                                             sl.size, d_seq=d[3].data_ptr()))
                keep_op = np.ones(sl.size, bool)
                keep_op[7] = False
                x[sl[keep_op]], z[sl[keep_op]] = nx[keep_op], nz[keep_op]
            else:  # host Leaves and Enters (the copying path) plus plain moves
                out = rng.choice(np.nonzero(live)[0], 100, replace=False)
                inn = rng.choice(np.nonzero(~live)[0], 100, replace=False)
                ex = rng.uniform(-wl.L / 4, wl.L / 4, 100).astype(np.float32)
                ez = rng.uniform(-wl.L / 4, wl.L / 4, 100).astype(np.float32)

                def churn(w):
                    w.leave_batch(out)
                    w.enter_batch(0, inn.astype(np.uint32), ex, ez)
                total += both(churn)
                live[out] = False
                live[inn] = True
                x[inn], z[inn] = ex, ez
        assert total > 0
        for i in rng.choice(np.nonzero(live)[0], 50, replace=False):
            np.testing.assert_array_equal(wc.neighbors(int(i)), wv.neighbors(int(i)))
    finally:
        wc.close()
        wv.close()


def test_committed_events_delivered_on_device_error_gpu():
    """A flush whose device batch held a bad op (here an explicit seq below the
    flush's floor) commits without that op and reports the problem; its other
    events must still reach the caller (GwaoiError.events), or the callers'
    InterestedIn/By would drift from the engine for good."""
    torch = pytest.importorskip("torch")
    with World(16) as w:
        s = w.space_create(D)
        for i in range(10):
            w.enter(s, i, 0.0, 0.0)
        assert flush(w)[0].size == 90
        floor = w.info()["next_seq"]
        ds = torch.tensor([0, 1], dtype=torch.int32, device="cuda")
        dx = torch.tensor([5000.0, 7000.0], device="cuda")
        dz = torch.tensor([0.0, 0.0], device="cuda")
        dq = torch.tensor([floor + 5, floor - 3], dtype=torch.int64, device="cuda")  # op 1 is stale: dropped
        torch.cuda.synchronize()
        w.moved_batch_device(ds.data_ptr(), dx.data_ptr(), dz.data_ptr(), 2, d_seq=dq.data_ptr())
        with pytest.raises(GwaoiError) as ei:
            w.tick()
        assert ei.value.code == -1 and ei.value.events is not None
        ent, lev = ei.value.events
        assert ent.shape[0] == 0
        assert sorted(map(tuple, lev.tolist())) == sorted([(0, i) for i in range(1, 10)] + [(i, 0) for i in range(1, 10)])
        assert w.neighbors(0).size == 0 and w.neighbors(1).tolist() == [2, 3, 4, 5, 6, 7, 8, 9]
        w.moved(1, 5000.0, 0.0)  # the world goes on
        ent, lev = flush(w)
        assert ent.size == 2 and lev.size == 16


def test_failed_event_regrow_poisons_world_gpu():
    """A failure after the flush's kernels rewrote the per-slot records but
    before the commit (here an injected failure of the event-buffer regrow)
    leaves host and device apart: the world refuses every later call."""
    w = World(64, event_capacity=16, test_flags=GWAOI_F_TEST_REGROW_FAIL)
    try:
        s = w.space_create(D)
        for i in range(20):
            w.enter(s, i, 0.0, 0.0)  # 380 directed enters > 16
        with pytest.raises(GwaoiError) as ei:
            w.tick()
        assert ei.value.code == -4
        for call in (lambda: w.enter(s, 30, 1.0, 1.0), lambda: w.moved(0, 1.0, 1.0), w.tick,
                     lambda: w.neighbors(0)):
            with pytest.raises(GwaoiError) as ej:
                call()
            assert ej.value.code == -5 and "failed flush" in str(ej.value)
    finally:
        w.close()


def test_async_tick_overlaps_next_calls_gpu():
    """gwaoi_tick_begin / _end: the calls made while a flush is in flight (a staged
    host batch with repeats, Enters, Leaves, single Moves, a device batch) are
    validated at once and queued for the NEXT flush.  Every flush's events equal
    those of a world driven with blocking ticks and the same call order."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(23)
    n = 30000
    wl = make_workload("cfg2", n=n)
    slots, x0, z0, _ = wl.initial()
    k0 = n - 3000
    live = np.zeros(n, bool)
    live[:k0] = True
    x, z = x0.copy(), z0.copy()
    keep = []

    def calls(t):
        """This tick's calls as closures over a world."""
        out = []
        live_prev = live.copy()  # device batches may only move slots live at the previous flush
        pool = np.nonzero(live)[0]
        sl = rng.choice(pool, 20000).astype(np.uint32)  # repeats included
        nx = (x[sl] + rng.uniform(-3, 3, sl.size)).astype(np.float32)
        nz = (z[sl] + rng.uniform(-3, 3, sl.size)).astype(np.float32)
        out.append(lambda w, a=sl, b=nx, c=nz: w.moved_batch(a, b, c))
        x[sl], z[sl] = nx, nz
        for i in rng.choice(np.nonzero(~live)[0], 200, replace=False):
            xi, zi = np.float32(x[i]), np.float32(z[i])
            out.append(lambda w, i=int(i), xi=xi, zi=zi: w.enter(0, i, xi, zi))
            live[i] = True
        for i in rng.choice(np.nonzero(live)[0], 150, replace=False):
            out.append(lambda w, i=int(i): w.leave(i))
            live[i] = False
        j = int(np.nonzero(live)[0][t])
        xj = np.float32(x[j] + 60)
        out.append(lambda w, j=j, xj=xj: w.moved(j, xj, z[j]))
        x[j] = xj
        ds = rng.choice(np.nonzero(live & live_prev)[0], 5000, replace=False).astype(np.uint32)
        dx = (x[ds] + rng.uniform(-2, 2, ds.size)).astype(np.float32)
        dz = (z[ds] + rng.uniform(-2, 2, ds.size)).astype(np.float32)
        x[ds], z[ds] = dx, dz
        tens = [torch.from_numpy(v).cuda() for v in (ds.astype(np.int32), dx, dz)]
        torch.cuda.synchronize()
        keep.append(tens)
        out.append(lambda w, tt=tens: w.moved_batch_device(tt[0].data_ptr(), tt[1].data_ptr(), tt[2].data_ptr(),
                                                           tt[0].numel()))
        return out

    with World(n) as wa, World(n) as wb:
        for w in (wa, wb):
            w.space_create(wl.D)
            w.enter_batch(0, slots[:k0], x0[:k0], z0[:k0])
        wa.tick()
        wb.tick()
        ticks = [calls(t) for t in range(5)]
        for c in ticks[0]:
            c(wa)
        wa.tick_begin()
        with pytest.raises(GwaoiError):
            wa.tick_begin()  # one flush at a time
        with pytest.raises(GwaoiError):
            wa.neighbors(0)  # not while a flush is in flight
        for t in range(5):
            for c in ticks[t]:
                c(wb)
            eb, lb = wb.tick()
            if t + 1 < 5:
                for c in ticks[t + 1]:
                    c(wa)  # queued while flush t is in flight
            ea, la = wa.tick_end()
            np.testing.assert_array_equal(pair_keys(ea), pair_keys(eb), err_msg=f"flush {t}: enters")
            np.testing.assert_array_equal(pair_keys(la), pair_keys(lb), err_msg=f"flush {t}: leaves")
            assert ea.shape[0] > 0 and la.shape[0] > 0
            if t + 1 < 5:
                wa.tick_begin()
        with pytest.raises(GwaoiError):
            wa.tick_end()  # nothing in flight
        for i in np.nonzero(live)[0][::2003]:
            np.testing.assert_array_equal(wa.neighbors(int(i)), wb.neighbors(int(i)))


def test_events_csr_regroups_events_gpu():
    """gwaoi_events_csr: the flush's directed events regrouped by their first entity,
    each row sorted with its leaves first; the same multiset as the event pairs,
    including a pair that leaves one space and enters another in the same flush."""
    rng = np.random.default_rng(41)
    n = 20000
    wl = make_workload("cfg2", n=n)
    slots, x0, z0, _ = wl.initial()
    with World(n, max_spaces=2) as w:
        s0 = w.space_create(wl.D)
        s1 = w.space_create(wl.D)
        w.enter_batch(s0, slots, x0, z0)
        w.tick()
        for t in range(3):
            sl, nx, nz = wl.tick(t)
            w.moved_batch(sl, nx, nz)
            for i in rng.choice(n, 300, replace=False):  # space changes of neighbours at the same spot
                w.leave(int(i))
                w.enter(s1 if t % 2 == 0 else s0, int(i), wl.x[i], wl.z[i])
            ent, lev = w.tick()
            off, items = w.events_csr()
            assert off.size == n + 1 and off[-1] == items.size == ent.shape[0] + lev.shape[0]
            rows = np.repeat(np.arange(n, dtype=np.uint64), np.diff(off).astype(np.int64))
            b = (items & np.uint32(0x7FFFFFFF)).astype(np.uint64)
            is_enter = (items & np.uint32(0x80000000)) != 0
            keys = (rows << np.uint64(32)) | b
            np.testing.assert_array_equal(np.sort(keys[is_enter]), pair_keys(ent))
            np.testing.assert_array_equal(np.sort(keys[~is_enter]), pair_keys(lev))
            for r in range(0, n, 97):  # each row sorted: leaves (bit 31 clear) first, each part by b
                row = items[off[r]:off[r + 1]]
                assert np.all(row[:-1] <= row[1:])


def test_events_csr_long_rows_gpu():
    """Rows past one lane's insertion sort: a populate flush with a co-located crowd of
    5000 (rows of 4999 items: LDS-sorted runs + block merge) and a 60-entity crowd
    beside a 1500-entity one (rows of 59 .. 1559: one LDS run), then a flush where
    the big crowd leaves -- every row sorted and the CSR equal to the event pairs."""
    rng = np.random.default_rng(43)
    n = 5000 + 1500 + 60 + 3000
    x = np.zeros(n, np.float32)
    z = np.zeros(n, np.float32)
    x[5000:6500] = rng.uniform(1000, 1100, 1500)
    z[5000:6500] = rng.uniform(1000, 1100, 1500)
    x[6500:6560] = rng.uniform(1050, 1150, 60)
    z[6500:6560] = rng.uniform(1000, 1100, 60)
    x[6560:] = rng.uniform(-50000, 50000, n - 6560)  # sparse background: short rows
    z[6560:] = rng.uniform(-50000, 50000, n - 6560)
    order = rng.permutation(n).astype(np.uint32)
    with World(n) as w:
        s = w.space_create(100.0)
        w.enter_batch(s, order, x[order], z[order])
        for flush in range(2):
            ent, lev = w.tick()
            off, items = w.events_csr()
            assert off[-1] == items.size == ent.shape[0] + lev.shape[0]
            lens = np.diff(off)
            if flush == 0:
                assert lens.max() == 4999 and np.sum((lens > 32) & (lens < 4096)) > 1000
            rows = np.repeat(np.arange(n, dtype=np.uint64), lens.astype(np.int64))
            b = (items & np.uint32(0x7FFFFFFF)).astype(np.uint64)
            is_enter = (items & np.uint32(0x80000000)) != 0
            keys = (rows << np.uint64(32)) | b
            np.testing.assert_array_equal(np.sort(keys[is_enter]), pair_keys(ent))
            np.testing.assert_array_equal(np.sort(keys[~is_enter]), pair_keys(lev))
            starts = off[:-1][lens > 1]
            for r in np.nonzero(lens > 1)[0]:
                row = items[off[r]:off[r + 1]]
                assert np.all(row[:-1] <= row[1:]), f"flush {flush} row {r} ({row.size} items) not sorted"
            assert starts.size > 0
            if flush == 0:
                w.leave_batch(np.arange(5000, dtype=np.uint32))  # next flush: 5000 rows of 4999 leaves


def _device_events(w, ne, nl):
    """Copy the last committed flush's device events (gwaoi_events_device) to the host."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    e, l = w.events_device()
    out = []
    for ptr, n in ((e, ne), (l, nl)):
        a = np.empty((n, 2), np.uint32)
        if n:
            assert hip.hipMemcpy(a.ctypes.data, ptr, a.nbytes, 2) == 0  # hipMemcpyDeviceToHost
        out.append(a)
    return out


@pytest.mark.parametrize("event_capacity,repeats", [(0, False), (3000, False), (0, True)])
def test_speculative_next_flush_matches_serial_gpu(event_capacity, repeats):
    """gwaoi_tick_finish(NEXT): the next flush queued before the commit of the one in
    flight (device Moved batches only) gives every flush the events of the serial path -- also when the
    flush in flight overflows its event buffer and is re-run after its successor
    (event_capacity=3000), when a batch moves slots more than once (repeats: the last
    call wins), and when a host call in flight forces the fallback."""
    torch = pytest.importorskip("torch")
    n = 20000
    wa, wb = make_workload("cfg2", n=n), make_workload("cfg2", n=n)
    slots, x0, z0, _ = wa.initial()
    ticks = 24
    batches, host = [], []
    rng = np.random.default_rng(99)
    for t in range(ticks):
        sl, nx, nz = wa.tick(t)
        if repeats:  # 2,000 extra moves of 300 slots, after and before their regular move
            extra = rng.integers(0, 300, 2000).astype(sl.dtype)
            ex = (x0[extra] + rng.uniform(-20, 20, extra.size)).astype(np.float32)
            ez = (z0[extra] + rng.uniform(-20, 20, extra.size)).astype(np.float32)
            cut = sl.size // 2
            sl = np.concatenate([sl[:cut], extra, sl[cut:]])
            nx = np.concatenate([nx[:cut], ex, nx[cut:]])
            nz = np.concatenate([nz[:cut], ez, nz[cut:]])
        host.append((sl, nx, nz))
        batches.append([torch.from_numpy(a).to("cuda:0") for a in (sl.astype(np.int32), nx, nz)])
    torch.cuda.synchronize()
    cap = 2 * n if repeats else n  # a speculative launch takes at most max_slots ops
    with World(cap, event_capacity=event_capacity) as A, World(cap) as B:
        for w in (A, B):
            s = w.space_create(wa.D)
            w.enter_batch(s, slots, x0, z0)
            w.tick()
        A.moved_batch_device(*(b.data_ptr() for b in batches[0]), host[0][0].size)
        A.tick_begin()
        caps = []
        for t in range(ticks):
            if t + 1 < ticks:
                A.moved_batch_device(*(b.data_ptr() for b in batches[t + 1]), host[t + 1][0].size)
                if t == 4:  # a host call queued in flight: this tick takes the fallback path
                    A.moved(7, 123.0, 456.0)
                ne, nl = A.tick_end_begin_device()
            else:
                ne, nl = A.tick_end_device()
            ga, la = _device_events(A, ne, nl)
            caps.append(A.info()["event_capacity"])
            sl, nx, nz = host[t]
            B.moved_batch(sl, nx, nz)
            if t == 5:
                B.moved(7, 123.0, 456.0)
            gb, lb = B.tick()
            np.testing.assert_array_equal(pair_keys(ga), pair_keys(gb), err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(pair_keys(la), pair_keys(lb), err_msg=f"tick {t}: leaves")
        d = A.debug_counters()
        assert d["speculative_launches"] >= ticks - 3
        assert d["premarked_runs"] == 0  # GWAOI_F_BATCH_READY is gone (ABI 5)
        # the two event sets match each other's capacity without outgrowing it (was: x1.25 per flush)
        assert caps[-1] == caps[ticks // 2], caps
        if event_capacity:
            assert d["event_regrows"] > 0
        for i in range(0, n, 997):
            np.testing.assert_array_equal(A.neighbors(i), B.neighbors(i))


def test_speculative_regrows_with_growing_crowd_gpu():
    """Event counts that rise flush after flush (the space contracts every tick) with a
    small event capacity: the speculative pipeline overflows and regrows its event sets
    several times back to back, while the twin set and the shared scratch drift apart.
    Every flush must still deliver the serial path's events: a flush compares its total
    with the capacity its pair passes were launched with, not with a buffer another
    flush grew since (finish_flight)."""
    torch = pytest.importorskip("torch")
    n, ticks = 20000, 14
    rng = np.random.default_rng(7)
    L = float(np.sqrt(n * 1250.0))
    x = rng.uniform(-L / 2, L / 2, n).astype(np.float32)
    z = rng.uniform(-L / 2, L / 2, n).astype(np.float32)
    slots = np.arange(n, dtype=np.uint32)
    host, dev = [], []
    px, pz = x, z
    for t in range(ticks):
        order = rng.permutation(n).astype(np.uint32)
        px = (px * np.float32(0.8) + rng.uniform(-1, 1, n).astype(np.float32)).astype(np.float32)
        pz = (pz * np.float32(0.8) + rng.uniform(-1, 1, n).astype(np.float32)).astype(np.float32)
        host.append((order, px[order], pz[order]))
        dev.append([torch.from_numpy(a).to("cuda:0") for a in (order.astype(np.int32), px[order], pz[order])])
    torch.cuda.synchronize()
    with World(n, event_capacity=2000) as A, World(n) as B:
        for w in (A, B):
            s = w.space_create(D)
            w.enter_batch(s, slots, x, z)
            w.tick()
        A.moved_batch_device(*(b.data_ptr() for b in dev[0]), n)
        A.tick_begin()
        totals = []
        for t in range(ticks):
            if t + 1 < ticks:
                A.moved_batch_device(*(b.data_ptr() for b in dev[t + 1]), n)
                ne, nl = A.tick_end_begin_device()
            else:
                ne, nl = A.tick_end_device()
            ga, la = _device_events(A, ne, nl)
            B.moved_batch(*host[t])
            gb, lb = B.tick()
            totals.append(ne + nl)
            np.testing.assert_array_equal(pair_keys(ga), pair_keys(gb), err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(pair_keys(la), pair_keys(lb), err_msg=f"tick {t}: leaves")
        d = A.debug_counters()
        assert d["event_regrows"] >= 2, (d, totals)
        assert d["speculative_launches"] >= ticks - 2
        assert totals[-1] > 4 * totals[1], totals
        for i in range(0, n, 1999):
            np.testing.assert_array_equal(A.neighbors(i), B.neighbors(i))


def test_cell_size_switch_keeps_parity_gpu(oracle_mod):
    """Automatic cell size (gwaoi_config.cells_per_dist = 0): a sparse uniform space
    switches the grids to D/2, a contracted one back to D/3 (two flushes recommending
    the other size rebuild every grid; that flush takes the radix sort, the others the
    incremental merge).  Events equal a world with a fixed D/4 grid and the closed form
    at every flush, across both switches."""
    n = 20000
    rng = np.random.default_rng(5)
    L = float(np.sqrt(n * 1250.0))
    x = rng.uniform(-L / 2, L / 2, n).astype(np.float32)
    z = rng.uniform(-L / 2, L / 2, n).astype(np.float32)
    slots = np.arange(n, dtype=np.uint32)
    seq = np.zeros(n, np.uint64)
    sp = np.zeros(n, np.uint32)
    with World(n) as A, World(n, cells_per_dist=4.0) as B:
        for w in (A, B):
            s = w.space_create(D)
            w.enter_batch(s, slots, x, z)
        seq[:] = 1 + np.arange(n, dtype=np.uint64)
        nxt = n + 1
        ea, _ = flush(A)
        eb, _ = flush(B)
        np.testing.assert_array_equal(ea, eb)
        prev = oracle_mod.closed_form_pairs(x, z, seq, sp, {0: D})
        np.testing.assert_array_equal(ea, prev)
        cpd = [A.debug_counters()["cells_per_dist"]]
        for t in range(12):
            order = rng.permutation(n).astype(np.uint32)
            shrink = np.float32(0.88) if 4 <= t < 8 else np.float32(1.0)  # ticks 4-7: the crowd thickens
            x = (x * shrink + rng.uniform(-1, 1, n).astype(np.float32)).astype(np.float32)
            z = (z * shrink + rng.uniform(-1, 1, n).astype(np.float32)).astype(np.float32)
            for w in (A, B):
                w.moved_batch(order, x[order], z[order])
            seq[order] = nxt + np.arange(n, dtype=np.uint64)
            nxt += n
            ea, la = flush(A)
            eb, lb = flush(B)
            cur = oracle_mod.closed_form_pairs(x, z, seq, sp, {0: D})
            np.testing.assert_array_equal(ea, eb, err_msg=f"tick {t}: enters vs fixed grid")
            np.testing.assert_array_equal(la, lb, err_msg=f"tick {t}: leaves vs fixed grid")
            np.testing.assert_array_equal(ea, np.setdiff1d(cur, prev), err_msg=f"tick {t}: enters vs closed form")
            np.testing.assert_array_equal(la, np.setdiff1d(prev, cur), err_msg=f"tick {t}: leaves vs closed form")
            prev = cur
            cpd.append(A.debug_counters()["cells_per_dist"])
        # sparse start (about 32 neighbours each): D/2; crowded end (about 90): back to D/3
        assert cpd[0] == 3 and 2 in cpd[1:5] and cpd[-1] == 3, cpd
        assert A.debug_counters()["cell_size_switches"] == 2, cpd
        assert B.debug_counters()["cell_size_switches"] == 0


def test_device_enter_leave_batches_match_host_calls_gpu(oracle_mod):
    """gwaoi_enter_batch_device / gwaoi_leave_batch_device (the strip worlds' boundary
    crossers, Space.go:211,243) give the events of the same Enter/Leave calls made on the
    host, with implicit and explicit seqs, mixed with a device Moved batch in one flush;
    the host mirror is rebuilt from the frame for the next host call (neighbors, Leave)."""
    torch = pytest.importorskip("torch")
    n = 30000
    wl = make_workload("cfg2", n=n)
    slots, x0, z0, _ = wl.initial()
    half = n // 2
    dev = "cuda:0"
    with World(n) as A, World(n) as B:
        for w in (A, B):
            s = w.space_create(wl.D)
            w.enter_batch(s, slots[:half], x0[:half], z0[:half])
            w.tick()
        # flush 1: device Enters of the second half (implicit seqs) + device moves of the first
        sl, nx, nz = wl.tick(0)
        keep = sl < half
        msl, mx, mz = sl[keep], nx[keep], nz[keep]
        d = [torch.from_numpy(a).to(dev) for a in (slots[half:].astype(np.int32), x0[half:], z0[half:],
                                                   msl.astype(np.int32), mx, mz)]
        torch.cuda.synchronize()
        box = (float(x0[half:].min()), float(z0[half:].min()), float(x0[half:].max()), float(z0[half:].max()))
        A.enter_batch_device(0, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n - half, box=box)
        with pytest.raises(GwaoiError):  # the host mirror is stale until the flush
            A.moved(0, 1.0, 1.0)
        A.moved_batch_device(d[3].data_ptr(), d[4].data_ptr(), d[5].data_ptr(), msl.size)
        B.enter_batch(0, slots[half:], x0[half:], z0[half:])
        B.moved_batch(msl, mx, mz)
        ea, la = flush(A)
        eb, lb = flush(B)
        np.testing.assert_array_equal(ea, eb)
        np.testing.assert_array_equal(la, lb)
        assert A.info()["live"] == n
        # flush 2: device Leaves of 5000 slots + explicit-seq device moves of the rest
        gone = np.arange(0, n, 6, dtype=np.uint32)[:5000]
        rest = np.setdiff1d(slots, gone)
        rx = (wl.x[rest] + np.float32(0.5)).astype(np.float32)
        rz = (wl.z[rest] - np.float32(0.5)).astype(np.float32)
        base = A.info()["next_seq"]
        sq = base + np.arange(rest.size, dtype=np.uint64)
        d2 = [torch.from_numpy(a).to(dev) for a in (gone.astype(np.int32), rest.astype(np.int32), rx, rz,
                                                    sq.view(np.int64))]
        torch.cuda.synchronize()
        A.leave_batch_device(0, d2[0].data_ptr(), gone.size)
        A.moved_batch_device(d2[1].data_ptr(), d2[2].data_ptr(), d2[3].data_ptr(), rest.size, d_seq=d2[4].data_ptr())
        B.leave_batch(gone)
        B.moved_batch(rest, rx, rz)
        ea, la = flush(A)
        eb, lb = flush(B)
        np.testing.assert_array_equal(ea, eb)
        np.testing.assert_array_equal(la, lb)
        assert A.info()["live"] == n - gone.size
        # host calls again: the mirror is rebuilt from the frame
        for i in (1, 2, 7, 12345, int(rest[-1])):
            np.testing.assert_array_equal(A.neighbors(i), B.neighbors(i))
        with pytest.raises(GwaoiError):
            A.neighbors(int(gone[3]))  # left: not in the frame
        for w in (A, B):
            w.leave(int(rest[0]))
            w.enter(0, int(gone[0]), 10.0, 20.0)
        ea, la = flush(A)
        eb, lb = flush(B)
        np.testing.assert_array_equal(ea, eb)
        np.testing.assert_array_equal(la, lb)


def test_device_enter_of_live_slot_poisons_gpu():
    """A device Enter batch naming a live slot breaks the frame's live count: the flush
    fails and the world refuses further calls (the rules of gwaoi_enter_batch_device)."""
    torch = pytest.importorskip("torch")
    with World(64) as w:
        w.space_create(D)
        for i in range(4):
            w.enter(0, i, float(i), 0.0)
        w.tick()
        d = [torch.tensor([2, 9], dtype=torch.int32, device="cuda:0"),
             torch.tensor([5.0, 6.0], dtype=torch.float32, device="cuda:0"),
             torch.tensor([0.0, 0.0], dtype=torch.float32, device="cuda:0")]
        torch.cuda.synchronize()
        w.enter_batch_device(0, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), 2)
        with pytest.raises(GwaoiError) as ei:
            w.tick()
        assert "live" in str(ei.value)
        with pytest.raises(GwaoiError):
            w.moved(1, 0.0, 0.0)


def test_zero_copy_batches_match_host_batches_gpu(oracle_mod):
    """gwaoi_moved_batch_stage / _commit (moves written straight into pinned staging, checked
    on the device) == gwaoi_moved_batch, serial and pipelined with gwaoi_tick_finish(NEXT|HOST) (the
    event copy beside the next flush) and with gwaoi_tick_finish(NEXT|HOST) + gwaoi_events_host;
    a partial commit, a batch after an Enter in the same flush (host-checked, space column),
    and a dead slot dropped and reported by the flush."""
    wl = make_workload("cfg3", n=40000)
    slots, x0, z0, _ = wl.initial()
    with World(wl.n) as A, World(wl.n) as B:
        for w in (A, B):
            s = w.space_create(wl.D)
            w.enter_batch(s, slots[:-10], x0[:-10], z0[:-10])
            w.tick()
        # serial: stage 1.5x, fill and commit the tick's moves
        for t in range(3):
            sl, nx, nz = wl.tick(t)
            keep = sl < wl.n - 10
            sl, nx, nz = sl[keep], nx[keep], nz[keep]
            vs, vx, vz = A.stage_moves(sl.size + sl.size // 2)
            vs[:sl.size], vx[:sl.size], vz[:sl.size] = sl, nx, nz
            A.commit_moves(sl.size)
            B.moved_batch(sl, nx, nz)
            ea, la = A.tick()
            eb, lb = B.tick()
            np.testing.assert_array_equal(pair_keys(ea), pair_keys(eb))
            np.testing.assert_array_equal(pair_keys(la), pair_keys(lb))
        # the caller's own pinned buffer (gwaoi_pinned_alloc + gwaoi_moved_batch_pinned)
        sl, nx, nz = wl.tick(30)
        keep = sl < wl.n - 10
        sl, nx, nz = sl[keep], nx[keep], nz[keep]
        ptr, views = A.pinned_batch(sl.size)
        views[0][:], views[1][:], views[2][:] = sl, nx, nz
        A.moved_batch_pinned(views, sl.size)
        B.moved_batch(sl, nx, nz)
        ea, la = A.tick()
        eb, lb = B.tick()
        A.free_pinned_batch(ptr)
        np.testing.assert_array_equal(pair_keys(ea), pair_keys(eb))
        np.testing.assert_array_equal(pair_keys(la), pair_keys(lb))
        # an Enter queued first: the staged batch then carries the space column (host-checked)
        new = slots[-10:]
        for w in (A, B):
            w.enter_batch(0, new, x0[-10:], z0[-10:])
        sl, nx, nz = wl.tick(3)
        vs, vx, vz = A.stage_moves(sl.size)
        vs[:], vx[:], vz[:] = sl, nx, nz
        A.commit_moves(sl.size)
        B.moved_batch(sl, nx, nz)
        ea, la = A.tick()
        eb, lb = B.tick()
        np.testing.assert_array_equal(pair_keys(ea), pair_keys(eb))
        np.testing.assert_array_equal(pair_keys(la), pair_keys(lb))
        # a host batch between _stage and _commit stays out of the reservation (queued as host ops
        # ahead of the committed batch: commit order is call order)
        sl, nx, nz = wl.tick(20)
        s2, x2, z2 = wl.tick(21)
        vs, vx, vz = A.stage_moves(sl.size)
        vs[:], vx[:], vz[:] = sl, nx, nz
        A.moved_batch(s2, x2, z2)
        np.testing.assert_array_equal(vs, sl)  # the reserved words were not overwritten
        A.commit_moves(sl.size)
        B.moved_batch(s2, x2, z2)
        B.moved_batch(sl, nx, nz)
        ea, la = A.tick()
        eb, lb = B.tick()
        np.testing.assert_array_equal(pair_keys(ea), pair_keys(eb))
        np.testing.assert_array_equal(pair_keys(la), pair_keys(lb))
        # pipelined: batch t+1 staged while flush t runs, tick_end_begin returns t's events
        host = [wl.tick(4 + t) for t in range(5)]
        vs, vx, vz = A.stage_moves(host[0][0].size)
        vs[:], vx[:], vz[:] = host[0]
        A.commit_moves(host[0][0].size)
        A.tick_begin()
        for t in range(5):
            if t + 1 < 5:
                sl, nx, nz = host[t + 1]
                vs, vx, vz = A.stage_moves(sl.size)
                vs[:], vx[:], vz[:] = sl, nx, nz
                A.commit_moves(sl.size)
                ea, la = A.tick_end_begin()
            else:
                ea, la = A.tick_end()
            B.moved_batch(*host[t])
            eb, lb = B.tick()
            np.testing.assert_array_equal(pair_keys(ea), pair_keys(eb), err_msg=f"pipelined tick {t}")
            np.testing.assert_array_equal(pair_keys(la), pair_keys(lb), err_msg=f"pipelined tick {t}")
        assert A.debug_counters()["speculative_launches"] >= 3
        # pipelined with the copy-out left running (gwaoi_tick_finish(NEXT|HOST)): batch t+1 queued from
        # the caller's pinned buffer, tick t-1's events taken (gwaoi_events_host), then t finished
        host = [wl.tick(9 + t) for t in range(5)]
        ptrs, got = [], []

        def put(b):
            ptr, views = A.pinned_batch(b[0].size)
            views[0][:], views[1][:], views[2][:] = b
            ptrs.append(ptr)
            A.moved_batch_pinned(views, b[0].size)

        put(host[0])
        A.tick_begin()
        for t in range(5):
            if t + 1 < 5:
                put(host[t + 1])
                if t:
                    got.append(A.events_host())
                counts = A.tick_end_begin_async()
            else:
                got.append(A.events_host())
                got.append(A.tick_end())
        assert counts == (len(got[3][0]), len(got[3][1]))
        for t in range(5):
            B.moved_batch(*host[t])
            eb, lb = B.tick()
            np.testing.assert_array_equal(pair_keys(got[t][0]), pair_keys(eb), err_msg=f"async tick {t}")
            np.testing.assert_array_equal(pair_keys(got[t][1]), pair_keys(lb), err_msg=f"async tick {t}")
        for p in ptrs:
            A.free_pinned_batch(p)
        # the same with one event per mirrored pair copied out (gwaoi_tick_finish(NEXT|PAIRS)):
        # the pairs and their mirrors are the directed events
        host = [wl.tick(14 + t) for t in range(4)]
        ptrs, got = [], []
        put(host[0])
        A.tick_begin()
        for t in range(4):
            if t + 1 < 4:
                put(host[t + 1])
                if t:
                    got.append(A.pairs_host())
                ne, nl = A.tick_end_begin_pairs_async()
            else:
                got.append(A.pairs_host())
                got.append(A.tick_end())
        with pytest.raises(GwaoiError):
            A.pairs_host()  # the last copy-out (tick_end) holds directed events
        for t in range(4):
            B.moved_batch(*host[t])
            eb, lb = B.tick()
            ea, la = got[t]
            if t < 3:  # pairs: mirror them
                assert ea.shape[0] * 2 == len(eb) and la.shape[0] * 2 == len(lb)
                ea, la = np.concatenate([ea, ea[:, ::-1]]), np.concatenate([la, la[:, ::-1]])
            np.testing.assert_array_equal(pair_keys(ea), pair_keys(eb), err_msg=f"pairs tick {t}")
            np.testing.assert_array_equal(pair_keys(la), pair_keys(lb), err_msg=f"pairs tick {t}")
        for p in ptrs:
            A.free_pinned_batch(p)
        # a commit without a copy-out (gwaoi_tick_device) leaves the host copy and its counts
        # alone: gwaoi_events_host still describes the buffer it points at
        prev = A.events_host()
        A.moved_batch(*wl.tick(20))
        ne, nl = A.tick_device()
        again = A.events_host()
        assert (len(again[0]), len(again[1])) == (len(prev[0]), len(prev[1]))
        assert (ne, nl) != (len(prev[0]), len(prev[1]))
        np.testing.assert_array_equal(again[0], prev[0])
        np.testing.assert_array_equal(again[1], prev[1])
        # a move of a slot that is not live: dropped on the device, reported by the flush
        A.leave(5)
        A.tick()
        vs, vx, vz = A.stage_moves(2)
        vs[:], vx[:], vz[:] = [5, 6], [1.0, 2.0], [3.0, 4.0]
        A.commit_moves(2)
        with pytest.raises(GwaoiError) as ei:
            A.tick()
        assert ei.value.code == -3  # GWAOI_ESTATE, the flush committed
        np.testing.assert_array_equal(A.snapshot()["x"][A.snapshot()["slot"] == 6], [np.float32(2.0)])


@pytest.mark.parametrize("cfg,n,seed,mode", [("cfg3", 30000, 5, "fused"), ("cfg2", 20000, 9, "fused"),
                                             ("cfg3", 30000, 6, "scr2"), ("cfg2", 20000, 10, "sequence")])
def test_sparse_flushes_match_full_flushes_and_oracle_gpu(oracle_mod, cfg, n, seed, mode):
    """The sparse flush (a few Moved calls: events against the frame in place, the frame patched
    in place, a cell changer shifted into its new cell) gives exactly the events of the full
    flush and of the sequential oracle, flush after flush; the full flushes in between start
    from the patched frame.  Batches of 1-300 moves: host calls (< 64) and staged host batches
    (64..256), repeated slots, steps across cells and rows, and teleports far enough that the
    shifts are declined (the full flush runs instead).  mode: the one-launch form (fused), the
    same with two-event scratch rows so that busy ops fall back to the kernel sequence (scr2),
    and the kernel sequence alone (GWAOI_SPARSE_FUSED=0)."""
    tf = {"scr2": GWAOI_F_TEST_SPARSE_SCR2, "sequence": GWAOI_F_TEST_SPARSE_SEQUENCE}.get(mode, 0)
    wl = make_workload(cfg, n=n, seed=seed)
    slots, x0, z0, _ = wl.initial()
    m = oracle_mod.XZList(wl.D, n)
    rng = np.random.default_rng(seed)
    px, pz = x0.astype(np.float32).copy(), z0.astype(np.float32).copy()
    lo, hi = float(min(px.min(), pz.min())), float(max(px.max(), pz.max()))
    with World(n, test_flags=tf) as A, World(n, sparse=False) as B:
        for w in (A, B):
            s = w.space_create(wl.D)
            w.enter_batch(s, slots, x0, z0)
            w.tick()
        for i in range(n):
            m.enter(int(slots[i]), x0[i], z0[i])
        m.take_events()
        sizes = [1, 1, 2, 5, 17, 63, 64, 100, 256, 257, 1, 3]
        for it in range(48):
            k = sizes[it % len(sizes)]
            if it % 16 == 15:
                k = n  # a full flush of every entity, from the patched frame
            sl = rng.choice(n, k, replace=k >= n or rng.random() < 0.5).astype(np.uint32)  # repeats
            u = rng.random(k)
            step = np.where(u < 0.75, rng.uniform(-1, 1, k), np.where(u < 0.97, rng.uniform(-45, 45, k), 0.0))
            nx = (px[sl] + step.astype(np.float32)).astype(np.float32)
            nz = (pz[sl] + rng.uniform(-1, 1, k).astype(np.float32) * np.where(u < 0.9, 1.0, 60.0)).astype(np.float32)
            tele = u >= 0.97
            nx[tele] = rng.uniform(lo, hi, int(tele.sum())).astype(np.float32)
            nz[tele] = rng.uniform(lo, hi, int(tele.sum())).astype(np.float32)
            if k < 64:
                for s_, x_, z_ in zip(sl.tolist(), nx.tolist(), nz.tolist()):
                    A.moved(s_, x_, z_)
            else:
                A.moved_batch(sl, nx, nz)
            B.moved_batch(sl, nx, nz)
            m.moved_batch(sl, nx, nz)
            for s_, x_, z_ in zip(sl.tolist(), nx.tolist(), nz.tolist()):  # the last op of a slot wins
                px[s_], pz[s_] = x_, z_
            ea, la = (pair_keys(e) for e in A.tick())
            eb, lb = (pair_keys(e) for e in B.tick())
            oe, ol = oracle_mod.net_events(*m.take_events())
            np.testing.assert_array_equal(ea, oe, err_msg=f"flush {it} ({k} moves): sparse-world enters")
            np.testing.assert_array_equal(la, ol, err_msg=f"flush {it} ({k} moves): sparse-world leaves")
            np.testing.assert_array_equal(eb, oe, err_msg=f"flush {it}: full-world enters")
            np.testing.assert_array_equal(lb, ol, err_msg=f"flush {it}: full-world leaves")
            if it % 6 == 5:  # the patched frame answers cell queries exactly
                for i in rng.choice(n, 24, replace=False).tolist():
                    np.testing.assert_array_equal(A.neighbors(i), m.neighbors(i).astype(np.uint32))
        d = A.debug_counters()
        assert d["sparse_flushes"] >= 20, d
        assert (d["sparse_unfused"] > 0) == (mode == "scr2"), d
        assert B.debug_counters()["sparse_flushes"] == 0


@pytest.mark.parametrize("fused", [True, False])
def test_sparse_flushes_multi_space_gpu(fused):
    """Sparse flushes in a world of several spaces whose coordinates overlap (each space its own
    grid, space-major cells): a mover's partners come from its own space only, and the frame
    patch (shifts into a new cell) keeps every space's cell ranges exact.  Each flush equals the
    full-flush world's; the spaces' sizes differ (one nearly empty), and some moves cross many
    cells."""
    rng = np.random.default_rng(31)
    sizes = [4000, 2500, 7, 1500]
    n = sum(sizes)
    with World(n + 16, max_spaces=8, test_flags=0 if fused else GWAOI_F_TEST_SPARSE_SEQUENCE) as A, World(n + 16, max_spaces=8, sparse=False) as B:
        spaces = [(A.space_create(D), B.space_create(D)) for _ in sizes]
        lo = 0
        x = np.empty(n, np.float32)
        z = np.empty(n, np.float32)
        for (sa, sb), k in zip(spaces, sizes):
            sl = np.arange(lo, lo + k, dtype=np.uint32)
            x[lo:lo + k] = rng.uniform(-800, 800, k).astype(np.float32)
            z[lo:lo + k] = rng.uniform(-800, 800, k).astype(np.float32)
            A.enter_batch(sa, sl, x[lo:lo + k], z[lo:lo + k])
            B.enter_batch(sb, sl, x[lo:lo + k], z[lo:lo + k])
            lo += k
        A.tick()
        B.tick()
        for it in range(30):
            k = int(rng.choice([1, 3, 20, 70, 200]))
            sl = rng.choice(n, k, replace=True).astype(np.uint32)
            step = np.where(rng.random(k) < 0.8, rng.uniform(-2, 2, k), rng.uniform(-150, 150, k)).astype(np.float32)
            nx = (x[sl] + step).astype(np.float32)
            nz = (z[sl] + rng.uniform(-2, 2, k).astype(np.float32)).astype(np.float32)
            A.moved_batch(sl, nx, nz)
            B.moved_batch(sl, nx, nz)
            for s_, x_, z_ in zip(sl.tolist(), nx.tolist(), nz.tolist()):
                x[s_], z[s_] = x_, z_
            ea, la = (pair_keys(e) for e in A.tick())
            eb, lb = (pair_keys(e) for e in B.tick())
            np.testing.assert_array_equal(ea, eb, err_msg=f"flush {it} ({k} moves): enters")
            np.testing.assert_array_equal(la, lb, err_msg=f"flush {it} ({k} moves): leaves")
            if it % 10 == 9:
                for i in rng.choice(n, 20, replace=False).tolist():
                    np.testing.assert_array_equal(A.neighbors(i), B.neighbors(i))
        assert A.debug_counters()["sparse_flushes"] >= 20


def test_tick_finish_modes_and_states_gpu():
    """gwaoi_tick_finish: unknown mode bits -> GWAOI_EINVAL and nothing happens; no flush in
    flight -> GWAOI_ESTATE; GWAOI_END_HOST / GWAOI_END_PAIRS copies are what events_host /
    pairs_host return (pairs_host after a directed copy and events_host after a pairs copy
    -> GWAOI_ESTATE); mode 0 leaves the last host copy and its counts as they were."""
    from goworld_amd._lib import GWAOI_END_HOST, GWAOI_END_NEXT, GWAOI_END_PAIRS
    with World(64) as w:
        s = w.space_create(D)
        for i in range(10):
            w.enter(s, i, float(i), 0.0)
        with pytest.raises(GwaoiError) as ei:
            w.finish(0)
        assert ei.value.code == -3  # nothing in flight
        w.tick_begin()
        with pytest.raises(GwaoiError) as ei:
            w.finish(8)
        assert ei.value.code == -1  # unknown bit: the flush stays in flight
        ne, nl = w.finish(GWAOI_END_HOST)
        assert (ne, nl) == (90, 0)
        ent, lev = w.events_host()
        assert len(ent) == 90 and len(lev) == 0
        with pytest.raises(GwaoiError):
            w.pairs_host()
        w.moved(0, 500.0, 0.0)  # 0 leaves 9 neighbours: 18 directed leaves
        w.tick_begin()
        ne, nl = w.finish(GWAOI_END_NEXT | GWAOI_END_PAIRS)
        assert (ne, nl) == (0, 18)
        pe, pl = w.pairs_host()
        assert len(pe) == 0 and len(pl) == 9
        with pytest.raises(GwaoiError):
            w.events_host()
        w.finish(0)  # the (empty) next flush; the pairs copy stays what pairs_host returns
        pe2, pl2 = w.pairs_host()
        np.testing.assert_array_equal(pl2, pl)
