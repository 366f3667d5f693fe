"""BASELINE configs 4 and 5 at their own sizes on the GPU,
checked against the closed form of SURVEY.md Appendix B evaluated by the
multithreaded C oracle (oracle/closed_form.c cf_diff / cf_rows).

* cfg4: the block of spaces one rank holds at 8 GPUs -- 1024 independent
  spaces x 2000 entities (2.05M entities, one manager per space,
  engine/entity/Space.go:33) in one world: the populate flush (count +
  order-independent checksum), three steady ticks of device-resident move
  batches and one churn tick (teleports inside spaces, Leaves, Enters, space
  changes) bit-exact, and 1,000 sampled neighbour rows.
* cfg5 in strips: a 2^22-entity space at config 5's density cut into 8
  x-strips on cuda:0 (loopback exchange, goworld_amd.strips.local_tick); the
  union of the strips' events vs the closed-form diff of the whole space:
  populate by count + checksum, then ticks with teleports across strips,
  churn and entities on edges / halo bounds bit-exact.
* cfg5 one world: the full 2^24-entity space as one world (the 1-GPU bench
  run): one steady tick bit-exact plus 1,000 sampled neighbour rows.

Parity is against the restatement (go-aoi itself is absent: DESIGN.md §2).
Progress lines are printed (run with -s) so a long phase never looks hung.
"""
import time

import numpy as np
import pytest

from goworld_amd import World, pair_keys
from goworld_amd.workload import make_workload

pytestmark = pytest.mark.gpu


def _log(t0, msg):
    print(f"  [{time.perf_counter() - t0:6.1f}s] {msg}", flush=True)


def _checksum_pairs(O, pairs):
    k = (pairs[:, 0].astype(np.uint64) << np.uint64(32)) | pairs[:, 1].astype(np.uint64)
    return O.key_checksum(k)


def _device_batch(torch, sl, nx, nz):
    d = [torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0") for a in (sl.astype(np.int32), nx, nz)]
    torch.cuda.synchronize()
    return d


@pytest.mark.timeout(900)
def test_cfg4_rank_block_1024_spaces_vs_closed_form_gpu(oracle_mod):
    """The 1024-space block of one rank at 8 GPUs (DispatcherService.go:529-540 places
    whole spaces on game processes; here on GPUs, goworld_amd.shard.assign_spaces)."""
    torch = pytest.importorskip("torch")
    O = oracle_mod
    t0 = time.perf_counter()
    ns, per = 1024, 2000
    wl = make_workload("cfg4", n_spaces=ns, per_space=per)
    n = wl.n
    spare = 4000
    N = n + spare
    x = np.zeros(N, np.float32)
    z = np.zeros(N, np.float32)
    seq = np.zeros(N, np.uint64)
    sp = np.full(N, O.DEAD, np.uint32)
    Ds = {s: wl.D for s in range(ns)}
    with World(N, max_spaces=ns, device=0) as w:
        spaces = [w.space_create(wl.D) for _ in range(ns)]
        assert spaces == list(range(ns))
        slots, x0, z0, sp0 = wl.initial()
        nxt = 1
        for s in range(ns):  # Space.enter of every entity, space by space
            sel = slice(s * per, (s + 1) * per)
            w.enter_batch(s, slots[sel], x0[sel], z0[sel])
            seq[slots[sel]] = nxt + np.arange(per, dtype=np.uint64)
            nxt += per
        x[:n], z[:n], sp[:n] = x0, z0, sp0
        before = (np.zeros(N, np.float32), np.zeros(N, np.float32), np.zeros(N, np.uint64),
                  np.full(N, O.DEAD, np.uint32))
        ent, lev = w.tick()
        want_e, want_l = O.closed_form_diff(before, (x, z, seq, sp), Ds)
        assert lev.shape[0] == 0 and want_l.size == 0
        assert ent.shape[0] == want_e.size > 50_000_000
        assert _checksum_pairs(O, ent) == O.key_checksum(want_e), "populate flush: enter multiset"
        _log(t0, f"populate: {ent.shape[0]} directed enters (count + checksum)")
        del ent, want_e

        for t in range(3):  # steady ticks, every entity moves in a random global call order
            sl, nx, nz = wl.tick(t)
            d = _device_batch(torch, sl, nx, nz)
            before = (x.copy(), z.copy(), seq.copy(), sp.copy())
            w.moved_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), sl.size)
            x[sl], z[sl] = nx, nz
            seq[sl] = nxt + np.arange(sl.size, dtype=np.uint64)
            nxt += sl.size
            ge, gl = w.tick()
            want_e, want_l = O.closed_form_diff(before, (x, z, seq, sp), Ds)
            assert want_e.size > 100_000 and want_l.size > 100_000
            np.testing.assert_array_equal(pair_keys(ge), want_e, err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(pair_keys(gl), want_l, err_msg=f"tick {t}: leaves")
            _log(t0, f"steady tick {t}: {want_e.size} enters / {want_l.size} leaves bit-exact")

        # churn: teleports inside the space in the device batch, then host Leaves, Enters of new
        # slots (some into other spaces than before: a slot re-entered elsewhere) and Moved calls
        rng = np.random.default_rng(0xC4)
        before = (x.copy(), z.copy(), seq.copy(), sp.copy())
        sl, nx, nz = wl.tick(3)
        nx, nz = nx.copy(), nz.copy()
        tele = rng.random(sl.size) < 0.01
        nx[tele] = (rng.uniform(-0.45, 0.45, tele.sum()) * wl.L).astype(np.float32)
        nz[tele] = (rng.uniform(-0.45, 0.45, tele.sum()) * wl.L).astype(np.float32)
        d = _device_batch(torch, sl, nx, nz)
        w.moved_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), sl.size)
        x[sl], z[sl] = nx, nz
        seq[sl] = nxt + np.arange(sl.size, dtype=np.uint64)
        nxt += sl.size
        leavers = rng.choice(n, 6000, replace=False)
        for i in leavers:
            w.leave(int(i))
            sp[i] = O.DEAD
        # new slots, and a third of the leavers re-entering another space in the same flush
        back = leavers[:2000]
        for k, i in enumerate(np.concatenate([np.arange(n, N), back])):
            i = int(i)
            s = int(rng.integers(0, ns))
            xi = np.float32(rng.uniform(-0.5, 0.5) * wl.L)
            zi = np.float32(rng.uniform(-0.5, 0.5) * wl.L)
            w.enter(s, i, xi, zi)
            x[i], z[i], seq[i], sp[i] = xi, zi, nxt, s
            nxt += 1
        live = np.nonzero(sp != O.DEAD)[0]
        for i in rng.choice(live, 3000, replace=False):
            xi = np.float32(x[i] + np.float32(rng.uniform(-30, 30)))
            zi = np.float32(z[i] + np.float32(rng.uniform(-30, 30)))
            w.moved(int(i), xi, zi)
            x[i], z[i], seq[i] = xi, zi, nxt
            nxt += 1
        ge, gl = w.tick()
        want_e, want_l = O.closed_form_diff(before, (x, z, seq, sp), Ds)
        np.testing.assert_array_equal(pair_keys(ge), want_e, err_msg="churn tick: enters")
        np.testing.assert_array_equal(pair_keys(gl), want_l, err_msg="churn tick: leaves")
        _log(t0, f"churn tick: {want_e.size} enters / {want_l.size} leaves bit-exact")

        q = rng.choice(np.nonzero(sp != O.DEAD)[0], 1000, replace=False)
        rows = O.closed_form_rows(x, z, seq, sp, Ds, q)
        for i, r in zip(q, rows):
            np.testing.assert_array_equal(w.neighbors(int(i)), r, err_msg=f"neighbours of {i}")
        _log(t0, "1000 sampled rows match")


@pytest.mark.timeout(900)
def test_cfg5_eight_strips_2p22_vs_closed_form_gpu(oracle_mod):
    """8 x-strips of one 2^22-entity space at config 5's density (L = sqrt(N * 1250))."""
    torch = pytest.importorskip("torch")
    from goworld_amd.strips import HALO_WORDS, StripShard, as_words, local_tick
    from strip_scenario import D, Scenario, split_by_owner
    O = oracle_mod
    t0 = time.perf_counter()
    n0 = 1 << 22
    sc = Scenario(n0=n0, spare=20000, n_strips=8, seed=0x5EED0005, teleports=400, pair_teleports=40,
                  churn=2000, edge_hops=400)
    shards = [StripShard(sc.max_slots, D, sc.edges, r, device=0) for r in range(8)]
    Ds = {0: D}
    try:
        st = sc.state()
        for t in range(4):
            kind, sl, nx, nz, seq, px = sc.tick()
            per = split_by_owner(kind, sl, nx, nz, seq, px, sc.edges)
            ops = [as_words(o, HALO_WORDS).to("cuda:0") for o in per]
            torch.cuda.synchronize()
            local_tick(shards, ops)
            evs = [sh.events() for sh in shards]
            after = sc.state()
            want_e, want_l = O.closed_form_diff(st, after, Ds)
            st = after
            if t == 0:
                got = np.concatenate([e for e, _ in evs])
                assert sum(l.shape[0] for _, l in evs) == 0 and want_l.size == 0
                assert got.shape[0] == want_e.size > 100_000_000
                assert _checksum_pairs(O, got) == O.key_checksum(want_e), "populate: enter multiset"
                _log(t0, f"populate: {got.shape[0]} directed enters over 8 strips (count + checksum)")
                del got
                continue
            ge = np.concatenate([pair_keys(e) for e, _ in evs])
            gl = np.concatenate([pair_keys(l) for _, l in evs])
            assert np.unique(ge).size == ge.size and np.unique(gl).size == gl.size, f"tick {t}: duplicates"
            np.testing.assert_array_equal(np.sort(ge), want_e, err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(np.sort(gl), want_l, err_msg=f"tick {t}: leaves")
            assert want_e.size > 100_000 and want_l.size > 100_000
            _log(t0, f"tick {t}: {want_e.size} enters / {want_l.size} leaves bit-exact over 8 strips")
        live = sum(sh.world.info()["live"] for sh in shards)
        assert live > int(np.count_nonzero(sc.live))  # owned entities + ghosts
    finally:
        for sh in shards:
            sh.close()


@pytest.mark.timeout(900)
def test_cfg5_one_world_2p24_steady_tick_gpu(oracle_mod):
    """The whole 2^24-entity space as one world on one GPU (bench --workload cfg5 at N=1)."""
    torch = pytest.importorskip("torch")
    O = oracle_mod
    t0 = time.perf_counter()
    wl = make_workload("cfg5")
    n = wl.n
    assert n == 1 << 24
    seq = np.zeros(n, np.uint64)
    sp = np.zeros(n, np.uint32)
    Ds = {0: wl.D}
    with World(n, device=0) as w:
        s = w.space_create(wl.D)
        slots, x0, z0, _ = wl.initial()
        w.enter_batch(s, slots, x0, z0)
        seq[:] = 1 + np.arange(n, dtype=np.uint64)
        nxt = n + 1
        ne, nl = w.tick_device()  # populate: events stay in HBM
        assert nl == 0 and ne > 400_000_000
        _log(t0, f"populate: {ne} directed enters (in HBM)")
        x, z = x0.copy(), z0.copy()
        for t in range(2):
            sl, nx, nz = wl.tick(t)
            d = _device_batch(torch, sl, nx, nz)
            before = (x.copy(), z.copy(), seq.copy(), sp.copy())
            w.moved_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), sl.size)
            x[sl], z[sl] = nx, nz
            seq[sl] = nxt + np.arange(sl.size, dtype=np.uint64)
            nxt += sl.size
            del d
            ge, gl = w.tick()
            want_e, want_l = O.closed_form_diff(before, (x, z, seq, sp), Ds)
            assert want_e.size > 1_000_000 and want_l.size > 1_000_000
            np.testing.assert_array_equal(pair_keys(ge), want_e, err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(pair_keys(gl), want_l, err_msg=f"tick {t}: leaves")
            _log(t0, f"steady tick {t}: {want_e.size} enters / {want_l.size} leaves bit-exact")
        rng = np.random.default_rng(0xC5)
        q = rng.choice(n, 1000, replace=False)
        rows = O.closed_form_rows(x, z, seq, sp, Ds, q)
        for i, r in zip(q, rows):
            np.testing.assert_array_equal(w.neighbors(int(i)), r, err_msg=f"neighbours of {i}")
        _log(t0, "1000 sampled rows match")
