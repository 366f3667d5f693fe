"""Config 3 at its own size and density on the GPU: 1M entities, 256 Gaussian
crowd hotspots (~1953 entities each at sigma 250) + uniform background --
the configuration BASELINE.json quotes its metric on.

The HIP path (through the C ABI) is checked against the closed form of
SURVEY.md Appendix B evaluated by the multithreaded C oracle
(oracle/closed_form.c cf_diff), flush by flush:

* the populate flush (84.8M directed enters): count + order-independent
  checksum of the key multiset (too large to sort inside a test);
* three steady ticks of device-resident move batches (every entity moves by
  U(-1,1), seeded call order): enter / leave sets bit-exact;
* one churn tick: teleports inside the device batch, host Leaves, host
  Enters of new slots and plain host Moved calls, all in one flush (the mixed
  op path): bit-exact;
* 1,000 sampled entities: gwaoi_neighbors == the closed-form row.

The rare paths of the combined pass that only crowds reach -- a wave's LDS
event buffer overflowing (sweep replay) and the survivor queue draining in
the middle of a sweep -- are asserted through gwaoi_debug_counters.
Parity is against the restatement (go-aoi itself is absent: DESIGN.md §2).
"""
import numpy as np
import pytest

from goworld_amd import World, pair_keys
from goworld_amd.workload import make_workload

pytestmark = pytest.mark.gpu


def _keys(pairs):
    return pair_keys(pairs)


@pytest.mark.timeout(600)
def test_cfg3_full_density_vs_closed_form_gpu(oracle_mod):
    torch = pytest.importorskip("torch")
    O = oracle_mod
    wl = make_workload("cfg3")
    n = wl.n
    extra = 2000  # slots entering in the churn tick
    N = n + extra
    Ds = {0: wl.D}
    x = np.zeros(N, np.float32)
    z = np.zeros(N, np.float32)
    seq = np.zeros(N, np.uint64)
    sp = np.full(N, O.DEAD, np.uint32)
    dev = "cuda:0"
    with World(N, device=0) as w:
        s = w.space_create(wl.D)
        slots, x0, z0, _ = wl.initial()
        w.enter_batch(s, slots, x0, z0)
        before = (x.copy(), z.copy(), seq.copy(), sp.copy())
        x[:n], z[:n] = x0, z0
        seq[:n] = 1 + np.arange(n, dtype=np.uint64)
        sp[:n] = 0
        nxt = n + 1
        ent, lev = w.tick()
        want_e, want_l = O.closed_form_diff(before, (x, z, seq, sp), Ds)
        assert lev.shape[0] == 0 and want_l.size == 0
        assert ent.shape[0] == want_e.size > 80_000_000
        k = (ent[:, 0].astype(np.uint64) << np.uint64(32)) | ent[:, 1].astype(np.uint64)
        assert O.key_checksum(k) == O.key_checksum(want_e), "populate flush: enter multiset"
        del ent, k, want_e
        d0 = w.debug_counters()

        # ---- steady ticks: device-resident move batches
        for t in range(3):
            sl, nx, nz = wl.tick(t)
            ds = torch.from_numpy(sl.astype(np.int32)).to(dev)
            dx = torch.from_numpy(nx).to(dev)
            dz = torch.from_numpy(nz).to(dev)
            torch.cuda.synchronize()
            before = (x.copy(), z.copy(), seq.copy(), sp.copy())
            w.moved_batch_device(ds.data_ptr(), dx.data_ptr(), dz.data_ptr(), sl.size)
            x[sl], z[sl] = nx, nz
            seq[sl] = nxt + np.arange(sl.size, dtype=np.uint64)
            nxt += sl.size
            ge, gl = w.tick()
            want_e, want_l = O.closed_form_diff(before, (x, z, seq, sp), Ds)
            assert want_e.size > 100_000 and want_l.size > 100_000
            np.testing.assert_array_equal(_keys(ge), want_e, err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(_keys(gl), want_l, err_msg=f"tick {t}: leaves")
        d1 = w.debug_counters()

        # ---- churn tick: teleports in the device batch + host Leave / Enter / Moved
        rng = np.random.default_rng(0xC3)
        before = (x.copy(), z.copy(), seq.copy(), sp.copy())
        sl, nx, nz = wl.tick(3)
        tele = rng.random(sl.size) < 0.01
        nx = nx.copy()
        nz = nz.copy()
        nx[tele] = (rng.uniform(-0.4, 0.4, tele.sum()) * wl.L).astype(np.float32)
        nz[tele] = (rng.uniform(-0.4, 0.4, tele.sum()) * wl.L).astype(np.float32)
        ds = torch.from_numpy(sl.astype(np.int32)).to(dev)
        dx = torch.from_numpy(nx).to(dev)
        dz = torch.from_numpy(nz).to(dev)
        torch.cuda.synchronize()
        w.moved_batch_device(ds.data_ptr(), dx.data_ptr(), dz.data_ptr(), sl.size)
        x[sl], z[sl] = nx, nz
        seq[sl] = nxt + np.arange(sl.size, dtype=np.uint64)
        nxt += sl.size
        leavers = rng.choice(n, 5000, replace=False)
        for i in leavers:
            w.leave(int(i))
            sp[i] = O.DEAD
        for j in range(extra):  # new entities, half of them into hotspot crowds
            i = n + j
            src = int(rng.integers(n // 2, n)) if j % 2 else int(rng.integers(0, n // 2))
            xi = np.float32(x[src] + np.float32(rng.uniform(-5, 5)))
            zi = np.float32(z[src] + np.float32(rng.uniform(-5, 5)))
            w.enter(s, i, xi, zi)
            x[i], z[i], seq[i], sp[i] = xi, zi, nxt, 0
            nxt += 1
        live = np.nonzero(sp != O.DEAD)[0]
        for i in rng.choice(live, 3000, replace=False):  # plain Moved calls after the batch (one may hit a
            xi = np.float32(x[i] + np.float32(rng.uniform(-40, 40)))  # new slot: Enter then Moved in one flush)
            zi = np.float32(z[i] + np.float32(rng.uniform(-40, 40)))
            w.moved(int(i), xi, zi)
            x[i], z[i], seq[i] = xi, zi, nxt
            nxt += 1
        ge, gl = w.tick()
        want_e, want_l = O.closed_form_diff(before, (x, z, seq, sp), Ds)
        np.testing.assert_array_equal(_keys(ge), want_e, err_msg="churn tick: enters")
        np.testing.assert_array_equal(_keys(gl), want_l, err_msg="churn tick: leaves")
        assert want_l.size > 1_000_000  # the leavers' pairs and the teleports'

        # ---- the relation itself, sampled
        q = rng.choice(np.nonzero(sp != O.DEAD)[0], 1000, replace=False)
        rows = O.closed_form_rows(x, z, seq, sp, Ds, q)
        for i, r in zip(q, rows):
            np.testing.assert_array_equal(w.neighbors(int(i)), r, err_msg=f"neighbours of {i}")
        d2 = w.debug_counters()

    steady = {k: d1[k] - d0[k] for k in d0}
    print(f"\ndebug counters: populate {d0}\n steady(3 ticks) {steady}\n total {d2}")
    # the crowds' populate and churn flushes reach the combined pass's rare paths: LDS
    # event-buffer overflow + replay, and survivor-queue drains in the middle of a sweep
    assert d2["combined_replays"] > 0
    assert d2["combined_queue_drains"] > 0
