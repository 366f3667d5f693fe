"""The benchmarked flush form, pinned at the benchmarked configuration.

bench.py's headline tick is a GWAOI_F_UNIQUE_MOVES world (no last-op claims, no repeated-slot
fixup) whose device move batches are chained by gwaoi_tick_finish(NEXT): flush t+1 is queued on
the GPU before flush t's summary is read, so it runs on the grid chosen from t-1's boxes and in
the combined-pass tile schedule that flush t-1 measured.  This test runs exactly that at 1M
entities (bench.py's seed, 256 crowd hotspots + uniform background) and checks every tick's
enter and leave sets bit-exact against the closed form of SURVEY.md Appendix B
(oracle/closed_form.c), then 500 sampled neighbour rows.

Reference: XZListAOIManager.Moved (/root/reference/engine/entity/Space.go:259), one call per move;
go-aoi itself is absent, so parity is against the restatement.
"""
import numpy as np
import pytest

from goworld_amd import World, pair_keys
from goworld_amd.workload import make_workload

from test_unique_moves_gpu import _device_events

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_cfg3_unique_moves_chained_ticks_vs_closed_form_gpu(oracle_mod):
    torch = pytest.importorskip("torch")
    O = oracle_mod
    wl = make_workload("cfg3")  # bench.py's rank-0 seed (0x5EED0003)
    n = wl.n
    ticks = 5  # tick 0 follows the populate (radix) flush; ticks 1-4 use a schedule a steady flush measured
    Ds = {0: wl.D}
    host = [wl.tick(t) for t in range(ticks)]
    dev = [[torch.from_numpy(a).to("cuda:0") for a in (sl.astype(np.int32), nx, nz)] for sl, nx, nz in host]
    torch.cuda.synchronize()
    x = np.zeros(n, np.float32)
    z = np.zeros(n, np.float32)
    seq = np.zeros(n, np.uint64)
    sp = np.full(n, O.DEAD, np.uint32)
    with World(n, unique_moves=True, device=0) as w:
        s = w.space_create(wl.D)
        slots, x0, z0, _ = wl.initial()
        w.enter_batch(s, slots, x0, z0)
        ne0, nl0 = w.tick_device()
        assert nl0 == 0 and ne0 > 80_000_000
        x[slots], z[slots] = x0, z0
        seq[slots] = 1 + np.arange(n, dtype=np.uint64)
        sp[slots] = 0
        nxt = n + 1
        d0 = w.debug_counters()
        w.moved_batch_device(*(b.data_ptr() for b in dev[0]), host[0][0].size)
        w.tick_begin()
        for t in range(ticks):
            before = (x.copy(), z.copy(), seq.copy(), sp.copy())
            if t + 1 < ticks:  # tick t+1's batch registered while flush t runs, then queued before t's summary
                w.moved_batch_device(*(b.data_ptr() for b in dev[t + 1]), host[t + 1][0].size)
                ne, nl = w.tick_end_begin_device()
            else:
                ne, nl = w.tick_end_device()
            ge, gl = _device_events(w, ne, nl)  # flush t's events (flush t+1 writes the other set)
            sl, nx, nz = host[t]
            x[sl], z[sl] = nx, nz
            seq[sl] = nxt + np.arange(sl.size, dtype=np.uint64)
            nxt += sl.size
            want_e, want_l = O.closed_form_diff(before, (x, z, seq, sp), Ds)
            assert want_e.size > 100_000 and want_l.size > 100_000
            np.testing.assert_array_equal(pair_keys(ge), want_e, err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(pair_keys(gl), want_l, err_msg=f"tick {t}: leaves")
        d1 = w.debug_counters()
        assert d1["unique_flushes"] - d0["unique_flushes"] == ticks, (d0, d1)
        assert d1["speculative_launches"] - d0["speculative_launches"] == ticks - 1, (d0, d1)
        # the speculative launches after the first ran their first kernels on the early stream, beside the
        # pair passes and finish of the flush before it (the first has no predecessor's mid event; a
        # flush on a new grid has no incremental sort and runs alone)
        assert d1["overlapped_flushes"] - d0["overlapped_flushes"] >= ticks - 3, (d0, d1)
        assert d1["incremental_sorts"] - d0["incremental_sorts"] >= ticks - 1, (d0, d1)
        rng = np.random.default_rng(0xC3C3)
        q = rng.choice(n, 500, replace=False)
        rows = O.closed_form_rows(x, z, seq, sp, Ds, q)
        for i, r in zip(q, rows):
            np.testing.assert_array_equal(np.sort(w.neighbors(int(i))), r, err_msg=f"neighbours of {i}")
