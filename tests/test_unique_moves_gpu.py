"""GWAOI_F_UNIQUE_MOVES: Moved batches that never repeat a slot within a flush are applied
without the last-op claims and the repeated-slot fixup (include/gwaoi.h).  The flush must give
exactly the events of the claims path, and a batch that breaks the promise must be reported
(GWAOI_ESTATE) by the flush that applied it, with the world still usable.

Reference: XZListAOIManager.Moved (/root/reference/engine/entity/Space.go:259) -- one call per
move, the last call of a slot wins; the oracle restates it (oracle/xzlist.c)."""
import numpy as np
import pytest

from goworld_amd import World, pair_keys
from goworld_amd._lib import GwaoiError
from goworld_amd.workload import make_workload
from oracle import oracle

pytestmark = pytest.mark.gpu

ESTATE = -3


def _device_events(w, ne, nl):
    """Copy the last committed flush's device events (gwaoi_events_device) to the host."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    e, l = w.events_device()
    out = []
    for ptr, k in ((e, ne), (l, nl)):
        a = np.empty((k, 2), np.uint32)
        if k:
            assert hip.hipMemcpy(a.ctypes.data, ptr, a.nbytes, 2) == 0  # hipMemcpyDeviceToHost
        out.append(a)
    return out


def _positions(w, n):
    """(x, z) per slot [0, n) from the frame snapshot (NaN: not live)."""
    snap = w.snapshot()
    out = np.full((n, 2), np.nan, np.float32)
    out[snap["slot"], 0] = snap["x"]
    out[snap["slot"], 1] = snap["z"]
    return out


@pytest.mark.parametrize("spec", [False, True])
def test_unique_moves_match_claims_and_oracle_gpu(spec):
    """Unique batches (every entity once per tick, in a random order) on a flagged world, against
    the same batches on an unflagged world (claims + fixup), tick by tick, both event lists;
    speculative (gwaoi_tick_finish(NEXT)) or serial flushes; neighbour sets against the
    sequential oracle at the end."""
    torch = pytest.importorskip("torch")
    n, ticks = 20000, 10
    wa = make_workload("cfg2", n=n)
    slots, x0, z0, _ = wa.initial()
    host = [wa.tick(t) for t in range(ticks)]
    dev = [[torch.from_numpy(a).to("cuda:0") for a in (sl.astype(np.int32), nx, nz)] for sl, nx, nz in host]
    torch.cuda.synchronize()
    ref = oracle.XZList(wa.D, n)
    for i in range(n):
        ref.enter(int(slots[i]), x0[i], z0[i])
    with World(n, unique_moves=True) as A, World(n) as B:
        for w in (A, B):
            s = w.space_create(wa.D)
            w.enter_batch(s, slots, x0, z0)
            w.tick()
        if spec:
            A.moved_batch_device(*(b.data_ptr() for b in dev[0]), host[0][0].size)
            A.tick_begin()
        for t in range(ticks):
            if spec:
                if t + 1 < ticks:
                    A.moved_batch_device(*(b.data_ptr() for b in dev[t + 1]), host[t + 1][0].size)
                    ne, nl = A.tick_end_begin_device()
                else:
                    ne, nl = A.tick_end_device()
            else:
                A.moved_batch_device(*(b.data_ptr() for b in dev[t]), host[t][0].size)
                ne, nl = A.tick_device()
            ga, la = _device_events(A, ne, nl)
            B.moved_batch_device(*(b.data_ptr() for b in dev[t]), host[t][0].size)
            gb, lb = _device_events(B, *B.tick_device())
            np.testing.assert_array_equal(pair_keys(ga), pair_keys(gb), err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(pair_keys(la), pair_keys(lb), err_msg=f"tick {t}: leaves")
            sl, nx, nz = host[t]
            for k in range(sl.size):
                ref.moved(int(sl[k]), nx[k], nz[k])
        da, db = A.debug_counters(), B.debug_counters()
        assert da["unique_flushes"] == ticks, da
        assert db["unique_flushes"] == 0, db
        for i in range(0, n, 499):
            want = np.sort(np.asarray(ref.neighbors(i), dtype=np.uint32))
            np.testing.assert_array_equal(np.sort(A.neighbors(i)), want, err_msg=f"entity {i}")


def test_unique_moves_repeated_slot_is_reported_gpu():
    """A flagged world given a batch that moves one slot twice: the flush commits, returns
    GWAOI_ESTATE (ERR_DUP_SLOT, found by keygen's written-entry count), and the slot holds one of
    its two positions.  A later batch that moves a slot that is not live: GWAOI_ESTATE (move
    dropped, no DUP: the dropped op is counted).  The flushes after each error report nothing
    (the apply's error word and drop count are reset for the next flush without a prologue), and a
    unique tick that moves every entity brings the world back in step with a claims world.  Three
    clean ticks first, so that the bad batches meet the steady flush (previous grid, no prologue)."""
    torch = pytest.importorskip("torch")
    n, warm = 5000, 3
    wa = make_workload("cfg2", n=n)
    slots, x0, z0, _ = wa.initial()
    clean = [wa.tick(t) for t in range(warm)]
    sl0, nx0, nz0 = wa.tick(warm)
    # one slot moved twice: an extra move appended after its regular one
    v = int(sl0[17])
    sl = np.concatenate([sl0, [v]]).astype(np.uint32)
    nx = np.concatenate([nx0, [np.float32(nx0[17] + 3.0)]]).astype(np.float32)
    nz = np.concatenate([nz0, [np.float32(nz0[17] - 2.0)]]).astype(np.float32)
    after = [wa.tick(warm + 1 + t) for t in range(3)]
    # a batch naming slot n (never entered) besides the regular moves
    sl2, nx2, nz2 = after[1]
    bad = (np.concatenate([sl2, [n]]).astype(np.uint32), np.concatenate([nx2, [np.float32(1.0)]]),
           np.concatenate([nz2, [np.float32(2.0)]]))

    def dev(b):
        return [torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0") for a in (b[0].astype(np.int32), b[1], b[2])]

    d_clean = [dev(b) for b in clean]
    d0 = dev((sl, nx, nz))
    d_after = [dev(after[0]), dev(bad), dev(after[2])]
    torch.cuda.synchronize()
    with World(n + 1, unique_moves=True) as A, World(n + 1) as B:
        for w in (A, B):
            s = w.space_create(wa.D)
            w.enter_batch(s, slots, x0, z0)
            w.tick()
            for b, h in zip(d_clean, clean):
                w.moved_batch_device(*(t.data_ptr() for t in b), h[0].size)
                w.tick_device()
        A.moved_batch_device(*(b.data_ptr() for b in d0), sl.size)
        with pytest.raises(GwaoiError) as ei:
            A.tick_device()
        assert ei.value.code == ESTATE, str(ei.value)
        assert "UNIQUE" in str(ei.value)
        B.moved_batch_device(*(b.data_ptr() for b in d0), sl.size)
        B.tick_device()
        # the repeated slot holds one of its two moves; every other slot is the claims world's
        xa = _positions(A, n)
        xb = _positions(B, n)
        cand = {(float(nx0[17]), float(nz0[17])), (float(nx[-1]), float(nz[-1]))}
        assert (float(xa[v][0]), float(xa[v][1])) in cand
        others = np.arange(n) != v
        np.testing.assert_array_equal(xa[others], xb[others])
        # a clean unique tick (no stale error), then the dead-slot batch, then a clean one
        for w in (A, B):
            w.moved_batch_device(*(b.data_ptr() for b in d_after[0]), after[0][0].size)
            w.tick_device()
        for w in (A, B):
            w.moved_batch_device(*(b.data_ptr() for b in d_after[1]), bad[0].size)
            with pytest.raises(GwaoiError) as ei:
                w.tick_device()
            assert ei.value.code == ESTATE and "not live" in str(ei.value), str(ei.value)
        for w in (A, B):
            w.moved_batch_device(*(b.data_ptr() for b in d_after[2]), after[2][0].size)
            w.tick_device()
        np.testing.assert_array_equal(_positions(A, n), _positions(B, n))
        for i in range(0, n, 97):
            np.testing.assert_array_equal(np.sort(A.neighbors(i)), np.sort(B.neighbors(i)))
        assert A.debug_counters()["unique_flushes"] == warm + 4


def test_unique_moves_on_an_empty_world_report_and_do_not_leak_gpu():
    """Moves of slots that are not live, on a flagged world with no entity yet: the flush has no
    entry (keygen does not run, only its fold), yet it must report the dropped moves
    (GWAOI_ESTATE), and the apply's error word and drop count must not leak into the next flushes."""
    torch = pytest.importorskip("torch")
    n = 3000
    wa = make_workload("cfg2", n=n)
    slots, x0, z0, _ = wa.initial()
    sl, nx, nz = wa.tick(0)
    d0 = [torch.from_numpy(a).to("cuda:0") for a in (sl.astype(np.int32), nx, nz)]
    ticks = [wa.tick(1 + t) for t in range(3)]
    dt = [[torch.from_numpy(a).to("cuda:0") for a in (b[0].astype(np.int32), b[1], b[2])] for b in ticks]
    torch.cuda.synchronize()
    with World(n, unique_moves=True) as A, World(n) as B:
        s = A.space_create(wa.D)
        A.moved_batch_device(*(b.data_ptr() for b in d0), sl.size)
        with pytest.raises(GwaoiError) as ei:
            A.tick_device()
        assert ei.value.code == ESTATE and "not live" in str(ei.value), str(ei.value)
        sb = B.space_create(wa.D)
        for w, sp in ((A, s), (B, sb)):
            w.enter_batch(sp, slots, x0, z0)
            w.tick()
            for b, h in zip(dt, ticks):  # clean unique ticks: no error may surface
                w.moved_batch_device(*(t.data_ptr() for t in b), h[0].size)
                w.tick_device()
        np.testing.assert_array_equal(_positions(A, n), _positions(B, n))
        for i in range(0, n, 101):
            np.testing.assert_array_equal(np.sort(A.neighbors(i)), np.sort(B.neighbors(i)))
