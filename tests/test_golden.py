"""Golden fixtures (tests/golden/, made by make_golden.py from the oracle).

CPU: the fixtures load without pickles, the KAT fixtures hold the
hand-derived Appendix C expectations, the sequential restatement replays
every fixture to the recorded events, and the final relation equals the
closed form (Appendix B).  GPU: libgwaoi replays every fixture through the
C ABI to the recorded per-flush events and final neighbour sets, bit-exact.
"""
import numpy as np
import pytest

import golden_util as G

NAMES = G.names()


def key(a, b):
    return (a << 32) | b


def test_fixture_inventory():
    for need in ("kat_r1", "kat_r2", "kat_t1", "kat_t2_t3", "kat_l1", "cfg1_1k_50t", "lattice64",
                 "multispace16x128"):
        assert need in NAMES


def test_kat_fixtures_match_appendix_c():
    r1 = G.load("kat_r1")
    e, l = G.expected(r1, 0)
    assert e.tolist() == [key(0, 1), key(1, 0)] and l.size == 0
    e, l = G.expected(r1, 1)
    assert e.size == 0 and l.tolist() == [key(0, 1), key(1, 0)]
    r2 = G.load("kat_r2")
    assert G.expected(r2, 0)[0].tolist() == [key(0, 1), key(1, 0)]
    assert G.expected(r2, 1)[1].tolist() == [key(0, 1), key(1, 0)]
    t1 = G.load("kat_t1")
    e, _ = G.expected(t1, 0)
    assert e.size == 90 and len({int(k) >> 32 for k in e}) == 10
    t23 = G.load("kat_t2_t3")
    e, _ = G.expected(t23, 0)
    pairs = sorted({tuple(sorted((int(k) >> 32, int(k) & 0xFFFFFFFF))) for k in e})
    assert pairs == [(0, 1), (0, 2), (0, 3), (1, 3), (1, 4), (2, 3)]
    l1 = G.load("kat_l1")
    e, l = G.expected(l1, 1)
    assert e.size == 0 and l.size == 14
    assert all((int(k) >> 32) == 3 or (int(k) & 0xFFFFFFFF) == 3 for k in l)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_replays_fixture(oracle_mod, name):
    fx = G.load(name)
    orc = oracle_mod.SpacesOracle({i: d for i, d in enumerate(fx["space_D"])}, int(fx["max_slots"]))

    def apply_op(kind, slot, x, z, sp):
        if kind == G.ENTER:
            orc.enter(sp, slot, x, z)
        elif kind == G.LEAVE:
            orc.leave(slot)
        else:
            orc.moved(slot, x, z)

    def flush():
        es, ls = [], []
        for m in orc.mgr.values():
            e, l = oracle_mod.net_events(*m.take_events())
            es.append(e)
            ls.append(l)
        return (np.sort(np.concatenate(es)) if es else np.empty(0, np.uint64),
                np.sort(np.concatenate(ls)) if ls else np.empty(0, np.uint64))

    for i, (e, l) in G.replay(fx, apply_op, flush):
        ee, el = G.expected(fx, i)
        np.testing.assert_array_equal(e, ee)
        np.testing.assert_array_equal(l, el)
    np.testing.assert_array_equal(orc.pairs(), fx["final_pairs"])


@pytest.mark.parametrize("name", NAMES)
def test_fixture_final_relation_is_closed_form(oracle_mod, name):
    fx = G.load(name)
    x, z, seq, sp = G.final_state(fx)
    cf = oracle_mod.closed_form_pairs(x, z, seq, sp, {i: d for i, d in enumerate(fx["space_D"])})
    np.testing.assert_array_equal(cf, fx["final_pairs"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_replays_fixture(name):
    from goworld_amd import World, pair_keys
    fx = G.load(name)
    nsp = len(fx["space_D"])
    with World(int(fx["max_slots"]), max_spaces=nsp) as w:
        ids = [w.space_create(d) for d in fx["space_D"]]

        def apply_op(kind, slot, x, z, sp):
            if kind == G.ENTER:
                w.enter(ids[sp], slot, x, z)
            elif kind == G.LEAVE:
                w.leave(slot)
            else:
                w.moved(slot, x, z)

        def flush():
            e, l = w.tick()
            return pair_keys(e), pair_keys(l)

        for i, (e, l) in G.replay(fx, apply_op, flush):
            ee, el = G.expected(fx, i)
            np.testing.assert_array_equal(e, ee, err_msg=f"{name} flush {i} enters")
            np.testing.assert_array_equal(l, el, err_msg=f"{name} flush {i} leaves")
        got = []
        live = np.nonzero(G.final_state(fx)[3] != 0xFFFFFFFF)[0]
        for s in live.tolist():
            nb = w.neighbors(s)
            if nb.size:
                got.append((np.uint64(s) << np.uint64(32)) | nb.astype(np.uint64))
        got = np.sort(np.concatenate(got)) if got else np.empty(0, np.uint64)
        np.testing.assert_array_equal(got, fx["final_pairs"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["lattice64", "multispace16x128", "cfg1_1k_50t"])
def test_gpu_freeze_restore_keeps_relation(name):
    """f4: freeze (gwaoi_snapshot) after the whole fixture, restore into a fresh
    world (gwaoi_restore, original seq order): the first flush enters exactly
    the frozen relation, bit for bit (EntityManager.go:554-656)."""
    from goworld_amd import World, pair_keys
    fx = G.load(name)
    nsp = len(fx["space_D"])
    with World(int(fx["max_slots"]), max_spaces=nsp) as w:
        ids = [w.space_create(d) for d in fx["space_D"]]

        def apply_op(kind, slot, x, z, sp):
            if kind == G.ENTER:
                w.enter(ids[sp], slot, x, z)
            elif kind == G.LEAVE:
                w.leave(slot)
            else:
                w.moved(slot, x, z)

        for _ in G.replay(fx, apply_op, lambda: w.tick()):
            pass
        snap = w.snapshot()
    x, z, seq, sp = G.final_state(fx)
    live = np.nonzero(sp != 0xFFFFFFFF)[0]
    assert np.array_equal(np.sort(snap["slot"]), live)
    o = np.argsort(snap["slot"])
    assert np.array_equal(snap["x"][o], x[live]) and np.array_equal(snap["z"][o], z[live])
    # the frozen seqs order the entities exactly as the call stream did
    assert np.array_equal(np.argsort(snap["seq"][o], kind="stable"), np.argsort(seq[live], kind="stable"))
    perm = np.random.default_rng(5).permutation(snap["slot"].size)  # any input order (Go map order)
    with World(int(fx["max_slots"]), max_spaces=nsp) as w2:
        for d in fx["space_D"]:
            w2.space_create(d)
        w2.restore({k: v[perm] for k, v in snap.items()})
        e, l = w2.tick()
        assert l.size == 0
        np.testing.assert_array_equal(pair_keys(e), fx["final_pairs"])
