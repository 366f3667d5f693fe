"""Entity position sync around the AOI path (include/gwaoi_sync.h): client
packet decode (GameService.go:392-404), CollectEntitySyncInfos fan-out
(Entity.go:1221-1267) and the routing of AOI events to client create/destroy
messages (Entity.go:236-246, GameClient.go:37-59).

CPU tests pin the restatement (oracle/entity_sync.py) on hand-built cases;
GPU tests run the seeded scenario of tests/sync_scenario.py through the
C ABI and compare every flush with the restatement: enter/leave pairs
bit-exact, sync records and client messages as exact multisets per gate.
Parity unpinned against GoWorld itself (Go is absent; the reference holds
no fixture for these packets) -- the record layouts follow the reference's
Packet.Append* order (Entity.go:1233-1251) and its little-endian floats.
"""
import struct

import numpy as np
import pytest

import sync_scenario as SS
from oracle import oracle
from oracle.entity_sync import SIF_NEIGHBOR, SIF_OWN, GameEntities, records_by_gate

EID = [bytes([65 + i]) * 16 for i in range(6)]
CID = [bytes([97 + i]) * 16 for i in range(6)]


def rec(eid, x, y, z, yaw):
    return eid + struct.pack("<4f", x, y, z, yaw)


# ------------------------------------------------------------------ CPU ------

def small_world():
    g = GameEntities({0: 100.0}, 8)
    for i in range(4):
        g.create(EID[i], i, 10.0 * i, 1.0, 0.0, 0.5)
    g.set_client(0, 1, CID[0])
    g.set_client(1, 2, CID[1])
    g.set_syncing(0, True)
    g.set_syncing(1, False)
    g.set_syncing(2, True)
    for i in range(3):  # entity 3 never enters a space
        g.enter_space(i, 0, 10.0 * i, 1.0, 0.0)
    return g


def test_enter_sets_both_flags_and_interest_is_symmetric():
    g = small_world()
    for e in g.by_slot.values():
        assert e.In == e.By
    assert g.by_slot[0].flags == SIF_OWN | SIF_NEIGHBOR
    assert g.by_slot[3].flags == 0
    out = g.collect()
    # own records of 0 and 1, plus one per (entity, interested neighbour with a client)
    assert sorted(out) == [1, 2]
    assert len(out[1]) == 1 + 2 and len(out[2]) == 1 + 2
    assert g.collect() == {}  # flags cleared


def test_packet_decode_rules():
    g = small_world()
    g.collect()
    pkt = rec(EID[0], 5.0, 2.0, 0.0, 1.0) + rec(EID[1], 7.0, 2.0, 0.0, 1.0) + rec(b"?" * 16, 0, 0, 0, 0) \
        + rec(EID[3], 1.0, 1.0, 1.0, 1.0) + rec(EID[2], 30.0, 3.0, 0.0, 2.0) + rec(EID[0], 6.0, 4.0, 0.0, 2.5)
    g.handle_sync_packet(pkt)
    e0, e1, e2, e3 = (g.by_slot[i] for i in range(4))
    assert (e0.x, e0.y, e0.yaw) == (6.0, 4.0, 2.5)         # last record wins
    assert e1.x == 10.0 and e1.flags == 0                  # not syncing from its client
    assert e3.x == 30.0 and e3.flags == 0                  # not syncing from its client
    assert e0.flags == SIF_NEIGHBOR and e2.flags == SIF_NEIGHBOR  # fromClient: no own-client record
    out = g.collect()
    # e0 and e2 moved; interested clients: e0 <- {1 (gate 2)}, e2 <- {0 (gate 1), 1 (gate 2)}
    assert out == {1: sorted([CID[0] + EID[2] + struct.pack("<4f", 30, 3, 0, 2)]),
                   2: sorted([CID[1] + EID[0] + struct.pack("<4f", 6, 4, 0, 2.5),
                              CID[1] + EID[2] + struct.pack("<4f", 30, 3, 0, 2)])}


def test_left_entity_keeps_own_record():
    g = small_world()
    g.collect()
    g.set_position_yaw(0, 1.0, 1.0, 1.0, 1.0)
    g.leave_space(0)
    assert g.by_slot[0].By == set()
    out = g.collect()
    assert out == {1: [CID[0] + EID[0] + struct.pack("<4f", 1, 1, 1, 1)]}


def test_nilspace_entity_keeps_position_gets_yaw_and_flags():
    """Entity.setPositionYaw of an entity outside every space: e.Space is
    nilSpace (EntityManager.go:250, Space.go:240), not nil, so the call goes on
    to nilSpace.move, which returns before `entity.Position = newPos` because
    nilSpace has no AOI manager (Space.go:253-257); yaw and the sync flags are
    still set (Entity.go:1196-1204).  CollectEntitySyncInfos then sends the own
    client the STALE position with the NEW yaw (Entity.go:1228-1239)."""
    g = small_world()
    g.set_client(3, 1, CID[3])
    g.set_syncing(3, True)
    g.collect()
    e3 = g.by_slot[3]
    g.handle_sync_packet(rec(EID[3], 50.0, 9.0, 50.0, 1.25))  # from the client: neighbour flag only
    assert (e3.x, e3.y, e3.z) == (30.0, 1.0, 0.0) and e3.yaw == np.float32(1.25)
    assert e3.flags == SIF_NEIGHBOR and e3.By == set()
    assert g.collect() == {}  # no own-client flag, nobody interested
    assert g.set_position_yaw(3, 60.0, 8.0, 60.0, -2.0)  # server side: both flags
    assert e3.x == 30.0 and e3.flags == SIF_OWN | SIF_NEIGHBOR
    assert g.collect() == {1: [CID[3] + EID[3] + struct.pack("<4f", 30.0, 1.0, 0.0, -2.0)]}


def test_space_without_aoi_enter_move_leave():
    """Space.enter of a space without AOI (or of an entity type without AOI,
    Space.go:210) sets Position and both flags but calls no AOI manager;
    moves inside it keep Position (Space.go:254-256) and change yaw."""
    g = small_world()
    g.set_client(3, 2, CID[3])
    g.collect()
    e3 = g.by_slot[3]
    g.enter_plain_space(3, 9, 5.0, 6.0, 7.0)
    assert (e3.x, e3.y, e3.z) == (5.0, 6.0, 7.0) and e3.flags == SIF_OWN | SIF_NEIGHBOR
    assert g.collect() == {2: [CID[3] + EID[3] + struct.pack("<4f", 5.0, 6.0, 7.0, 0.5)]}
    g.set_position_yaw(3, 0.0, 0.0, 0.0, 3.0)
    assert (e3.x, e3.z, e3.yaw) == (5.0, 7.0, np.float32(3.0))
    assert g.collect() == {2: [CID[3] + EID[3] + struct.pack("<4f", 5.0, 6.0, 7.0, 3.0)]}
    # the entity is 5 units from entity 0 of the AOI space, yet no AOI relation exists
    assert g.by_slot[0].In == {1, 2} and 3 not in g.by_slot[0].By
    g.leave_space(3)
    assert e3.space is None and g.collect() == {}


def test_left_aoi_entity_moves_keep_last_aoi_position():
    """After Space.leave the entity is in nilSpace: a server move sends its own
    client the position it had when it left, with the new yaw."""
    g = small_world()
    g.collect()
    g.set_position_yaw(0, 3.0, 4.0, 5.0, 0.25)
    g.leave_space(0)
    g.collect()
    g.set_position_yaw(0, 100.0, 100.0, 100.0, -1.0)
    assert g.collect() == {1: [CID[0] + EID[0] + struct.pack("<4f", 3.0, 4.0, 5.0, -1.0)]}


def test_scenario_oracle_consistency():
    sc = SS.make(n=200, flushes=3)

    def check(i, g):
        for e in g.by_slot.values():
            assert e.In == e.By
            if e.aoi:
                assert sorted(e.By) == g.aoi.neighbors(e.slot).tolist()
            else:
                assert not e.By and not e.In
        g.collect()

    SS.run_oracle(sc, check)


# ------------------------------------------------------------------ GPU ------

def expected(sc):
    exp = []

    def on_flush(i, g):
        raw = g.take_raw()  # every space its own manager (a pair may leave in one and enter in another)
        ent, lev = oracle.net_events(*raw)
        cre, des = g.net_client_events(*raw)
        exp.append({"sync": g.collect(), "enter": ent, "leave": lev, "create": cre, "destroy": des})

    SS.run_oracle(sc, on_flush)
    return exp


def check_run(sc, device_payload=None):
    from goworld_amd import World, pair_keys
    exp = expected(sc)
    seen = []

    def on_flush(i, w, ent=None, lev=None):
        e = exp[i]
        if ent is not None:
            assert np.array_equal(pair_keys(ent), e["enter"]), f"flush {i}: enter pairs"
            assert np.array_equal(pair_keys(lev), e["leave"]), f"flush {i}: leave pairs"
            cre, des = w.collect_client_events()
            assert records_by_gate(cre) == e["create"], f"flush {i}: create messages"
            assert records_by_gate(des) == e["destroy"], f"flush {i}: destroy messages"
        got = records_by_gate(w.collect_sync_infos())
        assert got == e["sync"], f"flush {i}: sync records"
        seen.append(sum(len(v) for v in got.values()))

    with World(sc["n"], max_spaces=4, device=0) as w:
        SS.run_gpu(sc, w, on_flush, device_payload)
    assert len(seen) == len(sc["flushes"]) + 1 and min(seen) > 0


@pytest.mark.gpu
def test_sync_host_packets_match_oracle():
    check_run(SS.make(seed=11))


@pytest.mark.gpu
def test_sync_device_packets_match_oracle():
    import torch

    def dev(b):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8).to("cuda:0")
        torch.cuda.synchronize()
        return t.data_ptr(), t

    check_run(SS.make(seed=12, n=900, flushes=4), device_payload=dev)


@pytest.mark.gpu
def test_sync_dense_crowd_regrows_fanout_scratch():
    """Every entity inside everyone's window (a 60 x 60 square, D = 100 / 60):
    ~250 records per receiver, past the fan-out scratch's first size (32 words
    per entry), so the first collect regrows it and reruns the hits pass."""
    check_run(SS.make(seed=13, n=600, n_outside=20, flushes=2, L=60.0))


@pytest.mark.gpu
def test_sync_output_regrows_between_collects():
    """A small collect (10 entities in the spaces), then a dense one (the other
    entities enter a 60 x 60 square): the write pass, launched behind the hits
    pass without a host round trip, finds the previous collect's output too
    small and writes nothing; the host regrows the output and relaunches it."""
    sc = SS.make(seed=14, n=800, n_outside=20, flushes=2, L=60.0)
    enters = [op for op in sc["setup"] if op[0] == "enter"]
    keep = {op[1] for op in enters[:10]}
    sc["setup"] = [op for op in sc["setup"] if op[0] != "enter" or op[1] in keep]
    sc["flushes"].insert(0, [op for op in enters if op[1] not in keep])
    check_run(sc)


@pytest.mark.gpu
def test_sync_errors():
    from goworld_amd import GwaoiError, World
    with World(16, device=0) as w:
        sp = w.space_create(100.0)
        w.entity_bind([0, 1], [EID[0], EID[1]])
        w.entity_bind([0], [EID[0]])  # same binding again: no-op
        with pytest.raises(GwaoiError):
            w.entity_bind([2], [EID[0]])  # id taken
        with pytest.raises(GwaoiError):
            w.entity_bind([0], [EID[2]])  # slot taken
        w.set_position_yaw(0, 1, 2, 3, 4)  # nilSpace: yaw + flags, Position stays (Space.go:253-257)
        with pytest.raises(GwaoiError):
            w.set_position_yaw(99, 1, 2, 3, 4)  # slot out of range
        w.entity_enter_plain(1, 1.0, 2.0, 3.0)  # a space without AOI
        with pytest.raises(GwaoiError):
            w.entity_enter_plain(1, 1.0, 2.0, 3.0)  # already in a space without AOI
        with pytest.raises(GwaoiError):
            w.enter(sp, 1, 0.0, 0.0)  # in a space already (Space.enter panics, Space.go:193-195)
        w.entity_leave_plain(1)
        with pytest.raises(GwaoiError):
            w.entity_leave_plain(1)  # not in a space without AOI
        w.enter(sp, 0, 0.0, 0.0)
        with pytest.raises(GwaoiError):
            w.entity_enter_plain(0, 1.0, 2.0, 3.0)  # in an AOI space (Space.enter panics, Space.go:193-195)
        with pytest.raises(GwaoiError):
            w.collect_sync_infos()  # ops queued since the last flush
        w.tick()
        w.entity_unbind(1)
        w.entity_bind([2], [EID[1]])  # the id is free again
        with pytest.raises(GwaoiError):
            w.entity_unbind(1)
        assert w.collect_sync_infos() == {}  # no client anywhere


@pytest.mark.gpu
def test_sync_fanout_full_size_sampled():
    """100k entities, every entity in one client packet: the records each
    sampled receiver gets are exactly one per neighbour of the flush (queried
    through gwaoi_neighbors) carrying that neighbour's packet record, and every
    record sits in its receiver's gate (size-independent property)."""
    from goworld_amd import World
    from goworld_amd.workload import make_workload
    wl = make_workload("cfg2", n=100_000)
    n = wl.n
    rng = np.random.default_rng(3)
    eids = np.frombuffer(b"".join(b"E%015d" % s for s in range(n)), np.uint8).reshape(n, 16)
    has = rng.random(n) < 0.5
    gate = (1 + np.arange(n) % 3).astype(np.uint16)
    with World(n, device=0) as w:
        sp = w.space_create(float(wl.D))
        slots, x0, z0, _ = wl.initial()
        w.entity_bind(slots, eids)
        for s in np.nonzero(has)[0]:
            w.entity_set_client(int(s), int(gate[s]), b"C%015d" % int(s))
        for s in range(n):
            w.entity_set_syncing(s, True)
        w.enter_batch(sp, slots, x0, z0)
        w.tick()
        w.collect_sync_infos()  # Space.enter flags
        sl, nx, nz = wl.tick(0)
        y = rng.uniform(0, 5, n).astype(np.float32)
        yaw = rng.uniform(-3, 3, n).astype(np.float32)
        pay = b"".join(bytes(eids[s]) + struct.pack("<4f", nx[k], y[k], nz[k], yaw[k]) for k, s in enumerate(sl))
        w.sync_from_clients(pay)
        w.tick()
        recs = w.collect_sync_infos()
        pos = {int(s): (nx[k], y[k], nz[k], yaw[k]) for k, s in enumerate(sl)}
        by_client = {}
        for g, a in recs.items():
            for r in a:
                cid = bytes(r[:16])
                assert int(cid[1:]) % 3 + 1 == g, "record in another gate than its receiver"
                by_client.setdefault(cid, []).append(bytes(r))
        assert sum(len(v) for v in recs.values()) > 0
        for b in rng.choice(np.nonzero(has)[0], 300, replace=False):
            b = int(b)
            cid = b"C%015d" % b
            exp = sorted(cid + bytes(eids[a]) + struct.pack("<4f", *pos[int(a)]) for a in w.neighbors(b))
            assert sorted(by_client.get(cid, [])) == exp, f"receiver {b}"


@pytest.mark.gpu
def test_sync_repeated_records_outside_spaces_list_each_slot_once():
    """More client records than max_slots, all for syncing entities outside every
    AOI space (nilSpace): k_decode lists such a slot for its own-client record at
    most once (atomic flag claim), so its per-slot list cannot overflow; the
    collects match the restatement (GameService.go:392-404, Entity.go:1221-1267)."""
    from goworld_amd import World
    n, reps = 8, 5
    eids = [bytes([70 + i]) * 16 for i in range(n)]
    cids = [bytes([110 + i]) * 16 for i in range(n)]
    g = GameEntities({0: 100.0}, n)
    with World(n, device=0) as w:
        w.entity_bind(list(range(n)), eids)
        for i in range(n):
            g.create(eids[i], i, 0.0, 0.0, 0.0, 0.0)
            w.entity_set_client(i, 1 + i % 2, cids[i])
            g.set_client(i, 1 + i % 2, cids[i])
            w.entity_set_syncing(i, True)
            g.set_syncing(i, True)
        assert records_by_gate(w.collect_sync_infos()) == g.collect()
        pkt = b"".join(rec(eids[i], float(k), 1.0, float(i), 0.25 * k) for k in range(reps) for i in range(n))
        w.sync_from_clients(pkt)
        g.handle_sync_packet(pkt)
        w.tick()
        assert records_by_gate(w.collect_sync_infos()) == g.collect() == {}
        for i in range(0, n, 2):  # server-side moves: own-client records with the stale position
            w.set_position_yaw(i, 9.0, 9.0, 9.0, -1.0)
            g.set_position_yaw(i, 9.0, 9.0, 9.0, -1.0)
        w.sync_from_clients(pkt)
        g.handle_sync_packet(pkt)
        w.tick()
        got = records_by_gate(w.collect_sync_infos())
        assert got == g.collect() and sum(len(v) for v in got.values()) == n // 2
