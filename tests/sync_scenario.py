"""Seeded entity-sync scenario shared by the CPU and GPU sync tests.

A game process with entities over two AOI spaces and one space without AOI:
clients on several gates, some entities not syncing from their client, some
never in a space (nilSpace), some in the space without AOI, some unknown ids
in the client packets, duplicated records, server-side moves (also of
entities outside every AOI space: Position stays, yaw and flags change,
Entity.go:1189-1205 with Space.go:253-257), leaves and re-enters (space
changes) between packets.  Each flush is a list
of ops in call order; `run_oracle` / `run_gpu` apply them to the sequential
restatement (oracle/entity_sync.py) and to libgwaoi.
"""
from __future__ import annotations

import struct

import numpy as np

GATES = [1, 2, 300, 65535]


def make(seed=7, n=600, n_outside=40, flushes=6, L=700.0):
    rng = np.random.default_rng(seed)
    ids = set()
    while len(ids) < n:
        ids.add(bytes(rng.integers(0, 256, 16, dtype=np.uint8)))
    ids = sorted(ids)
    rng.shuffle(ids)
    ent = []
    for s in range(n):
        has_client = rng.random() < 0.7
        ent.append({
            "slot": s, "eid": ids[s],
            "gate": int(rng.choice(GATES)) if has_client else None,
            "cid": bytes(rng.integers(0, 256, 16, dtype=np.uint8)) if has_client else None,
            "syncing": bool(rng.random() < 0.8),
            "pos": [np.float32(v) for v in (rng.uniform(-L / 2, L / 2), rng.uniform(0, 10), rng.uniform(-L / 2, L / 2),
                                            rng.uniform(-3, 3))],
        })
    spaces = {0: 100.0, 1: 60.0}
    in_space = {e["slot"]: (e["slot"] % 2) for e in ent[: n - n_outside]}
    plain = {e["slot"] for e in ent[n - n_outside:] if e["slot"] % 2 == 0}  # in the space without AOI
    setup = [("set_pos", e["slot"], *e["pos"]) for e in ent]
    setup += [("enter", s, sp) for s, sp in in_space.items()]
    setup += [("enter_plain", s) for s in sorted(plain)]
    cur = {e["slot"]: list(e["pos"]) for e in ent}
    space_of = dict(in_space)
    flush_ops = []
    for f in range(flushes):
        ops = []
        live = sorted(space_of)
        outside = sorted(set(range(n)) - set(space_of))  # nilSpace or the space without AOI

        def step(s, big=False):
            p = cur[s]
            d = 150.0 if big else 4.0
            p[0] = np.float32(p[0] + np.float32(rng.uniform(-d, d)))
            p[2] = np.float32(p[2] + np.float32(rng.uniform(-d, d)))
            p[1] = np.float32(rng.uniform(0, 10))
            p[3] = np.float32(rng.uniform(-3, 3))
            return p

        for s in rng.choice(live, size=min(25, len(live)), replace=False):
            p = step(int(s))
            ops.append(("server_move", int(s), *p))
        for s in rng.choice(outside, size=min(6, len(outside)), replace=False):
            p = step(int(s))  # Position stays stale in the reference: only yaw and the flags change
            ops.append(("server_move", int(s), *p))
        ops.append(("packet", packet(rng, ent, cur, step, 0.6)))
        # the space without AOI: leave to nilSpace, or enter it from nilSpace
        for s in rng.choice(outside, size=min(4, len(outside)), replace=False):
            s = int(s)
            if s in plain:
                ops.append(("leave_plain", s))
                plain.discard(s)
            else:
                p = step(s, big=True)
                ops.append(("set_pos", s, *p))
                ops.append(("enter_plain", s))
                plain.add(s)
        # leaves / re-enters / space changes
        for s in rng.choice(live, size=8, replace=False):
            s = int(s)
            ops.append(("leave", s))
            del space_of[s]
            if rng.random() < 0.6:
                sp = int(rng.integers(0, 2))
                p = step(s, big=True)
                ops.append(("set_pos", s, *p))
                ops.append(("enter", s, sp))
                space_of[s] = sp
        if f % 2 == 0:
            ops.append(("packet", packet(rng, ent, cur, step, 0.2)))
        flush_ops.append(ops)
    return {"ent": ent, "spaces": spaces, "setup": setup, "flushes": flush_ops, "n": n}


def packet(rng, ent, cur, step, frac):
    """32-byte records: EntityID + x,y,z,yaw little-endian (GameService.go:392-404)."""
    recs = []
    for e in ent:
        if rng.random() < frac:
            p = step(e["slot"])
            recs.append(e["eid"] + struct.pack("<4f", *p))
            if rng.random() < 0.05:  # a duplicate later in the packet (last one wins)
                p = step(e["slot"])
                recs.append(e["eid"] + struct.pack("<4f", *p))
    for _ in range(5):  # unknown entity ids (destroyed before the packet arrived)
        recs.append(bytes(rng.integers(0, 256, 16, dtype=np.uint8)) + struct.pack("<4f", 1, 2, 3, 4))
    order = rng.permutation(len(recs))
    return b"".join(recs[i] for i in order)


def run_oracle(sc, on_flush):
    from oracle.entity_sync import GameEntities
    g = GameEntities(sc["spaces"], sc["n"])
    for e in sc["ent"]:
        g.create(e["eid"], e["slot"], *e["pos"])
        if e["cid"] is not None:
            g.set_client(e["slot"], e["gate"], e["cid"])
        g.set_syncing(e["slot"], e["syncing"])
    pend = {}

    def apply(op):
        k = op[0]
        if k == "set_pos":
            pend[op[1]] = op[2:]
            g.set_position_yaw_noflags(op[1], *op[2:])
        elif k == "enter":
            x, y, z, _ = pend.pop(op[1])
            g.enter_space(op[1], op[2], x, y, z)
        elif k == "enter_plain":
            x, y, z, _ = pend.pop(op[1])
            g.enter_plain_space(op[1], 9, x, y, z)
        elif k in ("leave", "leave_plain"):
            g.leave_space(op[1])
        elif k == "server_move":
            assert g.set_position_yaw(op[1], *op[2:], from_client=False)
        elif k == "packet":
            g.handle_sync_packet(op[1])

    for op in sc["setup"]:
        apply(op)
    on_flush(0, g)
    for i, ops in enumerate(sc["flushes"]):
        for op in ops:
            apply(op)
        on_flush(i + 1, g)
    return g


def run_gpu(sc, w, on_flush, device_payload=None):
    """Drive a goworld_amd.World; device_payload(bytes) -> (ptr, keepalive) puts packets in HBM."""
    sp_ids = {k: w.space_create(D) for k, D in sc["spaces"].items()}
    ent = sc["ent"]
    w.entity_bind([e["slot"] for e in ent], [e["eid"] for e in ent])
    for e in ent:
        if e["cid"] is not None:
            w.entity_set_client(e["slot"], e["gate"], e["cid"])
        w.entity_set_syncing(e["slot"], e["syncing"])
    keep = []

    def apply(op):
        k = op[0]
        if k == "set_pos":
            w.entity_set_position_yaw(op[1], *op[2:])
            apply.last[op[1]] = op[2:]
        elif k == "enter":
            x, _, z, _ = apply.last[op[1]]
            w.enter(sp_ids[op[2]], op[1], x, z)
        elif k == "enter_plain":
            x, y, z, _ = apply.last[op[1]]
            w.entity_enter_plain(op[1], x, y, z)
        elif k == "leave":
            w.leave(op[1])
        elif k == "leave_plain":
            w.entity_leave_plain(op[1])
        elif k == "server_move":
            w.set_position_yaw(op[1], *op[2:])
        elif k == "packet":
            if device_payload is None:
                w.sync_from_clients(op[1])
            else:
                ptr, obj = device_payload(op[1])
                keep.append(obj)
                w.sync_from_clients_device(ptr, len(op[1]) // 32)

    apply.last = {}
    for op in sc["setup"]:
        apply(op)
    w.tick()
    on_flush(0, w)
    for i, ops in enumerate(sc["flushes"]):
        for op in ops:
            apply(op)
        ent_ev, lev_ev = w.tick()
        keep.clear()
        on_flush(i + 1, w, ent_ev, lev_ev)
