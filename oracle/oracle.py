"""ctypes front-end of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline, never as a product path.

* ``XZList``   -- one go-aoi ``XZListAOIManager`` restated sequentially
  (oracle/xzlist.c).
* ``SpacesOracle`` -- one ``XZList`` per space, global slot ids, the way
  GoWorld gives every Space its own manager (engine/entity/Space.go:33,105).
* ``closed_form_pairs`` -- the batch relation of SURVEY.md Appendix B
  (oracle/closed_form.c).
* ``WireHost`` -- the gate / dispatcher sync regroups as a host C loop
  (oracle/wire_host.c), bench.py's wire_leg comparator.

PARITY UNPINNED: go-aoi (go.mod:29) is absent and the reference holds no AOI
fixture; see DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

OP_MOVED, OP_ENTER, OP_LEAVE = 0, 1, 2
EV_ENTER, EV_LEAVE = 1, 2
DEAD = 0xFFFFFFFF


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        vp, f, i32, i64, sz = C.c_void_p, C.c_float, C.c_int32, C.c_int64, C.c_size_t
        L.xz_new.restype = vp
        L.xz_new.argtypes = [f, i32]
        L.xz_free.argtypes = [vp]
        L.xz_set_record.argtypes = [vp, C.c_int]
        for name in ("xz_enter", "xz_moved"):
            getattr(L, name).argtypes = [vp, i32, f, f]
            getattr(L, name).restype = C.c_int
        L.xz_leave.argtypes = [vp, i32]
        L.xz_leave.restype = C.c_int
        L.xz_apply.argtypes = [vp, i64, vp, vp, vp, vp]
        L.xz_apply.restype = i64
        L.xz_moved_batch.argtypes = [vp, i64, vp, vp, vp]
        L.xz_moved_batch.restype = i64
        L.xz_bulk_enter.argtypes = [vp, i64, vp, vp, vp]
        L.xz_bulk_enter.restype = C.c_int
        L.xz_counts.argtypes = [vp, C.POINTER(i64), C.POINTER(i64)]
        L.xz_num_events.argtypes = [vp]
        L.xz_num_events.restype = sz
        L.xz_take_events.argtypes = [vp, vp, vp, vp, sz]
        L.xz_take_events.restype = sz
        L.xz_neighbors.argtypes = [vp, i32, vp, i32]
        L.xz_neighbors.restype = i32
        L.xz_neighbor_count.argtypes = [vp, i32]
        L.xz_neighbor_count.restype = i32
        L.xz_total_pairs.argtypes = [vp]
        L.xz_total_pairs.restype = i64
        L.xz_check.argtypes = [vp]
        L.xz_check.restype = C.c_int
        L.cf_pairs.argtypes = [i64, vp, vp, vp, vp, vp, C.POINTER(C.POINTER(C.c_uint64))]
        L.cf_pairs.restype = i64
        L.cf_free.argtypes = [vp]
        L.cf_pred.argtypes = [f, f, f, f, f]
        L.cf_pred.restype = C.c_int
        L.cf_diff.argtypes = [i64] + [vp] * 9 + [C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(i64),
                                                 C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(i64), C.c_int]
        L.cf_diff.restype = C.c_int
        L.cf_rows.argtypes = [i64, vp, vp, vp, vp, vp, i64, vp, vp, C.POINTER(C.POINTER(C.c_uint32))]
        L.cf_rows.restype = i64
        L.cg_new.argtypes = [i64, f, C.c_int]
        L.cg_new.restype = vp
        L.cg_free.argtypes = [vp]
        L.cg_init.argtypes = [vp, vp, vp]
        L.cg_init.restype = i64
        L.cg_tick.argtypes = [vp, i64, vp, vp, vp, C.POINTER(i64), C.POINTER(i64)]
        L.wh_map_new.argtypes = [i64, vp, vp]
        L.wh_map_new.restype = vp
        L.wh_map_free.argtypes = [vp]
        L.wh_gate_from_clients.argtypes = [vp, i64, C.c_uint32, vp, vp, vp]
        L.wh_gate_from_clients.restype = i64
        for name in ("wh_dispatcher_to_games", "wh_gate_to_clients"):
            getattr(L, name).argtypes = [vp, i64, vp, C.c_uint32, vp, vp, vp]
            getattr(L, name).restype = i64
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class XZList:
    """Sequential go-aoi XZListAOIManager restatement over local ids [0, cap)."""

    def __init__(self, D: float, cap: int, record: bool = True):
        self._L = lib()
        self._m = self._L.xz_new(C.c_float(D), cap)
        self._L.xz_set_record(self._m, 1 if record else 0)
        self.cap = cap

    def __del__(self):
        if getattr(self, "_m", None):
            self._L.xz_free(self._m)
            self._m = None

    def enter(self, i, x, z):
        if self._L.xz_enter(self._m, int(i), C.c_float(x), C.c_float(z)):
            raise RuntimeError(f"Enter({i}) on a live AOI")

    def leave(self, i):
        if self._L.xz_leave(self._m, int(i)):
            raise RuntimeError(f"Leave({i}) on an AOI that never entered")

    def moved(self, i, x, z):
        if self._L.xz_moved(self._m, int(i), C.c_float(x), C.c_float(z)):
            raise RuntimeError(f"Moved({i}) on an AOI that never entered")

    def apply(self, ops, ids, xs, zs):
        ops = np.ascontiguousarray(ops, np.uint8)
        ids = np.ascontiguousarray(ids, np.int32)
        xs = np.ascontiguousarray(xs, np.float32)
        zs = np.ascontiguousarray(zs, np.float32)
        bad = self._L.xz_apply(self._m, ops.size, _p(ops), _p(ids), _p(xs), _p(zs))
        if bad >= 0:
            raise RuntimeError(f"op {bad} rejected")

    def bulk_enter(self, ids, xs, zs):
        """Same state as Enter(ids[i]) for i in order on an empty manager, without events."""
        ids = np.ascontiguousarray(ids, np.int32)
        xs = np.ascontiguousarray(xs, np.float32)
        zs = np.ascontiguousarray(zs, np.float32)
        if self._L.xz_bulk_enter(self._m, ids.size, _p(ids), _p(xs), _p(zs)):
            raise RuntimeError("bulk_enter needs an empty manager and fresh ids")

    def moved_batch(self, ids, xs, zs):
        ids = np.ascontiguousarray(ids, np.int32)
        xs = np.ascontiguousarray(xs, np.float32)
        zs = np.ascontiguousarray(zs, np.float32)
        bad = self._L.xz_moved_batch(self._m, ids.size, _p(ids), _p(xs), _p(zs))
        if bad >= 0:
            raise RuntimeError(f"move {bad} rejected")

    def counts(self):
        e, l = C.c_int64(), C.c_int64()
        self._L.xz_counts(self._m, C.byref(e), C.byref(l))
        return e.value, l.value

    def take_events(self):
        n = self._L.xz_num_events(self._m)
        t = np.empty(n, np.uint8)
        a = np.empty(n, np.int32)
        b = np.empty(n, np.int32)
        self._L.xz_take_events(self._m, _p(t), _p(a), _p(b), n)
        return t, a, b

    def neighbors(self, i):
        cnt = self._L.xz_neighbor_count(self._m, int(i))
        out = np.empty(max(cnt, 1), np.int32)
        self._L.xz_neighbors(self._m, int(i), _p(out), out.size)
        return np.sort(out[:cnt])

    def pairs(self):
        """All directed neighbour pairs as sorted uint64 keys (a<<32|b), local ids."""
        keys = []
        for i in range(self.cap):
            nb = self.neighbors(i)
            if nb.size:
                keys.append((np.uint64(i) << np.uint64(32)) | nb.astype(np.uint64))
        return np.sort(np.concatenate(keys)) if keys else np.empty(0, np.uint64)

    def check(self):
        return self._L.xz_check(self._m)


class SpacesOracle:
    """One XZList per space over global slots, replaying a GoWorld op stream.

    Ops are applied in seq order exactly as Space.enter/leave/move would call
    the manager (engine/entity/Space.go:211,243,259).  Events are kept as
    (type, a_slot, b_slot).
    """

    def __init__(self, D_by_space, max_slots: int, record: bool = True):
        self.D = {int(k): float(v) for k, v in D_by_space.items()}
        self.max_slots = max_slots
        self.mgr = {}
        self.local = {}  # slot -> (space, local id)
        self.free = {}
        self.next_local = {}
        self.local_to_slot = {}
        self.record = record

    def _m(self, sp):
        if sp not in self.mgr:
            self.mgr[sp] = XZList(self.D[sp], self.max_slots, self.record)
            self.local_to_slot[sp] = np.full(self.max_slots, -1, np.int64)
        return self.mgr[sp]

    def enter(self, sp, slot, x, z):
        m = self._m(sp)
        lid = slot  # local id == slot keeps the mapping trivial
        m.enter(lid, x, z)
        self.local[slot] = sp
        self.local_to_slot[sp][lid] = slot

    def leave(self, slot):
        sp = self.local.pop(slot)
        self.mgr[sp].leave(slot)

    def moved(self, slot, x, z):
        self.mgr[self.local[slot]].moved(slot, x, z)

    def moved_batch(self, slots, xs, zs):
        """Moves whose slots all live in one space (the common batched case)."""
        sps = {self.local[int(s)] for s in slots[:1]}
        sp = sps.pop()
        self.mgr[sp].moved_batch(slots, xs, zs)

    def take_events(self, with_space: bool = False):
        """(type, a, b) of every callback since the last call, manager by
        manager (call order within a space); with_space: also the space of
        each event, so that a net diff can keep every space its own manager."""
        ts, as_, bs, ss = [], [], [], []
        for sp, m in self.mgr.items():
            t, a, b = m.take_events()
            ts.append(t); as_.append(a); bs.append(b); ss.append(np.full(t.size, sp, np.int64))
        if not ts:
            e = (np.empty(0, np.uint8), np.empty(0, np.int32), np.empty(0, np.int32))
            return e + (np.empty(0, np.int64),) if with_space else e
        out = (np.concatenate(ts), np.concatenate(as_), np.concatenate(bs))
        return out + (np.concatenate(ss),) if with_space else out

    def pairs(self):
        keys = [m.pairs() for m in self.mgr.values()]
        keys = [k for k in keys if k.size]
        return np.sort(np.concatenate(keys)) if keys else np.empty(0, np.uint64)

    def neighbors(self, slot):
        if slot not in self.local:
            return np.empty(0, np.int32)
        return self.mgr[self.local[slot]].neighbors(slot)


def closed_form_pairs(x, z, seq, sp, D_by_space):
    """Directed neighbour pairs of the closed form (Appendix B), sorted uint64 keys."""
    L = lib()
    x = np.ascontiguousarray(x, np.float32)
    z = np.ascontiguousarray(z, np.float32)
    seq = np.ascontiguousarray(seq, np.uint64)
    sp = np.ascontiguousarray(sp, np.uint32)
    live = sp[sp != DEAD]
    nsp = int(live.max()) + 1 if live.size else 1
    D = np.zeros(nsp, np.float32)
    for k, v in D_by_space.items():
        if int(k) < nsp:
            D[int(k)] = v
    out = C.POINTER(C.c_uint64)()
    n = L.cf_pairs(x.size, _p(x), _p(z), _p(seq), _p(sp), _p(D), C.byref(out))
    res = np.ctypeslib.as_array(out, shape=(n,)).copy() if n else np.empty(0, np.uint64)
    L.cf_free(C.cast(out, C.c_void_p))
    return res


class CpuGrid:
    """CPU-grid comparator (oracle/cpu_grid.c): one space, every tick the relation
    recomputed on all host cores with a cell grid and diffed against the last."""

    def __init__(self, x, z, D, threads):
        self._L = lib()
        x = np.ascontiguousarray(x, np.float32)
        z = np.ascontiguousarray(z, np.float32)
        self._g = self._L.cg_new(x.size, C.c_float(D), int(threads))
        self.pairs = self._L.cg_init(self._g, _p(x), _p(z))

    def tick(self, slots, x, z):
        s = np.ascontiguousarray(slots, np.int32)
        x = np.ascontiguousarray(x, np.float32)
        z = np.ascontiguousarray(z, np.float32)
        ne, nl = C.c_int64(), C.c_int64()
        self._L.cg_tick(self._g, s.size, _p(s), _p(x), _p(z), C.byref(ne), C.byref(nl))
        return ne.value, nl.value

    def __del__(self):
        if getattr(self, "_g", None):
            self._L.cg_free(self._g)
            self._g = None


def _space_d(sp_arrays, D_by_space):
    nsp = 1
    for sp in sp_arrays:
        live = sp[sp != DEAD]
        if live.size:
            nsp = max(nsp, int(live.max()) + 1)
    D = np.zeros(nsp, np.float32)
    for k, v in D_by_space.items():
        if int(k) < nsp:
            D[int(k)] = v
    return D


def _state(x, z, seq, sp):
    return (np.ascontiguousarray(x, np.float32), np.ascontiguousarray(z, np.float32),
            np.ascontiguousarray(seq, np.uint64), np.ascontiguousarray(sp, np.uint32))


def closed_form_diff(before, after, D_by_space, threads=None):
    """Net events of one flush from the closed form at two states (Appendix B,
    per-tick recipe): ``before``/``after`` = (x, z, seq, space) per entity, space
    DEAD when not live.  Returns sorted uint64 keys (enter, leave), both
    directions.  An entity that changed space leaves every old pair and enters
    every new one.  Multithreaded C (oracle/closed_form.c cf_diff)."""
    L = lib()
    b = _state(*before)
    a = _state(*after)
    n = b[0].size
    D = _space_d([b[3], a[3]], D_by_space)
    threads = threads or max(1, min(16, len(os.sched_getaffinity(0))))
    pe, pl = C.POINTER(C.c_uint64)(), C.POINTER(C.c_uint64)()
    ne, nl = C.c_int64(), C.c_int64()
    L.cf_diff(n, *[_p(v) for v in b], *[_p(v) for v in a], _p(D), C.byref(pe), C.byref(ne), C.byref(pl),
              C.byref(nl), threads)
    ent = np.ctypeslib.as_array(pe, shape=(ne.value,)).copy() if ne.value else np.empty(0, np.uint64)
    lev = np.ctypeslib.as_array(pl, shape=(nl.value,)).copy() if nl.value else np.empty(0, np.uint64)
    L.cf_free(C.cast(pe, C.c_void_p))
    L.cf_free(C.cast(pl, C.c_void_p))
    return ent, lev


def closed_form_rows(x, z, seq, sp, D_by_space, query):
    """Sorted closed-form neighbour list of every entity in ``query``: list of uint32 arrays."""
    L = lib()
    st = _state(x, z, seq, sp)
    D = _space_d([st[3]], D_by_space)
    q = np.ascontiguousarray(query, np.int32)
    off = np.zeros(q.size + 1, np.int64)
    out = C.POINTER(C.c_uint32)()
    tot = L.cf_rows(st[0].size, *[_p(v) for v in st], _p(D), q.size, _p(q), _p(off), C.byref(out))
    flat = np.ctypeslib.as_array(out, shape=(tot,)).copy() if tot else np.empty(0, np.uint32)
    L.cf_free(C.cast(out, C.c_void_p))
    return [flat[off[k]:off[k + 1]] for k in range(q.size)]


def key_checksum(keys: np.ndarray) -> tuple:
    """(count, sum of SplitMix64(key) mod 2^64) of a uint64 key multiset: an
    order-independent fingerprint for relations too large to sort in a test."""
    k = np.asarray(keys, np.uint64)
    with np.errstate(over="ignore"):
        z = k + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        return int(k.size), int(np.sum(z, dtype=np.uint64))


def pred(wx, wz, lx, lz, D):
    """P_W(L): does W's window [fl32(w-D), fl32(w+D)]^2 contain L?"""
    return bool(lib().cf_pred(C.c_float(wx), C.c_float(wz), C.c_float(lx), C.c_float(lz), C.c_float(D)))


def events_to_keys(t, a, b):
    """Split an event stream into sorted uint64 key arrays (enter, leave)."""
    a = np.asarray(a).astype(np.uint64)
    b = np.asarray(b).astype(np.uint64)
    k = (a << np.uint64(32)) | b
    return np.sort(k[t == EV_ENTER]), np.sort(k[t == EV_LEAVE])


def net_events(t, a, b, sp=None):
    """Net per-flush diff of a sequential event stream: (enter keys, leave keys).

    The sequential manager can emit a transient enter+leave of one pair within
    a flush; the batch engine reports only the net change.
    With ``sp`` (the space of each event) every space is its own manager: a
    pair that leaves in one space and enters in another inside the flush
    (both entities changed space) keeps both events, as the GPU path reports
    them.
    """
    a = np.asarray(a).astype(np.int64)
    b = np.asarray(b).astype(np.int64)
    s = np.zeros(a.size, np.int64) if sp is None else np.asarray(sp).astype(np.int64)
    state = {}
    for ti, ai, bi, si in zip(t.tolist(), a.tolist(), b.tolist(), s.tolist()):
        k = (si, (ai << 32) | bi)
        d = 1 if ti == EV_ENTER else -1
        state[k] = state.get(k, 0) + d
    ent = np.array(sorted(k for (_, k), v in state.items() if v > 0), np.uint64)
    lev = np.array(sorted(k for (_, k), v in state.items() if v < 0), np.uint64)
    for v in state.values():
        assert v in (-1, 0, 1), "unbalanced event stream"
    return ent, lev


class WireHost:
    """Host C restatement of the gate / dispatcher sync regroups (oracle/wire_host.c):
    the CPU comparator of bench.py's wire_leg.  Tables: entity id -> game, client
    id -> proxy index.  Each call returns (keys, offsets, records bytes array) like
    the GPU regroups of include/gwaoi_wire.h."""

    def __init__(self, entity_ids=None, games=None, client_ids=None, client_index=None):
        self._L = lib()
        self._g = self._c = None
        self.max_game = self.max_client = 0
        if entity_ids is not None:
            ids = np.ascontiguousarray(entity_ids, np.uint8).reshape(-1)
            v = np.ascontiguousarray(games, np.uint32)
            self._g = self._L.wh_map_new(v.size, _p(ids), _p(v))
            self.max_game = int(v.max()) if v.size else 0
        if client_ids is not None:
            ids = np.ascontiguousarray(client_ids, np.uint8).reshape(-1)
            v = np.ascontiguousarray(client_index, np.uint32)
            self._c = self._L.wh_map_new(v.size, _p(ids), _p(v))
            self.max_client = int(v.max()) if v.size else 0

    def __del__(self):
        for h in (getattr(self, "_g", None), getattr(self, "_c", None)):
            if h:
                self._L.wh_map_free(h)

    def _out(self, n, max_key, rec):
        return (np.empty(max_key + 2, np.uint32), np.empty(max_key + 3, np.uint64), np.empty(max(n, 1) * rec, np.uint8))

    def gate_from_clients(self, rec, n_disp):
        rec = np.ascontiguousarray(rec, np.uint8).reshape(-1)
        n = rec.size // 32
        k, o, out = self._out(n, n_disp, 32)
        g = self._L.wh_gate_from_clients(_p(rec), n, n_disp, _p(k), _p(o), _p(out))
        return k[:g], o[:g + 1], out[:int(o[g]) * 32]

    def dispatcher_to_games(self, rec):
        rec = np.ascontiguousarray(rec, np.uint8).reshape(-1)
        n = rec.size // 32
        k, o, out = self._out(n, self.max_game, 32)
        g = self._L.wh_dispatcher_to_games(_p(rec), n, self._g, self.max_game, _p(k), _p(o), _p(out))
        return k[:g], o[:g + 1], out[:int(o[g]) * 32]

    def gate_to_clients(self, rec):
        rec = np.ascontiguousarray(rec, np.uint8).reshape(-1)
        n = rec.size // 48
        k, o, out = self._out(n, self.max_client, 32)
        g = self._L.wh_gate_to_clients(_p(rec), n, self._c, self.max_client, _p(k), _p(o), _p(out))
        return k[:g], o[:g + 1], out[:int(o[g]) * 32]
