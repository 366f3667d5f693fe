"""Host-side mirror of the AOI interface GoWorld's engine uses (go-aoi v0.2.0,
package ``aoi``), backed by libgwaoi.

Reference interface and the Python names that mirror it:

    aoi.AOI                       -> AOI            (embedded in Entity, Entity.go:55)
    aoi.InitAOI(aoi, dist, data, cb) -> init_aoi    (Entity.go:210)
    aoi.AOICallback{OnEnterAOI, OnLeaveAOI} -> AOICallback (Entity.go:227-233)
    aoi.AOIManager{Enter, Leave, Moved}     -> XZListAOIManager.enter/leave/moved
                                               (Space.go:211,221,243,259)
    aoi.NewXZListAOIManager(dist) -> AOIWorld.new_xzlist_aoi_manager
                                               (Space.go:105)

The one semantic difference, documented in DESIGN.md: go-aoi fires the
callbacks synchronously inside every Enter/Leave/Moved; here calls are queued
(in call order = seq order) and ``AOIWorld.flush()`` runs the GPU tick and
replays the NET per-flush diff -- leaves first, then enters, each pair as
(A.OnXxx(B), B.OnXxx(A)) like go-aoi's adjust.  Final interest sets equal the
sequential manager's.  Misuse that makes go-aoi panic
(Moved/Leave of an AOI that never entered, Enter twice) raises AOIError at
the call, like the reference's panic.

Slots: the C ABI names entities by u32 slot (cgo may not keep Go pointers).
An AOI keeps its slot while it is in a space; a slot released by Leave is
only reused after the next flush, so every event of a flush names exactly
one AOI.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Protocol

import numpy as np

from ._lib import GwaoiError, World


class AOIError(RuntimeError):
    """Misuse the reference would panic on (go-aoi / Space.go gwlog.Panicf)."""


class AOICallback(Protocol):
    def on_enter_aoi(self, other: "AOI") -> None: ...

    def on_leave_aoi(self, other: "AOI") -> None: ...


class AOI:
    """Per-entity AOI record (go-aoi ``AOI``): coordinates, distance, user data
    (GoWorld stores the *Entity, Entity.go:228) and the callback."""

    __slots__ = ("x", "y", "dist", "data", "callback", "_slot", "_mgr")

    def __init__(self):
        self.x = np.float32(0.0)
        self.y = np.float32(0.0)  # world Z (GoWorld passes pos.Z as y)
        self.dist = np.float32(0.0)
        self.data = None
        self.callback: Optional[AOICallback] = None
        self._slot = -1
        self._mgr: Optional["XZListAOIManager"] = None

    @property
    def slot(self) -> int:
        return self._slot


def init_aoi(aoi: AOI, dist, data, callback: AOICallback) -> None:
    """go-aoi InitAOI (Entity.go:210).  The XZ-list manager uses its own
    distance; the per-AOI one is stored and otherwise ignored, as in go-aoi."""
    aoi.dist = np.float32(dist)
    aoi.data = data
    aoi.callback = callback


_ENTER, _LEAVE, _MOVED = 1, 2, 0


class AOIWorld:
    """All AOI managers of one process on one GPU (one libgwaoi world).

    GoWorld has one manager per space (Space.go:33); each
    ``new_xzlist_aoi_manager`` is one space of this world, and one flush
    computes every space at once.
    """

    def __init__(self, max_entities: int, max_spaces: int = 1, device: int = -1, **kw):
        self.world = World(max_entities, max_spaces=max_spaces, device=device, **kw)
        self.max_entities = max_entities
        self._by_slot: List[Optional[AOI]] = [None] * max_entities
        self._free = list(range(max_entities - 1, -1, -1))
        self._quarantine: List[int] = []
        # op log in call order: runs are submitted as batches at flush
        self._kind: List[int] = []
        self._slot: List[int] = []
        self._x: List[float] = []
        self._z: List[float] = []
        self._space: List[int] = []

    def close(self):
        self.world.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def new_xzlist_aoi_manager(self, dist) -> "XZListAOIManager":
        """go-aoi NewXZListAOIManager(dist) (Space.go:105)."""
        if not np.float32(dist) > 0:
            raise AOIError(f"aoi distance must be > 0, got {dist}")  # Space.go:92 panics likewise
        return XZListAOIManager(self, self.world.space_create(np.float32(dist)), np.float32(dist))

    # ---- op queue
    def _log(self, kind, slot, x, z, space):
        self._kind.append(kind)
        self._slot.append(slot)
        self._x.append(x)
        self._z.append(z)
        self._space.append(space)

    def _submit(self):
        """Hand the queued calls to the C ABI in call order, as batches of runs."""
        kind = self._kind
        n = len(kind)
        i = 0
        W = self.world
        while i < n:
            k, sp = kind[i], self._space[i]
            j = i + 1
            while j < n and kind[j] == k and (k != _ENTER or self._space[j] == sp):
                j += 1
            sl = np.asarray(self._slot[i:j], np.uint32)
            if k == _MOVED:
                W.moved_batch(sl, np.asarray(self._x[i:j], np.float32), np.asarray(self._z[i:j], np.float32))
            elif k == _ENTER:
                W.enter_batch(sp, sl, np.asarray(self._x[i:j], np.float32), np.asarray(self._z[i:j], np.float32))
            else:
                W.leave_batch(sl)
            i = j
        self._kind, self._slot, self._x, self._z, self._space = [], [], [], [], []

    def flush(self):
        """Run the tick and replay the net callbacks.  Returns (n_enter, n_leave)
        directed events."""
        self._submit()
        err = None
        try:
            ent, lev = self.world.tick()
        except GwaoiError as e:  # committed with a dropped op: replay the events, then report
            if e.events is None:
                raise
            ent, lev = e.events
            err = e
        by = self._by_slot
        for a, b in lev.tolist():
            A = by[a]
            A.callback.on_leave_aoi(by[b])
        for a, b in ent.tolist():
            A = by[a]
            A.callback.on_enter_aoi(by[b])
        for s in self._quarantine:
            A = by[s]
            if A is not None and A._mgr is None and A._slot == s:  # still out of every space
                A._slot = -1
                by[s] = None
                self._free.append(s)
        self._quarantine = []
        if err is not None:
            raise err
        return len(ent), len(lev)

    def neighbors(self, aoi: AOI) -> List[AOI]:
        """Current neighbour set of `aoi` as of the last flush (debug/parity)."""
        if aoi._slot < 0:
            return []
        return [self._by_slot[s] for s in self.world.neighbors(aoi._slot).tolist()]


class XZListAOIManager:
    """go-aoi AOIManager for one space (Enter / Leave / Moved)."""

    def __init__(self, world: AOIWorld, space: int, dist):
        self._w = world
        self.space = space
        self.dist = dist

    def enter(self, aoi: AOI, x, y) -> None:
        """Space.go:211,221 -- aoiMgr.Enter(&entity.aoi, pos.X, pos.Z)."""
        if aoi._mgr is not None:
            raise AOIError("Enter of an AOI that is already in a space")
        x, y = np.float32(x), np.float32(y)
        if not (np.isfinite(x) and np.isfinite(y)):
            raise AOIError("non-finite coordinate")
        W = self._w
        if aoi._slot < 0:
            if not W._free:
                raise AOIError("no free AOI slot (raise max_entities)")
            aoi._slot = W._free.pop()
            W._by_slot[aoi._slot] = aoi
        aoi._mgr = self
        aoi.x, aoi.y = x, y
        W._log(_ENTER, aoi._slot, x, y, self.space)

    def leave(self, aoi: AOI) -> None:
        """Space.go:243 -- aoiMgr.Leave(&entity.aoi)."""
        if aoi._mgr is not self:
            raise AOIError("Leave of an AOI that is not in this space")
        aoi._mgr = None
        W = self._w
        W._log(_LEAVE, aoi._slot, 0.0, 0.0, self.space)
        # the slot stays bound to this AOI until the flush has replayed its
        # leaves; a re-Enter before then keeps it (leave + enter in one flush)
        W._quarantine.append(aoi._slot)

    def moved(self, aoi: AOI, x, y) -> None:
        """Space.go:259 -- aoiMgr.Moved(&entity.aoi, pos.X, pos.Z)."""
        if aoi._mgr is not self:
            raise AOIError("Moved of an AOI that is not in this space")
        x, y = np.float32(x), np.float32(y)
        if not (np.isfinite(x) and np.isfinite(y)):
            raise AOIError("non-finite coordinate")
        aoi.x, aoi.y = x, y
        self._w._log(_MOVED, aoi._slot, x, y, self.space)

    def flush(self):
        """Flush the whole world (all spaces share one GPU tick)."""
        return self._w.flush()

    def close(self):
        self._w.world.space_destroy(self.space)


class EntityInterest:
    """The reference consumer of the callbacks: Entity.OnEnterAOI/OnLeaveAOI ->
    interest/uninterest (Entity.go:227-246) over EntitySets (entity_map.go:44-66).
    ``interested_in`` == the AOI neighbour set; ``interested_by`` mirrors it."""

    __slots__ = ("id", "aoi", "interested_in", "interested_by")

    def __init__(self, eid, dist):
        self.id = eid
        self.aoi = AOI()
        self.interested_in = set()
        self.interested_by = set()
        init_aoi(self.aoi, dist, self, self)

    def on_enter_aoi(self, other: AOI) -> None:
        o = other.data
        self.interested_in.add(o)
        o.interested_by.add(self)

    def on_leave_aoi(self, other: AOI) -> None:
        o = other.data
        self.interested_in.discard(o)
        o.interested_by.discard(self)


__all__ = ["AOI", "AOICallback", "AOIError", "AOIWorld", "EntityInterest", "GwaoiError", "XZListAOIManager",
           "init_aoi"]
