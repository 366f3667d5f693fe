"""CPU restatement of GoWorld's entity position sync -- TEST INFRASTRUCTURE ONLY.

Only tests/ and bench.py's cpu_baseline leg may use this module, and only as
the checker, never as a product path.  It drives the sequential go-aoi
restatement (oracle.SpacesOracle) the way GoWorld's entity layer does and
restates, in plain Python:

* ``handle_sync_packet``   GameService.HandleSyncPositionYawFromClient
  (components/game/GameService.go:392-404): 32-byte records
  ``EntityID[16] + x,y,z,yaw`` float32 little-endian (netutil.NETWORK_ENDIAN
  = binary.LittleEndian, engine/netutil/PacketConnection.go:31), each one
  ``entity.OnSyncPositionYawFromClient`` (engine/entity/EntityManager.go:484-493):
  unknown id -> skipped; ``Entity.syncPositionYawFromClient`` (Entity.go:430-435):
  only while syncing from the client.
* ``set_position_yaw``      Entity.setPositionYaw (Entity.go:1189-1205):
  Space.move (Space.go:253-261) -> Position + Moved only in a space with an
  AOI manager; yaw and the flags sifSyncNeighborClients (+ sifSyncOwnClient
  unless from the client) in every case.  An entity outside every space is in
  nilSpace (``entity.Space = nilSpace``, EntityManager.go:250,293 and
  Space.go:240), never nil, so the early return of Entity.go:1191-1194 is not
  taken: in nilSpace and in a space without AOI, Position stays stale while
  yaw and the flags change.
* ``enter_plain_space``     Space.enter (Space.go:188-226) of a space without
  AOI (EnableAOI never called) or of an entity type without AOI
  (IsUseAOI false): Position and both flags, no AOI call.
* ``collect``               CollectEntitySyncInfos (Entity.go:1221-1267): per
  flagged entity, a 48-byte record ``ClientID + EntityID + x,y,z,yaw`` to its
  own client (sifSyncOwnClient) and to the client of every entity in its
  InterestedBy set (sifSyncNeighborClients), per gate; flags cleared.
* AOI callbacks             Entity.OnEnterAOI/OnLeaveAOI -> interest/uninterest
  (Entity.go:227-246): InterestedIn/InterestedBy, and the client create /
  destroy messages of GameClient.sendCreateEntity/sendDestroyEntity
  (GameClient.go:37-59), logged as records per gate.

Records are compared as sorted multisets per gate: the reference iterates Go
maps, so their order is unspecified.
"""
from __future__ import annotations

import struct

import numpy as np

from .oracle import EV_ENTER, EV_LEAVE, SpacesOracle

SIF_OWN, SIF_NEIGHBOR = 1, 2


class Ent:
    __slots__ = ("eid", "slot", "space", "aoi", "x", "y", "z", "yaw", "gate", "cid", "syncing", "flags", "In", "By")

    def __init__(self, eid: bytes, slot: int):
        self.eid, self.slot = eid, slot
        self.space = None
        self.x = self.y = self.z = self.yaw = np.float32(0)
        self.aoi = False  # space (if any) has an AOI manager and the entity uses AOI
        self.gate, self.cid = None, None
        self.syncing = False
        self.flags = 0
        self.In, self.By = set(), set()


def f32(v) -> np.float32:
    return np.float32(v)


class GameEntities:
    """Entities of one game process over the sequential AOI oracle."""

    def __init__(self, D_by_space, max_slots: int):
        self.aoi = SpacesOracle(D_by_space, max_slots)
        self.by_eid: dict[bytes, Ent] = {}
        self.by_slot: dict[int, Ent] = {}
        self.creates: dict[int, list] = {}   # gate -> [48-byte create records], callback order
        self.destroys: dict[int, list] = {}  # gate -> [32-byte destroy records]
        self.raw: list = []                  # (type, a, b, space) callbacks since take_raw()

    # ---- entity table
    def create(self, eid: bytes, slot: int, x=0.0, y=0.0, z=0.0, yaw=0.0):
        e = Ent(eid, slot)
        e.x, e.y, e.z, e.yaw = f32(x), f32(y), f32(z), f32(yaw)
        self.by_eid[eid] = e
        self.by_slot[slot] = e
        return e

    def set_client(self, slot, gate=None, cid=None):
        e = self.by_slot[slot]
        e.gate, e.cid = (None, None) if cid is None else (int(gate), bytes(cid))

    def set_syncing(self, slot, syncing=True):
        self.by_slot[slot].syncing = bool(syncing)

    def set_position_yaw_noflags(self, slot, x, y, z, yaw):
        e = self.by_slot[slot]
        e.x, e.y, e.z, e.yaw = f32(x), f32(y), f32(z), f32(yaw)

    # ---- AOI callbacks (Entity.go:227-246)
    def _replay(self):
        t, a, b, sp = self.aoi.take_events(with_space=True)
        if t.size:
            self.raw.append((t, a, b, sp))
        for k in range(t.size):
            ea, eb = self.by_slot[int(a[k])], self.by_slot[int(b[k])]
            if t[k] == EV_ENTER:
                ea.In.add(eb.slot)
                eb.By.add(ea.slot)
                if ea.cid is not None:
                    self.creates.setdefault(ea.gate, []).append(
                        ea.cid + eb.eid + struct.pack("<4f", eb.x, eb.y, eb.z, eb.yaw))
            else:
                ea.In.discard(eb.slot)
                eb.By.discard(ea.slot)
                if ea.cid is not None:
                    self.destroys.setdefault(ea.gate, []).append(ea.cid + eb.eid)

    # ---- Space.enter / leave / move (Space.go:188-261)
    def enter_space(self, slot, sp, x, y, z):
        """Space.enter (Space.go:188-226): Position, both sync flags, Enter."""
        e = self.by_slot[slot]
        assert e.space is None, "Space.enter: entity not in nilSpace (Space.go:193-195 panics)"
        e.space, e.aoi = sp, True
        e.x, e.y, e.z = f32(x), f32(y), f32(z)
        e.flags |= SIF_OWN | SIF_NEIGHBOR
        self.aoi.enter(sp, slot, e.x, e.z)
        self._replay()

    def enter_plain_space(self, slot, sp, x, y, z):
        """Space.enter (Space.go:188-226) without an AOI call: the space has no
        AOI manager, or the entity type does not use AOI (Space.go:210)."""
        e = self.by_slot[slot]
        assert e.space is None, "Space.enter: entity not in nilSpace (Space.go:193-195 panics)"
        e.space, e.aoi = ("plain", sp), False
        e.x, e.y, e.z = f32(x), f32(y), f32(z)
        e.flags |= SIF_OWN | SIF_NEIGHBOR

    def leave_space(self, slot):
        """Space.leave (Space.go:228-251): back to nilSpace; Leave only with AOI (Space.go:242)."""
        e = self.by_slot[slot]
        if e.aoi:
            self.aoi.leave(slot)
        e.space, e.aoi = None, False
        self._replay()

    def set_position_yaw(self, slot, x, y, z, yaw, from_client=False):
        """Entity.setPositionYaw (Entity.go:1189-1205).  e.Space is never nil
        for a created entity (nilSpace), so every call reaches Space.move, which
        returns before touching Position when the space has no AOI manager
        (Space.go:253-257): only then are Position and the AOI relation updated."""
        e = self.by_slot[slot]
        if e.aoi:
            e.x, e.y, e.z = f32(x), f32(y), f32(z)
            self.aoi.moved(slot, e.x, e.z)
            self._replay()
        e.yaw = f32(yaw)
        e.flags |= SIF_NEIGHBOR
        if not from_client:
            e.flags |= SIF_OWN
        return True

    def handle_sync_packet(self, payload: bytes):
        """HandleSyncPositionYawFromClient (GameService.go:392-404)."""
        for i in range(0, len(payload), 32):
            eid = bytes(payload[i:i + 16])
            x, y, z, yaw = struct.unpack("<4f", payload[i + 16:i + 32])
            e = self.by_eid.get(eid)          # EntityManager.go:485-490
            if e is None or not e.syncing:    # Entity.go:432
                continue
            self.set_position_yaw(e.slot, x, y, z, yaw, from_client=True)

    def collect(self) -> dict:
        """CollectEntitySyncInfos (Entity.go:1221-1267): {gate: sorted list of 48-byte records}."""
        out: dict[int, list] = {}
        for e in self.by_eid.values():
            fl = e.flags
            if not fl:
                continue
            e.flags = 0
            info = struct.pack("<4f", e.x, e.y, e.z, e.yaw)
            if fl & SIF_OWN and e.cid is not None:
                out.setdefault(e.gate, []).append(e.cid + e.eid + info)
            if fl & SIF_NEIGHBOR:
                for s in e.By:
                    n = self.by_slot[s]
                    if n.cid is not None:
                        out.setdefault(n.gate, []).append(n.cid + e.eid + info)
        return {g: sorted(v) for g, v in out.items()}

    def take_raw(self):
        """(type, a, b, space) arrays of every callback since the last call."""
        r, self.raw = self.raw, []
        if not r:
            return (np.empty(0, np.uint8), np.empty(0, np.int32), np.empty(0, np.int32),
                    np.empty(0, np.int64))
        return tuple(np.concatenate([x[i] for x in r]) for i in range(4))

    def net_client_events(self, t, a, b, sp=None):
        """Client messages of a flush's NET diff at the flush's final state (the GPU
        path's granularity): ({gate: sorted create records}, {gate: sorted destroy records})."""
        from .oracle import net_events
        ent, lev = net_events(t, a, b, sp)
        cre, des = {}, {}
        for k in ent:
            ea, eb = self.by_slot[int(k >> np.uint64(32))], self.by_slot[int(k & np.uint64(0xFFFFFFFF))]
            if ea.cid is not None:
                cre.setdefault(ea.gate, []).append(ea.cid + eb.eid + struct.pack("<4f", eb.x, eb.y, eb.z, eb.yaw))
        for k in lev:
            ea, eb = self.by_slot[int(k >> np.uint64(32))], self.by_slot[int(k & np.uint64(0xFFFFFFFF))]
            if ea.cid is not None:
                des.setdefault(ea.gate, []).append(ea.cid + eb.eid)
        return {g: sorted(v) for g, v in cre.items()}, {g: sorted(v) for g, v in des.items()}

    def take_client_events(self):
        c, d = self.creates, self.destroys
        self.creates, self.destroys = {}, {}
        return c, d


def records_by_gate(d: dict) -> dict:
    """{gate: (n,R) uint8 array} (library output) -> {gate: sorted list of bytes}, empty gates dropped."""
    out = {}
    for g, a in d.items():
        rows = sorted(bytes(r) for r in np.asarray(a))
        if rows:
            out[int(g)] = rows
    return out
