"""CPU restatement of GoWorld's position-sync wire path between game, dispatcher
and gate -- TEST INFRASTRUCTURE ONLY.

Only tests/ may use this module, and only as the checker of the GPU regroup
kernels (goworld_amd/csrc/gwaoi_wire.hip, include/gwaoi_wire.h).  It restates,
in plain Python over bytes:

* ``gate_from_clients``     GateService.handleSyncPositionYawFromClient
  (components/gate/GateService.go:398-405) appends each client's record
  ``EntityID[16] + x,y,z,yaw`` (16 B, proto.SYNC_INFO_SIZE_PER_ENTITY,
  engine/proto/proto.go:137) to the pending packet of the entity's dispatcher,
  ``dispatchercluster.EntityIDToDispatcherID`` (dispatchercluster.go:108-110):
  ``(id[14]*256 + id[15]) % dispatcherNum + 1`` (dispatchercluster/hash.go:7-12);
  tryFlushPendingSyncPackets (GateService.go:407-425) sends every non-empty
  packet.  Records keep their arrival order inside a packet.
* ``dispatcher_to_games``   DispatcherService.handleSyncPositionYawFromClient
  (components/dispatcher/DispatcherService.go:786-811): each 32-B record goes
  to the pending packet of ``entityDispatchInfos[eid].gameid``; an entity
  without dispatch info is dropped (the Warnf branch); sendEntitySyncInfosToGames
  (:813-825) sends one packet per game.  Arrival order inside a packet.
* ``gate_to_clients``       GateService.handleSyncPositionYawOnClients
  (GateService.go:346-371): the game's 48-B records ``ClientID[16] +
  EntityID[16] + x,y,z,yaw`` are grouped by ClientID (``dispatch[clientid] =
  append(..., data...)``, arrival order inside a client) and each connected
  client (``gs.clientProxies[clientid] != nil``) gets one packet of its 32-B
  ``EntityID + x,y,z,yaw`` records; records of unknown clients are dropped.

Groups are returned as ``{destination: bytes}``; the reference iterates Go
maps, so the order of the groups is unspecified (only the order inside one).
"""
from __future__ import annotations

from typing import Dict, Mapping

ID = 16            # common.ENTITYID_LENGTH / CLIENTID_LENGTH (uuid)
SYNC = 16          # proto.SYNC_INFO_SIZE_PER_ENTITY: x, y, z, yaw float32
REC = ID + SYNC    # EntityID + sync info
REC_ON_CLIENTS = ID + ID + SYNC


def dispatcher_of(eid: bytes, n_dispatchers: int) -> int:
    """dispatchercluster.EntityIDToDispatcherID (dispatchercluster.go:108; hash.go:7-12)."""
    return (eid[14] * 256 + eid[15]) % n_dispatchers + 1


def gate_from_clients(payload: bytes, n_dispatchers: int) -> Dict[int, bytes]:
    out: Dict[int, bytearray] = {}
    for i in range(0, len(payload), REC):
        rec = payload[i:i + REC]
        out.setdefault(dispatcher_of(rec[:ID], n_dispatchers), bytearray()).extend(rec)
    return {k: bytes(v) for k, v in out.items()}


def dispatcher_to_games(payload: bytes, game_of: Mapping[bytes, int]) -> Dict[int, bytes]:
    out: Dict[int, bytearray] = {}
    for i in range(0, len(payload), REC):
        rec = payload[i:i + REC]
        g = game_of.get(rec[:ID])
        if g is None:  # "synced from client, but dispatch info is not found"
            continue
        out.setdefault(g, bytearray()).extend(rec)
    return {k: bytes(v) for k, v in out.items()}


def gate_to_clients(payload: bytes, connected: Mapping[bytes, int]) -> Dict[int, bytes]:
    """connected: ClientID -> the caller's index of that client proxy."""
    dispatch: Dict[bytes, bytearray] = {}
    for i in range(0, len(payload), REC_ON_CLIENTS):
        cid = payload[i:i + ID]
        dispatch.setdefault(cid, bytearray()).extend(payload[i + ID:i + REC_ON_CLIENTS])
    return {connected[c]: bytes(d) for c, d in dispatch.items() if c in connected}
