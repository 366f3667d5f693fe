/*
 * gwaoi_sync.h -- entity position sync on the GPU: the callers either side of
 * the AOI path, on the same world and
 * stream as gwaoi.h.
 *
 *   reference (file:line, /root/reference)                      replaced by
 *   ------------------------------------------------------     ------------------------------------
 *   GameService.HandleSyncPositionYawFromClient                 gwaoi_sync_from_clients(_device)
 *     components/game/GameService.go:392-404  (32-B records:
 *     EntityID[16] + x,y,z,yaw float32 little-endian)
 *   entity.OnSyncPositionYawFromClient  EntityManager.go:484-493 (ID lookup; unknown IDs are skipped)
 *   Entity.syncPositionYawFromClient    Entity.go:430-435       (only if SetClientSyncing(true))
 *   Entity.SetClientSyncing             Entity.go:437-440       gwaoi_entity_set_syncing
 *   Entity.setPositionYaw / SetPosition Entity.go:1185-1205     gwaoi_set_position_yaw
 *   Space.enter / Space.leave without AOI (no EnableAOI, or IsUseAOI false)
 *     Space.go:188-251                                        gwaoi_entity_enter_plain / _leave_plain
 *   CollectEntitySyncInfos              Entity.go:1221-1267     gwaoi_collect_sync_infos(_device)
 *     (per-gate MT_SYNC_POSITION_YAW_ON_CLIENTS payloads of 48-B records:
 *      ClientID[16] + EntityID[16] + x,y,z,yaw float32)
 *   Entity.interest / uninterest -> GameClient.sendCreateEntity / sendDestroyEntity
 *     Entity.go:236-246, GameClient.go:37-59                    gwaoi_collect_client_events
 *
 * Entity ids and client ids are the reference's 16-byte strings
 * (common.ENTITYID_LENGTH = common.CLIENTID_LENGTH = uuid.UUID_LENGTH = 16,
 * engine/common/types.go:9,46).  The world keeps, per slot: the entity id
 * (device hash table id -> slot, for the packet decode), the client
 * (gate id + client id, or none), the syncing-from-client flag, the last
 * synced position and yaw (AOI itself uses X/Z only), and the sync flags
 * (sifSyncOwnClient / sifSyncNeighborClients, Entity.go:1198-1203).
 *
 * Ordering.  Sync calls share the world's call order: a decoded packet is a
 * device Moved batch queued after everything before it; the last write of a
 * slot's Y/yaw wins exactly as the sequential calls would leave it.
 * gwaoi_collect_* read the state of the last flush (gwaoi_tick*): call them
 * with no queued op (GWAOI_ESTATE otherwise), as GoWorld does (the collect
 * runs after the position packets of the tick have been handled,
 * GameService.go:171-183).
 *
 * Records of one gate come in an unspecified order (the reference iterates Go
 * maps); the multiset per gate is exact.
 */
#ifndef GWAOI_SYNC_H
#define GWAOI_SYNC_H

#include <stddef.h>
#include <stdint.h>

#include "gwaoi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GWAOI_ID_LEN 16          /* EntityID / ClientID bytes                                   */
#define GWAOI_SYNC_IN_REC 32     /* client -> game record: EntityID + x,y,z,yaw                 */
#define GWAOI_SYNC_OUT_REC 48    /* game -> gate record: ClientID + EntityID + x,y,z,yaw        */
#define GWAOI_DESTROY_REC 32     /* game -> gate destroy record: ClientID + EntityID            */
#define GWAOI_MAX_GATES 1024     /* distinct gate ids a world may route to                      */

#define GWAOI_SIF_OWN_CLIENT 1u       /* sifSyncOwnClient       */
#define GWAOI_SIF_NEIGHBOR_CLIENTS 2u /* sifSyncNeighborClients */

/* Per-gate output of a collect: gate g (id gate_ids[g]) owns records
 * [offsets[g], offsets[g+1]).  Host pointers are world-owned and valid until
 * the next collect of the same kind; `records` is host memory for
 * gwaoi_collect_sync_infos and device memory for the _device form. */
typedef struct {
    uint32_t n_gates;
    const uint16_t *gate_ids;
    const uint64_t *offsets;   /* n_gates + 1 entries, in records */
    const uint8_t *records;    /* offsets[n_gates] * record bytes */
} gwaoi_gate_records;

/* ---- per-entity state ---------------------------------------------------- */
/* Bind a slot to its entity id (entity creation).  GWAOI_ESTATE if the id is
 * bound to another slot or the slot to another id. */
int gwaoi_entity_bind(gwaoi_world *w, uint32_t slot, const uint8_t eid[GWAOI_ID_LEN]);
int gwaoi_entity_bind_batch(gwaoi_world *w, const uint32_t *slots, const uint8_t *eids, size_t n);
/* Drop the id of a slot (entity destroyed); also clears its client. */
int gwaoi_entity_unbind(gwaoi_world *w, uint32_t slot);
/* Entity.SetClient: gate id + client id; clientid == NULL clears the client. */
int gwaoi_entity_set_client(gwaoi_world *w, uint32_t slot, uint16_t gate_id, const uint8_t *clientid);
/* Entity.SetClientSyncing. */
int gwaoi_entity_set_syncing(gwaoi_world *w, uint32_t slot, int syncing);
/* Position and yaw of a slot as the sync records report them, without a
 * Moved call or a sync flag (entity creation; before gwaoi_enter, which sets
 * both sync flags as Space.enter does, Space.go:203-205). */
int gwaoi_entity_set_position_yaw(gwaoi_world *w, uint32_t slot, float x, float y, float z, float yaw);

/* Space.enter of a space without AOI (EnableAOI never called), or of an
 * entity type without AOI (IsUseAOI false, Space.go:210): Position = (x,y,z)
 * and both sync flags (Space.go:201-205), no AOI call; the entity has no AOI
 * neighbours there.  GWAOI_ESTATE unless the slot is in nilSpace (neither in
 * an AOI space nor in another space without AOI: Space.go:193-195 panics).
 * gwaoi_enter of a slot in such a space is GWAOI_ESTATE too. */
int gwaoi_entity_enter_plain(gwaoi_world *w, uint32_t slot, float x, float y, float z);
/* Space.leave of that space: back to nilSpace (GWAOI_ESTATE if not in one). */
int gwaoi_entity_leave_plain(gwaoi_world *w, uint32_t slot);

/* ---- moves ---------------------------------------------------------------- */
/* Entity.setPositionYaw(pos, yaw, fromClient=false) (server-side move).  A
 * created entity is never in a nil space: outside every space it is in
 * nilSpace (EntityManager.go:250,293; Space.go:240), so Space.move always
 * runs.  In an AOI space: a Moved(x, z) plus Position and yaw.  In nilSpace
 * or a space without AOI, Space.move returns before Position
 * (Space.go:253-257): only yaw changes.  Both sync flags either way; the
 * own-client record then carries the stale Position with the new yaw. */
int gwaoi_set_position_yaw(gwaoi_world *w, uint32_t slot, float x, float y, float z, float yaw);

/* HandleSyncPositionYawFromClient: decode n_rec 32-B records (host memory)
 * on the GPU into one device Moved batch, in record order.  Records whose
 * id is unknown or whose entity is not syncing from its client are skipped
 * silently, as in the reference.  The others are setPositionYaw(fromClient):
 * in an AOI space a Moved plus Position and yaw, elsewhere yaw only (as
 * above); every applied record raises sifSyncNeighborClients. */
int gwaoi_sync_from_clients(gwaoi_world *w, const uint8_t *payload, size_t n_rec);
/* Same, payload already in device memory of the world's GPU (16-B aligned);
 * it must stay valid until the next gwaoi_tick*. */
int gwaoi_sync_from_clients_device(gwaoi_world *w, const uint8_t *d_payload, size_t n_rec);

/* ---- collect ---------------------------------------------------------------- */
/* CollectEntitySyncInfos: for every flagged entity, a record to its own
 * client (sifSyncOwnClient) and to the client of every entity interested in
 * it (sifSyncNeighborClients, the go-aoi relation of the last flush); then
 * clears every flag.  Records go to host memory. */
int gwaoi_collect_sync_infos(gwaoi_world *w, gwaoi_gate_records *out);
/* Same; records stay in device memory. */
int gwaoi_collect_sync_infos_device(gwaoi_world *w, gwaoi_gate_records *out);
/* The last flush's events routed to clients: enter (a,b) with a client on a
 * -> create record (a's ClientID, b's EntityID, b's x,y,z,yaw: 48 B);
 * leave (a,b) -> destroy record (a's ClientID, b's EntityID: 32 B).  The
 * caller adds type name and client data per record (GameClient.go:37-53).
 * Host memory. */
int gwaoi_collect_client_events(gwaoi_world *w, gwaoi_gate_records *creates, gwaoi_gate_records *destroys);

#ifdef __cplusplus
}
#endif

#endif /* GWAOI_SYNC_H */
