/*
 * gwaoi_wire.h -- the position-sync wire path between GoWorld's gate,
 * dispatcher and game processes, regrouped on the GPU.
 *
 * Three byte regroups of the per-tick sync records, each replacing one
 * reference handler:
 *
 *   gwaoi_wire_gate_from_clients   GateService.handleSyncPositionYawFromClient
 *                                  + tryFlushPendingSyncPackets
 *                                  (components/gate/GateService.go:398-425)
 *   gwaoi_wire_dispatcher_to_games DispatcherService.handleSyncPositionYawFromClient
 *                                  + sendEntitySyncInfosToGames
 *                                  (components/dispatcher/DispatcherService.go:786-825)
 *   gwaoi_wire_gate_to_clients     GateService.handleSyncPositionYawOnClients
 *                                  (components/gate/GateService.go:346-371)
 *
 * Records (little-endian, netutil.NETWORK_ENDIAN):
 *   from clients / to games:  EntityID[16] | x, y, z, yaw float32      32 B
 *   on clients (game output): ClientID[16] | EntityID[16] | x,y,z,yaw  48 B
 *                             (gwaoi_collect_sync_infos' records, gwaoi_sync.h)
 *   to one client:            EntityID[16] | x, y, z, yaw              32 B
 *
 * Every regroup is stable: inside a destination, records keep their arrival
 * order (the reference appends to one packet per destination).  Destinations
 * come out in increasing key order (the reference iterates a Go map: any
 * order).  Records whose destination is unknown are dropped and counted, as
 * the reference drops them.
 *
 * One handle per process side (a gate or a dispatcher), on one device and
 * one HIP stream; not thread-safe.  Every call returns GWAOI_OK or a negative
 * gwaoi_status (gwaoi.h) and never aborts.
 */
#ifndef GWAOI_WIRE_H
#define GWAOI_WIRE_H

#include "gwaoi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gwaoi_wire gwaoi_wire;

/* One regroup's output, valid until the next regroup call on the handle.
 * Group k: destination keys[k], records [offsets[k], offsets[k+1]) of
 * `records` (rec_bytes each).  keys/offsets are host arrays; records are
 * device memory for the _device calls, host memory otherwise. */
typedef struct {
    uint32_t n_groups;
    const uint32_t *keys;
    const uint64_t *offsets; /* n_groups + 1 */
    const uint8_t *records;
    uint32_t rec_bytes;
    uint64_t n_dropped;      /* records with an unknown destination */
} gwaoi_wire_groups;

int gwaoi_wire_create(int device, gwaoi_wire **out);
void gwaoi_wire_destroy(gwaoi_wire *w);
const char *gwaoi_wire_last_error(gwaoi_wire *w);

/* Dispatcher side: entityDispatchInfos[eid].gameid (DispatcherService.go),
 * set (insert or overwrite) / removed for n 16-byte entity ids. */
int gwaoi_wire_set_entity_games(gwaoi_wire *w, const uint8_t *entity_ids, const uint16_t *game_ids, size_t n);
int gwaoi_wire_remove_entities(gwaoi_wire *w, const uint8_t *entity_ids, size_t n);

/* Gate side: gs.clientProxies (GateService.go): connected clients, each with
 * the caller's index of its proxy (the group key of gate_to_clients). */
int gwaoi_wire_set_clients(gwaoi_wire *w, const uint8_t *client_ids, const uint32_t *client_index, size_t n);
int gwaoi_wire_remove_clients(gwaoi_wire *w, const uint8_t *client_ids, size_t n);

/* Gate: n client records (32 B) -> one group per dispatcher id
 * (EntityIDToDispatcherID: (id[14]*256 + id[15]) % n_dispatchers + 1,
 * engine/dispatchercluster/hash.go:7-12, dispatchercluster.go:108-110). */
int gwaoi_wire_gate_from_clients(gwaoi_wire *w, const uint8_t *records, size_t n, uint32_t n_dispatchers,
                                 gwaoi_wire_groups *out);
int gwaoi_wire_gate_from_clients_device(gwaoi_wire *w, const uint8_t *d_records, size_t n, uint32_t n_dispatchers,
                                        gwaoi_wire_groups *out);

/* Dispatcher: n records (32 B) -> one group per game id; entities without a
 * game (no dispatch info) are dropped. */
int gwaoi_wire_dispatcher_to_games(gwaoi_wire *w, const uint8_t *records, size_t n, gwaoi_wire_groups *out);
int gwaoi_wire_dispatcher_to_games_device(gwaoi_wire *w, const uint8_t *d_records, size_t n,
                                          gwaoi_wire_groups *out);

/* Gate: n records on clients (48 B) -> one group of 32-B records per
 * connected client (key = its client_index); unknown clients are dropped. */
int gwaoi_wire_gate_to_clients(gwaoi_wire *w, const uint8_t *records, size_t n, gwaoi_wire_groups *out);
int gwaoi_wire_gate_to_clients_device(gwaoi_wire *w, const uint8_t *d_records, size_t n, gwaoi_wire_groups *out);

#ifdef __cplusplus
}
#endif

#endif /* GWAOI_WIRE_H */
