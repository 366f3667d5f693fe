/*
 * oracle/wire_host.c -- CPU BASELINE ONLY (bench.py's wire_leg; tests pin it
 * against oracle/wire.py).  The gate / dispatcher position-sync regroups of
 * GoWorld restated as a plain single-threaded C host loop, the comparator for
 * the GPU regroups of include/gwaoi_wire.h:
 *
 *   wh_gate_from_clients   GateService.handleSyncPositionYawFromClient +
 *                          tryFlushPendingSyncPackets (GateService.go:398-425):
 *                          32-B client records grouped by dispatcher
 *                          (id[14]*256 + id[15]) % n + 1 (dispatchercluster/hash.go:7-12)
 *   wh_dispatcher_to_games DispatcherService.handleSyncPositionYawFromClient +
 *                          sendEntitySyncInfosToGames (DispatcherService.go:786-825):
 *                          32-B records grouped by the entity's game (a map
 *                          lookup of the 16-B id); unknown entities dropped
 *   wh_gate_to_clients     GateService.handleSyncPositionYawOnClients
 *                          (GateService.go:346-371): 48-B records [client id |
 *                          entity id | x y z yaw] -> 32-B records per connected
 *                          client (a map lookup of the client id); unknown dropped
 *
 * Each regroup is the reference's "append to the destination's packet" as a
 * stable two-pass counting regroup over dense destination keys: pass 1 keys and
 * counts, a prefix sum, pass 2 copies.  Outputs: keys[] of the non-empty
 * destinations in key order, off[ngroups+1] (records), out = records grouped.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint8_t *keys; /* 16 B per bucket */
    uint32_t *vals; /* 0xFFFFFFFF = empty */
    uint64_t mask;
} whmap;

static uint64_t h16(const uint8_t *k) {
    uint64_t a, b;
    memcpy(&a, k, 8);
    memcpy(&b, k + 8, 8);
    uint64_t z = a ^ (b * 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void *wh_map_new(int64_t n, const uint8_t *ids, const uint32_t *vals) {
    whmap *m = (whmap *)calloc(1, sizeof(whmap));
    uint64_t cap = 1024;
    while (cap < 2 * (uint64_t)n) cap <<= 1;
    m->mask = cap - 1;
    m->keys = (uint8_t *)malloc(cap * 16);
    m->vals = (uint32_t *)malloc(cap * 4);
    memset(m->vals, 0xFF, cap * 4);
    for (int64_t i = 0; i < n; i++) {
        uint64_t h = h16(ids + 16 * i) & m->mask;
        while (m->vals[h] != 0xFFFFFFFFu && memcmp(m->keys + 16 * h, ids + 16 * i, 16)) h = (h + 1) & m->mask;
        memcpy(m->keys + 16 * h, ids + 16 * i, 16);
        m->vals[h] = vals[i];
    }
    return m;
}

void wh_map_free(void *p) {
    whmap *m = (whmap *)p;
    if (!m) return;
    free(m->keys);
    free(m->vals);
    free(m);
}

static uint32_t map_get(const whmap *m, const uint8_t *k) {
    uint64_t h = h16(k) & m->mask;
    while (m->vals[h] != 0xFFFFFFFFu) {
        if (!memcmp(m->keys + 16 * h, k, 16)) return m->vals[h];
        h = (h + 1) & m->mask;
    }
    return 0xFFFFFFFFu;
}

/* regroup n records of rec_in bytes by dest[i] (0xFFFFFFFF = dropped) into
 * rec_out-byte records (the last rec_out bytes of each input record) */
static int64_t regroup(const uint8_t *in, int64_t n, size_t rec_in, size_t rec_out, const uint32_t *dest,
                       uint32_t max_key, uint32_t *keys, uint64_t *off, uint8_t *out) {
    uint64_t *cnt = (uint64_t *)calloc((size_t)max_key + 2, sizeof(uint64_t));
    for (int64_t i = 0; i < n; i++)
        if (dest[i] != 0xFFFFFFFFu) cnt[dest[i]]++;
    int64_t g = 0;
    uint64_t run = 0;
    for (uint32_t k = 0; k <= max_key; k++) {
        const uint64_t c = cnt[k];
        cnt[k] = run;
        if (c) {
            keys[g] = k;
            off[g++] = run;
        }
        run += c;
    }
    off[g] = run;
    for (int64_t i = 0; i < n; i++) {
        const uint32_t d = dest[i];
        if (d == 0xFFFFFFFFu) continue;
        memcpy(out + rec_out * cnt[d]++, in + rec_in * i + (rec_in - rec_out), rec_out);
    }
    free(cnt);
    return g;
}

int64_t wh_gate_from_clients(const uint8_t *rec, int64_t n, uint32_t n_disp, uint32_t *keys, uint64_t *off,
                             uint8_t *out) {
    uint32_t *dest = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n ? n : 1));
    for (int64_t i = 0; i < n; i++) {
        const uint8_t *id = rec + 32 * i;
        dest[i] = ((uint32_t)id[14] * 256u + id[15]) % n_disp + 1u;
    }
    const int64_t g = regroup(rec, n, 32, 32, dest, n_disp, keys, off, out);
    free(dest);
    return g;
}

int64_t wh_dispatcher_to_games(const uint8_t *rec, int64_t n, const void *games, uint32_t max_game, uint32_t *keys,
                               uint64_t *off, uint8_t *out) {
    uint32_t *dest = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n ? n : 1));
    for (int64_t i = 0; i < n; i++) dest[i] = map_get((const whmap *)games, rec + 32 * i);
    const int64_t g = regroup(rec, n, 32, 32, dest, max_game, keys, off, out);
    free(dest);
    return g;
}

int64_t wh_gate_to_clients(const uint8_t *rec, int64_t n, const void *clients, uint32_t max_client, uint32_t *keys,
                           uint64_t *off, uint8_t *out) {
    uint32_t *dest = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n ? n : 1));
    for (int64_t i = 0; i < n; i++) dest[i] = map_get((const whmap *)clients, rec + 48 * i);
    const int64_t g = regroup(rec, n, 48, 32, dest, max_client, keys, off, out);
    free(dest);
    return g;
}
