/*
 * gwaoi_strips.h -- one x-strip of a single oversized space, tiled over
 * several GPUs (BASELINE config 5; SURVEY.md §8e "Partitioning (config 5)").
 *
 * GoWorld gives every Space exactly one AOI manager (engine/entity/Space.go:33,
 * :105).  A space too large for one GPU is cut into x-strips; strip r owns
 * the entities with x in [edges[r-1], edges[r]).  Each rank runs a normal
 * gwaoi world (include/gwaoi.h) that holds its owned entities plus the
 * ghosts within the halo H of its strip, fed with the GLOBAL call order as
 * explicit seqs (gwaoi_*_seq), and keeps only the events its strip owns:
 *
 *   enter (a,b) -- kept by the rank owning a after the tick,
 *   leave (a,b) -- kept by the rank owning a before the tick,
 *
 * so the union over ranks is the net diff of the whole space, exact and
 * duplicate-free.  With H = 2*D + teleport + 1 every pair whose relation can
 * change is visible to the rank that reports it, except pairs of two
 * "teleporters" (|dx| > teleport in one tick); those are all-gathered and
 * decided directly from their before/after states.  DESIGN.md §5 has the
 * argument.
 *
 * Per tick, on every rank:
 *   1. gwaoi_strips_route(ops)  -- the owned entities' Enter/Moved/Leave of this
 *      tick (their owner before the tick receives them) become halo records
 *      per destination rank + teleport records; returns the counts, and
 *      gwaoi_strips_route_kinds how many of each destination's records are
 *      ENTER / LEAVE (and the box of the ENTER positions).
 *   2. gwaoi_strips_route_scatter(send, tele) -- writes them, grouped by
 *      destination rank, into caller device buffers.
 *   3. the caller exchanges them (counts on the host, records point to point
 *      over RCCL / xGMI; teleports to every rank) -- see goworld_amd/strips.py.
 *   4. gwaoi_strips_tick_async(local, recv, tele_all, enters, leaves, box) --
 *      queues: its own and the received records become device Leave / Enter /
 *      Moved batches of the world (gwaoi.h), the world flushes, and its events
 *      are filtered to the ones this strip owns.  Nothing waits: the next
 *      gwaoi_strips_route (or gwaoi_strips_wait / _events) completes the tick
 *      with the same host wait that brings the route's counts, so a tick has
 *      ONE host wait.  gwaoi_strips_tick does 4. and waits (two waits: it
 *      reads the record kinds back first).
 *
 * Single-threaded per strip, on the world's stream.  All counts are records.
 */
#ifndef GWAOI_STRIPS_H
#define GWAOI_STRIPS_H

#include "gwaoi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GWAOI_MAX_STRIPS 64

enum { GWAOI_HALO_MOVE = 0, GWAOI_HALO_ENTER = 1, GWAOI_HALO_LEAVE = 2 };

typedef struct {  /* 24 B: one op as it travels between strips             */
    uint32_t slot; /* global entity slot                                    */
    float x, z;    /* position after the op                                 */
    uint32_t kind; /* GWAOI_HALO_*: as input, the AOIManager call (Moved /  */
                   /* Enter / Leave); as sent, the op for the receiver      */
    uint64_t seq;  /* global call order                                     */
} gwaoi_halo_rec;

typedef struct {    /* 40 B: an entity that teleported this tick           */
    uint32_t slot;
    uint32_t flags; /* bit0 present before, bit1 present after             */
    float px, pz;   /* before                                               */
    uint64_t pseq;
    float x, z;     /* after                                                */
    uint64_t seq;
} gwaoi_tele_rec;

typedef struct {
    uint32_t n_strips;   /* 1 .. GWAOI_MAX_STRIPS                                    */
    uint32_t rank;       /* this strip                                               */
    const float *edges;  /* n_strips-1 increasing interior x edges                   */
    float aoi_distance;  /* D of the space (the world space must use the same)       */
    float teleport;      /* |dx| per tick above which an entity is a teleporter      */
                         /* (<= 0: D/8)                                              */
} gwaoi_strips_config;

typedef struct gwaoi_strips gwaoi_strips;

/* Creates the strip layer on `w`, whose space `space` is this strip's part of
 * the big space.  The world must hold the global slot range (max_slots). */
int gwaoi_strips_create(gwaoi_world *w, uint32_t space, const gwaoi_strips_config *cfg, gwaoi_strips **out);
int gwaoi_strips_destroy(gwaoi_strips *s);
/* Halo width H (x distance around the strip whose entities are mirrored). */
int gwaoi_strips_halo(const gwaoi_strips *s, float *halo);

/* 1. Route this tick's ops of the entities this strip owned after the last
 * tick (Moved / Leave) or that enter the space inside it (Enter).  d_ops is
 * device memory, one op per entity at most, in any order; it must be complete
 * before the call (the world's stream does not wait for the producer's
 * stream).  counts[0..n_strips-1]
 * = records for each destination rank, counts[n_strips] = teleport records.
 * Returns GWAOI_ESTATE if an op names an entity this strip does not own. */
int gwaoi_strips_route(gwaoi_strips *s, const gwaoi_halo_rec *d_ops, size_t n, uint64_t *counts);
/* 1'. The same route with the count exchange on the device (multi-GPU: no
 * host collective per tick).  _begin queues the route and writes this
 * strip's count row to d_row (device, gwaoi_strips_route_row_words words):
 *   [records to each strip (n_strips) | teleport records |
 *    per destination: ENTER, LEAVE, ENTER box x0 z0 x1 z1 (6 words each; the
 *    box as order-preserving ints) | route error word];
 * nothing waits.  The caller then gathers the rows of all strips, in rank
 * order, into d_matrix (n_strips rows) on the world's stream (an RCCL
 * all-gather over xGMI: goworld_amd/strips.py), and _end copies the matrix
 * to host memory owned by the strip (*h_matrix, valid until the next _end)
 * with the tick's one host wait, which also completes the previous tick.
 * counts and gwaoi_strips_route_kinds as after gwaoi_strips_route; _end
 * fails if any strip's row carries a route error. */
int gwaoi_strips_route_row_words(const gwaoi_strips *s, uint32_t *words);
int gwaoi_strips_route_begin(gwaoi_strips *s, const gwaoi_halo_rec *d_ops, size_t n, uint32_t *d_row);
int gwaoi_strips_route_end(gwaoi_strips *s, const uint32_t *d_matrix, const uint32_t **h_matrix, uint64_t *counts);
/* 2. Write the routed records: d_send holds sum(counts[0..n_strips-1])
 * records grouped by destination rank (rank order), d_tele counts[n_strips].
 * Returns after the writes completed (the caller's transport may read them). */
int gwaoi_strips_route_scatter(gwaoi_strips *s, gwaoi_halo_rec *d_send, gwaoi_tele_rec *d_tele);
/* 4. Apply this rank's own records (d_local: its slice of d_send, never sent),
 * the records received from the other ranks and the all-gathered teleport
 * records, flush the world and keep this strip's events.  The inputs must
 * be complete (the caller synchronised its transport). */
int gwaoi_strips_tick(gwaoi_strips *s, const gwaoi_halo_rec *d_local, size_t n_local, const gwaoi_halo_rec *d_recv,
                      size_t n_recv, const gwaoi_tele_rec *d_tele, size_t n_tele, uint64_t *n_enter,
                      uint64_t *n_leave);
/* After gwaoi_strips_route: per destination rank q (n_strips entries each),
 * the ENTER and LEAVE records among counts[q] and the box {x0, z0, x1, z1} of
 * the ENTER positions (+inf, +inf, -inf, -inf when none).  A receiver sums
 * them over the senders for gwaoi_strips_tick_async. */
int gwaoi_strips_route_kinds(const gwaoi_strips *s, uint64_t *enters, uint64_t *leaves, float *enter_boxes);
/* 4. (asynchronous) As gwaoi_strips_tick, with the receiver's ENTER / LEAVE
 * record counts over d_local + d_recv and the box of their positions (NULL:
 * unknown) taken from the senders' gwaoi_strips_route_kinds.  Queues the tick
 * on the world's stream and returns; the inputs must stay valid until it
 * completes (the next gwaoi_strips_route, gwaoi_strips_wait, _events,
 * _events_device or _destroy).  Problems found on the device are reported
 * by the call that completes it.  The records are not validated before the
 * world consumes them: a bad record (slot out of range, a kind that is not
 * MOVE / ENTER / LEAVE, an ENTER of a slot the strip holds, a MOVE / LEAVE of
 * one it does not) fails that completing call, and the strip is unusable
 * from then on -- every later call returns GWAOI_ESTATE, and its world is
 * poisoned when a record reached it in the wrong state (gwaoi_tick).  An
 * unknown kind reaches the world as a no-op.  gwaoi_strips_tick validates
 * first and leaves the state untouched on such an error. */
int gwaoi_strips_tick_async(gwaoi_strips *s, const gwaoi_halo_rec *d_local, size_t n_local,
                            const gwaoi_halo_rec *d_recv, size_t n_recv, const gwaoi_tele_rec *d_tele, size_t n_tele,
                            uint64_t n_enter_recs, uint64_t n_leave_recs, const float *enter_box);
/* Complete the queued tick (host wait if needed); its event counts. */
int gwaoi_strips_wait(gwaoi_strips *s, uint64_t *n_enter, uint64_t *n_leave);
/* Host waits (stream synchronisations) of the strip layer so far (tests, bench). */
int gwaoi_strips_host_waits(const gwaoi_strips *s, uint64_t *waits);
/* Device pointers of this strip's events of the last tick (layout of
 * gwaoi_events: enter pairs, then leave pairs, a0,b0,a1,b1,...). */
int gwaoi_strips_events_device(gwaoi_strips *s, const uint32_t **d_enter, const uint32_t **d_leave);
/* Copy them to host memory owned by the strip layer (valid until the next tick). */
int gwaoi_strips_events(gwaoi_strips *s, gwaoi_events *out);
const char *gwaoi_strips_last_error(gwaoi_strips *s);

#ifdef __cplusplus
}
#endif
#endif /* GWAOI_STRIPS_H */
