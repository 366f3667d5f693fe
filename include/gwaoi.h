/*
 * gwaoi.h -- C ABI of the MI355X-native AOI engine for GoWorld (libgwaoi.so).
 *
 * Drop-in boundary for GoWorld's `aoi.AOIManager` (go-aoi v0.2.0,
 * /root/reference/go.mod:29) as engine/entity/Space drives it:
 *
 *   reference call                                   replaced by
 *   ---------------------------------------------   -------------------------------
 *   aoi.NewXZListAOIManager(d)   Space.go:105         gwaoi_space_create
 *   (space destroyed)            Space.go:33          gwaoi_space_destroy
 *   aoiMgr.Enter(&e.aoi, x, z)   Space.go:211,221     gwaoi_enter / gwaoi_enter_batch
 *   aoiMgr.Leave(&e.aoi)         Space.go:243         gwaoi_leave / gwaoi_leave_batch
 *   aoiMgr.Moved(&e.aoi, x, z)   Space.go:259         gwaoi_moved / gwaoi_moved_batch(_device)
 *   AOICallback.OnEnterAOI(o)    Entity.go:227-229    replay of gwaoi_events.enter
 *   AOICallback.OnLeaveAOI(o)    Entity.go:231-233    replay of gwaoi_events.leave
 *   aoi.InitAOI(&e.aoi, ...)     Entity.go:210        caller-side slot handle (uint32)
 *
 * Semantics.  A world holds many independent spaces (one go-aoi manager
 * each).  Enter/Leave/Moved are queued in call order; each call gets the next
 * sequence number, exactly as the sequential manager would process it.
 * gwaoi_tick() flushes the queue: it computes the neighbour relation of every
 * space at the queued state on the GPU and returns the NET enter/leave events
 * since the previous flush.  After replaying them (leaves first, then enters)
 * the callers' InterestedIn/InterestedBy sets are bit-identical to those the
 * sequential XZListAOIManager produces for the same call sequence: pair {A,B}
 * is a neighbour iff P_W(L) holds at the current positions, W being the one
 * of A,B whose Enter/Moved came last and
 *     P_W(L) = L.x >= fl32(W.x-D) && L.x <= fl32(W.x+D)
 *           && L.z >= fl32(W.z-D) && L.z <= fl32(W.z+D)        (float32).
 * A transient enter+leave of one pair inside one flush is not reported (the
 * reference would emit both callbacks; the final sets are the same).
 *
 * Slots.  Go pointers cannot be retained by C (cgo rule), so entities are
 * named by caller-chosen uint32 slots in [0, max_slots).  A slot may not be
 * reused for a different entity before the next flush.
 *
 * Errors.  Every call returns 0 or a negative gwaoi_status and never aborts.
 * Misuse that panics in the reference (Moved/Leave before Enter, Enter twice,
 * EnableAOI with d <= 0, Space.go:92-102) returns GWAOI_ESTATE / GWAOI_EINVAL.
 *
 * Threading.  A world is single-threaded (GoWorld's GameService goroutine,
 * components/game/GameService.go:88-186); it owns one HIP stream on one GPU.
 */
#ifndef GWAOI_H
#define GWAOI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GWAOI_ABI_VERSION 6  /* 6: gwaoi_debug.overlapped_flushes; 5: GWAOI_F_TEST_* flags replace environment switches, GWAOI_F_BATCH_READY ignored */

typedef struct gwaoi_world gwaoi_world;

typedef enum {
    GWAOI_OK = 0,
    GWAOI_EINVAL = -1,     /* null pointer, bad size, aoi distance <= 0          */
    GWAOI_EBADSLOT = -2,   /* slot >= max_slots                                   */
    GWAOI_ESTATE = -3,     /* Enter on a live slot; Leave/Moved on a non-live one */
    GWAOI_ENOMEM = -4,     /* host or device allocation failed                    */
    GWAOI_EDEVICE = -5,    /* HIP runtime error (see gwaoi_last_error)            */
    GWAOI_ENONFINITE = -6, /* NaN or infinite coordinate                          */
    GWAOI_EBADSPACE = -7,  /* unknown / destroyed space id, or too many spaces    */
    GWAOI_EBUSY = -8,      /* space destroyed while entities are still in it      */
    GWAOI_ECAPACITY = -9   /* more than 2^32-1 events in one flush                */
} gwaoi_status;

typedef struct {
    uint32_t max_slots;      /* slot handles are in [0, max_slots)                   */
    uint32_t max_spaces;     /* space ids are in [0, max_spaces)                      */
    int32_t device;          /* HIP device ordinal, -1 = the calling thread's current */
    uint32_t flags;          /* GWAOI_F_*                                             */
    uint64_t event_capacity; /* initial device event capacity in pairs (0 = default) */
    float cells_per_dist;    /* grid cells per AOI distance (0 = automatic, from 3.0) */
} gwaoi_config;

#define GWAOI_F_TIMING 1u /* time every pipeline stage with HIP events (gwaoi_stage_times) */
#define GWAOI_F_NO_SPARSE 2u /* never take the sparse flush (every flush rebuilds the frame; A/B, tests) */
/* Accepted for compatibility and ignored since ABI 5.  (Until then: the next flush's last-op
 * claims stored beside the flush in flight.  Measured slower at 1M entities, DESIGN.md §3 step 1,
 * and removed with the side stream it needed.) */
#define GWAOI_F_BATCH_READY 4u
/* The Moved batches of one flush never name a slot twice (a per-tick position array with one
 * entry per moving entity).  A flush of plain device Moved batches (gwaoi_moved_batch_device,
 * or gwaoi_moved_batch's staged batches) then applies every move without the last-op claims
 * and the repeated-slot fixup.  The promise is checked on the device: keygen counts the frame
 * entries the moves wrote, and a flush with fewer than its moves commits, with the repeated
 * slot's position unspecified (each move writes its 16-B record with one store, so in practice
 * one of its moves, not necessarily the last), and returns GWAOI_ESTATE (gwaoi_last_error also
 * names any other problem the device found in that flush).  Batches with explicit seqs, decoded sync batches and mixed queues keep the
 * claims.  Measured at 1M entities: DESIGN.md §3 step 2. */
#define GWAOI_F_UNIQUE_MOVES 8u
/* Test and diagnostics flags: they select a slower or failing path so that tests can compare
 * it with the default one.  Not for production worlds. */
#define GWAOI_F_TEST_FORCE_RADIX 0x100u      /* every flush sorts the frame with the full radix sort  */
#define GWAOI_F_TEST_FORCE_COPY 0x200u       /* S' is always copied from the previous frame            */
#define GWAOI_F_TEST_BUCKETED 0x400u         /* Moved batches take the bucketed apply at any size       */
#define GWAOI_F_TEST_REGROW_FAIL 0x800u      /* an event-buffer regrow fails (the poison path)          */
#define GWAOI_F_TEST_SPARSE_SEQUENCE 0x1000u /* the sparse flush runs its kernel sequence, not one launch */
#define GWAOI_F_TEST_SPARSE_SCR2 0x2000u     /* sparse one-launch scratch rows of 2 events per kind     */
#define GWAOI_F_TEST_CHECK_STAGES 0x4000u    /* wait after every flush stage (names a faulting stage)   */

typedef struct {
    uint64_t n_enter;      /* directed enter events; replay pair (a,b) as a.OnEnterAOI(b) */
    uint64_t n_leave;      /* directed leave events; replay pair (a,b) as a.OnLeaveAOI(b) */
    const uint32_t *enter; /* 2*n_enter uint32: a0,b0,a1,b1,...  (world-owned host memory,  */
    const uint32_t *leave; /* 2*n_leave uint32                     valid until the next tick) */
} gwaoi_events;

typedef struct {
    uint64_t ticks;        /* completed flushes                       */
    uint64_t next_seq;     /* sequence number the next call gets      */
    uint32_t live;         /* live entities after the last flush      */
    uint32_t spaces;       /* spaces currently created                */
    uint32_t total_cells;  /* grid cells of the last flush            */
    uint32_t pending_ops;  /* calls queued since the last flush       */
    uint64_t event_capacity;
    uint32_t max_slots;    /* creation config                         */
    uint32_t max_spaces;
} gwaoi_info;

/* Counters of the rare paths of the flush pipeline, summed over flushes
 * since the world was created (tests assert that a workload reached them). */
typedef struct {
    uint64_t flushes;
    uint64_t combined_replays;      /* combined-pass waves whose LDS event buffer overflowed (sweep replayed) */
    uint64_t combined_queue_drains; /* combined-pass survivor queues drained in the middle of a sweep         */
    uint64_t special_global;        /* special-pass lanes whose events spilled past their LDS slots          */
    uint64_t event_regrows;         /* flushes that grew the device event buffer and re-ran the pair passes  */
    uint64_t speculative_launches;  /* flushes GWAOI_END_NEXT queued before the commit of the       */
                                    /* one in flight                                                         */
    uint64_t cell_size_switches;    /* flushes that rebuilt every grid with another automatic cell size      */
    uint32_t cells_per_dist;        /* cells per AOI distance of the grids in use (2 or 3 when automatic)    */
    uint32_t pad;
    uint64_t incremental_sorts;     /* flush launches whose frame sort was the per-cell merge (grid unchanged) */
    uint64_t sparse_flushes;        /* flushes of a few Moved calls done on the frame in place (gwaoi_tick*) */
    uint64_t sparse_declined;       /* sparse flushes that fell back to the full one (long shifts, capacity)  */
    uint64_t premarked_runs;        /* always 0 since ABI 5 (GWAOI_F_BATCH_READY is ignored)                 */
    uint64_t sparse_unfused;        /* sparse flushes that ran the kernel sequence (an op outgrew its row)    */
    uint64_t unique_flushes;        /* flushes applied without last-op claims (GWAOI_F_UNIQUE_MOVES)          */
    uint64_t overlapped_flushes;    /* speculative flushes whose first kernels ran beside the pair passes and */
                                    /* finish of the flush before them (two streams)                        */
} gwaoi_debug;

typedef struct {
    char name[32];
    double ms;             /* accumulated device time (HIP events)     */
    uint64_t calls;
} gwaoi_stage_time;

/* ---- world / space lifetime ---------------------------------------------- */
int gwaoi_world_create(const gwaoi_config *cfg, gwaoi_world **out);
int gwaoi_world_destroy(gwaoi_world *w);

/* aoi.NewXZListAOIManager(aoi_distance)  -- Space.EnableAOI, Space.go:91-107 */
int gwaoi_space_create(gwaoi_world *w, float aoi_distance, uint32_t *space_out);
int gwaoi_space_destroy(gwaoi_world *w, uint32_t space);

/* ---- AOIManager calls (queued; seq = call order) ---------------------------- */
int gwaoi_enter(gwaoi_world *w, uint32_t space, uint32_t slot, float x, float z);
int gwaoi_leave(gwaoi_world *w, uint32_t slot);
int gwaoi_moved(gwaoi_world *w, uint32_t slot, float x, float z);

/* Batched forms (array order = call order).  Validated as a whole: on error
 * nothing is queued.  gwaoi_moved_batch copies the arrays before it returns
 * (batches of 64+ moves into pinned staging, sent with one async H2D), so the
 * caller may reuse them at once. */
int gwaoi_enter_batch(gwaoi_world *w, uint32_t space, const uint32_t *slots, const float *x,
                      const float *z, size_t n);
int gwaoi_leave_batch(gwaoi_world *w, const uint32_t *slots, size_t n);
int gwaoi_moved_batch(gwaoi_world *w, const uint32_t *slots, const float *x, const float *z,
                      size_t n);

/* Moves whose arrays already live in device memory of the world's GPU (the
 * per-tick position-sync batch, GameService.go:392-404).  The pointers must
 * stay valid until the next gwaoi_tick*.  Only slots live at the previous
 * flush may appear; violations and non-finite coordinates are detected on the
 * device and reported by the next tick (the offending moves are dropped). */
int gwaoi_moved_batch_device(gwaoi_world *w, const uint32_t *d_slots, const float *d_x,
                             const float *d_z, size_t n);

/* ---- explicit sequence numbers ---------------------------------------------
 * The relation depends on call order only through each entity's seq (the
 * one of A,B whose Enter/Moved came last owns the window test).  These forms
 * take the seq from the caller instead of the world's counter: for a world
 * that is one strip of a larger space fed by several hosts (gwaoi_strips.h),
 * and to restore frozen AOI state with its original order (EntityManager.go
 * freeze/restore, :554-656).  Rules: an explicit seq must be >= the next
 * seq the world would hand out (gwaoi_info.next_seq; host calls check it and
 * return GWAOI_EINVAL) and the caller keeps them unique; afterwards the
 * world's counter continues above it.  Device seqs are checked on the device
 * against the flush's floor (violations: the op is dropped, the tick returns
 * GWAOI_EINVAL).  After a device explicit batch, no other call may be queued
 * before the next flush (GWAOI_ESTATE). */
int gwaoi_enter_seq(gwaoi_world *w, uint32_t space, uint32_t slot, float x, float z, uint64_t seq);
int gwaoi_moved_seq(gwaoi_world *w, uint32_t slot, float x, float z, uint64_t seq);
int gwaoi_moved_batch_device_seq(gwaoi_world *w, const uint32_t *d_slots, const float *d_x, const float *d_z,
                                 const uint64_t *d_seq, size_t n);

/* ---- structural device batches ----------------------------------------------
 * Enter / Leave calls whose slots live in device memory (Space.go:211,243): the
 * entities crossing into / out of a strip world (gwaoi_strips.h) without a host
 * round trip.  The host learns only the counts, so the world's per-slot host
 * mirror goes stale; it is rebuilt from the device on the next host call that
 * needs it (a host Enter/Leave/Moved/batch, gwaoi_neighbors), which returns
 * GWAOI_ESTATE while such a batch is queued and not yet flushed.  Rules, checked
 * on the device: an entered slot is not live when the flush begins, a left slot
 * is live (the host counts it out of `space`), each slot appears once in the
 * flush.  A violation breaks
 * the frame's live count: the flush fails and the world is poisoned.
 * gwaoi_enter_batch_device: d_seq NULL = implicit seqs (call order), else
 * explicit seqs (rules above); box = {x0, z0, x1, z1} holding every entered
 * position (sizes the space's grid), or NULL.  Not while a flush is in flight,
 * nor on a world with an entity-sync layer (gwaoi_sync.h). */
int gwaoi_enter_batch_device(gwaoi_world *w, uint32_t space, const uint32_t *d_slots, const float *d_x,
                             const float *d_z, const uint64_t *d_seq, size_t n, const float *box);
int gwaoi_leave_batch_device(gwaoi_world *w, uint32_t space, const uint32_t *d_slots, size_t n);

/* ---- flush ------------------------------------------------------------------ */
/* Run the tick and copy its events to host memory.  If the device found a bad
 * op in a device batch (dropped; GWAOI_ESTATE / GWAOI_ENONFINITE /
 * GWAOI_EINVAL) the flush still commits and *out holds its events: replay
 * them.  Other failures leave *out empty. */
int gwaoi_tick(gwaoi_world *w, gwaoi_events *out);
/* Run the tick; events stay in device memory (see gwaoi_events_device). */
int gwaoi_tick_device(gwaoi_world *w, uint64_t *n_enter, uint64_t *n_leave);

/* Asynchronous flush: gwaoi_tick == gwaoi_tick_begin + gwaoi_tick_finish(GWAOI_END_HOST).
 * _begin closes the op queue, queues the whole pipeline on the GPU and returns
 * at once.  Until _finish, the AOIManager calls (enter / leave / moved and their
 * batch forms, except explicit-seq device batches) stay available: they are
 * validated and numbered at the call -- a gwaoi_moved_batch is also staged
 * and sent to the GPU on a copy stream, overlapping the flush -- and queued
 * for the NEXT flush when _finish commits this one.  Everything else
 * (neighbours, snapshot/restore, the sync layer, another _begin) returns
 * GWAOI_ESTATE while a flush is in flight. */
int gwaoi_tick_begin(gwaoi_world *w);

/* gwaoi_tick_finish: wait for the flush in flight, commit it, and return its
 * status and counts (directed events; zero unless it committed).  `mode` is an
 * OR of:
 *   GWAOI_END_NEXT   begin the next flush with the calls queued meanwhile (the
 *                    steady game loop: one call per tick, the next flush in
 *                    flight on return whenever this one committed).  When those
 *                    calls are device Moved batches only (implicit seqs, no
 *                    Enter / Leave / space change, no host op) and the flush in
 *                    flight has no explicit-seq batch, the next flush is queued
 *                    on the GPU BEFORE this one's summary is waited for, so the
 *                    GPU runs the two back to back (a second buffer set; an
 *                    event-buffer overflow of the first is still re-run
 *                    exactly).
 *   GWAOI_END_HOST   copy the events to host memory: gwaoi_events_host returns
 *                    them (with GWAOI_END_NEXT the copy runs beside the next
 *                    flush and gwaoi_events_host waits for it, so a caller can
 *                    queue the next tick's batch -- e.g. gwaoi_moved_batch_pinned
 *                    -- while the copy runs).
 *   GWAOI_END_PAIRS  as GWAOI_END_HOST with half the bytes: the flush reports
 *                    every relation change as the mirrored pair (a,b),(b,a), and
 *                    only (a,b) is copied.  gwaoi_pairs_host returns them:
 *                    n_enter / n_leave pairs, each entry (a,b) standing for the
 *                    events (a,b) and (b,a) -- OnEnterAOI / OnLeaveAOI on both
 *                    entities.  (The counts returned here are directed events.)
 * Events stay in device memory in every mode (gwaoi_events_device).
 *
 * Buffer lifetime, the one rule for every flush-ending call: events in device
 * memory (gwaoi_events_device, gwaoi_events_csr_device) are valid until the
 * next commit; events in host memory (gwaoi_tick's *out, gwaoi_events_host,
 * gwaoi_pairs_host, gwaoi_events_csr) until the next call that copies events to
 * host memory (gwaoi_tick, or gwaoi_tick_finish with GWAOI_END_HOST /
 * GWAOI_END_PAIRS).  gwaoi_events_host / gwaoi_pairs_host always describe the
 * last host copy, whatever committed since; after a GWAOI_END_PAIRS copy
 * gwaoi_events_host (and gwaoi_pairs_host after any other) returns
 * GWAOI_ESTATE. */
#define GWAOI_END_NEXT 1u
#define GWAOI_END_HOST 2u
#define GWAOI_END_PAIRS 4u
int gwaoi_tick_finish(gwaoi_world *w, uint32_t mode, uint64_t *n_enter, uint64_t *n_leave);
int gwaoi_events_host(gwaoi_world *w, gwaoi_events *out);
int gwaoi_pairs_host(gwaoi_world *w, gwaoi_events *out);

/* ---- zero-copy host move batches ---------------------------------------------
 * The per-tick position batch written straight into the world's pinned staging
 * memory, as a cgo adapter appends each client's (slot, x, z) while it decodes
 * the sync packets (GameService.go:392-404, HandleSyncPositionYawFromClient):
 * _stage reserves room for up to n moves and returns the three arrays; the
 * caller fills a prefix of them and _commit(k) queues those k moves as one
 * Moved batch (array order = call order) and starts their one H2D copy on a
 * copy stream.  Nothing is read on the host: a move of a slot that is not
 * live, an out-of-range slot or a non-finite coordinate is dropped on the
 * device and reported by the flush (as gwaoi_moved_batch_device).  When an
 * Enter / Leave is queued in the same flush before it, the batch is checked
 * on the host instead (a slot's space may have changed; errors as
 * gwaoi_moved_batch: nothing is queued).  One reservation at a time;
 * available while a flush is in flight (the batch joins the next flush).
 * GWAOI_ECAPACITY: the staging memory holds this flush's batches already
 * (commit, flush, then stage again). */
int gwaoi_moved_batch_stage(gwaoi_world *w, size_t n, uint32_t **slots, float **x, float **z);
int gwaoi_moved_batch_commit(gwaoi_world *w, size_t n);
/* The same from batch arrays the caller keeps in pinned memory it got from
 * gwaoi_pinned_alloc (a cgo adapter's per-tick move buffers, filled as the
 * sync packets arrive during the game tick): the H2D copies read them in place,
 * so the arrays must stay unchanged until the flush that takes the batch has
 * returned.  Checked on the device as above (on the host after an Enter /
 * Leave of the same flush). */
int gwaoi_moved_batch_pinned(gwaoi_world *w, const uint32_t *slots, const float *x, const float *z, size_t n);
int gwaoi_pinned_alloc(gwaoi_world *w, size_t bytes, void **out);
int gwaoi_pinned_free(gwaoi_world *w, void *p);
/* Device pointers of the last committed tick's events (same layout as
 * gwaoi_events); valid until the next commit, also while a later flush is in
 * flight (it writes the other event buffer). */
int gwaoi_events_device(gwaoi_world *w, const uint32_t **d_enter, const uint32_t **d_leave);

/* The last tick's events regrouped by entity (built on the GPU on request), for
 * a replay entity by entity -- Entity.go:236-246 touches a's InterestedIn and
 * b's InterestedBy per event (a,b); events come in pairs, so row s lists every
 * change of s's InterestedIn AND of s's InterestedBy:
 *   row s = items[offsets[s] .. offsets[s+1]),  offsets has max_slots + 1 entries,
 *   item  = b               : leave (s, b)
 *         = b | 0x80000000  : enter (s, b)
 * sorted ascending within the row, so its leaves come first (an entity that
 * changed space may leave and re-enter the same partner in one flush), each
 * part by b.  Host memory (world-owned, valid until the next flush) or device
 * memory.  GWAOI_ESTATE while a flush is in flight. */
#define GWAOI_CSR_ENTER 0x80000000u
int gwaoi_events_csr(gwaoi_world *w, const uint32_t **offsets, const uint32_t **items, uint64_t *n_items);
int gwaoi_events_csr_device(gwaoi_world *w, const uint32_t **d_offsets, const uint32_t **d_items, uint64_t *n_items);

/* ---- freeze / restore (EntityManager.go:554-656, Space.go:118-125) ----------
 * gwaoi_snapshot copies the AOI state of the last flush in frame order:
 * slot, space, x, z and the seq of the entity's last Enter/Moved.  *n_out =
 * live entities (also when it exceeds cap; nothing is copied then).
 * gwaoi_restore re-enters such a state into a world with no queued op, in
 * seq order, so the restored relation is the frozen one bit for bit (the
 * reference re-enters in Go map order, Appendix D.6 of SURVEY.md, which may
 * flip ownership-dependent pairs).  The entities keep their original seqs
 * when every one of them is >= the world's next seq (a fresh world, or one
 * whose counter is below the snapshot's -- required for a strip world,
 * gwaoi_strips.h, whose halo records carry global seqs); otherwise they get
 * fresh seqs in the frozen order.  Spaces must exist; the next gwaoi_tick
 * reports every restored pair as an enter. */
int gwaoi_snapshot(gwaoi_world *w, uint32_t *slots, uint32_t *spaces, float *x, float *z, uint64_t *seq,
                   size_t cap, size_t *n_out);
int gwaoi_restore(gwaoi_world *w, const uint32_t *slots, const uint32_t *spaces, const float *x, const float *z,
                  const uint64_t *seq, size_t n);

/* ---- queries ----------------------------------------------------------------- */
/* Neighbours of `slot` at the last flush (unsorted).  *n_out = total count even
 * when it exceeds cap. */
int gwaoi_neighbors(gwaoi_world *w, uint32_t slot, uint32_t *out, size_t cap, size_t *n_out);
int gwaoi_world_info(gwaoi_world *w, gwaoi_info *info);
int gwaoi_debug_counters(gwaoi_world *w, gwaoi_debug *out);
int gwaoi_stage_times(gwaoi_world *w, gwaoi_stage_time *out, size_t cap, size_t *n_out);
int gwaoi_reset_stage_times(gwaoi_world *w);
/* Time only the stages whose bit is set (bit i = entry i of gwaoi_stage_times);
 * 0 = no events at all.  GWAOI_F_TIMING at creation sets every bit.          */
int gwaoi_set_stage_timing(gwaoi_world *w, uint32_t stage_mask);
int gwaoi_sync(gwaoi_world *w);
void *gwaoi_stream(gwaoi_world *w); /* the world's hipStream_t */
/* Stream ordering without a host wait (a caller whose producers / consumers of
 * the world's device buffers run on another hipStream_t `other`):
 * gwaoi_stream_after: work queued on the world's stream from now on runs after
 * everything queued on `other` so far; gwaoi_stream_before: work queued on
 * `other` from now on runs after everything queued on the world's stream so far. */
int gwaoi_stream_after(gwaoi_world *w, void *other);
int gwaoi_stream_before(gwaoi_world *w, void *other);

const char *gwaoi_strerror(int status);
const char *gwaoi_last_error(gwaoi_world *w);
int gwaoi_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GWAOI_H */
