// Internal types shared by the host world (gwaoi_world.cpp) and the HIP
// kernels (gwaoi_kernels.hip).  Not part of the public ABI.
#pragma once

#include <cstddef>

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <new>

struct gwaoi_world;  // include/gwaoi.h

namespace gw {

// Every extern "C" entry point runs its body through api_guard: no C++
// exception (std::bad_alloc from a vector, a thread that cannot start, ...)
// may cross the C ABI into a cgo host, where it would end in std::terminate.
template <class F>
inline int api_guard(F &&f) noexcept {
    try {
        return f();
    } catch (const std::bad_alloc &) {
        return -4;  // GWAOI_ENOMEM
    } catch (...) {
        return -5;  // GWAOI_EDEVICE
    }
}

constexpr uint32_t SP_DEAD = 0xFFFFFFFFu;  // slot not live (or left this tick)
constexpr uint32_t SP_KEEP = 0xFFFFFFFEu;  // device move: keep the space of the previous flush
constexpr uint32_t SLOT_NONE = 0xFFFFFFFFu;  // op placeholder (skipped decoded sync record): no op

// Device-side validation flags (bit set = problem seen during the tick).
constexpr uint32_t ERR_NONFINITE = 1u;
constexpr uint32_t ERR_MOVE_DEAD = 2u;       // device move of a slot that is not live
constexpr uint32_t ERR_BAD_SLOT = 4u;
constexpr uint32_t ERR_COUNT_MISMATCH = 8u;  // host/device live-count disagreement (bug guard)
constexpr uint32_t ERR_SEQ = 16u;            // explicit device seq below the flush's floor
constexpr uint32_t ERR_ENTER_LIVE = 32u;     // device Enter of a slot live when the flush began
constexpr uint32_t ERR_DUP_SLOT = 64u;       // GWAOI_F_UNIQUE_MOVES flush whose moves named a slot twice

constexpr uint32_t TILE_A = 256;  // entities per pair-pass tile (= threads per workgroup)

// One entity state: position (go-aoi Coord = float32) and the sequence
// number of its last Enter/Moved call.  16 B, one vector access.
struct alignas(16) Rec16 {
    float x, z;
    unsigned long long s;
};

struct alignas(8) SlotSp {  // caller slot handle + space id (SP_DEAD = not live)
    uint32_t slot, sp;
};

// Per-slot table, indexed by the caller's slot, as three arrays: lastop[s] = (tick << 32 | op
// index) of the slot's last op this flush (the claims path only); rank[s] = its index in S'
// (previous frame order, or appended; 0xFFFFFFFF if not live); sp[s] = its space in S' before
// this flush's ops (SP_DEAD if not live).  Arrays, not one 16-B record, because the hot passes
// touch few of them per random slot: the unique-moves apply reads only rank, so its one random
// line per move comes from a 4 B-per-slot array (at 1M slots 4 MB, an XCD's L2; the record was
// 16 MB); the gather writes rank and sp; only the claims path reads all three.
struct SlotTab {
    unsigned long long *lastop;
    uint32_t *rank;
    uint32_t *sp;
};

// Uniform grid of one space for one flush.  Cell (cx,cz) of space s has the
// global cell key base + cz*gx + cx; its grid row cz is global row
// row_base + cz.  cellOf() is monotone in the coordinate, so a query range
// derived from conservative window bounds is complete.
struct SpaceGrid {
    float ox, oz;  // grid origin
    float inv;     // 1 / cell size
    float D;       // AOI distance of the space (go-aoi aoidist)
    uint32_t gx, gz;
    uint32_t base;
    uint32_t row_base;
};

// One flush's sorted state: entries [0, n) are the live entities ordered by
// cell key (space-major, then cz, cx), stable in the previous order.
struct FrameView {
    const Rec16 *rec;
    const SlotSp *ss;
    const uint32_t *cell_start;  // total_cells + 1 entries
    const SpaceGrid *grid;
    uint32_t n;
    uint32_t total_cells;
};


// Per-tick scalars written by device kernels.
struct TickScalars {
    uint32_t err;
    uint32_t ndrop;              // unique-moves flush: ops that wrote nothing (placeholders, dropped ops)
    unsigned long long counter;  // directed event pairs reserved by the pair passes
    float d_rel;                 // largest displacement / D of "near" entities
    float bmax;                  // largest |x|,|z| of live entities (new positions)
    unsigned long long seq_max;  // largest explicit seq of the device batches (0 = none)
    uint32_t ncoll;              // slots moved more than once in this flush (k_moves_apply_n)
    uint32_t n_unique;           // unique-moves flush: its ops (keygen's written entries + ndrop must match; 0 = no check)
    uint32_t dbg[4];             // path counters of this flush (DBG_*), copied to TickOut
    uint32_t err_apply;          // unique-moves apply's ERR_* bits (folded into err by the keygen fold, which resets it)
    uint32_t pad3[17];
    // One 128-B line per XCD shard q (zeroed by the prologue): [q][2..3] = the u64 length of
    // event stream q (the pair passes' event allocator: ev_phys).  Sharded because one device-scope atomic word saturates
    // at ~88 returning atomics per us (MI355X_MICROARCH.md, dequeue).
    uint32_t shard[8][32];
};
constexpr uint32_t EV_SHARDS = 8;
static_assert(offsetof(TickScalars, shard) % 128 == 0, "one line per shard");

// The pair passes' directed events go to EV_SHARDS virtual streams (one per XCD, allocated by
// that XCD's waves with one atomic per tile on the shard's own word), interleaved over the
// scratch buffer in chunks of EV_CHUNK pairs: stream q's chunk k is physical chunk k*8+q.  A
// tile's events are contiguous in its stream; a stream position is encoded (q << 60) | v.
constexpr uint32_t EV_CHUNK_LOG = 8;
constexpr uint64_t EV_CHUNK = 1ull << EV_CHUNK_LOG;
__host__ __device__ inline unsigned long long ev_phys(unsigned long long qv) {
    const unsigned long long q = qv >> 60, v = qv & ((1ull << 60) - 1);
    return (((v >> EV_CHUNK_LOG) * EV_SHARDS + q) << EV_CHUNK_LOG) | (v & (EV_CHUNK - 1));
}
__host__ __device__ inline unsigned long long ev_enc(uint32_t q, unsigned long long v) {
    return ((unsigned long long)q << 60) | v;
}
// The scratch extent n pairs can need at most: all of them in one stream, whose chunks are every
// EV_SHARDS-th physical chunk.
inline uint64_t ev_worst_extent(uint64_t n) {
    return ((n + EV_CHUNK - 1) >> EV_CHUNK_LOG) * EV_SHARDS * EV_CHUNK;
}

// Rare-path counters of one flush (gwaoi_debug_counters accumulates them).
enum : uint32_t {
    DBG_COMBINED_REPLAY = 0,  // k_combined waves whose event buffer (EVW) overflowed: sweep replayed
    DBG_COMBINED_DRAIN = 1,   // k_combined survivor-queue drains in the middle of a sweep (QCAP full)
    DBG_SPECIAL_GLOBAL = 2,   // special-pass lanes with more events than their LDS slots (global path)
    DBG_N = 4
};

// Device -> host block copied once per tick: result + per-space bbox.
struct TickOut {
    uint32_t n_enter;
    uint32_t n_total;
    uint32_t err;
    uint32_t pad;
    unsigned long long total64;
    unsigned long long seq_max;
    unsigned long long ext64;  // the scratch extent the pair passes reached (their 8 event streams interleaved)
    uint32_t dbg[4];  // TickScalars::dbg
    // followed by int4 bbox[n_spaces] (ordered-int min x, min z, max x, max z)
};

// ---- launchers (gwaoi_kernels.hip) ------------------------------------------
// S' entries base .. base+n_app-1 for the entering slots new_slots[] (host-checked, or a device
// Enter batch: slots out of range or live when the flush began are flagged and left dead).
void launch_init_appended(const uint32_t *new_slots, uint32_t n_app, uint32_t base, Rec16 *s_rec, SlotSp *s_ss,
                          SlotTab info, uint32_t max_slots, TickScalars *sc, hipStream_t st);
// One run of the op queue: ops j0 .. j0+n-1 of this flush.  sp == nullptr
// means a device-resident Moved batch (keep the space).  Op i gets seq
// seqs[i] when seqs is given (explicit: checked >= seq_floor, the largest
// folded into sc->seq_max when track_max), else seq0 + i.
void launch_ops_claim(const uint32_t *slots, uint32_t n, uint32_t j0, uint32_t max_slots,
                      SlotTab info, uint32_t tick_id, TickScalars *sc, hipStream_t st);
// sp == nullptr: every op has space sp_def (SP_KEEP: Moved; a space: Enter; SP_DEAD: Leave, whose
// x / z may be nullptr).
void launch_ops_apply(const uint32_t *slots, const float *x, const float *z, const uint32_t *sp, uint32_t sp_def,
                      uint32_t n, uint32_t j0, uint32_t max_slots, SlotTab info, uint32_t tick_id,
                      uint32_t n_total, const unsigned long long *seqs, uint64_t seq0, uint64_t seq_floor,
                      bool track_max, Rec16 *s_rec, SlotSp *s_ss, TickScalars *sc, hipStream_t st);
// A flush whose queue is only device Moved batches (<= MAX_MOVE_RUNS of them):
// single-pass claim+apply, then a fixup of the slots moved more than once.
constexpr uint32_t MAX_MOVE_RUNS = 4;
struct MoveRun {
    const uint32_t *ds;
    const float *dx, *dz;
    const unsigned long long *dseq;  // explicit seqs (nullptr: seq0 + i)
    const uint32_t *dsp;             // explicit space per op (nullptr: sp_def for every op)
    unsigned long long seq0;
    uint32_t j0, n;  // first op index in the flush, ops
    uint32_t sp_def; // SP_KEEP: Moved (keep the slot's space); a space: Enter; SP_DEAD: Leave
};
struct MoveRuns {
    MoveRun r[MAX_MOVE_RUNS];
    uint32_t count;
};
// s_ss == nullptr: a moves-only flush without the prologue's copy ("virtual S'":
// the spaces are the previous frame's, and an entry of S' not written by an op
// holds an older seq than seq_floor, so k_keygen takes the previous frame's
// record for it and writes it back).  n_marked: runs whose claims are stored
// already (by the prologue: run 0).
// unique (GWAOI_F_UNIQUE_MOVES): no run repeats a slot, so no claims are stored or compared and
// no fixup runs; keygen counts the entries the ops wrote and the scan's fold block checks the
// count against TickScalars::n_unique (ERR_DUP_SLOT).
// The re-apply of the slots moved more than once (k_moves_fixup's arguments).
struct FixupArgs {
    MoveRuns RS;
    uint32_t max_slots, tick, n_total, n_prev;
    unsigned long long seq_floor;
    SlotTab info;
    Rec16 *s_rec;
    SlotSp *s_ss;
    const Rec16 *p_rec;
    TickScalars *sc;
    const uint32_t *coll;
};
void launch_moves(const MoveRuns &RS, uint32_t max_slots, SlotTab info, uint32_t tick_id, uint32_t n_total,
                  uint64_t seq_floor, Rec16 *s_rec, SlotSp *s_ss, const Rec16 *p_rec, uint32_t n_prev,
                  TickScalars *sc, uint32_t *coll, uint32_t n_marked, bool unique, hipStream_t st);
// The same flush through slot buckets (gwaoi_kernels.hip k_mv_*), for worlds whose
// SlotInfo outgrows the MALL (max_slots > MV_MIN_SLOTS; moves_buckets(max_slots) <=
// MV_NB_MAX).  hist: moves_hist_elems(n ops, max_slots) uint32; scan_tmp:
// scan_tmp_elems of that; binned: 16 B per op (<= max_slots ops).
constexpr uint32_t MV_NB_MAX = 8192;
constexpr uint32_t MV_MIN_SLOTS = 1u << 22;
uint32_t moves_buckets(uint32_t max_slots);
size_t moves_hist_elems(uint32_t n, uint32_t max_slots);
void launch_moves_bucketed(const MoveRuns &RS, uint32_t max_slots, SlotTab info, uint32_t n_total,
                           uint64_t seq_floor, Rec16 *s_rec, SlotSp *s_ss, TickScalars *sc, uint32_t *hist,
                           uint32_t *scan_tmp, void *binned, hipStream_t st);
// Zero the per-tick counters and two ranges; bbox entries get the fold
// identity; S' <- the previous frame's first n_copy entries; and (mark != nullptr)
// the claims of a moves-only flush's first run.  n_unique: TickScalars::n_unique (0 = no check).
void launch_prologue(TickScalars *sc, uint32_t *z0, size_t n0, uint32_t *z1, size_t n1, int4 *bbox,
                     uint32_t n_spaces, uint32_t n_copy, const Rec16 *p_rec, const SlotSp *p_ss, Rec16 *s_rec,
                     SlotSp *s_ss, const MoveRun *mark, uint32_t max_slots, SlotTab info, uint32_t tick_id,
                     uint32_t n_unique, hipStream_t st);

// Cell keys of S' and the per-tick scalars d_rel / bmax (via per-block
// partials in blk, 2 * cdiv(n, 256) floats, then cdiv(n, 256) u32 counts of the
// entries this flush's ops wrote).  cnt64 != nullptr (grid
// unchanged): also per-cell entity counts (low word) and arrival counts
// (high word; arrival = cell differs from p_key[i], or i >= n_prev).
// S' entries i < n_prev whose seq is below seq_base (not written by this flush's
// ops) take the previous frame's record, written back into s_rec (see launch_moves).
// The prologue's per-flush zeroing, done by keygen instead when a unique-moves flush skips the
// prologue (its apply writes only sc->err_apply / sc->ndrop, which the keygen fold reads and
// resets, so they are zero when any flush begins): sc's counters, z1[0, n1), the bbox fold
// identity of n_spaces spaces, and sc->n_unique = n_unique.  sc == nullptr: nothing (the prologue ran).
struct TickZero {
    TickScalars *sc;
    uint32_t *z1;
    uint32_t n1;
    int4 *bbox;
    uint32_t n_spaces;
    uint32_t n_unique;
};
void launch_keygen(Rec16 *s_rec, const SlotSp *s_ss, uint32_t n_total, const SpaceGrid *grid,
                   uint32_t sentinel, uint32_t *keys, uint32_t *vals, const Rec16 *p_rec, const SlotSp *p_ss,
                   const SpaceGrid *p_grid, uint32_t n_prev, float *blk, TickScalars *sc, const uint32_t *p_key,
                   unsigned long long *cnt64, uint64_t seq_base, uint32_t *special, const TickZero &tz,
                   unsigned long long *tent, hipStream_t st);
// special (optional, cdiv(n_prev, TILE_A) words): keygen marks the previous-frame tiles that hold an
// entity the special pass must look at; launch_pairs skips the others.
// The stable sort of S' by key when the grid is the previous frame's: the
// new cell_start (from cnt64) plus, per cell, a merge of the entities that
// stayed with the arrivals.  Writes perm / skeys like radix_sort and the
// frame's cell_start (so no separate cell count).  tmp: incr_sort_tmp_elems
// words (the cell scan's tile totals);
// arr_pos: 3 (total_cells + 1) words (arrival cursors, per-cell shifts, changed cells).
size_t incr_sort_tmp_elems(size_t cells);
// true: the sort leaves cnt64 zero for the next flush (zeroed once when allocated)
bool scan_rezeroes_counts();
// The special pass (launch_pairs' arguments), run inside the incremental sort's arrival launch
// (k_arrive_special) when sp != nullptr; n_tiles = the previous frame's tiles.
struct SpecialJob {
    FrameView F;
    const Rec16 *O_rec;
    const SlotSp *O_ss;
    unsigned long long seq_base;
    TickScalars *sc;
    uint2 *tmp;
    uint64_t cap;
    uint32_t *tile_total;
    unsigned long long *tile_base;
    uint32_t tile_off, leave_off;
    const uint32_t *special;
    uint32_t n_tiles;
};
// The gather (launch_gather's arguments), run inside the incremental sort's merge launch
// (k_merge_gather) when gj != nullptr: block b gathers scan tile b's range of the new frame once it
// has merged the tile's changed cells, and writes bbox part b (incr_sort_tiles parts, which
// launch_finish folds).  The sort's perm / skeys are the gather's.
struct GatherJob {
    uint32_t n_new, n_prev;
    const Rec16 *s_rec;
    const SlotSp *s_ss;
    const Rec16 *p_rec;
    const SlotSp *p_ss;
    Rec16 *f_rec;
    SlotSp *f_ss;
    Rec16 *o_rec;
    uint4 *cand;
    const SpaceGrid *grid;
    SlotTab info;
    TickScalars *sc;
    int4 *bbox;
    uint32_t n_spaces;
    void *parts;
};
// scan tiles of a grid of total_cells cells (the fused gather's bbox parts)
uint32_t incr_sort_tiles(uint32_t total_cells);
void incremental_sort(const uint32_t *keys, uint32_t n_total, uint32_t n_prev, const uint32_t *p_key,
                      const uint32_t *p_cell_start, unsigned long long *cnt64, uint32_t total_cells,
                      uint32_t sentinel, uint32_t *cell_start, uint32_t *arr_pos, uint32_t *arr_idx,
                      unsigned long long *tmp, uint32_t *perm, uint32_t *skeys, const float *blk,
                      TickScalars *sc, const SpecialJob *sp, const GatherJob *gj, hipStream_t st);
// LSD radix sort of (key,val) pairs on `bits` low key bits.  Returns which
// buffer (0 or 1) holds the result.
struct SortBuffers {
    uint32_t *keys[2];
    uint32_t *vals[2];
    uint32_t *hist;      // >= radix_hist_elems(n)
    uint32_t *scan_tmp;  // scratch for the scan of hist
};
int radix_sort(SortBuffers &b, uint32_t n, int bits, hipStream_t st);
size_t radix_hist_elems(uint32_t n);
// Exclusive scan (in place allowed); `tmp` needs scan_tmp_elems(n) uint32.
void scan_exclusive(const uint32_t *in, uint32_t *out, size_t n, uint32_t *tmp, hipStream_t st);
size_t scan_tmp_elems(size_t n);

// New frame (f_rec/f_ss), previous state in the new order (o_rec), and the
// combined pass's candidate records cand = {x, z, old x, old z} (x, z NaN for a jumper).
void launch_gather(const uint32_t *perm, uint32_t n_new, uint32_t n_prev, const Rec16 *s_rec, const SlotSp *s_ss,
                   const Rec16 *p_rec, const SlotSp *p_ss, Rec16 *f_rec, SlotSp *f_ss, Rec16 *o_rec, uint4 *cand,
                   const SpaceGrid *grid, uint64_t seq_base, SlotTab info, const uint32_t *sorted_keys,
                   uint32_t sentinel, uint32_t n_total, TickScalars *sc, uint32_t *f_key, int4 *bbox,
                   uint32_t n_spaces, void *bbox_parts, hipStream_t st);
void launch_cell_count(const uint32_t *sorted_keys, uint32_t n, uint32_t *cnt, hipStream_t st);

// Combined pass over the new frame: blocks of TILE_A consecutive entries
// (O = previous state in the new order, NaN where not live in the same space).
// Directed event pairs go to tmp at an atomically reserved offset per block;
// block t's enter total/base are at [t], its leave total/base at [leave_off + t].
inline uint32_t combined_blocks(uint32_t n) { return (n + TILE_A - 1) / TILE_A; }
#ifndef GWAOI_CT
#define GWAOI_CT 256
#endif
// entities per k_combined tile (= threads per workgroup; the special pass keeps TILE_A)
constexpr uint32_t COMBINED_TILE = GWAOI_CT;
__host__ __device__ inline uint32_t combined_tiles(uint32_t n) { return (n + COMBINED_TILE - 1) / COMBINED_TILE; }
void launch_combined(FrameView F, const uint4 *cand, const Rec16 *O_rec, uint64_t seq_base, TickScalars *sc,
                     uint32_t *tmp_pairs, uint64_t cap, uint32_t *tile_total, unsigned long long *tile_base,
                     uint32_t leave_off, const uint32_t *tile_order, uint32_t *tile_work, uint8_t *ework,
                     hipStream_t st,
                     hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// The schedule: tile_order[1 + i] = the i-th tile of the XCD ranges laid end to end, heaviest first
// within each range; tile_order[2 + n_tiles + x] .. = the eight ranges' cuts (cumulative measured
// time, tile_work); tile_order[0] = the tile count it was built for (k_combined ignores it
// otherwise).  launch_finish builds it for the next flush when given the buffers.
// Special-entity pass over the previous frame in blocks of TILE_A entries
// (O = S', the new state in the previous order, with O_ss giving its space);
// block t's totals/bases at [tile_off + t] and [leave_off + tile_off + t].
void launch_pairs(FrameView F, const Rec16 *O_rec, const SlotSp *O_ss, uint64_t seq_base, TickScalars *sc,
                  uint32_t *tmp_pairs, uint64_t cap, uint32_t *tile_total, unsigned long long *tile_base,
                  uint32_t tile_off, uint32_t leave_off, const uint32_t *special, hipStream_t st);
// The flush's tail in one launch: every tile's events from tmp into tile order
// (`out` may be host-mapped pinned memory, and hbbox, when given, receives the
// folded per-space boxes there: the flush summary needs no copy)
// (a block's offset: the group totals the pair passes added, then its group's
// tile totals before it), the scalars of TickOut, and the per-space bbox fold
// (k_gather's parts).
// tile_total words for n_entries entries: the totals, one spare, then any group totals (all zeroed per flush)
size_t tile_total_elems(size_t n_entries);
// the first event of each mirrored pair of a flush's [enters | leaves] (n_pairs of them) into pinned host memory
void launch_pairs_out(const void *events, uint64_t n_pairs, void *dst, hipStream_t st);
void launch_finish(const uint32_t *tile_total, const unsigned long long *tile_base, uint32_t n_entries,
                   uint32_t n_enter_entries, const uint32_t *tmp_pairs,
                   uint32_t *out_pairs, uint64_t cap_tmp, uint64_t cap_out, const TickScalars *sc, TickOut *out,
                   uint32_t n_new, int4 *bbox, uint32_t n_spaces, void *parts_mem, uint32_t n_parts, int4 *hbbox,
                   const uint32_t *tile_work, uint32_t *tile_order, uint32_t *dcount, hipStream_t st);
// Size of k_gather's level-1 bbox parts (+ the fold's scratch part), folded by launch_finish;
// gather_parts: how many k_gather writes for n entries.
size_t bbox_part_bytes(uint32_t n);
uint32_t gather_parts(uint32_t n);
void launch_neighbors(FrameView F, SlotTab info, uint32_t slot, uint32_t *out, uint32_t cap,
                      uint32_t *count, hipStream_t st);
// Zero `n` uint32 (rare re-run path).
void launch_zero(uint32_t *p, size_t n, hipStream_t st);
// The flush's events [enters | leaves] (pairs) as per-slot rows (gwaoi_events_csr):
// off[n_rows + 1] (exclusive scan of the counts, cnt is scratch), items[n_total]
// = b | 0x80000000 for an enter, each row sorted (leaves first).
void launch_events_csr(const uint32_t *ev_pairs, uint64_t n_enter, uint64_t n_total, uint32_t n_rows, uint32_t *cnt,
                       uint32_t *off, uint32_t *scan_tmp, uint32_t *items, uint32_t *scratch, uint32_t *long_rows,
                       hipStream_t st);

// Sparse flush of k host Moved calls on a frame in place (gwaoi_sparse.hip): claims must be stored
// first (launch_ops_claim, this tick).  cnt: sparse_cnt_elems(k) words.  The flush's summary goes to
// res (TickOut.pad != 0: declined, nothing changed); its events [enters | leaves] to out (cap pairs).
size_t sparse_cnt_elems(uint32_t k);
// op_seq == nullptr: op j's seq is seq0 + j.
void launch_sparse(Rec16 *rec, SlotSp *ss, uint32_t *key, uint32_t *cell_start, const SpaceGrid *grid,
                   SlotTab info, const uint32_t *op_slot, const float *op_x, const float *op_z,
                   const unsigned long long *op_seq, uint64_t seq0, uint32_t k, uint32_t tick, uint32_t *cnt,
                   uint32_t *out, uint64_t cap, TickOut *res, hipStream_t st);
// The same flush in one launch for k <= sparse_fused_max() ops (no claims stored): scr holds
// 2 * scr_cap words per op, done one zeroed word (re-armed by the kernel).  TickOut.pad 3: an op
// outgrew its scratch row (nothing written; run launch_sparse instead).
uint32_t sparse_fused_max();
void launch_sparse_fused(Rec16 *rec, SlotSp *ss, uint32_t *key, uint32_t *cell_start, const SpaceGrid *grid,
                         SlotTab info, const uint32_t *op_slot, const float *op_x, const float *op_z,
                         const unsigned long long *op_seq, uint64_t seq0, uint32_t k, uint32_t *cnt, uint32_t *scr,
                         uint32_t scr_cap, uint32_t *done, uint32_t *out, uint64_t cap, TickOut *res, hipStream_t st);

// ---- world accessors for the entity-sync layer (gwaoi_sync.cpp) -------------
struct SyncState;
struct WorldView {
    FrameView F;           // frame of the last flush
    SlotTab info;  // per slot: .rank = index in F for slots in F
    hipStream_t st;
    uint32_t max_slots;
    size_t pending_ops;     // calls queued since the last flush (or a flush in flight)
    bool in_flight;         // gwaoi_tick_begin without its gwaoi_tick_finish yet
    const uint32_t *events; // last flush's events (device): [enters | leaves] as (a,b) pairs
    uint64_t n_enter, n_leave;
};
WorldView world_view(gwaoi_world *w);
SyncState *&world_sync(gwaoi_world *w);
void world_set_error(gwaoi_world *w, const char *msg);
// Queue a device Moved batch whose ops carry their space (a decoded position
// packet): op i moves d_slots[i] in space d_sp[i]; SLOT_NONE ops are no-ops.
int world_queue_decoded(gwaoi_world *w, const uint32_t *d_slots, const float *d_x, const float *d_z,
                        const uint32_t *d_sp, size_t n);
// The event buffer, device counts {n_enter, n_total} (written by the flush's k_finish) and event
// capacity of the flush in flight (gwaoi_tick_begin .. _end) or, when none is, of the last
// committed one: for work queued on the world's stream behind the flush (the strip filter).
// Events past the capacity were not written (the flush re-runs them at its end).
void world_flush_events(gwaoi_world *w, const uint32_t **events, const uint32_t **dcount, uint64_t *cap);
// Space of a slot in call order (as queued so far), SP_DEAD if not in one.
uint32_t world_slot_space(gwaoi_world *w, uint32_t slot);
// Hooks the world calls when a sync layer is attached.
void sync_note_slot(SyncState *s, uint32_t slot, uint32_t space_or_dead);
bool sync_slot_plain(const SyncState *s, uint32_t slot);  // in a space without AOI
void sync_destroy(SyncState *s);

}  // namespace gw
