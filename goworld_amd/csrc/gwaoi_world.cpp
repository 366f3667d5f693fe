// gwaoi_world.cpp -- host side of libgwaoi: the C ABI of include/gwaoi.h.
//
// Mirrors go-aoi's AOIManager contract as GoWorld's Space drives it
// (engine/entity/Space.go:105,211,221,243,259; callbacks Entity.go:227-246):
// calls are queued in order with increasing sequence numbers and flushed by
// gwaoi_tick(), which runs the HIP pipeline of gwaoi_kernels.hip and returns
// the net enter/leave events.  Device state lives in HBM between flushes:
// two sorted frames (previous / current) plus working buffers, all sized for
// max_slots entities at creation so that a flush never allocates unless the
// grid or the event buffer must grow.

#include "gwaoi_internal.h"
#include "../../include/gwaoi.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdio>
#ifdef GWAOI_EXP_HOSTTIME
#include <chrono>
#endif
#include <cstdlib>
#include <cstring>
#include <limits>
#include <new>
#include <string>
#include <thread>
#include <vector>

using gw::SpaceGrid;

// k_finish writes the flush summary (TickOut + per-space boxes) straight into
// pinned host memory: a copy after it would be a blit kernel of ~4 us per flush
// at config 3 (profiles/archive/r03_trace_base.txt)

namespace {

enum Stage { ST_APPLY, ST_KEYGEN, ST_SORT, ST_GATHER, ST_CELLS, ST_COMBINED, ST_SPECIAL, ST_FINISH, ST_D2H, ST_N };
const char *kStageNames[ST_N] = {"apply",    "keygen",  "sort",   "gather", "cells",
                                 "combined", "special", "finish", "d2h"};

struct DevFrame {
    gw::Rec16 *rec = nullptr;
    gw::SlotSp *ss = nullptr;
    uint32_t *key = nullptr;  // cell key of every entry (the next flush's "previous cell")
    uint32_t *cell_start = nullptr;
    size_t cell_cap = 0;  // entries allocated in cell_start
    SpaceGrid *grid = nullptr;
    std::vector<SpaceGrid> hgrid;  // host mirror of `grid` (upload only on change)
    uint32_t n = 0;
    uint32_t total_cells = 0;
};

struct SpaceHost {
    bool used = false;
    float D = 0.f;
    uint32_t alive = 0;
    bool have_bbox = false;  // device bbox of the last flush
    float bx0 = 0, bz0 = 0, bx1 = 0, bz1 = 0;
    bool pend = false;  // bbox of Enter positions queued since the last flush
    float px0 = 0, pz0 = 0, px1 = 0, pz1 = 0;
    SpaceGrid grid{};
    bool grid_valid = false;
};

enum RunKind : uint8_t { RUN_MOVE = 0, RUN_ENTER = 1, RUN_LEAVE = 2 };

struct Run {  // a stretch of the op queue: host ops [hbegin, hend) or a device batch
    bool device;
    uint8_t kind;    // device batch: RUN_MOVE, or a structural batch (gwaoi_enter/leave_batch_device)
    uint32_t space;  // RUN_ENTER / RUN_LEAVE: the space
    size_t hbegin, hend;
    const uint32_t *ds;
    const float *dx, *dz;
    const unsigned long long *dseq;  // explicit device seqs (nullptr: seq0 + i)
    const uint32_t *dsp;             // explicit space per op (nullptr: keep the slot's space)
    uint64_t seq0;
    size_t dn;
    bool checked;  // a host batch validated while staged (gwaoi_moved_batch): every slot live, finite positions
};

// Persistent host threads for the validation + staging of big move batches
// (a thread start per call costs ~20 us each; a tick stages 1M moves).
class StagePool {
  public:
    ~StagePool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread &t : th_) t.join();
    }
    // f(0) .. f(T-1), f(0) on the calling thread.  Falls back to running on the
    // caller when threads cannot be started.
    void run(unsigned T, const std::function<void(unsigned)> &f) {
        if (T <= 1) {  // inline: no wake-up of the workers
            if (T) f(0);
            return;
        }
        while (th_.size() + 1 < T) {
            try {
                const unsigned id = (unsigned)th_.size() + 1;
                th_.emplace_back([this, id] { loop(id); });
            } catch (...) {
                break;
            }
        }
        const unsigned Tw = std::min<unsigned>(T, (unsigned)th_.size() + 1);
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &f;
            T_ = Tw;
            left_ = Tw - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        for (unsigned t = Tw; t < T; ++t) f(t);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return left_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(unsigned id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)> *job;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (id >= T_) continue;
                job = job_;
            }
            (*job)(id);
            std::lock_guard<std::mutex> g(m_);
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)> *job_ = nullptr;
    unsigned T_ = 0, left_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// A call made while a flush is in flight (gwaoi_tick_begin .. _end): validated
// and given its seq at call time, queued for the next flush at the commit.
struct Deferred {
    enum Kind : uint8_t { MOVED, ENTER, LEAVE, RUN } kind;
    uint32_t slot, space;
    float x, z;
    uint64_t seq;
    Run run;  // RUN: a staged or device batch
};
struct DeferredBox {  // Enter/Moved positions of a deferred staged batch, per space
    uint32_t space;
    float x0, z0, x1, z1;
};

// Event capacities of one launch of the pair passes: the shared scratch (in pairs of the streams'
// interleaved extent) and the flush set's buffer (in events).
struct EvCaps {
    uint64_t tmp, out;
};

// The buffers one flush writes that the flush after it must leave alone while the
// first may still be re-run (event buffer regrow) or read by the caller: two
// sets, alternated per launch, so that flush t+1 can be launched before flush
// t's summary has reached the host (gwaoi_tick_finish with GWAOI_END_NEXT).
struct FlushSet {
    gw::Rec16 *srec = nullptr;  // S': previous frame + this flush's ops, previous order
    gw::SlotSp *sss = nullptr;
    gw::Rec16 *orec = nullptr;  // previous state in the new frame's order (NaN if absent)
    uint4 *cand = nullptr;      // combined-pass candidate records of the new frame (x, z, old x, old z; NaN = jumper)
    gw::TickScalars *sc = nullptr;
    uint32_t *events = nullptr;  // ev_cap (a,b) pairs: [enters | leaves] in tile order
    uint64_t ev_cap = 0;         // capacity in directed pairs
    // the pair passes' scratch (evtmp_cap pairs: per-tile chunks of the eight event streams) and the
    // per-tile event totals / stream positions: per set, so that a flush's pair passes and finish
    // can run while the next flush's first kernels (which zero the totals and write the special
    // pass's events) already run on the early stream
    uint32_t *evtmp = nullptr;
    uint64_t evtmp_cap = 0;
    uint32_t *tile_total = nullptr;
    unsigned long long *tile_base = nullptr;
    size_t tile_entries_cap = 0;
    hipEvent_t mid_ev = nullptr;  // recorded after the flush's early kernels (the next flush's early stream waits)
    void *bbox_parts = nullptr;  // bbox level-1 partials
    uint32_t n_parts = 0;        // ... written by the flush (k_gather's blocks or k_merge_gather's tiles)
    char *dev_out = nullptr;     // device counts (2 words) | int4 bbox[max_spaces] from kDevBBox on (the bbox fold)
    char *h_out = nullptr;       // pinned: the flush summary (TickOut + bbox)
    char *d_hout = nullptr;      // h_out as the device sees it: k_finish writes the summary there
    hipEvent_t done_ev = nullptr;  // recorded after the flush's last kernel
    hipEvent_t ev[ST_N][2] = {};   // stage timing
    bool ev_used[ST_N] = {};
};

}  // namespace

struct gwaoi_world {
    gwaoi_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t max_slots = 0, max_spaces = 0;
    float cells_per_dist = 1.0f;  // cells per AOI distance of the grids in use
    // Cell size by density (gwaoi_config.cells_per_dist == 0): clustered crowds want D/3,
    // sparse uniform worlds D/2 (fewer cells to scan and merge; config 5: 5.25 vs 5.91 ms,
    // config 4: 4.35 vs 4.95, config 3: 0.316 vs 0.283).  The measure is the mean number of
    // neighbours per entity, kept from the flushes' enter/leave counts.
    bool cells_auto = true;
    int64_t rel_pairs = 0;     // directed relation pairs after the last committed flush
    uint32_t cpd_streak = 0;   // consecutive flushes recommending another cell size
    float cpd_rec = 3.0f;

    // three frames: the last committed one, the one a flush in flight writes, and (while a
    // flush launched before the commit of the one in flight runs) the one that flush writes
    DevFrame fr[3];
    int cur = 0;  // fr[cur] = frame of the last committed flush
    FlushSet fs[2];
    int launch_set = 0;  // set the next launch uses (alternates)
    int last_set = 0;    // set of the last committed flush (its events)

    // working set (max_slots entries each)
    uint32_t *keys[2] = {nullptr, nullptr}, *vals[2] = {nullptr, nullptr};
    uint32_t *hist = nullptr;
    uint32_t *scan_tmp = nullptr;
    size_t scan_tmp_cap = 0;
    gw::SlotTab sinfo{};  // per slot: last op claim, S' index, space (three arrays)
    // incremental frame sort (grid unchanged): per-cell counts, arrival lists
    unsigned long long *cnt64 = nullptr, *scan64_tmp = nullptr;
    uint32_t *arr_pos = nullptr, *arr_idx = nullptr;
    uint32_t *coll = nullptr;  // slots moved twice in one flush (single-pass apply)
    uint32_t *special = nullptr;  // per previous-frame tile: keygen saw a special entity (the special pass's skip list)
    uint32_t *tile_work = nullptr;   // per combined tile: its measured time, then its candidates (k_combined)
    uint32_t *tile_order = nullptr;  // the next flush's combined tile order, heaviest first (k_tile_order)
    uint8_t *ework = nullptr;        // per frame entry: log2 of the candidates its lane swept (the next flush's deal)
    uint32_t *mv_hist = nullptr;  // bucketed apply: the bucket-major histogram, scanned (gw::launch_moves_bucketed)
    uint4 *mv_binned = nullptr;  // bucketed apply: the ops regrouped by slot bucket (16 B each)
    bool moves_bucketed = false;   // the bucketed apply (max_slots > MV_MIN_SLOTS; GWAOI_MOVES_BUCKETED forces it)
    size_t cnt64_cap = 0;
    // test and diagnostics flags (GWAOI_F_TEST_*, include/gwaoi.h)
    bool force_radix = false;  // always the full radix sort (checks the incremental sort against it)
    bool force_copy = false;   // S' always copied by the prologue (checks virtual S' against it)
    bool inject_regrow_fail = false;  // the event regrow fails (the poison path)
    hipEvent_t done_ev = nullptr;  // wait_stream's marker (polled)
    hipEvent_t order_ev = nullptr;  // gwaoi_stream_after / _before
    // Overlapped flushes (speculative launches only): flush t+1's early kernels (apply .. gather)
    // run on early_st while flush t's pair passes and finish still run on the stream.  gen counts
    // the enqueues on the stream from anything but a flush; an early stream may skip only work
    // the previous flush queued (gen unchanged since its launch: gen_launch).
    hipStream_t early_st = nullptr;
    uint64_t gen = 0, gen_launch = ~0ull;
    bool ovl_ok = false;   // set around a speculative launch (end_begin)
#ifdef GWAOI_EXP_HOSTTIME  // diagnostics build only: host time per phase of gwaoi_tick_finish(NEXT), printed at destroy
    double ht[6] = {};     // entry -> first kernel queued, launch total, wait for the summary, commit, call total, calls
    std::chrono::steady_clock::time_point ht_entry;
#endif
    bool mid_last = false;  // the last flush recorded its set's mid_ev
    bool check_stages = false;   // wait after every flush stage (fault diagnosis)
    const char *fault_stage = nullptr;  // stage at the first failed wait
    bool fault_before = false;          // ... the wait before it (else after it)
    uint32_t *new_slots_d = nullptr;
    uint32_t *op_slot = nullptr, *op_sp = nullptr;
    float *op_x = nullptr, *op_z = nullptr;
    unsigned long long *op_seq = nullptr;
    size_t op_cap = 0;
    float *blk = nullptr;        // keygen per-block partials
    uint32_t *nb_out = nullptr, *nb_count = nullptr;
    size_t nb_cap = 0;
    // per-slot rows of the last flush's events (gwaoi_events_csr), built on request
    uint32_t *csr_cnt = nullptr, *csr_off = nullptr, *csr_items = nullptr, *csr_long = nullptr;
    uint64_t csr_items_cap = 0;
    uint32_t *h_csr_off = nullptr, *h_csr_items = nullptr;
    uint64_t h_csr_items_cap = 0;
    uint64_t csr_tick = ~0ull;  // flush the device CSR belongs to

    // pinned host mirrors
    uint32_t *h_events = nullptr;
    uint64_t h_ev_cap = 0;
    SpaceGrid *h_grid = nullptr;

    // host bookkeeping
    std::vector<uint8_t> alive, in_frame, appended;
    std::vector<uint32_t> space_of;
    std::vector<SpaceHost> spaces;
    uint32_t n_space_ids = 0;  // 1 + highest space id ever created
    uint32_t n_spaces_live = 0;
    std::vector<uint32_t> h_op_slot, h_op_sp;
    std::vector<float> h_op_x, h_op_z;
    std::vector<unsigned long long> h_op_seq;
    std::vector<Run> runs;
    size_t n_ops = 0;
    // device Enter/Leave batches (gwaoi_enter/leave_batch_device) queued for the next flush: their
    // slots are known on the device only, so the per-slot host mirror (alive, space_of, in_frame)
    // goes stale and is rebuilt from the frame on demand (host_slots)
    uint32_t dev_app = 0;     // entries the queued device Enter batches append to S'
    bool dev_struct = false;  // a device Enter/Leave batch is queued
    bool slots_stale = false; // the host mirror misses device Enter/Leave batches of committed flushes
    // host move batches (gwaoi_moved_batch) staged as [slots | x | z | space] in pinned memory and sent
    // with one async H2D each (copy stream); they then run as device batches.  Two halves: the calls
    // queued while a flush is in flight stage into the half that flush does not read.
    uint32_t *h_stage[2] = {nullptr, nullptr}, *d_stage[2] = {nullptr, nullptr};
    size_t stage_cap[2] = {0, 0}, stage_used[2] = {0, 0};
    int stage_cur = 0;
    // sparse flush (gwaoi_sparse.hip): per-op counts and offsets, and the host ops' upload buffer
    // (sp_ops_layout: pinned -> device in one copy); off with GWAOI_F_NO_SPARSE
    uint32_t *sp_cnt = nullptr;
    uint8_t *h_sp_ops = nullptr, *d_sp_ops = nullptr;
    // the fused form (one launch; GWAOI_F_TEST_SPARSE_SEQUENCE: the kernel sequence): per-op scratch
    // rows of sp_scr_cap events per kind (GWAOI_F_TEST_SPARSE_SCR2: 2), and its arrival counter
    uint32_t *sp_scr = nullptr, *sp_done = nullptr;
    uint32_t sp_scr_cap = 512;
    bool sparse_fused = true;
    bool sparse_on = true;
    // zero-copy batch (gwaoi_moved_batch_stage / _commit): the caller fills [slots | x | z | space]
    size_t resv_n = 0;        // moves reserved (0: no reservation)
    uint32_t *resv_h = nullptr, *resv_d = nullptr;
    int resv_half = 0;
    // event copies to the host beside the next flush (gwaoi_tick_finish, GWAOI_END_HOST / _PAIRS)
    hipStream_t out_st = nullptr;
    hipEvent_t out_ev = nullptr;
    bool out_pending = false;  // a copy-out of events queued by gwaoi_tick_finish, not yet waited for
    bool out_pairs = false;    // ... of one event per mirrored pair (GWAOI_END_PAIRS)
    // the counts of the flush whose events h_events holds (a later commit without a copy-out, e.g.
    // gwaoi_tick_finish without a host mode, changes last_n_* but not the host copy)
    uint64_t out_n_enter = 0, out_n_leave = 0;
    uint32_t *d_h_events = nullptr;  // h_events as the device sees it (k_pairs_out writes through it)
    // GWAOI_F_UNIQUE_MOVES: the Moved batches of one flush never repeat a slot (no claims, no fixup)
    bool unique_moves = false;
    hipStream_t copy_st = nullptr;  // staging H2D copies
    hipEvent_t copy_ev = nullptr;   // recorded after the last staging copy
    bool copy_pending = false;      // the flush must wait for copy_ev
    StagePool pool;
    unsigned stage_threads = 8;  // host threads validating + staging one big batch
    std::vector<uint32_t> new_slots;
    std::vector<uint32_t> touched;  // slots whose liveness changed since the last flush
    // seq_next: the seq the next implicit call gets (advanced at queue time);
    // seq_floor: seq_next at the last flush = lower bound of this flush's seqs.
    uint64_t seq_next = 1, seq_floor = 1;
    bool space_ops_queued = false;  // an Enter or Leave is queued for the next flush
    bool dev_seq_pending = false;  // an explicit-seq device batch is queued (its max is known after the flush)
    uint32_t tick_id = 0;
    uint64_t ticks = 0;
    uint32_t n_alive = 0;
    // ---- flush in flight (gwaoi_tick_begin -> gwaoi_tick_finish).  The op queue (runs, host op
    // arrays, new_slots, touched) stays frozen until the commit: calls made meanwhile are
    // deferred, then queued for the next flush.
    bool in_flight = false;
    struct Flight {
        uint32_t tick_id;
        size_t entries;
        uint64_t seq_next;  // seq_next when the flush's queue was closed (the next flush's floor)
        uint64_t seq_base;  // the flush's seq floor (every seq of it is >= seq_base)
        bool dev_seq;       // it held an explicit-seq device batch
        int set;            // FlushSet it writes
        int p_idx, n_idx;   // previous / new frame
        const gw::SlotSp *s_ss_view;  // its S' spaces: the set's sss, or the previous frame's (virtual S')
        EvCaps cap;         // event capacities its pair passes were launched with (writes clipped to them)
        std::vector<uint8_t> touched_alive;  // liveness of touched[i] when the queue was closed
    } fl;

    std::vector<Deferred> deferred;
    std::vector<DeferredBox> deferred_boxes;
    uint64_t last_n_enter = 0, last_n_leave = 0;
    gwaoi_debug dbg{};  // rare-path counters, accumulated over flushes

    // stage timing: bit s of timing_mask = time stage s with HIP events
    uint32_t timing_mask = 0;
    double stage_ms[ST_N] = {};
    uint64_t stage_calls[ST_N] = {};

    std::string last_error;
    // A flush that failed after its kernels rewrote the per-slot records (SlotInfo) for a frame it
    // could not commit leaves host and device state apart: every later call returns GWAOI_EDEVICE.
    bool poisoned = false;
    std::string poison_msg;
    gw::SyncState *sync = nullptr;  // entity position-sync layer (gwaoi_sync.h), created on first use
};

namespace {

// A poisoned world refuses every call (see gwaoi_world::poisoned).
#define GW_LIVE(w)                                 \
    do {                                           \
        if ((w)->poisoned) {                       \
            (w)->last_error = (w)->poison_msg;     \
            return GWAOI_EDEVICE;                  \
        }                                          \
    } while (0)

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            w->last_error = std::string(#expr) + ": " + hipGetErrorString(e_);               \
            return GWAOI_EDEVICE;                                                             \
        }                                                                                     \
    } while (0)

template <class T>
int dalloc(gwaoi_world *w, T **p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void **)p, n * sizeof(T));
    if (e != hipSuccess) {
        w->last_error = std::string("hipMalloc: ") + hipGetErrorString(e);
        *p = nullptr;
        return e == hipErrorOutOfMemory ? GWAOI_ENOMEM : GWAOI_EDEVICE;
    }
    return GWAOI_OK;
}

template <class T>
void dfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

inline bool finite2(float x, float z) { return std::isfinite(x) && std::isfinite(z); }

void stage_begin(gwaoi_world *w, FlushSet &S, Stage s) {
    if (w->check_stages && !w->fault_stage && hipStreamSynchronize(w->stream) != hipSuccess) {
        w->fault_stage = kStageNames[s];
        w->fault_before = true;
    }
    if (!(w->timing_mask >> s & 1u)) return;
    (void)hipEventRecord(S.ev[s][0], w->stream);
    S.ev_used[s] = true;
}
void stage_end(gwaoi_world *w, FlushSet &S, Stage s) {
    if (w->check_stages && !w->fault_stage && hipStreamSynchronize(w->stream) != hipSuccess)
        w->fault_stage = kStageNames[s];
    if (!(w->timing_mask >> s & 1u)) return;
    (void)hipEventRecord(S.ev[s][1], w->stream);
}
void stage_collect(gwaoi_world *w, FlushSet &S) {
    for (int s = 0; s < ST_N; ++s) {
        if (!S.ev_used[s]) continue;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, S.ev[s][0], S.ev[s][1]) == hipSuccess) {
            w->stage_ms[s] += ms;
            w->stage_calls[s] += 1;
        }
        S.ev_used[s] = false;
    }
}

// Wait until the world's stream has drained.  The flush ends with a small D2H
// that the host needs at once; polling an event returns as soon as it lands,
// where the blocking wait of hipStreamSynchronize adds tens of microseconds of
// wake-up latency to every tick.
int wait_stream(gwaoi_world *w) {
    if (!w->done_ev) {
        HIP_TRY(hipStreamSynchronize(w->stream));
        return GWAOI_OK;
    }
    HIP_TRY(hipEventRecord(w->done_ev, w->stream));
    hipError_t e;
    while ((e = hipEventQuery(w->done_ev)) == hipErrorNotReady) __builtin_ia32_pause();
    HIP_TRY(e);
    return GWAOI_OK;
}

int ensure_scan_tmp(gwaoi_world *w, size_t n) {
    size_t need = gw::scan_tmp_elems(n) + 16;
    if (need <= w->scan_tmp_cap) return GWAOI_OK;
    w->gen++;  // (an enqueue on the stream that no flush made: the next flush's early kernels wait for it)
    HIP_TRY(hipStreamSynchronize(w->stream));
    dfree(w->scan_tmp);
    int rc = dalloc(w, &w->scan_tmp, need);
    if (rc) return rc;
    w->scan_tmp_cap = need;
    return GWAOI_OK;
}

// Room for `pairs` directed events in set S's event buffer and for a scratch extent of `extent`
// pairs in the shared scratch (the pair passes' eight event streams interleave there, so their
// extent may exceed the event count).  Grows only S's buffer: the other set may hold the events of
// a committed flush the caller has not read yet.  exact: grow S's buffer to `pairs` and no more
// (matching the twin set's capacity: with slack, the two sets would outgrow each other on every
// flush).
int ensure_events(gwaoi_world *w, FlushSet &S, uint64_t pairs, uint64_t extent, bool exact = false) {
    if (pairs <= S.ev_cap && extent <= S.evtmp_cap) return GWAOI_OK;
    w->gen++;
    HIP_TRY(hipStreamSynchronize(w->stream));
    int rc;
    if (pairs > S.ev_cap) {
        const uint64_t cap = exact ? pairs : std::max<uint64_t>(pairs + pairs / 4, S.ev_cap * 2);
        dfree(S.events);
        S.ev_cap = 0;
        if ((rc = dalloc(w, &S.events, 2 * cap))) return rc;
        S.ev_cap = cap;
    }
    if (extent > S.evtmp_cap) {
        const uint64_t cap = std::max<uint64_t>(extent + extent / 4, S.evtmp_cap * 2);
        dfree(S.evtmp);
        S.evtmp_cap = 0;
        if ((rc = dalloc(w, &S.evtmp, 2 * cap))) return rc;
        S.evtmp_cap = cap;
    }
    return GWAOI_OK;
}


int ensure_tile_entries(gwaoi_world *w, FlushSet &S, size_t entries) {
    if (entries + 1 <= S.tile_entries_cap) return GWAOI_OK;
    w->gen++;
    size_t cap = std::max<size_t>(entries + 1 + entries / 4, 1024);
    HIP_TRY(hipStreamSynchronize(w->stream));
    dfree(S.tile_total);
    dfree(S.tile_base);
    int rc;
    if ((rc = dalloc(w, &S.tile_total, gw::tile_total_elems(cap))) ||
        (rc = dalloc(w, &S.tile_base, cap))) {
        S.tile_entries_cap = 0;
        return rc;
    }
    S.tile_entries_cap = cap;
    return GWAOI_OK;
}

int wait_done(gwaoi_world *w, hipEvent_t ev);
// Waits for the copy-out gwaoi_tick_finish queued (before h_events is rewritten or freed).
int finish_out(gwaoi_world *w) {
    if (!w->out_pending) return GWAOI_OK;
    w->out_pending = false;
    return wait_done(w, w->out_ev);
}

int ensure_host_events(gwaoi_world *w, uint64_t pairs) {
    if (int rc = finish_out(w)) return rc;
    if (pairs <= w->h_ev_cap) return GWAOI_OK;
    uint64_t cap = std::max<uint64_t>(pairs + pairs / 4, 1024);
    if (w->h_events) (void)hipHostFree(w->h_events);
    w->h_events = w->d_h_events = nullptr;
    w->h_ev_cap = 0;
    // mapped and coherent: k_pairs_out writes it from the device, through its device address
    HIP_TRY(hipHostMalloc((void **)&w->h_events, 2 * cap * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
    HIP_TRY(hipHostGetDevicePointer((void **)&w->d_h_events, w->h_events, 0));
    w->h_ev_cap = cap;
    return GWAOI_OK;
}

int ensure_ops(gwaoi_world *w, size_t n) {
    if (n <= w->op_cap) return GWAOI_OK;
    w->gen++;  // (an enqueue on the stream that no flush made: the next flush's early kernels wait for it)
    size_t cap = std::max<size_t>(n, w->op_cap * 2);
    HIP_TRY(hipStreamSynchronize(w->stream));
    dfree(w->op_slot);
    dfree(w->op_sp);
    dfree(w->op_x);
    dfree(w->op_z);
    dfree(w->op_seq);
    int rc;
    if ((rc = dalloc(w, &w->op_slot, cap)) || (rc = dalloc(w, &w->op_sp, cap)) || (rc = dalloc(w, &w->op_x, cap)) ||
        (rc = dalloc(w, &w->op_z, cap)) || (rc = dalloc(w, &w->op_seq, cap))) {
        w->op_cap = 0;
        return rc;
    }
    w->op_cap = cap;
    return GWAOI_OK;
}

int ensure_incr(gwaoi_world *w, size_t cells) {
    const size_t need = cells + 1;
    if (need <= w->cnt64_cap) return GWAOI_OK;
    w->gen++;  // (an enqueue on the stream that no flush made: the next flush's early kernels wait for it)
    const size_t cap = std::max(need + need / 4, (size_t)1024);
    HIP_TRY(hipStreamSynchronize(w->stream));
    dfree(w->cnt64);
    dfree(w->scan64_tmp);
    dfree(w->arr_pos);
    w->cnt64_cap = 0;
    int rc;
    // arr_pos: the arrival cursors, the per-cell stayer shifts, the changed cells (incremental_sort)
    if ((rc = dalloc(w, &w->cnt64, cap)) || (rc = dalloc(w, &w->arr_pos, 3 * cap)) ||
        (rc = dalloc(w, &w->scan64_tmp, gw::incr_sort_tmp_elems(cap))))
        return rc;
    HIP_TRY(hipMemsetAsync(w->scan64_tmp, 0, gw::incr_sort_tmp_elems(cap) * sizeof(unsigned long long), w->stream));
    HIP_TRY(hipMemsetAsync(w->cnt64, 0, cap * sizeof(unsigned long long), w->stream));  // then kept zero by the sort
    w->cnt64_cap = cap;
    return GWAOI_OK;
}

int ensure_cells(gwaoi_world *w, DevFrame &f, size_t cells) {
    size_t need = cells + 1;
    if (need <= f.cell_cap) return GWAOI_OK;
    w->gen++;  // (an enqueue on the stream that no flush made: the next flush's early kernels wait for it)
    size_t cap = std::max(need + need / 4, (size_t)1024);
    HIP_TRY(hipStreamSynchronize(w->stream));
    dfree(f.cell_start);
    int rc = dalloc(w, &f.cell_start, cap);
    if (rc) {
        f.cell_cap = 0;
        return rc;
    }
    f.cell_cap = cap;
    return GWAOI_OK;
}

void push_host_op(gwaoi_world *w, uint32_t slot, float x, float z, uint32_t sp, uint64_t seq) {
    if (w->runs.empty() || w->runs.back().device) {
        Run r{};
        r.device = false;
        r.hbegin = r.hend = w->h_op_slot.size();
        w->runs.push_back(r);
    }
    w->h_op_slot.push_back(slot);
    w->h_op_x.push_back(x);
    w->h_op_z.push_back(z);
    w->h_op_sp.push_back(sp);
    w->h_op_seq.push_back(seq);
    w->runs.back().hend = w->h_op_slot.size();
    w->n_ops++;
}

void note_pending_bbox(SpaceHost &S, float x, float z) {
    if (!S.pend) {
        S.pend = true;
        S.px0 = S.px1 = x;
        S.pz0 = S.pz1 = z;
    } else {
        S.px0 = std::min(S.px0, x);
        S.px1 = std::max(S.px1, x);
        S.pz0 = std::min(S.pz0, z);
        S.pz1 = std::max(S.pz1, z);
    }
}

void mark_appended(gwaoi_world *w, uint32_t slot) {
    if (!w->in_frame[slot] && !w->appended[slot]) {
        w->appended[slot] = 1;
        w->new_slots.push_back(slot);
    }
}

// Queue the calls deferred while a flush was in flight, in call order, as if
// they had been made now (their seqs were taken at call time).
void replay_deferred(gwaoi_world *w) {
    for (const Deferred &q : w->deferred) {
        switch (q.kind) {
            case Deferred::ENTER:
                note_pending_bbox(w->spaces[q.space], q.x, q.z);
                mark_appended(w, q.slot);
                w->touched.push_back(q.slot);
                push_host_op(w, q.slot, q.x, q.z, q.space, q.seq);
                w->space_ops_queued = true;
                break;
            case Deferred::LEAVE:
                w->touched.push_back(q.slot);
                push_host_op(w, q.slot, 0.f, 0.f, gw::SP_DEAD, q.seq);
                w->space_ops_queued = true;
                break;
            case Deferred::MOVED:
                note_pending_bbox(w->spaces[q.space], q.x, q.z);
                push_host_op(w, q.slot, q.x, q.z, q.space, q.seq);
                break;
            case Deferred::RUN:
                w->runs.push_back(q.run);
                w->n_ops += q.run.dn;
                break;
        }
    }
    for (const DeferredBox &b : w->deferred_boxes) {
        note_pending_bbox(w->spaces[b.space], b.x0, b.z0);
        note_pending_bbox(w->spaces[b.space], b.x1, b.z1);
    }
    w->deferred.clear();
    w->deferred_boxes.clear();
}

void defer(gwaoi_world *w, Deferred::Kind k, uint32_t slot, uint32_t space, float x, float z, uint64_t seq) {
    Deferred q{};
    q.kind = k;
    q.slot = slot;
    q.space = space;
    q.x = x;
    q.z = z;
    q.seq = seq;
    w->deferred.push_back(q);
}

float o2f(int i) {
    int b = i ^ ((i >> 31) & 0x7FFFFFFF);
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}

// Choose the grid of every space for the coming flush.  Any grid is correct
// (cellOf is monotone and clamped); this only keeps cells near D wide and the
// cell count bounded by the population.
// The cell size for a mean of K neighbours per entity: entities per cell ~ (K / 4) / c^2 held
// near 1.3 (config 3: K = 85 -> D/3 or D/4; configs 4 and 5: K = 30-32 -> D/2).
// Only D/2 and D/3 are used (the measured sizes): D/3 from K = 5.33 * 3^2 = 48.  At config 3, D/3 against
// D/4 (round 4): the cell scan, merge and keygen shrink with the cell count, the combined pass grows,
// and the tick is 4 us shorter (241.3 vs 245.4 us, kernel traces).
float recommend_cells_per_dist(double K) { return std::sqrt(K / 5.33) >= 3.0 ? 3.0f : 2.0f; }

void choose_grids(gwaoi_world *w, uint32_t &total_cells, uint32_t &total_rows) {
    uint32_t base = 0, rows = 0;
    // two flushes in a row recommending another cell size: every grid is rebuilt with it (one
    // flush takes the full radix sort)
    bool rebuild = false;
    if (w->cells_auto && w->cpd_streak >= 2) {
        w->cells_per_dist = w->cpd_rec;
        w->cpd_streak = 0;
        rebuild = true;
        w->dbg.cell_size_switches++;
    }
    for (uint32_t s = 0; s < w->n_space_ids; ++s) {
        SpaceHost &S = w->spaces[s];
        SpaceGrid g{};
        g.D = S.used ? S.D : 1.0f;
        bool have = false;
        float x0 = 0, z0 = 0, x1 = 0, z1 = 0;
        if (S.used && S.have_bbox && S.alive) {
            have = true;
            x0 = S.bx0; z0 = S.bz0; x1 = S.bx1; z1 = S.bz1;
        }
        if (S.used && S.pend) {
            if (!have) {
                x0 = S.px0; z0 = S.pz0; x1 = S.px1; z1 = S.pz1;
                have = true;
            } else {
                x0 = std::min(x0, S.px0); z0 = std::min(z0, S.pz0);
                x1 = std::max(x1, S.px1); z1 = std::max(z1, S.pz1);
            }
        }
        if (!S.used || !have || S.alive == 0) {
            g.ox = g.oz = 0.f;
            g.inv = 1.0f / g.D;
            g.gx = g.gz = 1;
        } else {
            const double cap = std::max(64.0, 4.0 * (double)S.alive);
            bool keep = false;
            if (S.grid_valid) {
                const SpaceGrid &o = S.grid;
                const double C = 1.0 / (double)o.inv;
                const double ex1 = o.ox + C * o.gx, ez1 = o.oz + C * o.gz;
                const bool inside = x0 >= o.ox && z0 >= o.oz && x1 <= ex1 && z1 <= ez1;
                const double area_grid = (double)o.gx * o.gz * C * C;
                const double area_box = ((double)x1 - x0 + 4.0 * g.D) * ((double)z1 - z0 + 4.0 * g.D);
                keep = !rebuild && inside && (double)o.gx * o.gz <= cap && area_grid <= 4.0 * area_box + 1.0;
            }
            if (keep) {
                g = S.grid;
            } else {
                const double m = 2.0 * g.D;
                const double ox = (double)x0 - m, oz = (double)z0 - m;
                const double wdt = (double)x1 - x0 + 2 * m, hgt = (double)z1 - z0 + 2 * m;
                double C = (double)g.D / (double)w->cells_per_dist;
                double gx, gz;
                for (;;) {
                    gx = std::max(1.0, std::ceil(wdt / C));
                    gz = std::max(1.0, std::ceil(hgt / C));
                    if (gx * gz <= cap && gx <= 32768 && gz <= 32768) break;
                    C *= 1.25;
                }
                g.ox = (float)ox;
                g.oz = (float)oz;
                g.inv = (float)(1.0 / C);
                g.gx = (uint32_t)gx;
                g.gz = (uint32_t)gz;
            }
        }
        g.base = base;
        base += g.gx * g.gz;
        g.row_base = rows;
        rows += g.gz;
        w->h_grid[s] = g;
        if (S.used && S.alive) {
            S.grid = g;
            S.grid_valid = true;
        } else {
            S.grid_valid = false;
        }
    }
    total_cells = base;
    total_rows = rows;
}

gw::FrameView view_of(const DevFrame &f) {
    gw::FrameView v;
    v.rec = f.rec;
    v.ss = f.ss;
    v.cell_start = f.cell_start;
    v.grid = f.grid;
    v.n = f.n;
    v.total_cells = f.total_cells;
    return v;
}

int bitlen(uint32_t v) {
    int b = 0;
    while (v) {
        ++b;
        v >>= 1;
    }
    return b;
}

gw::TickOut *tick_out(FlushSet &S) { return reinterpret_cast<gw::TickOut *>(S.h_out); }
const int4 *tick_bbox(FlushSet &S) { return reinterpret_cast<const int4 *>(S.h_out + sizeof(gw::TickOut)); }
// The device boxes a line apart from the device counts: k_finish's copy block storing a count while
// its fold block's atomics land on the boxes shared one line and stalled both (6 us at config 3).
constexpr size_t kDevBBox = 256;
int4 *dev_bbox(FlushSet &S) { return reinterpret_cast<int4 *>(S.dev_out + kDevBBox); }
// the events of the last committed flush
uint32_t *last_events(gwaoi_world *w) { return w->fs[w->last_set].events; }

// Pair passes + deterministic reorder.  Block-total entries: [enter totals:
// new-frame blocks | previous-frame blocks] then [leave totals: same order];
// their exclusive scan is the final layout [enters | leaves] in block order.

// Returns the event capacities the passes were given (what the flush's finish must compare the
// count and the scratch extent against: the set's buffer or the shared scratch may grow later, by
// another flush's regrow).
// rerun: the flush's pair passes again after an event-buffer overflow.  By then a speculatively
// launched successor may have rebuilt the shared scheduling buffers (tile order, tile work, per-entry
// work) for the flush after it, so a re-run neither reads nor writes them, and keygen's special-tile
// flags may be the successor's too, so every tile is visited.
EvCaps launch_pair_passes(gwaoi_world *w, FlushSet &S, DevFrame &Fn, DevFrame &P, uint64_t seq_base,
                            const gw::SlotSp *s_ss_view, bool rerun = false, bool special_done = false) {
    hipStream_t st = w->stream;
    const uint32_t TBn = gw::combined_tiles(Fn.n), TBp = gw::combined_blocks(P.n);
    const uint32_t half = TBn + TBp, entries = 2 * half;
    gw::FrameView Vn = view_of(Fn), Vp = view_of(P);
    // the pair passes write their streams into the scratch (capacity evtmp_cap), and k_finish copies
    // them into the set's buffer (ev_cap); a larger extent or count is an overflow (re-run)
    const EvCaps caps{S.evtmp_cap, S.ev_cap};
    const uint64_t cap = caps.tmp;
    // timed with the launch's own start/end events (no marker packets)
    const bool tc = w->timing_mask >> ST_COMBINED & 1u;
    if (tc) S.ev_used[ST_COMBINED] = true;
    const bool order = !rerun;
    gw::launch_combined(Vn, S.cand, S.orec, seq_base, S.sc, S.evtmp, cap, S.tile_total, S.tile_base, half,
                        order ? w->tile_order : nullptr, order ? w->tile_work : nullptr, rerun ? nullptr : w->ework,
                        st,
                        tc ? S.ev[ST_COMBINED][0] : nullptr, tc ? S.ev[ST_COMBINED][1] : nullptr);
    if (!special_done) {  // (special_done: it ran in the sort's arrival launch)
        stage_begin(w, S, ST_SPECIAL);
        gw::launch_pairs(Vp, S.srec, s_ss_view, seq_base, S.sc, S.evtmp, cap, S.tile_total, S.tile_base, TBn,
                         half, rerun ? nullptr : w->special, st);
        stage_end(w, S, ST_SPECIAL);
    }
    // tile order + TickOut + the per-space bboxes for the next flush's grid (one launch)
    stage_begin(w, S, ST_FINISH);
    gw::launch_finish(S.tile_total, S.tile_base, entries, half, S.evtmp, S.events,
                      caps.tmp, caps.out, S.sc, reinterpret_cast<gw::TickOut *>(S.d_hout), Fn.n,
                      dev_bbox(S), w->n_space_ids, S.bbox_parts, S.n_parts,
                      reinterpret_cast<int4 *>(S.d_hout + sizeof(gw::TickOut)),
                      order ? w->tile_work : nullptr, order ? w->tile_order : nullptr,
                      reinterpret_cast<uint32_t *>(S.dev_out), st);
    stage_end(w, S, ST_FINISH);
    return caps;
}

int poison(gwaoi_world *w, int rc) {
    w->poisoned = true;
    w->poison_msg = "world unusable after a failed flush: " + w->last_error;
    w->last_error = w->poison_msg;
    return rc;
}

void replay_deferred(gwaoi_world *w);

// The flush, first half: close the op queue and launch the whole pipeline on
// the world's stream, ending with the D2H of the flush's summary (TickOut);
// returns without waiting.  Calls made until tick_finish are deferred (see
// Deferred).  A failure before any kernel was queued returns with nothing in
// flight.
int tick_launch(gwaoi_world *w) {
    hipStream_t st = w->stream;
    int rc;
    const uint32_t tick_id = ++w->tick_id;
    const uint64_t seq_base = w->seq_floor;  // every seq of this flush is >= seq_base > every earlier one
    const uint32_t n_ops = (uint32_t)w->n_ops;

    // the previous flush's frame, and one no flush that may still be re-run reads
    const int p_idx = w->cur, n_idx = (w->cur + 1) % 3;
    DevFrame &P = w->fr[p_idx];   // previous flush
    DevFrame &Fn = w->fr[n_idx];  // this flush
    const int set = w->launch_set;
    FlushSet &S = w->fs[set];
    const uint32_t n_prev = P.n;
    const uint32_t n_app_host = (uint32_t)w->new_slots.size();
    const uint32_t n_app = n_app_host + w->dev_app;
    const uint32_t n_total = n_prev + n_app;
    const uint32_t n_new = w->n_alive;

    (void)hipGetLastError();  // the launch check below must see this flush's launches only
    // a copy-out still reading a flush set's events (gwaoi_tick_finish) ends before this
    // flush writes into a set
    if (w->out_pending) HIP_TRY(hipStreamWaitEvent(st, w->out_ev, 0));
    // grid for this flush
    uint32_t total_cells = 0, total_rows = 0;
    choose_grids(w, total_cells, total_rows);
    for (uint32_t s = 0; s < w->n_space_ids; ++s) w->spaces[s].pend = false;  // consumed by this grid
    const size_t entries = 2 * ((size_t)gw::combined_tiles(n_new) + gw::combined_blocks(n_prev));
    if ((rc = ensure_cells(w, Fn, total_cells))) return rc;
    if ((rc = ensure_tile_entries(w, S, entries))) return rc;
    // a set whose twin grew on an overflow grows alike before its next flush (one re-run, not two)
    if (S.ev_cap < w->fs[set ^ 1].ev_cap && (rc = ensure_events(w, S, w->fs[set ^ 1].ev_cap, 0, true))) return rc;
    size_t host_ops = 0;
    for (const Run &r : w->runs)
        if (!r.device) host_ops += r.hend - r.hbegin;
    if ((rc = ensure_ops(w, host_ops))) return rc;
    const size_t scan_need = std::max<size_t>({gw::radix_hist_elems(std::max(n_total, 1u)), (size_t)total_cells + 1,
                                               (size_t)total_rows + 1, entries + 1});
    if ((rc = ensure_scan_tmp(w, scan_need))) return rc;
    Fn.total_cells = total_cells;
    Fn.n = n_new;

    const uint32_t ns = std::max(1u, w->n_space_ids);
    const bool grid_same = Fn.hgrid.size() == ns && !std::memcmp(Fn.hgrid.data(), w->h_grid, ns * sizeof(SpaceGrid));
    // the previous frame was cut with the same grid: its cells and keys are this flush's
    const bool incr = !w->force_radix && n_prev > 0 && P.total_cells == total_cells && P.hgrid.size() == ns &&
                      !std::memcmp(P.hgrid.data(), w->h_grid, ns * sizeof(SpaceGrid));
    if (incr && (rc = ensure_incr(w, total_cells))) return rc;
    // Overlap (speculative launches): this flush's early kernels (apply .. gather) go on the early
    // stream behind the previous flush's early kernels (its set's mid_ev), while that flush's pair
    // passes and finish still run on the stream; this flush's pair passes wait for its own early
    // kernels.  Nothing the early kernels touch is read or written by the previous flush's pair
    // passes or finish: the scratch, tile totals and boxes are per set, the frames rotate over three,
    // and the special pass rides on the arrival launch (it reads the previous frame early).  Only when
    // nothing else was queued on the stream since the previous flush's launch (gen), and with no
    // stage timing but the combined pass's.
#ifdef GWAOI_EXP_NO_OVERLAP  // diagnostics build only: one flush at a time (the A/B of the overlap)
    const bool ovl = false;
#else
    const bool ovl = w->ovl_ok && w->mid_last && w->gen == w->gen_launch && incr && n_prev > 0 &&
                     (w->timing_mask & ~(1u << ST_COMBINED)) == 0 && !w->check_stages;
#endif
    if (ovl) {
        st = w->early_st;
        HIP_TRY(hipStreamWaitEvent(st, w->fs[set ^ 1].mid_ev, 0));
        w->dbg.overlapped_flushes++;
    }
    if (!grid_same) {
        HIP_TRY(hipMemcpyAsync(Fn.grid, w->h_grid, sizeof(SpaceGrid) * ns, hipMemcpyHostToDevice, st));
        Fn.hgrid.assign(w->h_grid, w->h_grid + ns);
    }
    // the staged move batches' H2D copies (copy stream) land before the flush reads them
    if (w->copy_pending) {
        HIP_TRY(hipStreamWaitEvent(st, w->copy_ev, 0));
        w->copy_pending = false;
    }
    // device runs only (device Enter/Leave batches included: their ops carry the space, the appended
    // entries are initialised first and S' is copied, so the single-pass apply handles them)
    const bool moves_only = n_ops && host_ops == 0 && w->runs.size() <= gw::MAX_MOVE_RUNS && n_ops <= w->max_slots;
    // Virtual S': a flush of Moved batches only (or of nothing) changes no space and appends
    // no entry, so S' needs no copy of the previous frame: its spaces ARE the previous frame's,
    // and the records no op wrote are taken from the previous frame by k_keygen (seq check).
    const bool virt = n_app == 0 && host_ops == 0 && !w->dev_struct && (moves_only || n_ops == 0) && !w->force_copy;
    const gw::SlotSp *s_ss_view = virt ? P.ss : S.sss;
    gw::MoveRuns RS{};
    if (moves_only) {
        uint32_t j0 = 0;
        for (const Run &r : w->runs) {
            gw::MoveRun &m = RS.r[RS.count++];
            m.ds = r.ds; m.dx = r.dx; m.dz = r.dz; m.dseq = r.dseq; m.dsp = r.dsp; m.seq0 = r.seq0;
            m.sp_def = r.kind == RUN_MOVE ? gw::SP_KEEP : r.kind == RUN_ENTER ? r.space : gw::SP_DEAD;
            m.j0 = j0; m.n = (uint32_t)r.dn;
            j0 += (uint32_t)r.dn;
        }
    }
    // counters, tile totals, bbox fold identity; S' <- the previous frame unless virtual; the
    // first Moved run's claims
    const bool bucketed = moves_only && w->mv_binned;
    // GWAOI_F_UNIQUE_MOVES: plain device Moved batches (implicit seqs, the slot's own space) are
    // applied without last-op claims; keygen's written-entry count checks the promise
    bool uniq = w->unique_moves && moves_only && virt && !bucketed;
    for (const Run &r : w->runs)
        if (uniq && (!r.device || r.kind != RUN_MOVE || r.dseq || r.dsp)) uniq = false;
    const gw::MoveRun *mark = moves_only && !bucketed && !uniq ? &RS.r[0] : nullptr;
    if (uniq) w->dbg.unique_flushes++;
    const uint32_t n_unique = uniq ? (uint32_t)n_ops : 0u;
    const uint32_t n_copy = virt ? 0u : n_prev;
    // a unique-moves flush on the previous grid has no prologue: its apply writes only
    // sc->err_apply / ndrop (zero whenever a flush begins) and keygen does the zeroing (TickZero)
    gw::TickZero tz{};
    if (uniq && incr) {
        tz.sc = S.sc;
        tz.z1 = S.tile_total;
        tz.n1 = (uint32_t)gw::tile_total_elems(entries);
        tz.bbox = dev_bbox(S);
        tz.n_spaces = w->n_space_ids;
        tz.n_unique = n_unique;
    } else if (incr)
        gw::launch_prologue(S.sc, reinterpret_cast<uint32_t *>(w->cnt64),
                            gw::scan_rezeroes_counts() ? 0 : 2 * ((size_t)total_cells + 1), S.tile_total,
                            gw::tile_total_elems(entries), dev_bbox(S), w->n_space_ids, n_copy, P.rec, P.ss, S.srec, S.sss, mark,
                            w->max_slots, w->sinfo, tick_id, n_unique, st);
    else
        gw::launch_prologue(S.sc, Fn.cell_start, (size_t)total_cells + 1, S.tile_total, gw::tile_total_elems(entries), dev_bbox(S),
                            w->n_space_ids, n_copy, P.rec, P.ss, S.srec, S.sss, mark, w->max_slots, w->sinfo,
                            tick_id, n_unique, st);

    // ---- apply queued ops onto S'
    stage_begin(w, S, ST_APPLY);
    if (n_app_host) {
        HIP_TRY(hipMemcpyAsync(w->new_slots_d, w->new_slots.data(), n_app_host * sizeof(uint32_t),
                               hipMemcpyHostToDevice, st));
        gw::launch_init_appended(w->new_slots_d, n_app_host, n_prev, S.srec, S.sss, w->sinfo, w->max_slots, S.sc, st);
    }
    if (w->dev_app) {  // device Enter batches: their slots are appended after the host ones, in queue order
        uint32_t base = n_prev + n_app_host;
        for (const Run &r : w->runs)
            if (r.device && r.kind == RUN_ENTER) {
                gw::launch_init_appended(r.ds, (uint32_t)r.dn, base, S.srec, S.sss, w->sinfo, w->max_slots, S.sc, st);
                base += (uint32_t)r.dn;
            }
    }
    if (bucketed) {  // the per-tick position sync: ops regrouped by slot bucket, last op per slot in LDS
        gw::launch_moves_bucketed(RS, w->max_slots, w->sinfo, n_total, seq_base, S.srec, virt ? nullptr : S.sss,
                                  S.sc, w->mv_hist, w->scan_tmp, w->mv_binned, st);
    } else if (moves_only) {  // one pass + fixup of repeated slots (run 0's claims: the prologue)
#ifdef GWAOI_EXP_HOSTTIME
        if (w->ovl_ok)  // (speculative launches only: ht_entry is their gwaoi_tick_finish call's)
            w->ht[0] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w->ht_entry).count();
#endif
        gw::launch_moves(RS, w->max_slots, w->sinfo, tick_id, n_total, seq_base, S.srec, virt ? nullptr : S.sss,
                         P.rec, n_prev, S.sc, w->coll, 1u, uniq, st);
    } else if (n_ops) {
        // host runs -> device op buffers; device runs are read in place
        size_t hat = 0;
        for (const Run &r : w->runs) {
            if (r.device) continue;
            const size_t k = r.hend - r.hbegin;
            HIP_TRY(hipMemcpyAsync(w->op_slot + hat, w->h_op_slot.data() + r.hbegin, k * 4, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(w->op_x + hat, w->h_op_x.data() + r.hbegin, k * 4, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(w->op_z + hat, w->h_op_z.data() + r.hbegin, k * 4, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(w->op_sp + hat, w->h_op_sp.data() + r.hbegin, k * 4, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(w->op_seq + hat, w->h_op_seq.data() + r.hbegin, k * 8, hipMemcpyHostToDevice, st));
            hat += k;
        }
        for (int pass = 0; pass < 2; ++pass) {
            uint32_t j0 = 0;
            size_t hoff = 0;
            for (const Run &r : w->runs) {
                const uint32_t *sl;
                const float *xs, *zs;
                const uint32_t *sps;
                const unsigned long long *sq;
                uint64_t seq0 = 0;
                uint32_t k;
                const uint32_t sp_def = !r.device || r.kind == RUN_MOVE ? gw::SP_KEEP
                                        : r.kind == RUN_ENTER ? r.space : gw::SP_DEAD;
                if (r.device) {
                    sl = r.ds; xs = r.dx; zs = r.dz; sps = r.dsp; sq = r.dseq; seq0 = r.seq0; k = (uint32_t)r.dn;
                } else {
                    k = (uint32_t)(r.hend - r.hbegin);
                    sl = w->op_slot + hoff; xs = w->op_x + hoff; zs = w->op_z + hoff; sps = w->op_sp + hoff;
                    sq = w->op_seq + hoff;
                    hoff += k;
                }
                if (pass == 0)
                    gw::launch_ops_claim(sl, k, j0, w->max_slots, w->sinfo, tick_id, S.sc, st);
                else
                    gw::launch_ops_apply(sl, xs, zs, sps, sp_def, k, j0, w->max_slots, w->sinfo, tick_id, n_total, sq, seq0,
                                         seq_base, r.device && r.dseq, S.srec, S.sss, S.sc, st);
                j0 += k;
            }
        }
    }
    stage_end(w, S, ST_APPLY);

    // ---- keys (+ d_rel, bmax) and stable sort
    stage_begin(w, S, ST_KEYGEN);
    gw::launch_keygen(S.srec, s_ss_view, n_total, Fn.grid, total_cells, w->keys[0], w->vals[0], P.rec, P.ss, P.grid,
                      n_prev, w->blk, S.sc, P.key, incr ? w->cnt64 : nullptr, seq_base, w->special, tz,
                      incr ? w->scan64_tmp : nullptr, st);
    stage_end(w, S, ST_KEYGEN);
    stage_begin(w, S, ST_SORT);
    int which = 1;
    // the special pass rides on the sort's arrival launch (k_arrive_special) unless it is timed;
    // launch_pair_passes then skips its own launch
    const bool sp_fused = incr && !(w->timing_mask >> ST_SPECIAL & 1u) && n_prev > 0;
    gw::SpecialJob spj{};
    if (sp_fused) {
        const uint32_t TBn = gw::combined_tiles(n_new), TBp = gw::combined_blocks(n_prev);
        spj.F = view_of(P);
        spj.O_rec = S.srec;
        spj.O_ss = s_ss_view;
        spj.seq_base = seq_base;
        spj.sc = S.sc;
        spj.tmp = reinterpret_cast<uint2 *>(S.evtmp);
        spj.cap = S.evtmp_cap;
        spj.tile_total = S.tile_total;
        spj.tile_base = S.tile_base;
        spj.tile_off = TBn;
        spj.leave_off = TBn + TBp;
        spj.special = w->special;
        spj.n_tiles = TBp;
    }
    // the gather rides on the incremental sort's merge launch (k_merge_gather, one bbox part per
    // scan tile) unless it is timed or the grid has more scan tiles than the set has parts
#ifdef GWAOI_EXP_UNFUSED_GATHER  // diagnostics build only: the two launches
    const bool ga_fused = false;
#else
    const bool ga_fused = incr && !(w->timing_mask >> ST_GATHER & 1u) &&
                          gw::incr_sort_tiles(total_cells) <= gw::gather_parts(w->max_slots);
#endif
    S.n_parts = ga_fused ? gw::incr_sort_tiles(total_cells) : gw::gather_parts(n_new);
    gw::GatherJob gj{};
    if (ga_fused) {
        gj.n_new = n_new;
        gj.n_prev = n_prev;
        gj.s_rec = S.srec;
        gj.s_ss = s_ss_view;
        gj.p_rec = P.rec;
        gj.p_ss = P.ss;
        gj.f_rec = Fn.rec;
        gj.f_ss = Fn.ss;
        gj.o_rec = S.orec;
        gj.cand = S.cand;
        gj.grid = Fn.grid;
        gj.info = w->sinfo;
        gj.sc = S.sc;
        gj.bbox = dev_bbox(S);
        gj.n_spaces = w->n_space_ids;
        gj.parts = S.bbox_parts;
    }
    if (incr) {
        w->dbg.incremental_sorts++;
        gw::incremental_sort(w->keys[0], n_total, n_prev, P.key, P.cell_start, w->cnt64, total_cells,
                             total_cells, Fn.cell_start, w->arr_pos, w->arr_idx, w->scan64_tmp, w->vals[1],
                             Fn.key, w->blk, S.sc, sp_fused ? &spj : nullptr, ga_fused ? &gj : nullptr,
                             st);  // the sorted keys ARE the frame's
    } else {
        gw::SortBuffers sb;
        sb.keys[0] = w->keys[0];
        sb.keys[1] = w->keys[1];
        sb.vals[0] = w->vals[0];
        sb.vals[1] = w->vals[1];
        sb.hist = w->hist;
        sb.scan_tmp = w->scan_tmp;
        which = gw::radix_sort(sb, n_total, bitlen(total_cells), st);
    }
    stage_end(w, S, ST_SORT);
    const uint32_t *skeys = incr ? Fn.key : w->keys[which];
    const uint32_t *perm = w->vals[which];

    // ---- new frame + previous state in the new order
    if (!ga_fused) {
        stage_begin(w, S, ST_GATHER);
        gw::launch_gather(perm, n_new, n_prev, S.srec, s_ss_view, P.rec, P.ss, Fn.rec, Fn.ss, S.orec, S.cand,
                          Fn.grid, seq_base, w->sinfo, skeys, total_cells, n_total, S.sc, incr ? nullptr : Fn.key,
                          dev_bbox(S), w->n_space_ids, S.bbox_parts, st);
        stage_end(w, S, ST_GATHER);
    }

    // ---- cell_start = exclusive scan of entities per cell (zeroed by the prologue;
    // the incremental sort has written it already)
    if (!incr) {
        stage_begin(w, S, ST_CELLS);
        gw::launch_cell_count(skeys, n_new, Fn.cell_start, st);
        gw::scan_exclusive(Fn.cell_start, Fn.cell_start, (size_t)total_cells + 1, w->scan_tmp, st);
        stage_end(w, S, ST_CELLS);
    }

    // the early kernels' end: the next (speculative) flush's early stream starts behind it, and an
    // overlapped flush's pair passes wait for it on the stream
    w->mid_last = false;
    if (w->ovl_ok || ovl) {
        if (hipEventRecord(S.mid_ev, st) != hipSuccess ||
            (ovl && hipStreamWaitEvent(w->stream, S.mid_ev, 0) != hipSuccess)) {
            w->last_error = "flush mid event failed";
            return poison(w, GWAOI_EDEVICE);
        }
        w->mid_last = true;
    }
    st = w->stream;

    // ---- pair passes: combined over the new grid, special entities over the previous one
    const EvCaps ev_cap = launch_pair_passes(w, S, Fn, P, seq_base, s_ss_view, false, sp_fused);

    // from here on the device has rewritten SlotInfo for the new frame: any failure before the
    // commit below leaves the world inconsistent (poisoned)
    if (hipGetLastError() != hipSuccess) {
        w->last_error = "kernel launch failed";
        return poison(w, GWAOI_EDEVICE);
    }
    // (k_finish writes the summary straight into pinned host memory: no copy)
    if (hipEventRecord(S.done_ev, st) != hipSuccess) {
        w->last_error = "flush done event failed";
        return poison(w, GWAOI_EDEVICE);
    }
    // the queue is closed: what the commit needs of it
    w->in_flight = true;
    w->fl.tick_id = tick_id;
    w->fl.entries = entries;
    w->fl.seq_next = w->seq_next;
    w->fl.seq_base = seq_base;
    w->fl.dev_seq = w->dev_seq_pending;
    w->fl.set = set;
    w->fl.p_idx = p_idx;
    w->fl.n_idx = n_idx;
    w->fl.s_ss_view = s_ss_view;
    w->fl.cap = ev_cap;
    w->launch_set ^= 1;
    w->fl.touched_alive.resize(w->touched.size());
    for (size_t i = 0; i < w->touched.size(); ++i) w->fl.touched_alive[i] = w->alive[w->touched[i]];
    w->stage_cur ^= 1;  // calls made in flight stage into the other half (free: its flush has ended)
    w->stage_used[w->stage_cur] = 0;
    w->space_ops_queued = false;
    w->gen_launch = w->gen;
    return GWAOI_OK;
}

// Wait for a flush's summary: polls its event (a blocking wait adds tens of microseconds of wake-up).
int wait_done(gwaoi_world *w, hipEvent_t ev) {
    hipError_t e;
    while ((e = hipEventQuery(ev)) == hipErrorNotReady) __builtin_ia32_pause();
    HIP_TRY(e);
    return GWAOI_OK;
}

using Flight = decltype(gwaoi_world::fl);

// The host half of a flush's commit: its op queue becomes the world's state and
// the calls deferred while it was in flight are queued for the next flush.  r:
// the flush's summary (needed only after explicit-seq device batches; a
// speculative launch commits before the summary and never has those).
void commit_host(gwaoi_world *w, const gw::TickOut *r) {
    for (uint32_t s : w->new_slots) w->appended[s] = 0;
    w->new_slots.clear();
    for (size_t i = 0; i < w->touched.size(); ++i) w->in_frame[w->touched[i]] = w->fl.touched_alive[i];
    w->touched.clear();
    w->h_op_slot.clear();
    w->h_op_x.clear();
    w->h_op_z.clear();
    w->h_op_sp.clear();
    w->h_op_seq.clear();
    w->runs.clear();
    w->n_ops = 0;
    if (w->dev_struct) w->slots_stale = true;
    w->dev_app = 0;
    w->dev_struct = false;
    if (r && w->fl.dev_seq && r->seq_max >= w->seq_next) w->seq_next = r->seq_max + 1;  // no call was made in flight
    w->dev_seq_pending = false;
    w->seq_floor = w->fl.dev_seq ? w->seq_next : w->fl.seq_next;
    w->cur = w->fl.n_idx;
    w->in_flight = false;
    replay_deferred(w);
}

// The flush, second half, for flight f: wait for the summary, grow the event
// buffer and re-run the pair passes if needed, commit.  host_done: the host half
// was committed ahead (a speculative launch of the next flush followed it; that
// flush writes the other FlushSet and the third frame, so f's pair-pass inputs
// are intact for a re-run, which then runs after it on the stream).  On return
// the events are in the set's buffer (last_events).  *committed: the new frame
// became the world's state (the events are valid and must be delivered, even
// when the returned status reports a problem the device found in the queued
// ops).  A failure after the device kernels have rewritten the per-slot records
// but before the commit poisons the world.
int finish_flight(gwaoi_world *w, const Flight &f, bool host_done, bool *committed) {
    *committed = false;
    hipStream_t st = w->stream;
    int rc;
    FlushSet &S = w->fs[f.set];
    DevFrame &P = w->fr[f.p_idx];
    DevFrame &Fn = w->fr[f.n_idx];
    if (wait_done(w, S.done_ev) != GWAOI_OK) {
        w->last_error = "flush did not complete: " + w->last_error;
        if (w->fault_stage)
            w->last_error += std::string(" (first failed stage wait: ") + (w->fault_before ? "before " : "after ") +
                             w->fault_stage + ")";
        return poison(w, GWAOI_EDEVICE);
    }

    gw::TickOut r = *tick_out(S);
    if (r.total64 > 0xFFFFFFFFull) {
        w->last_error = "more than 2^32-1 events in one flush";
        return poison(w, GWAOI_ECAPACITY);
    }
    // compared with the capacities the passes had at launch: a regrow by another flush since then
    // (shared scratch, or the twin set's catch-up) does not make the clipped events complete.
    // The scratch extent is not the event count: the pair passes deal their pairs to the event
    // streams by the XCD each block lands on, so a re-run's extent may differ from the overflowed
    // run's.  The first re-run is sized for the extent seen; a second one for the worst case (every
    // pair in one stream), which cannot overflow.  The set's buffer is sized by the count.
    EvCaps cap_used = f.cap;
    for (int attempt = 0; r.total64 > cap_used.out || r.ext64 > cap_used.tmp; ++attempt) {  // grow, re-run
        stage_collect(w, S);
        if (w->inject_regrow_fail) {
            w->last_error = "event buffer regrow failed (injected)";
            return poison(w, GWAOI_ENOMEM);
        }
        if (attempt == 2) {
            w->last_error = "pair passes re-run: the event extent exceeds its worst-case bound";
            return poison(w, GWAOI_EDEVICE);
        }
        const uint64_t need = attempt == 0 ? r.ext64 : std::max<uint64_t>(r.ext64, gw::ev_worst_extent(r.total64));
        if ((rc = ensure_events(w, S, r.total64, need))) return poison(w, rc);
        (void)hipGetLastError();  // a failure of an unrelated earlier call is not this re-run's
        w->gen++;
        gw::launch_zero(S.tile_total, gw::tile_total_elems(f.entries), st);
        gw::launch_zero(&S.sc->shard[0][0], gw::EV_SHARDS * 32, st);  // event streams
        gw::launch_zero(S.sc->dbg, gw::DBG_N, st);
        cap_used = launch_pair_passes(w, S, Fn, P, f.seq_base, f.s_ss_view, true);
        if (cap_used.tmp < need || cap_used.out < r.total64) {
            w->last_error = "pair passes re-run: event buffers did not grow";
            return poison(w, GWAOI_EDEVICE);
        }
        w->dbg.event_regrows++;
        if (hipGetLastError() != hipSuccess || wait_stream(w) != GWAOI_OK) {
            w->last_error = "pair passes re-run failed: " + w->last_error;
            return poison(w, GWAOI_EDEVICE);
        }
        r = *tick_out(S);
        if (r.total64 > 0xFFFFFFFFull) {
            w->last_error = "more than 2^32-1 events in one flush";
            return poison(w, GWAOI_ECAPACITY);
        }
    }
    stage_collect(w, S);

    // ---- commit
    w->dbg.flushes++;
    w->dbg.combined_replays += r.dbg[gw::DBG_COMBINED_REPLAY];
    w->dbg.combined_queue_drains += r.dbg[gw::DBG_COMBINED_DRAIN];
    w->dbg.special_global += r.dbg[gw::DBG_SPECIAL_GLOBAL];
    w->last_n_enter = r.n_enter;
    w->last_n_leave = (uint64_t)r.n_total - r.n_enter;
    w->rel_pairs += (int64_t)w->last_n_enter - (int64_t)w->last_n_leave;
    if (w->cells_auto) {
        const float rec =
            recommend_cells_per_dist((double)std::max<int64_t>(w->rel_pairs, 0) / std::max<uint32_t>(1, Fn.n));
        if (rec != w->cells_per_dist) {
            w->cpd_streak = rec == w->cpd_rec ? w->cpd_streak + 1 : 1;
            w->cpd_rec = rec;
        } else {
            w->cpd_streak = 0;
        }
    }
    w->last_set = f.set;
    const int4 *bb = tick_bbox(S);
    for (uint32_t s = 0; s < w->n_space_ids; ++s) {
        SpaceHost &SH = w->spaces[s];
        if (SH.used && SH.alive && bb[s].x != 0x7FFFFFFF) {
            SH.have_bbox = true;
            SH.bx0 = o2f(bb[s].x);
            SH.bz0 = o2f(bb[s].y);
            SH.bx1 = o2f(bb[s].z);
            SH.bz1 = o2f(bb[s].w);
        } else {
            SH.have_bbox = false;
        }
    }
    if (!host_done) commit_host(w, &r);
    w->ticks++;
    *committed = true;
    // problems the device found in the queued ops: the frame is committed (the offending ops were
    // dropped), so the flush's events are valid and the caller still receives them
    if (r.err & (gw::ERR_COUNT_MISMATCH | gw::ERR_ENTER_LIVE)) {
        w->last_error = (r.err & gw::ERR_ENTER_LIVE)
                            ? "device Enter batch of a slot live when the flush began (frame count broken)"
                            : "live-count mismatch between host and device (a device Enter/Leave batch broke its "
                              "rules, or an internal error)";
        return poison(w, GWAOI_EDEVICE);
    }
    // every problem of the flush goes into last_error; the status is the first one's
    int st_err = GWAOI_OK;
    std::string msg;
    auto note = [&](uint32_t bits, int code, const char *text) {
        if (!(r.err & bits)) return;
        if (st_err == GWAOI_OK) st_err = code;
        msg += msg.empty() ? text : std::string("; ") + text;
    };
    note(gw::ERR_DUP_SLOT, GWAOI_ESTATE,
         "GWAOI_F_UNIQUE_MOVES: a slot was moved twice in one flush (its position is unspecified: in practice one "
         "of its moves, not necessarily the last)");
    note(gw::ERR_NONFINITE, GWAOI_ENONFINITE, "device batch held a non-finite coordinate (move dropped)");
    note(gw::ERR_SEQ, GWAOI_EINVAL, "device batch held an explicit seq below the flush's floor (op dropped)");
    note(gw::ERR_MOVE_DEAD | gw::ERR_BAD_SLOT, GWAOI_ESTATE, "device batch moved a slot that is not live (move dropped)");
    if (st_err != GWAOI_OK) w->last_error = msg;
    return st_err;
}

int tick_finish(gwaoi_world *w, bool *committed) { return finish_flight(w, w->fl, false, committed); }

// The sparse flush (gwaoi_sparse.hip): a queue of a few host Moved calls, nothing in flight,
// becomes events and an in-place patch of the committed frame, without the frame rebuild.
// Returns GWAOI_OK when it committed, 1 when it was not taken or the device declined it (nothing
// changed: the caller runs the full flush over the same queue), or an error.
constexpr size_t kSparseMaxOps = 256;
// the host ops of a sparse flush in one upload: [seq u64 x 256 | slot x 256 | x x 256 | z x 256]
constexpr size_t kSpSeq = 0, kSpSlot = 8 * kSparseMaxOps, kSpX = 12 * kSparseMaxOps, kSpZ = 16 * kSparseMaxOps;
constexpr size_t kSpOpsBytes = 20 * kSparseMaxOps;
int sparse_try(gwaoi_world *w) {
    if (!w->sparse_on || w->in_flight || w->n_ops == 0 || w->n_ops > kSparseMaxOps || !w->new_slots.empty() ||
        w->space_ops_queued || w->dev_app || w->dev_struct || w->dev_seq_pending || !w->deferred.empty() ||
        w->resv_n || w->ticks == 0 || w->runs.size() != 1)
        return 1;
    const Run &run = w->runs[0];
    // one stretch of host calls, or one host batch staged as a device batch (validated on the host,
    // implicit seqs, every slot in its own space); never a caller's device batch (checked on the device)
    if (run.device && (run.kind != RUN_MOVE || !run.checked || run.dseq || run.dsp)) return 1;
    DevFrame &P = w->fr[w->cur];
    if (P.n == 0) return 1;
    for (uint32_t sp : w->h_op_sp)
        if (sp == gw::SP_DEAD) return 1;
    const uint32_t k = (uint32_t)w->n_ops;
    hipStream_t st = w->stream;
    w->gen++;  // (the sparse flush's kernels: the next flush's early kernels wait for them)
    const int set = w->launch_set;
    FlushSet &S = w->fs[set];
    int rc;
    // the sparse flush is optional: a failed allocation of its buffers turns it off, and the full
    // flush runs over the same queue (nothing was launched yet)
    auto give_up = [&]() {
        w->sparse_on = false;
        w->dbg.sparse_declined++;
        return 1;
    };
    if (!w->sp_cnt && dalloc(w, &w->sp_cnt, gw::sparse_cnt_elems((uint32_t)kSparseMaxOps)) != GWAOI_OK) return give_up();
    if (!run.device && !w->h_sp_ops) {  // the host ops' one pinned upload buffer
        if (hipHostMalloc((void **)&w->h_sp_ops, kSpOpsBytes, hipHostMallocDefault) != hipSuccess) {
            w->h_sp_ops = nullptr;
            return give_up();
        }
        if (dalloc(w, &w->d_sp_ops, kSpOpsBytes) != GWAOI_OK) return give_up();
    }
    const bool fused = w->sparse_fused && k <= gw::sparse_fused_max();
    if (fused && !w->sp_scr) {
        if (dalloc(w, &w->sp_scr, (size_t)gw::sparse_fused_max() * 2 * w->sp_scr_cap) != GWAOI_OK ||
            dalloc(w, &w->sp_done, 1) != GWAOI_OK) {
            dfree(w->sp_scr);
            w->sparse_fused = false;  // the kernel sequence needs neither
        } else {
            HIP_TRY(hipMemsetAsync(w->sp_done, 0, sizeof(uint32_t), st));
        }
    }
    if (w->out_pending) HIP_TRY(hipStreamWaitEvent(st, w->out_ev, 0));  // a copy-out still reads S's events
    const uint32_t *d_slot = run.ds;
    const float *d_x = run.dx, *d_z = run.dz;
    const unsigned long long *d_seq = nullptr;
    if (!run.device) {  // one pinned upload (four pageable copies cost ~8 us each)
        std::memcpy(w->h_sp_ops + kSpSeq, w->h_op_seq.data(), k * 8);
        std::memcpy(w->h_sp_ops + kSpSlot, w->h_op_slot.data(), k * 4);
        std::memcpy(w->h_sp_ops + kSpX, w->h_op_x.data(), k * 4);
        std::memcpy(w->h_sp_ops + kSpZ, w->h_op_z.data(), k * 4);
        HIP_TRY(hipMemcpyAsync(w->d_sp_ops, w->h_sp_ops, kSpZ + k * 4, hipMemcpyHostToDevice, st));
        d_slot = reinterpret_cast<const uint32_t *>(w->d_sp_ops + kSpSlot);
        d_x = reinterpret_cast<const float *>(w->d_sp_ops + kSpX);
        d_z = reinterpret_cast<const float *>(w->d_sp_ops + kSpZ);
        d_seq = reinterpret_cast<const unsigned long long *>(w->d_sp_ops + kSpSeq);
    } else if (w->copy_pending) {  // the staged batch's H2D lands first
        HIP_TRY(hipStreamWaitEvent(st, w->copy_ev, 0));
        w->copy_pending = false;
    }
    const uint32_t tick_id = ++w->tick_id;
    gw::TickOut *res = reinterpret_cast<gw::TickOut *>(S.d_hout);
    auto run_sparse = [&](bool fused) -> int {
        if (fused) {
            gw::launch_sparse_fused(P.rec, P.ss, P.key, P.cell_start, P.grid, w->sinfo, d_slot, d_x, d_z, d_seq,
                                    run.seq0, k, w->sp_cnt, w->sp_scr, w->sp_scr_cap, w->sp_done, S.events,
                                    S.ev_cap, res, st);
        } else {
            gw::launch_ops_claim(d_slot, k, 0, w->max_slots, w->sinfo, tick_id, S.sc, st);
            gw::launch_sparse(P.rec, P.ss, P.key, P.cell_start, P.grid, w->sinfo, d_slot, d_x, d_z, d_seq, run.seq0,
                              k, tick_id, w->sp_cnt, S.events, S.ev_cap, res, st);
        }
        if (hipGetLastError() != hipSuccess || hipEventRecord(S.done_ev, st) != hipSuccess) {
            w->last_error = "sparse flush launch failed";
            return poison(w, GWAOI_EDEVICE);  // the frame may be half patched
        }
        if (wait_done(w, S.done_ev) != GWAOI_OK) {
            w->last_error = "sparse flush did not complete: " + w->last_error;
            return poison(w, GWAOI_EDEVICE);
        }
        return GWAOI_OK;
    };
    const bool use_fused = fused && w->sparse_fused;
    if ((rc = run_sparse(use_fused))) return rc;
    if (use_fused && tick_out(S)->pad == 3u) {  // an op outgrew its scratch row: the kernel sequence
        w->dbg.sparse_unfused++;
        if ((rc = run_sparse(false))) return rc;
    }
    const gw::TickOut r = *tick_out(S);
    if (r.pad) {  // declined on the device before any write to the frame
        w->dbg.sparse_declined++;
        return 1;
    }
    // ---- commit: the frame is patched in place (same frame index); the events are set S's
    w->dbg.flushes++;
    w->dbg.sparse_flushes++;
    w->last_n_enter = r.n_enter;
    w->last_n_leave = (uint64_t)r.n_total - r.n_enter;
    w->rel_pairs += (int64_t)w->last_n_enter - (int64_t)w->last_n_leave;
    w->last_set = set;
    w->launch_set ^= 1;
    w->h_op_slot.clear();
    w->h_op_x.clear();
    w->h_op_z.clear();
    w->h_op_sp.clear();
    w->h_op_seq.clear();
    w->runs.clear();
    w->n_ops = 0;
    w->seq_floor = w->seq_next;
    w->ticks++;
    // the staged batch was read (the stream was waited for): its staging words are free again
    if (run.device) w->stage_used[w->stage_cur] = 0;
    return GWAOI_OK;
}

// Whether the calls queued during the flush in flight allow launching the next
// flush before the one in flight has committed: device Moved batches only
// (implicit seqs, the space of every slot unchanged, no host op), and the flush
// in flight has no explicit-seq batch (its successor's seq floor is then known).
bool speculative_ok(gwaoi_world *w) {
    if (!w->in_flight || w->fl.dev_seq || !w->deferred_boxes.empty() || w->deferred.size() > gw::MAX_MOVE_RUNS)
        return false;
    size_t n = 0;
    for (const Deferred &q : w->deferred) {
        if (q.kind != Deferred::RUN || !q.run.device || q.run.dseq || q.run.dsp) return false;
        n += q.run.dn;
    }
    return n <= w->max_slots;
}

}  // namespace

// =============================================================== C ABI =======

extern "C" {

int gwaoi_abi_version(void) { return GWAOI_ABI_VERSION; }

const char *gwaoi_strerror(int s) {
    switch (s) {
        case GWAOI_OK: return "ok";
        case GWAOI_EINVAL: return "invalid argument";
        case GWAOI_EBADSLOT: return "slot out of range";
        case GWAOI_ESTATE: return "slot in wrong state (Enter on live / Leave or Moved on non-live)";
        case GWAOI_ENOMEM: return "out of memory";
        case GWAOI_EDEVICE: return "HIP device error";
        case GWAOI_ENONFINITE: return "non-finite coordinate";
        case GWAOI_EBADSPACE: return "unknown space";
        case GWAOI_EBUSY: return "space not empty";
        case GWAOI_ECAPACITY: return "event capacity exceeded";
        default: return "unknown status";
    }
}

const char *gwaoi_last_error(gwaoi_world *w) { return w ? w->last_error.c_str() : "null world"; }

int gwaoi_world_destroy(gwaoi_world *w) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
#ifdef GWAOI_EXP_HOSTTIME
    if (w->ht[5] > 0)
        fprintf(stderr, "hosttime per gwaoi_tick_finish (%.0f calls, %llu speculative): entry->first kernel %.1f us, launch %.1f, "
                "summary wait %.1f, commit %.1f (speculative calls); call %.1f (all)\n", w->ht[5],
                (unsigned long long)w->dbg.speculative_launches, w->ht[0] / std::max<double>(1, w->dbg.speculative_launches),
                w->ht[1] / std::max<double>(1, w->dbg.speculative_launches), w->ht[2] / std::max<double>(1, w->dbg.speculative_launches),
                w->ht[3] / std::max<double>(1, w->dbg.speculative_launches), w->ht[4] / w->ht[5]);
#endif
    if (w->stream) (void)hipStreamSynchronize(w->stream);
    if (w->early_st) (void)hipStreamSynchronize(w->early_st);
    if (w->copy_st) (void)hipStreamSynchronize(w->copy_st);
    if (w->out_st) (void)hipStreamSynchronize(w->out_st);
    if (w->sync) gw::sync_destroy(w->sync);
    w->sync = nullptr;
    for (DevFrame &f : w->fr) {
        dfree(f.rec); dfree(f.ss); dfree(f.key); dfree(f.cell_start); dfree(f.grid);
    }
    for (FlushSet &S : w->fs) {
        dfree(S.srec); dfree(S.sss); dfree(S.orec); dfree(S.cand); dfree(S.sc); dfree(S.events);
        dfree(S.bbox_parts); dfree(S.dev_out); dfree(S.evtmp); dfree(S.tile_total); dfree(S.tile_base);
        if (S.mid_ev) (void)hipEventDestroy(S.mid_ev);
        if (S.h_out) (void)hipHostFree(S.h_out);
        S.h_out = nullptr;
        for (int st = 0; st < ST_N; ++st)
            for (int q = 0; q < 2; ++q)
                if (S.ev[st][q]) (void)hipEventDestroy(S.ev[st][q]);
        if (S.done_ev) (void)hipEventDestroy(S.done_ev);
    }
    for (int i = 0; i < 2; ++i) { dfree(w->keys[i]); dfree(w->vals[i]); }
    dfree(w->hist); dfree(w->scan_tmp); dfree(w->sinfo.lastop); dfree(w->sinfo.rank); dfree(w->sinfo.sp); dfree(w->new_slots_d);
    dfree(w->cnt64); dfree(w->scan64_tmp); dfree(w->arr_pos); dfree(w->arr_idx); dfree(w->coll); dfree(w->special);
    dfree(w->tile_work); dfree(w->tile_order); dfree(w->ework);
    dfree(w->mv_hist); dfree(w->mv_binned);
    dfree(w->op_slot); dfree(w->op_sp); dfree(w->op_x); dfree(w->op_z); dfree(w->op_seq);
    dfree(w->sp_cnt); dfree(w->d_sp_ops); dfree(w->sp_scr); dfree(w->sp_done);
    if (w->h_sp_ops) (void)hipHostFree(w->h_sp_ops);
    dfree(w->blk);
    dfree(w->nb_out); dfree(w->nb_count);
    dfree(w->csr_cnt); dfree(w->csr_off); dfree(w->csr_items); dfree(w->csr_long);
    if (w->h_csr_off) (void)hipHostFree(w->h_csr_off);
    if (w->h_csr_items) (void)hipHostFree(w->h_csr_items);
    if (w->h_events) (void)hipHostFree(w->h_events);
    if (w->h_grid) (void)hipHostFree(w->h_grid);
    for (int h = 0; h < 2; ++h) {
        if (w->h_stage[h]) (void)hipHostFree(w->h_stage[h]);
        dfree(w->d_stage[h]);
    }
    if (w->copy_ev) (void)hipEventDestroy(w->copy_ev);
    if (w->copy_st) (void)hipStreamDestroy(w->copy_st);
    if (w->out_st) (void)hipStreamSynchronize(w->out_st);
    if (w->out_ev) (void)hipEventDestroy(w->out_ev);
    if (w->out_st) (void)hipStreamDestroy(w->out_st);
    if (w->done_ev) (void)hipEventDestroy(w->done_ev);
    if (w->order_ev) (void)hipEventDestroy(w->order_ev);
    if (w->stream) (void)hipStreamDestroy(w->stream);
    if (w->early_st) (void)hipStreamDestroy(w->early_st);
    delete w;
    return GWAOI_OK;
    });
}

int gwaoi_world_create(const gwaoi_config *cfg, gwaoi_world **out) {
    return gw::api_guard([&]() -> int {
    if (!cfg || !out || cfg->max_slots == 0 || cfg->max_spaces == 0 || cfg->max_slots > 0x7FFFFFF0u)
        return GWAOI_EINVAL;
    *out = nullptr;
    gwaoi_world *w = new (std::nothrow) gwaoi_world();
    if (!w) return GWAOI_ENOMEM;
    w->cfg = *cfg;
    w->max_slots = cfg->max_slots;
    w->max_spaces = cfg->max_spaces;
    w->cells_per_dist = cfg->cells_per_dist > 0.f ? cfg->cells_per_dist : 3.0f;
    w->cells_auto = !(cfg->cells_per_dist > 0.f);
    w->timing_mask = (cfg->flags & GWAOI_F_TIMING) ? (1u << ST_N) - 1u : 0u;
    w->sparse_on = !(cfg->flags & GWAOI_F_NO_SPARSE);
    // GWAOI_F_BATCH_READY is accepted and has no effect (include/gwaoi.h)
    w->unique_moves = (cfg->flags & GWAOI_F_UNIQUE_MOVES) != 0;
    w->sparse_fused = !(cfg->flags & GWAOI_F_TEST_SPARSE_SEQUENCE);
    if (cfg->flags & GWAOI_F_TEST_SPARSE_SCR2) w->sp_scr_cap = 2;
    w->force_radix = (cfg->flags & GWAOI_F_TEST_FORCE_RADIX) != 0;
    w->force_copy = (cfg->flags & GWAOI_F_TEST_FORCE_COPY) != 0;
    w->inject_regrow_fail = (cfg->flags & GWAOI_F_TEST_REGROW_FAIL) != 0;
    w->check_stages = (cfg->flags & GWAOI_F_TEST_CHECK_STAGES) != 0;
    int rc = GWAOI_OK;
    auto fail = [&](int code) {
        gwaoi_world_destroy(w);
        return code;
    };
    if (cfg->device >= 0) {
        hipError_t e = hipSetDevice(cfg->device);
        if (e != hipSuccess) {
            delete w;
            return GWAOI_EDEVICE;
        }
    }
    if (hipGetDevice(&w->device) != hipSuccess) {
        delete w;
        return GWAOI_EDEVICE;
    }
    if (hipStreamCreateWithFlags(&w->early_st, hipStreamNonBlocking) != hipSuccess) {
        w->early_st = nullptr;
        return fail(GWAOI_EDEVICE);
    }
    if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess) {
        w->stream = nullptr;
        return fail(GWAOI_EDEVICE);
    }
    if (hipStreamCreateWithFlags(&w->copy_st, hipStreamNonBlocking) != hipSuccess) {
        w->copy_st = nullptr;
        return fail(GWAOI_EDEVICE);
    }
    if (hipEventCreateWithFlags(&w->copy_ev, hipEventDisableTiming) != hipSuccess) {
        w->copy_ev = nullptr;
        return fail(GWAOI_EDEVICE);
    }
    if (hipStreamCreateWithFlags(&w->out_st, hipStreamNonBlocking) != hipSuccess) {
        w->out_st = nullptr;
        return fail(GWAOI_EDEVICE);
    }
    if (hipEventCreateWithFlags(&w->out_ev, hipEventDisableTiming) != hipSuccess) {
        w->out_ev = nullptr;
        return fail(GWAOI_EDEVICE);
    }
    const size_t N = w->max_slots;
    for (DevFrame &f : w->fr) {
        if ((rc = dalloc(w, &f.rec, N)) || (rc = dalloc(w, &f.ss, N)) || (rc = dalloc(w, &f.key, N)) ||
            (rc = dalloc(w, &f.grid, w->max_spaces)))
            return fail(rc);
        if ((rc = ensure_cells(w, f, 1))) return fail(rc);
    }
    const size_t out_bytes = sizeof(gw::TickOut) + sizeof(int4) * (size_t)w->max_spaces;
    for (FlushSet &S : w->fs) {
        if ((rc = dalloc(w, &S.srec, N)) || (rc = dalloc(w, &S.sss, N)) || (rc = dalloc(w, &S.orec, N)) ||
            (rc = dalloc(w, &S.cand, N)) || (rc = dalloc(w, &S.sc, 1)) ||
            (rc = dalloc(w, (char **)&S.bbox_parts, gw::bbox_part_bytes((uint32_t)N))) ||
            (rc = dalloc(w, &S.dev_out, kDevBBox + sizeof(int4) * (size_t)w->max_spaces)))
            return fail(rc);
        // S' records seq 0 (virtual S': never "written")
        if (hipMemset(S.srec, 0, N * sizeof(gw::Rec16)) != hipSuccess) return fail(GWAOI_EDEVICE);
        // err_apply / ndrop are zero whenever a flush begins (a flush without a prologue relies on it)
        if (hipMemset(S.sc, 0, sizeof(gw::TickScalars)) != hipSuccess) return fail(GWAOI_EDEVICE);
        // k_finish writes the summary here while the host polls done_ev: coherent (uncached, system
        // scope) memory, so that the writes are visible once the event is seen whatever the runtime's
        // default coherence of pinned allocations
        if (hipHostMalloc((void **)&S.h_out, out_bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&S.d_hout, S.h_out, 0) != hipSuccess)
            return fail(GWAOI_ENOMEM);
        std::memset(S.h_out, 0, out_bytes);
        for (int st = 0; st < ST_N; ++st)
            for (int q = 0; q < 2; ++q)
                if (hipEventCreate(&S.ev[st][q]) != hipSuccess) return fail(GWAOI_EDEVICE);
        if (hipEventCreateWithFlags(&S.done_ev, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.mid_ev, hipEventDisableTiming) != hipSuccess)
            return fail(GWAOI_EDEVICE);
    }
    if ((rc = dalloc(w, &w->keys[0], N)) || (rc = dalloc(w, &w->keys[1], N)) || (rc = dalloc(w, &w->vals[0], N)) ||
        (rc = dalloc(w, &w->vals[1], N)) || (rc = dalloc(w, &w->hist, gw::radix_hist_elems((uint32_t)N))) ||
        (rc = dalloc(w, &w->sinfo.lastop, N)) || (rc = dalloc(w, &w->sinfo.rank, N)) ||
        (rc = dalloc(w, &w->sinfo.sp, N)) || (rc = dalloc(w, &w->new_slots_d, N)) || (rc = dalloc(w, &w->arr_idx, N)) ||
        (rc = dalloc(w, &w->coll, N)) || (rc = dalloc(w, &w->blk, 3 * (N / 256 + 2))) ||
        (rc = dalloc(w, &w->special, N / 256 + 2)) || (rc = dalloc(w, &w->tile_work, 2 * (N / gw::COMBINED_TILE + 2))) ||
        (rc = dalloc(w, &w->tile_order, 1 + (size_t)gw::combined_tiles((uint32_t)N) + 16)) || (rc = dalloc(w, &w->ework, N)) ||
        (rc = dalloc(w, &w->nb_count, 1)))
        return fail(rc);
    if (hipMemset(w->tile_order, 0, sizeof(uint32_t)) != hipSuccess ||  // no order yet
        hipMemset(w->ework, 0, N * sizeof(uint8_t)) != hipSuccess)
        return fail(GWAOI_EDEVICE);
    // lastop = 0, rank = sp = 0xFFFFFFFF (not live)
    if (hipMemset(w->sinfo.rank, 0xFF, N * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(w->sinfo.sp, 0xFF, N * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(w->sinfo.lastop, 0, N * sizeof(unsigned long long)) != hipSuccess)
        return fail(GWAOI_EDEVICE);
    // the bucketed apply for worlds whose SlotInfo outgrows the MALL (GWAOI_F_TEST_BUCKETED forces it)
    w->moves_bucketed = N > gw::MV_MIN_SLOTS || (cfg->flags & GWAOI_F_TEST_BUCKETED);
    size_t mv_hist_n = 0;
    if (w->moves_bucketed && gw::moves_buckets((uint32_t)N) <= gw::MV_NB_MAX) {
        mv_hist_n = std::max(gw::moves_hist_elems((uint32_t)N, (uint32_t)N),
                             ((size_t)1 << 20) + 2 * (size_t)gw::moves_buckets((uint32_t)N) + 2);
        if ((rc = dalloc(w, &w->mv_hist, mv_hist_n)) || (rc = dalloc(w, &w->mv_binned, N))) return fail(rc);
    }
    if ((rc = ensure_scan_tmp(w, std::max(gw::radix_hist_elems((uint32_t)N), mv_hist_n)))) return fail(rc);
    for (FlushSet &S : w->fs)
        if ((rc = ensure_tile_entries(w, S, 2 * ((size_t)gw::combined_tiles((uint32_t)N) + gw::combined_blocks((uint32_t)N)))))
            return fail(rc);
    if ((rc = ensure_ops(w, 1024))) return fail(rc);
    for (FlushSet &S : w->fs)
        if ((rc = ensure_events(w, S, cfg->event_capacity ? cfg->event_capacity : std::max<uint64_t>(4 * N, 1 << 16),
                                cfg->event_capacity ? cfg->event_capacity : std::max<uint64_t>(4 * N, 1 << 16))))
            return fail(rc);
    if (hipHostMalloc((void **)&w->h_grid, sizeof(SpaceGrid) * w->max_spaces, hipHostMallocDefault) != hipSuccess)
        return fail(GWAOI_ENOMEM);
    if (hipEventCreateWithFlags(&w->done_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->order_ev, hipEventDisableTiming) != hipSuccess)
        return fail(GWAOI_EDEVICE);
    w->alive.assign(N, 0);
    w->in_frame.assign(N, 0);
    w->appended.assign(N, 0);
    w->space_of.assign(N, gw::SP_DEAD);
    w->spaces.resize(w->max_spaces);
    *out = w;
    return GWAOI_OK;
    });
}

int gwaoi_space_create(gwaoi_world *w, float d, uint32_t *space_out) {
    return gw::api_guard([&]() -> int {
    if (!w || !space_out) return GWAOI_EINVAL;
    if (!(d > 0.f) || !std::isfinite(d)) return GWAOI_EINVAL;  // "defaultAOIDistance < 0" panic, Space.go:92-94
    for (uint32_t s = 0; s < w->max_spaces; ++s) {
        SpaceHost &S = w->spaces[s];
        if (S.used) continue;
        // an id freed in this flush may still own pairs in the previous frame
        if (s < w->n_space_ids && S.grid_valid) continue;
        S = SpaceHost();
        S.used = true;
        S.D = d;
        w->n_space_ids = std::max(w->n_space_ids, s + 1);
        w->n_spaces_live++;
        *space_out = s;
        return GWAOI_OK;
    }
    return GWAOI_EBADSPACE;
    });
}

int gwaoi_space_destroy(gwaoi_world *w, uint32_t space) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    if (space >= w->n_space_ids || !w->spaces[space].used) return GWAOI_EBADSPACE;
    if (w->spaces[space].alive) return GWAOI_EBUSY;
    w->spaces[space].used = false;
    w->n_spaces_live--;
    return GWAOI_OK;
    });
}

namespace {

// The per-slot host mirror for a host call that reads it: rebuilt from the last committed frame
// after device Enter/Leave batches (the frame holds exactly the live slots); GWAOI_ESTATE while
// such a batch is queued or in flight (its slots are not known on the host yet).
int host_slots(gwaoi_world *w) {
    w->gen++;  // (an enqueue on the stream that no flush made: the next flush's early kernels wait for it)
    if (w->dev_struct || (w->in_flight && w->slots_stale)) {
        w->last_error = "a device Enter/Leave batch is queued or in flight: flush before host per-slot calls";
        return GWAOI_ESTATE;
    }
    if (!w->slots_stale) return GWAOI_OK;
    const DevFrame &F = w->fr[w->cur];
    std::vector<gw::SlotSp> ss(F.n);
    if (F.n) {
        HIP_TRY(hipMemcpyAsync(ss.data(), F.ss, F.n * sizeof(gw::SlotSp), hipMemcpyDeviceToHost, w->stream));
        HIP_TRY(hipStreamSynchronize(w->stream));
    }
    std::fill(w->alive.begin(), w->alive.end(), 0);
    std::fill(w->in_frame.begin(), w->in_frame.end(), 0);
    std::fill(w->space_of.begin(), w->space_of.end(), gw::SP_DEAD);
    for (const gw::SlotSp &e : ss) {
        if (e.slot >= w->max_slots) continue;
        w->alive[e.slot] = 1;
        w->in_frame[e.slot] = 1;
        w->space_of[e.slot] = e.sp;
    }
    w->slots_stale = false;
    return GWAOI_OK;
}

// Explicit seqs must keep call order: >= the next implicit seq, and nothing
// host-side may follow an explicit device batch inside one flush (its
// largest seq is only known after the flush).
int check_seq(gwaoi_world *w, const uint64_t *seq) {
    if (w->dev_seq_pending) return GWAOI_ESTATE;
    if (seq && *seq < w->seq_next) return GWAOI_EINVAL;
    return GWAOI_OK;
}
uint64_t take_seq(gwaoi_world *w, const uint64_t *seq) {
    const uint64_t s = seq ? *seq : w->seq_next;
    w->seq_next = s + 1;
    return s;
}

int enter_impl(gwaoi_world *w, uint32_t space, uint32_t slot, float x, float z, const uint64_t *seq) {
    if (!w) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (int rc = host_slots(w)) return rc;
    if (slot >= w->max_slots) return GWAOI_EBADSLOT;
    if (space >= w->n_space_ids || !w->spaces[space].used) return GWAOI_EBADSPACE;
    if (w->alive[slot]) return GWAOI_ESTATE;
    if (w->sync && gw::sync_slot_plain(w->sync, slot)) return GWAOI_ESTATE;  // in a space without AOI
    if (!finite2(x, z)) return GWAOI_ENONFINITE;
    if (int rc = check_seq(w, seq)) return rc;
    w->alive[slot] = 1;
    w->space_of[slot] = space;
    w->n_alive++;
    if (w->sync) gw::sync_note_slot(w->sync, slot, space);
    SpaceHost &S = w->spaces[space];
    S.alive++;
    const uint64_t sq = take_seq(w, seq);
    w->space_ops_queued = true;
    if (w->in_flight) {
        defer(w, Deferred::ENTER, slot, space, x, z, sq);
        return GWAOI_OK;
    }
    note_pending_bbox(S, x, z);
    mark_appended(w, slot);
    w->touched.push_back(slot);
    push_host_op(w, slot, x, z, space, sq);
    return GWAOI_OK;
}

int moved_impl(gwaoi_world *w, uint32_t slot, float x, float z, const uint64_t *seq) {
    if (!w) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (int rc = host_slots(w)) return rc;
    if (slot >= w->max_slots) return GWAOI_EBADSLOT;
    if (!w->alive[slot]) return GWAOI_ESTATE;
    if (!finite2(x, z)) return GWAOI_ENONFINITE;
    if (int rc = check_seq(w, seq)) return rc;
    const uint64_t sq = take_seq(w, seq);
    if (w->in_flight) {
        defer(w, Deferred::MOVED, slot, w->space_of[slot], x, z, sq);
        return GWAOI_OK;
    }
    note_pending_bbox(w->spaces[w->space_of[slot]], x, z);
    push_host_op(w, slot, x, z, w->space_of[slot], sq);
    return GWAOI_OK;
}


// Room for `words` more staged words.  1: no room without moving a buffer that a queued
// batch still points into (the caller then queues the batch as host ops).
int ensure_stage(gwaoi_world *w, size_t words) {
    const int h = w->stage_cur;
    // an open reservation (gwaoi_moved_batch_stage) owns the words past stage_used until its commit:
    // nothing else may stage into them, and the buffer it points into must not move
    if (w->resv_n) return 1;
    if (w->stage_used[h] + words <= w->stage_cap[h]) return GWAOI_OK;
    if (w->stage_used[h]) return 1;
    const size_t cap = std::max<size_t>({2 * words, 2 * w->stage_cap[h], (size_t)4 << 16});
    HIP_TRY(hipStreamSynchronize(w->copy_st));  // no staging copy may still read the old buffer
    if (w->h_stage[h]) (void)hipHostFree(w->h_stage[h]);
    w->h_stage[h] = nullptr;
    dfree(w->d_stage[h]);
    w->stage_cap[h] = 0;
    HIP_TRY(hipHostMalloc((void **)&w->h_stage[h], cap * sizeof(uint32_t), hipHostMallocDefault));
    if (int rc = dalloc(w, &w->d_stage[h], cap)) return rc;
    w->stage_cap[h] = cap;
    // grow the other half alike while no flush reads it, so that the first flush that stages
    // into it (the next one begun with gwaoi_tick_begin) does not pay the pinned allocation
    const int o = h ^ 1;
    if (!w->in_flight && w->stage_used[o] == 0 && w->stage_cap[o] < cap) {
        if (w->h_stage[o]) (void)hipHostFree(w->h_stage[o]);
        w->h_stage[o] = nullptr;
        dfree(w->d_stage[o]);
        w->stage_cap[o] = 0;
        if (hipHostMalloc((void **)&w->h_stage[o], cap * sizeof(uint32_t), hipHostMallocDefault) == hipSuccess &&
            dalloc(w, &w->d_stage[o], cap) == GWAOI_OK)
            w->stage_cap[o] = cap;
    }
    return GWAOI_OK;
}

struct StageBox {  // positions of one space seen by one staging chunk
    float x0, z0, x1, z1;
    bool any;
};

// Validate moves [lo, hi) in call order (the checks and their order of gwaoi_moved) and write them
// into the staging words h = [slots | x | z | space] (n each).  Returns the first bad index (hi if
// none) with its status in *st; boxes[space] gathers the chunk's positions.
size_t stage_chunk(const gwaoi_world *w, const uint32_t *slots, const float *x, const float *z, size_t n,
                   size_t lo, size_t hi, uint32_t *h, bool with_space, StageBox *boxes, int *st) {
    uint32_t *hs = h, *hsp = h + 3 * n;
    float *hx = reinterpret_cast<float *>(h + n), *hz = reinterpret_cast<float *>(h + 2 * n);
    // a live slot has a space (space_of == SP_DEAD <=> !alive): one random lookup per move
    const uint32_t *space_of = w->space_of.data();
    const uint32_t ms = w->max_slots;
    // The running box of the current space stays in registers: updated through a StageBox in
    // memory, every float store to hx/hz may alias it and the loop became a load-store chain.
    uint32_t bsp = gw::SP_DEAD;
    float bx0 = 0.f, bz0 = 0.f, bx1 = 0.f, bz1 = 0.f;
    auto fold = [&]() {
        if (bsp == gw::SP_DEAD) return;
        StageBox &b = boxes[bsp];
        if (!b.any) {
            b = StageBox{bx0, bz0, bx1, bz1, true};
        } else {
            b.x0 = std::min(b.x0, bx0); b.x1 = std::max(b.x1, bx1);
            b.z0 = std::min(b.z0, bz0); b.z1 = std::max(b.z1, bz1);
        }
    };
    for (size_t i = lo; i < hi; ++i) {
        if (i + 16 < hi) __builtin_prefetch(space_of + std::min(slots[i + 16], ms - 1));
        const uint32_t sl = slots[i];
        const float xi = x[i], zi = z[i];
        if (sl >= ms) { *st = GWAOI_EBADSLOT; return i; }
        const uint32_t sp = space_of[sl];
        if (sp == gw::SP_DEAD) { *st = GWAOI_ESTATE; return i; }
        if (!finite2(xi, zi)) { *st = GWAOI_ENONFINITE; return i; }
        hs[i] = sl; hx[i] = xi; hz[i] = zi;
        if (with_space) hsp[i] = sp;
        if (sp != bsp) {
            fold();
            bsp = sp;
            bx0 = bx1 = xi;
            bz0 = bz1 = zi;
        } else {
            bx0 = std::min(bx0, xi); bx1 = std::max(bx1, xi);
            bz0 = std::min(bz0, zi); bz1 = std::max(bz1, zi);
        }
    }
    fold();
    *st = GWAOI_OK;
    return hi;
}

// A host move batch with room in the staging area (ensure_stage): validate + stage it on up to
// kStageThreads host threads, send it with one async H2D and queue it as a device batch with seqs
// seq_next.. and the slot's space at call time (explicit, so a slot that entered earlier in this
// flush moves exactly as a host op would).  Nothing is queued if any move is rejected.
constexpr size_t kStageThreadMin = 1 << 13;  // moves per extra thread (65,536 moves: 8 threads, 0.39 -> ~0.06 ms)
constexpr size_t kStageMin = 64;             // host move batches of this many moves or more are staged

int stage_moves(gwaoi_world *w, const uint32_t *slots, const float *x, const float *z, size_t n) {
    const int half = w->stage_cur;
    // the space column is needed only when an Enter/Leave of this flush precedes the batch (a slot
    // that entered in this flush must move in its new space); otherwise every slot keeps its space
    const bool with_space = w->space_ops_queued;
    const size_t words = (with_space ? 4 : 3) * n;
    uint32_t *h = w->h_stage[half] + w->stage_used[half], *d = w->d_stage[half] + w->stage_used[half];
    const size_t nsp = std::max(1u, w->n_space_ids);
    unsigned T = (unsigned)std::min<size_t>(w->stage_threads, std::max<size_t>(1, n / kStageThreadMin));
    T = std::min(T, std::max(1u, std::thread::hardware_concurrency()));
    const size_t stride = nsp + 4;  // >= 64 B between the threads' boxes: no false sharing
    std::vector<StageBox> boxes((size_t)T * stride, StageBox{0, 0, 0, 0, false});
    std::vector<size_t> bad(T, 0);
    std::vector<int> st(T, GWAOI_OK);
    const size_t chunk = (n + T - 1) / T;
    w->pool.run(T, [&](unsigned t) {
        const size_t lo = std::min(n, t * chunk), hi = std::min(n, lo + chunk);
        bad[t] = stage_chunk(w, slots, x, z, n, lo, hi, h, with_space, boxes.data() + (size_t)t * stride, &st[t]);
    });
    for (unsigned t = 0; t < T; ++t)  // chunks are in call order: the first bad chunk has the first bad move
        if (st[t] != GWAOI_OK) return st[t];
    HIP_TRY(hipMemcpyAsync(d, h, words * sizeof(uint32_t), hipMemcpyHostToDevice, w->copy_st));
    HIP_TRY(hipEventRecord(w->copy_ev, w->copy_st));
    w->copy_pending = true;
    w->stage_used[half] += words;
    Run r{};
    r.device = true;
    r.ds = d;
    r.dx = reinterpret_cast<const float *>(d + n);
    r.dz = reinterpret_cast<const float *>(d + 2 * n);
    r.dsp = with_space ? d + 3 * n : nullptr;
    r.seq0 = w->seq_next;
    r.dn = n;
    r.checked = true;
    w->seq_next += n;
    for (unsigned t = 0; t < T; ++t)
        for (size_t sp = 0; sp < nsp; ++sp) {
            const StageBox &b = boxes[(size_t)t * stride + sp];
            if (!b.any) continue;
            if (w->in_flight) {
                w->deferred_boxes.push_back(DeferredBox{(uint32_t)sp, b.x0, b.z0, b.x1, b.z1});
            } else {
                note_pending_bbox(w->spaces[sp], b.x0, b.z0);
                note_pending_bbox(w->spaces[sp], b.x1, b.z1);
            }
        }
    if (w->in_flight) {
        Deferred q{};
        q.kind = Deferred::RUN;
        q.run = r;
        w->deferred.push_back(q);
    } else {
        w->runs.push_back(r);
        w->n_ops += n;
    }
    return GWAOI_OK;
}

}  // namespace

int gwaoi_enter(gwaoi_world *w, uint32_t space, uint32_t slot, float x, float z) {
    return gw::api_guard([&]() -> int {
    return enter_impl(w, space, slot, x, z, nullptr);
    });
}

int gwaoi_enter_seq(gwaoi_world *w, uint32_t space, uint32_t slot, float x, float z, uint64_t seq) {
    return gw::api_guard([&]() -> int {
    return enter_impl(w, space, slot, x, z, &seq);
    });
}

int gwaoi_leave(gwaoi_world *w, uint32_t slot) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (int rc = host_slots(w)) return rc;
    if (slot >= w->max_slots) return GWAOI_EBADSLOT;
    if (!w->alive[slot]) return GWAOI_ESTATE;
    if (w->dev_seq_pending) return GWAOI_ESTATE;
    w->alive[slot] = 0;
    w->spaces[w->space_of[slot]].alive--;
    w->space_of[slot] = gw::SP_DEAD;
    w->n_alive--;
    if (w->sync) gw::sync_note_slot(w->sync, slot, gw::SP_DEAD);
    w->space_ops_queued = true;
    if (w->in_flight) {
        defer(w, Deferred::LEAVE, slot, gw::SP_DEAD, 0.f, 0.f, w->seq_next);
        return GWAOI_OK;
    }
    w->touched.push_back(slot);
    push_host_op(w, slot, 0.f, 0.f, gw::SP_DEAD, w->seq_next);  // a Leave's seq is never compared
    return GWAOI_OK;
    });
}

int gwaoi_moved(gwaoi_world *w, uint32_t slot, float x, float z) { return gw::api_guard([&]() -> int { return moved_impl(w, slot, x, z, nullptr); }); }

int gwaoi_moved_seq(gwaoi_world *w, uint32_t slot, float x, float z, uint64_t seq) {
    return gw::api_guard([&]() -> int {
    return moved_impl(w, slot, x, z, &seq);
    });
}

int gwaoi_enter_batch(gwaoi_world *w, uint32_t space, const uint32_t *slots, const float *x, const float *z,
                      size_t n) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && (!slots || !x || !z))) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (space >= w->n_space_ids || !w->spaces[space].used) return GWAOI_EBADSPACE;
    if (w->dev_seq_pending) return GWAOI_ESTATE;
    if (int rc = host_slots(w)) return rc;
    // validate the whole batch first (duplicates inside the batch are Enter-twice)
    std::vector<uint32_t> seen;
    seen.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        if (slots[i] >= w->max_slots) return GWAOI_EBADSLOT;
        if (w->alive[slots[i]]) return GWAOI_ESTATE;
        if (!finite2(x[i], z[i])) return GWAOI_ENONFINITE;
        seen.push_back(slots[i]);
    }
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end()) return GWAOI_ESTATE;
    for (size_t i = 0; i < n; ++i) gwaoi_enter(w, space, slots[i], x[i], z[i]);
    return GWAOI_OK;
    });
}

int gwaoi_leave_batch(gwaoi_world *w, const uint32_t *slots, size_t n) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && !slots)) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->dev_seq_pending) return GWAOI_ESTATE;
    if (int rc = host_slots(w)) return rc;
    std::vector<uint32_t> seen(slots, slots + n);
    for (size_t i = 0; i < n; ++i) {
        if (slots[i] >= w->max_slots) return GWAOI_EBADSLOT;
        if (!w->alive[slots[i]]) return GWAOI_ESTATE;
    }
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end()) return GWAOI_ESTATE;
    for (size_t i = 0; i < n; ++i) gwaoi_leave(w, slots[i]);
    return GWAOI_OK;
    });
}

int gwaoi_moved_batch(gwaoi_world *w, const uint32_t *slots, const float *x, const float *z, size_t n) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && (!slots || !x || !z))) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->dev_seq_pending) return GWAOI_ESTATE;
    if (int rc = host_slots(w)) return rc;
    // Batches of kStageMin+ moves go through pinned staging as one device batch (single-pass
    // move apply); without room (or if the staging allocation failed) they queue as host ops.
    if (n >= kStageMin && n <= 0xFFFFFFFFull - w->n_ops && ensure_stage(w, 4 * n) == GWAOI_OK)
        return stage_moves(w, slots, x, z, n);
    for (size_t i = 0; i < n; ++i) {
        if (slots[i] >= w->max_slots) return GWAOI_EBADSLOT;
        if (!w->alive[slots[i]]) return GWAOI_ESTATE;
        if (!finite2(x[i], z[i])) return GWAOI_ENONFINITE;
    }
    for (size_t i = 0; i < n; ++i) gwaoi_moved(w, slots[i], x[i], z[i]);
    return GWAOI_OK;
    });
}

int gwaoi_moved_batch_device(gwaoi_world *w, const uint32_t *d_slots, const float *d_x, const float *d_z,
                             size_t n) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && (!d_slots || !d_x || !d_z))) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (!n) return GWAOI_OK;
    if (n > 0xFFFFFFFFull - w->n_ops) return GWAOI_EINVAL;
    if (w->dev_seq_pending) return GWAOI_ESTATE;
    Run r{};
    r.device = true;
    r.ds = d_slots;
    r.dx = d_x;
    r.dz = d_z;
    r.dseq = nullptr;
    r.seq0 = w->seq_next;
    r.dn = n;
    w->seq_next += n;
    if (w->in_flight) {
        Deferred q{};
        q.kind = Deferred::RUN;
        q.run = r;
        w->deferred.push_back(q);
        return GWAOI_OK;
    }
    w->runs.push_back(r);
    w->n_ops += n;
    return GWAOI_OK;
    });
}

int gwaoi_moved_batch_device_seq(gwaoi_world *w, const uint32_t *d_slots, const float *d_x, const float *d_z,
                                 const uint64_t *d_seq, size_t n) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && (!d_slots || !d_x || !d_z || !d_seq))) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->in_flight) return GWAOI_ESTATE;
    if (!n) return GWAOI_OK;
    if (n > 0xFFFFFFFFull - w->n_ops) return GWAOI_EINVAL;
    Run r{};
    r.device = true;
    r.ds = d_slots;
    r.dx = d_x;
    r.dz = d_z;
    r.dseq = reinterpret_cast<const unsigned long long *>(d_seq);
    r.seq0 = 0;
    r.dn = n;
    w->runs.push_back(r);
    w->n_ops += n;
    w->dev_seq_pending = true;
    return GWAOI_OK;
    });
}

int gwaoi_enter_batch_device(gwaoi_world *w, uint32_t space, const uint32_t *d_slots, const float *d_x,
                             const float *d_z, const uint64_t *d_seq, size_t n, const float *box) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && (!d_slots || !d_x || !d_z))) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (space >= w->n_space_ids || !w->spaces[space].used) return GWAOI_EBADSPACE;
    if (w->in_flight || w->sync) return GWAOI_ESTATE;
    if (!d_seq && w->dev_seq_pending) return GWAOI_ESTATE;
    if (!n) return GWAOI_OK;
    if (n > (size_t)w->max_slots - w->n_alive || n > 0xFFFFFFFFull - w->n_ops) return GWAOI_ECAPACITY;
    if (box && !(std::isfinite(box[0]) && std::isfinite(box[1]) && std::isfinite(box[2]) && std::isfinite(box[3]) &&
                 box[0] <= box[2] && box[1] <= box[3]))
        return GWAOI_EINVAL;
    Run r{};
    r.device = true;
    r.kind = RUN_ENTER;
    r.space = space;
    r.ds = d_slots;
    r.dx = d_x;
    r.dz = d_z;
    r.dseq = reinterpret_cast<const unsigned long long *>(d_seq);
    r.seq0 = d_seq ? 0 : w->seq_next;
    r.dn = n;
    if (!d_seq) w->seq_next += n;
    else w->dev_seq_pending = true;
    w->runs.push_back(r);
    w->n_ops += n;
    w->dev_app += (uint32_t)n;
    w->dev_struct = true;
    w->space_ops_queued = true;
    w->n_alive += (uint32_t)n;
    SpaceHost &S = w->spaces[space];
    S.alive += (uint32_t)n;
    if (box) {
        note_pending_bbox(S, box[0], box[1]);
        note_pending_bbox(S, box[2], box[3]);
    }
    return GWAOI_OK;
    });
}

int gwaoi_leave_batch_device(gwaoi_world *w, uint32_t space, const uint32_t *d_slots, size_t n) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && !d_slots)) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (space >= w->n_space_ids || !w->spaces[space].used) return GWAOI_EBADSPACE;
    if (w->in_flight || w->sync) return GWAOI_ESTATE;
    if (!n) return GWAOI_OK;
    if (n > w->spaces[space].alive || n > 0xFFFFFFFFull - w->n_ops) return GWAOI_ESTATE;
    Run r{};
    r.device = true;
    r.kind = RUN_LEAVE;
    r.space = space;
    r.ds = d_slots;
    // a Leave has no position: the slot array stands in for x and z (read, never used)
    r.dx = r.dz = reinterpret_cast<const float *>(d_slots);
    r.seq0 = w->seq_next;  // a Leave's seq is never compared
    r.dn = n;
    w->runs.push_back(r);
    w->n_ops += n;
    w->dev_struct = true;
    w->space_ops_queued = true;
    w->n_alive -= (uint32_t)n;
    w->spaces[space].alive -= (uint32_t)n;
    return GWAOI_OK;
    });
}

int gwaoi_moved_batch_stage(gwaoi_world *w, size_t n, uint32_t **slots, float **x, float **z) {
    return gw::api_guard([&]() -> int {
    if (!w || !slots || !x || !z || n == 0 || n > 0xFFFFFFFFull - w->n_ops) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->resv_n || w->dev_seq_pending) return GWAOI_ESTATE;
    if (int rc = ensure_stage(w, 4 * n)) {
        if (rc == 1) {
            w->last_error = "staging memory holds this flush's batches: flush before staging more";
            return GWAOI_ECAPACITY;
        }
        return rc;
    }
    const int h = w->stage_cur;
    w->resv_half = h;
    w->resv_n = n;
    w->resv_h = w->h_stage[h] + w->stage_used[h];
    w->resv_d = w->d_stage[h] + w->stage_used[h];
    *slots = w->resv_h;
    *x = reinterpret_cast<float *>(w->resv_h + n);
    *z = reinterpret_cast<float *>(w->resv_h + 2 * n);
    return GWAOI_OK;
    });
}

int gwaoi_moved_batch_commit(gwaoi_world *w, size_t k) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    GW_LIVE(w);
    const size_t n = w->resv_n;
    if (!n || k > n) return n ? GWAOI_EINVAL : GWAOI_ESTATE;
    w->resv_n = 0;
    if (w->resv_half != w->stage_cur) return GWAOI_ESTATE;  // a flush launched in between took that half
    if (!k) return GWAOI_OK;
    uint32_t *h = w->resv_h, *d = w->resv_d;
    // After an Enter / Leave queued in this flush a slot's space may differ from its space at the
    // flush's start: the space column is filled (and the batch checked) on the host then.
    const bool with_space = w->space_ops_queued;
    if (with_space) {
        if (int rc = host_slots(w)) return rc;
        std::vector<StageBox> boxes(std::max(1u, w->n_space_ids), StageBox{0, 0, 0, 0, false});
        int st = GWAOI_OK;
        const float *hx = reinterpret_cast<const float *>(h + n), *hz = reinterpret_cast<const float *>(h + 2 * n);
        if (stage_chunk(w, h, hx, hz, n, 0, k, h, true, boxes.data(), &st) != k) return st;
        for (size_t sp = 0; sp < boxes.size(); ++sp) {
            const StageBox &b = boxes[sp];
            if (!b.any) continue;
            if (w->in_flight) {
                w->deferred_boxes.push_back(DeferredBox{(uint32_t)sp, b.x0, b.z0, b.x1, b.z1});
            } else {
                note_pending_bbox(w->spaces[sp], b.x0, b.z0);
                note_pending_bbox(w->spaces[sp], b.x1, b.z1);
            }
        }
    }
    const size_t words = (with_space ? 4 : 3) * n;
    HIP_TRY(hipMemcpyAsync(d, h, words * sizeof(uint32_t), hipMemcpyHostToDevice, w->copy_st));
    HIP_TRY(hipEventRecord(w->copy_ev, w->copy_st));
    w->copy_pending = true;
    w->stage_used[w->resv_half] += 4 * n;
    Run r{};
    r.device = true;
    r.ds = d;
    r.dx = reinterpret_cast<const float *>(d + n);
    r.dz = reinterpret_cast<const float *>(d + 2 * n);
    r.dsp = with_space ? d + 3 * n : nullptr;
    r.seq0 = w->seq_next;
    r.dn = k;
    w->seq_next += k;
    if (w->in_flight) {
        Deferred q{};
        q.kind = Deferred::RUN;
        q.run = r;
        w->deferred.push_back(q);
    } else {
        w->runs.push_back(r);
        w->n_ops += k;
    }
    return GWAOI_OK;
    });
}

int gwaoi_moved_batch_pinned(gwaoi_world *w, const uint32_t *slots, const float *x, const float *z, size_t n) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && (!slots || !x || !z)) || n > 0xFFFFFFFFull - w->n_ops) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->dev_seq_pending || w->resv_n) return GWAOI_ESTATE;
    if (!n) return GWAOI_OK;
    // after an Enter / Leave of this flush a slot's space may have changed: host-checked staging
    if (w->space_ops_queued) return gwaoi_moved_batch(w, slots, x, z, n);
    if (int rc = ensure_stage(w, 3 * n)) {
        if (rc == 1) {
            w->last_error = "staging memory holds this flush's batches: flush before queueing more";
            return GWAOI_ECAPACITY;
        }
        return rc;
    }
    const int h = w->stage_cur;
    uint32_t *d = w->d_stage[h] + w->stage_used[h];
    HIP_TRY(hipMemcpyAsync(d, slots, n * sizeof(uint32_t), hipMemcpyHostToDevice, w->copy_st));
    HIP_TRY(hipMemcpyAsync(d + n, x, n * sizeof(float), hipMemcpyHostToDevice, w->copy_st));
    HIP_TRY(hipMemcpyAsync(d + 2 * n, z, n * sizeof(float), hipMemcpyHostToDevice, w->copy_st));
    HIP_TRY(hipEventRecord(w->copy_ev, w->copy_st));
    w->copy_pending = true;
    w->stage_used[h] += 3 * n;
    Run r{};
    r.device = true;
    r.ds = d;
    r.dx = reinterpret_cast<const float *>(d + n);
    r.dz = reinterpret_cast<const float *>(d + 2 * n);
    r.seq0 = w->seq_next;
    r.dn = n;
    w->seq_next += n;
    if (w->in_flight) {
        Deferred q{};
        q.kind = Deferred::RUN;
        q.run = r;
        w->deferred.push_back(q);
    } else {
        w->runs.push_back(r);
        w->n_ops += n;
    }
    return GWAOI_OK;
    });
}

int gwaoi_pinned_alloc(gwaoi_world *w, size_t bytes, void **out) {
    return gw::api_guard([&]() -> int {
    if (!w || !out || !bytes) return GWAOI_EINVAL;
    *out = nullptr;
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return GWAOI_ENOMEM;
    }
    return GWAOI_OK;
    });
}

int gwaoi_pinned_free(gwaoi_world *w, void *p) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    if (p) HIP_TRY(hipHostFree(p));
    return GWAOI_OK;
    });
}

}  // extern "C"

namespace gw {

WorldView world_view(gwaoi_world *w) {
    w->gen++;  // (an enqueue on the stream that no flush made: the next flush's early kernels wait for it)
    WorldView v{};
    v.F = view_of(w->fr[w->cur]);
    v.info = w->sinfo;
    v.st = w->stream;
    v.max_slots = w->max_slots;
    v.pending_ops = w->n_ops + w->deferred.size() + (w->in_flight ? 1 : 0);
    v.in_flight = w->in_flight;
    v.events = last_events(w);
    v.n_enter = w->last_n_enter;
    v.n_leave = w->last_n_leave;
    return v;
}

SyncState *&world_sync(gwaoi_world *w) { return w->sync; }

void world_set_error(gwaoi_world *w, const char *msg) { w->last_error = msg; }

void world_flush_events(gwaoi_world *w, const uint32_t **events, const uint32_t **dcount, uint64_t *cap) {
    FlushSet &S = w->fs[w->in_flight ? w->fl.set : w->last_set];
    *events = S.events;
    *dcount = reinterpret_cast<const uint32_t *>(S.dev_out);
    *cap = w->in_flight ? w->fl.cap.out : S.ev_cap;  // events the set's buffer holds (clipped to it)
}

uint32_t world_slot_space(gwaoi_world *w, uint32_t slot) {
    if (host_slots(w) != GWAOI_OK) return SP_DEAD;
    return slot < w->max_slots && w->alive[slot] ? w->space_of[slot] : SP_DEAD;
}

int world_queue_decoded(gwaoi_world *w, const uint32_t *d_slots, const float *d_x, const float *d_z,
                        const uint32_t *d_sp, size_t n) {
    GW_LIVE(w);
    if (w->in_flight) return GWAOI_ESTATE;
    if (!n) return GWAOI_OK;
    if (n > 0xFFFFFFFFull - w->n_ops) return GWAOI_EINVAL;
    if (w->dev_seq_pending) return GWAOI_ESTATE;
    Run r{};
    r.device = true;
    r.ds = d_slots;
    r.dx = d_x;
    r.dz = d_z;
    r.dsp = d_sp;
    r.seq0 = w->seq_next;
    r.dn = n;
    w->runs.push_back(r);
    w->n_ops += n;
    w->seq_next += n;
    return GWAOI_OK;
}

}  // namespace gw

extern "C" {

int gwaoi_tick_begin(gwaoi_world *w) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->in_flight) return GWAOI_ESTATE;
    return tick_launch(w);
    });
}

}  // extern "C"

namespace {

// gwaoi_tick_finish(GWAOI_END_NEXT): finish the flush in flight, begin the next one (speculatively,
// before the finished one's summary is read, when the queue allows it).
int end_begin(gwaoi_world *w, bool *committed_out) {
    bool committed = false;
    int rc, lrc = GWAOI_OK;
    if (speculative_ok(w)) {
        // the next flush goes on the stream first, then the host waits for the one in flight:
        // no idle gap on the GPU between the two
        const Flight f = w->fl;
        commit_host(w, nullptr);
        w->ovl_ok = true;
#ifdef GWAOI_EXP_HOSTTIME
        const auto h0 = std::chrono::steady_clock::now();
#endif
        lrc = tick_launch(w);
        w->ovl_ok = false;
        if (lrc == GWAOI_OK) w->dbg.speculative_launches++;
#ifdef GWAOI_EXP_HOSTTIME
        const auto h1 = std::chrono::steady_clock::now();
        (void)wait_done(w, w->fs[f.set].done_ev);
        const auto h2 = std::chrono::steady_clock::now();
#endif
        rc = finish_flight(w, f, true, &committed);
#ifdef GWAOI_EXP_HOSTTIME
        const auto h3 = std::chrono::steady_clock::now();
        w->ht[1] += std::chrono::duration<double, std::micro>(h1 - h0).count();
        w->ht[2] += std::chrono::duration<double, std::micro>(h2 - h1).count();
        w->ht[3] += std::chrono::duration<double, std::micro>(h3 - h2).count();
#endif
    } else {
        rc = tick_finish(w, &committed);
        if (committed && !w->poisoned) lrc = tick_launch(w);
    }
    *committed_out = committed;
    return rc != GWAOI_OK ? rc : lrc;
}

// Queues the copy of the committed flush's events to h_events on the copy-out stream (directed
// events, or one per mirrored pair); gwaoi_events_host / gwaoi_pairs_host wait for it.
// regrows: the regrow count before the flush ended (a re-run of its pair passes ends later than
// its done event).
int copy_out(gwaoi_world *w, bool pairs, uint64_t regrows) {
    const uint64_t tot = w->last_n_enter + w->last_n_leave;
    if (int rc2 = ensure_host_events(w, std::max<uint64_t>(tot, 1))) return poison(w, rc2);
    FlushSet &S = w->fs[w->last_set];
    w->out_pairs = pairs;
    w->out_n_enter = w->last_n_enter;
    w->out_n_leave = w->last_n_leave;
    if (tot) {
        // ordered after the flush's last kernel (its event's release makes the writes visible to the
        // copy engine); after a re-run of its pair passes, after the wait that followed the re-run
        HIP_TRY(hipStreamWaitEvent(w->out_st, w->dbg.event_regrows != regrows ? w->done_ev : S.done_ev, 0));
        if (pairs) {
            gw::launch_pairs_out(S.events, tot / 2, w->d_h_events, w->out_st);
            HIP_TRY(hipGetLastError());
        } else {
            HIP_TRY(hipMemcpyAsync(w->h_events, S.events, 2 * tot * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   w->out_st));
        }
        HIP_TRY(hipEventRecord(w->out_ev, w->out_st));
        w->out_pending = true;
    }
    return GWAOI_OK;
}

// The flush's end with its events copied to host memory on its own stream, no next flush
// (gwaoi_tick, gwaoi_tick_finish(GWAOI_END_HOST)): the copy is the D2H stage of the stage timing.
int end_host(gwaoi_world *w, bool *committed) {
    w->gen++;  // (an enqueue on the stream that no flush made: the next flush's early kernels wait for it)
    int rc = tick_finish(w, committed);
    if (!*committed) return rc;
    // committed: deliver the events whatever the status (InterestedIn/By must follow the frame)
    const uint64_t tot = w->last_n_enter + w->last_n_leave;
    if (int rc2 = ensure_host_events(w, std::max<uint64_t>(tot, 1)))
        return poison(w, rc2);  // the committed events cannot reach the caller
    w->out_pairs = false;
    w->out_n_enter = w->last_n_enter;
    w->out_n_leave = w->last_n_leave;
    FlushSet &S = w->fs[w->last_set];
    stage_begin(w, S, ST_D2H);
    if (tot) {
        hipError_t e = hipMemcpyAsync(w->h_events, S.events, 2 * tot * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                      w->stream);
        if (e != hipSuccess) {
            w->last_error = std::string("event D2H: ") + hipGetErrorString(e);
            return poison(w, GWAOI_EDEVICE);
        }
        if (int rw = wait_stream(w)) return poison(w, rw);
    }
    stage_end(w, S, ST_D2H);
    if (w->timing_mask) {
        (void)hipStreamSynchronize(w->stream);
        stage_collect(w, S);
    }
    return rc;
}

}  // namespace

extern "C" {

int gwaoi_tick_finish(gwaoi_world *w, uint32_t mode, uint64_t *n_enter, uint64_t *n_leave) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    if (n_enter) *n_enter = 0;
    if (n_leave) *n_leave = 0;
    if (mode & ~(GWAOI_END_NEXT | GWAOI_END_HOST | GWAOI_END_PAIRS)) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (!w->in_flight) return GWAOI_ESTATE;
    const bool next = (mode & GWAOI_END_NEXT) != 0, pairs = (mode & GWAOI_END_PAIRS) != 0;
    const bool host = pairs || (mode & GWAOI_END_HOST) != 0;
    if (host) {
        // the host copy is being replaced: until this flush's copy is queued it holds nothing
        if (int rw = finish_out(w)) return poison(w, rw);
        w->out_n_enter = w->out_n_leave = 0;
        w->out_pairs = pairs;
    }
    bool committed = false;
    int rc;
#ifdef GWAOI_EXP_HOSTTIME
    w->ht_entry = std::chrono::steady_clock::now();
    struct HtCall {
        gwaoi_world *w;
        ~HtCall() {
            w->ht[4] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w->ht_entry).count();
            w->ht[5] += 1.0;
        }
    } ht_call{w};
#endif
    if (host && !next && !pairs) {
        rc = end_host(w, &committed);
    } else {
        const uint64_t regrows = w->dbg.event_regrows;
        rc = next ? end_begin(w, &committed) : tick_finish(w, &committed);
        if (committed && host)
            if (int rc2 = copy_out(w, pairs, regrows)) return rc2;
    }
    if (committed) {
        if (n_enter) *n_enter = w->last_n_enter;
        if (n_leave) *n_leave = w->last_n_leave;
    }
    return rc;
    });
}

int gwaoi_events_host(gwaoi_world *w, gwaoi_events *out) {
    return gw::api_guard([&]() -> int {
    if (!w || !out) return GWAOI_EINVAL;
    out->n_enter = out->n_leave = 0;
    out->enter = out->leave = nullptr;
    GW_LIVE(w);
    if (w->out_pairs) return GWAOI_ESTATE;  // the last copy-out holds pairs: gwaoi_pairs_host
    if (int rw = finish_out(w)) return poison(w, rw);
    out->n_enter = w->out_n_enter;
    out->n_leave = w->out_n_leave;
    out->enter = w->h_events;
    out->leave = w->h_events ? w->h_events + 2 * w->out_n_enter : nullptr;
    return GWAOI_OK;
    });
}

int gwaoi_pairs_host(gwaoi_world *w, gwaoi_events *out) {
    return gw::api_guard([&]() -> int {
    if (!w || !out) return GWAOI_EINVAL;
    out->n_enter = out->n_leave = 0;
    out->enter = out->leave = nullptr;
    GW_LIVE(w);
    if (!w->out_pairs) return GWAOI_ESTATE;
    if (int rw = finish_out(w)) return poison(w, rw);
    out->n_enter = w->out_n_enter / 2;
    out->n_leave = w->out_n_leave / 2;
    out->enter = w->h_events;
    out->leave = w->h_events ? w->h_events + w->out_n_enter : nullptr;
    return GWAOI_OK;
    });
}


int gwaoi_tick_device(gwaoi_world *w, uint64_t *n_enter, uint64_t *n_leave) {
    const int sp = w ? gw::api_guard([&]() -> int {
        GW_LIVE(w);
        return sparse_try(w);
    }) : 1;
    if (sp <= 0) {
        if (n_enter) *n_enter = sp == GWAOI_OK ? w->last_n_enter : 0;
        if (n_leave) *n_leave = sp == GWAOI_OK ? w->last_n_leave : 0;
        return sp;
    }
    if (int rc = gwaoi_tick_begin(w)) {
        if (n_enter) *n_enter = 0;
        if (n_leave) *n_leave = 0;
        return rc;
    }
    return gwaoi_tick_finish(w, 0u, n_enter, n_leave);
}

int gwaoi_events_device(gwaoi_world *w, const uint32_t **d_enter, const uint32_t **d_leave) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    if (d_enter) *d_enter = last_events(w);
    if (d_leave) *d_leave = last_events(w) + 2 * w->last_n_enter;
    return GWAOI_OK;
    });
}

int gwaoi_tick(gwaoi_world *w, gwaoi_events *out) {
    if (!w || !out) return GWAOI_EINVAL;
    out->n_enter = out->n_leave = 0;
    out->enter = out->leave = nullptr;
    const int sp = gw::api_guard([&]() -> int {
        GW_LIVE(w);
        const int rc = sparse_try(w);
        if (rc != GWAOI_OK) return rc;
        // the sparse flush's events to host memory
        const uint64_t tot = w->last_n_enter + w->last_n_leave;
        if (int rc2 = ensure_host_events(w, std::max<uint64_t>(tot, 1))) return poison(w, rc2);
        w->out_pairs = false;
        w->out_n_enter = w->last_n_enter;
        w->out_n_leave = w->last_n_leave;
        if (tot) {
            HIP_TRY(hipMemcpyAsync(w->h_events, w->fs[w->last_set].events, 2 * tot * sizeof(uint32_t),
                                   hipMemcpyDeviceToHost, w->stream));
            if (int rw = wait_stream(w)) return poison(w, rw);
        }
        out->n_enter = w->last_n_enter;
        out->n_leave = w->last_n_leave;
        out->enter = w->h_events;
        out->leave = w->h_events + 2 * w->last_n_enter;
        return GWAOI_OK;
    });
    if (sp <= 0) return sp;  // committed sparse flush, or an error
    if (int rc = gwaoi_tick_begin(w)) return rc;
    return gw::api_guard([&]() -> int {
        bool committed = false;
        const int rc = end_host(w, &committed);
        if (committed) {
            out->n_enter = w->out_n_enter;
            out->n_leave = w->out_n_leave;
            out->enter = w->h_events;
            out->leave = w->h_events + 2 * w->out_n_enter;
        }
        return rc;
    });
}

namespace {

// Build the last flush's event rows on the device (once per flush).
int build_csr(gwaoi_world *w) {
    w->gen++;  // (an enqueue on the stream that no flush made: the next flush's early kernels wait for it)
    const uint64_t tot = w->last_n_enter + w->last_n_leave;
    if (w->csr_tick == w->ticks) return GWAOI_OK;
    const size_t rows = w->max_slots;
    if (!w->csr_cnt) {
        int rc;
        if ((rc = dalloc(w, &w->csr_cnt, rows + 1)) || (rc = dalloc(w, &w->csr_off, rows + 1)) ||
            (rc = dalloc(w, &w->csr_long, rows)))
            return rc;
    }
    if (tot > w->csr_items_cap) {
        HIP_TRY(hipStreamSynchronize(w->stream));
        dfree(w->csr_items);
        w->csr_items_cap = 0;
        const uint64_t cap = std::max<uint64_t>(tot + tot / 4, 1 << 16);
        if (int rc = dalloc(w, &w->csr_items, 2 * cap)) return rc;  // items | merge scratch of long rows
        w->csr_items_cap = cap;
    }
    if (int rc = ensure_scan_tmp(w, rows + 1)) return rc;
    gw::launch_events_csr(last_events(w), w->last_n_enter, tot, (uint32_t)rows, w->csr_cnt, w->csr_off, w->scan_tmp,
                          w->csr_items, w->csr_items + w->csr_items_cap, w->csr_long, w->stream);
    HIP_TRY(hipGetLastError());
    w->csr_tick = w->ticks;
    return GWAOI_OK;
}

}  // namespace

int gwaoi_events_csr_device(gwaoi_world *w, const uint32_t **d_offsets, const uint32_t **d_items, uint64_t *n_items) {
    return gw::api_guard([&]() -> int {
    if (!w || !d_offsets || !d_items) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->in_flight) return GWAOI_ESTATE;
    if (int rc = build_csr(w)) return rc;
    *d_offsets = w->csr_off;
    *d_items = w->csr_items;
    if (n_items) *n_items = w->last_n_enter + w->last_n_leave;
    return GWAOI_OK;
    });
}

int gwaoi_events_csr(gwaoi_world *w, const uint32_t **offsets, const uint32_t **items, uint64_t *n_items) {
    return gw::api_guard([&]() -> int {
    if (!w || !offsets || !items) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->in_flight) return GWAOI_ESTATE;
    if (int rc = build_csr(w)) return rc;
    const uint64_t tot = w->last_n_enter + w->last_n_leave;
    if (!w->h_csr_off) HIP_TRY(hipHostMalloc((void **)&w->h_csr_off, ((size_t)w->max_slots + 1) * 4, hipHostMallocDefault));
    if (tot > w->h_csr_items_cap) {
        if (w->h_csr_items) (void)hipHostFree(w->h_csr_items);
        w->h_csr_items = nullptr;
        w->h_csr_items_cap = 0;
        const uint64_t cap = std::max<uint64_t>(tot + tot / 4, 1 << 16);
        HIP_TRY(hipHostMalloc((void **)&w->h_csr_items, cap * 4, hipHostMallocDefault));
        w->h_csr_items_cap = cap;
    }
    w->gen++;
    HIP_TRY(hipMemcpyAsync(w->h_csr_off, w->csr_off, ((size_t)w->max_slots + 1) * 4, hipMemcpyDeviceToHost, w->stream));
    if (tot) HIP_TRY(hipMemcpyAsync(w->h_csr_items, w->csr_items, tot * 4, hipMemcpyDeviceToHost, w->stream));
    if (int rc = wait_stream(w)) return rc;
    *offsets = w->h_csr_off;
    *items = w->h_csr_items;
    if (n_items) *n_items = tot;
    return GWAOI_OK;
    });
}

int gwaoi_neighbors(gwaoi_world *w, uint32_t slot, uint32_t *out, size_t cap, size_t *n_out) {
    return gw::api_guard([&]() -> int {
    if (!w || (cap && !out)) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->in_flight) return GWAOI_ESTATE;
    if (slot >= w->max_slots) return GWAOI_EBADSLOT;
    if (n_out) *n_out = 0;
    if (int rc = host_slots(w)) return rc;
    if (!w->in_frame[slot]) return GWAOI_ESTATE;
    const size_t need = std::max<size_t>(cap, 1);
    if (need > w->nb_cap) {
        dfree(w->nb_out);
        int rc = dalloc(w, &w->nb_out, need);
        if (rc) return rc;
        w->nb_cap = need;
    }
    const DevFrame &F = w->fr[w->cur];
    w->gen++;
    HIP_TRY(hipMemsetAsync(w->nb_count, 0, sizeof(uint32_t), w->stream));
    gw::launch_neighbors(view_of(F), w->sinfo, slot, w->nb_out, (uint32_t)std::min<size_t>(cap, 0xFFFFFFFFu),
                         w->nb_count, w->stream);
    HIP_TRY(hipGetLastError());
    uint32_t cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, w->nb_count, sizeof(uint32_t), hipMemcpyDeviceToHost, w->stream));
    HIP_TRY(hipStreamSynchronize(w->stream));
    const size_t k = std::min<size_t>(cnt, cap);
    if (k) {
        HIP_TRY(hipMemcpyAsync(out, w->nb_out, k * sizeof(uint32_t), hipMemcpyDeviceToHost, w->stream));
        HIP_TRY(hipStreamSynchronize(w->stream));
    }
    if (n_out) *n_out = cnt;
    return GWAOI_OK;
    });
}

int gwaoi_snapshot(gwaoi_world *w, uint32_t *slots, uint32_t *spaces, float *x, float *z, uint64_t *seq,
                   size_t cap, size_t *n_out) {
    return gw::api_guard([&]() -> int {
    if (!w || !n_out) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->in_flight) return GWAOI_ESTATE;
    const DevFrame &F = w->fr[w->cur];
    *n_out = F.n;
    if (F.n > cap || !F.n) return GWAOI_OK;
    if (!slots || !spaces || !x || !z || !seq) return GWAOI_EINVAL;
    std::vector<gw::Rec16> rec(F.n);
    std::vector<gw::SlotSp> ss(F.n);
    w->gen++;
    HIP_TRY(hipMemcpyAsync(rec.data(), F.rec, F.n * sizeof(gw::Rec16), hipMemcpyDeviceToHost, w->stream));
    HIP_TRY(hipMemcpyAsync(ss.data(), F.ss, F.n * sizeof(gw::SlotSp), hipMemcpyDeviceToHost, w->stream));
    HIP_TRY(hipStreamSynchronize(w->stream));
    for (uint32_t i = 0; i < F.n; ++i) {
        slots[i] = ss[i].slot;
        spaces[i] = ss[i].sp;
        x[i] = rec[i].x;
        z[i] = rec[i].z;
        seq[i] = rec[i].s;
    }
    return GWAOI_OK;
    });
}

int gwaoi_restore(gwaoi_world *w, const uint32_t *slots, const uint32_t *spaces, const float *x, const float *z,
                  const uint64_t *seq, size_t n) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && (!slots || !spaces || !x || !z || !seq))) return GWAOI_EINVAL;
    GW_LIVE(w);
    if (w->n_ops || w->dev_seq_pending || w->in_flight) return GWAOI_ESTATE;
    if (int rc = host_slots(w)) return rc;
    std::vector<size_t> ord(n);
    for (size_t i = 0; i < n; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return seq[a] < seq[b]; });
    // validate everything before queueing anything
    std::vector<uint32_t> seen(slots, slots + n);
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end()) return GWAOI_ESTATE;
    for (size_t k = 0; k < n; ++k) {
        const size_t i = ord[k];
        if (slots[i] >= w->max_slots) return GWAOI_EBADSLOT;
        if (w->alive[slots[i]]) return GWAOI_ESTATE;
        if (spaces[i] >= w->n_space_ids || !w->spaces[spaces[i]].used) return GWAOI_EBADSPACE;
        if (!finite2(x[i], z[i])) return GWAOI_ENONFINITE;
        if (k && seq[i] == seq[ord[k - 1]]) return GWAOI_EINVAL;
    }
    // The original seqs when they all lie at or above the world's next seq (a fresh world, or one
    // whose counter is below the snapshot's): then gwaoi_snapshot after the restore returns them
    // unchanged, which strip worlds (halo records carry global seqs) rely on.  Otherwise fresh seqs
    // in the frozen order: the relation inside the world only compares seqs, so it is the frozen
    // one either way.
    const bool keep = n == 0 || seq[ord[0]] >= w->seq_next;
    for (size_t k = 0; k < n; ++k) {
        const size_t i = ord[k];
        if (int rc = enter_impl(w, spaces[i], slots[i], x[i], z[i], keep ? &seq[i] : nullptr)) return rc;
    }
    return GWAOI_OK;
    });
}

int gwaoi_world_info(gwaoi_world *w, gwaoi_info *info) {
    return gw::api_guard([&]() -> int {
    if (!w || !info) return GWAOI_EINVAL;
    info->ticks = w->ticks;
    info->next_seq = w->seq_next;
    info->live = w->fr[w->cur].n;
    info->spaces = w->n_spaces_live;
    info->total_cells = w->fr[w->cur].total_cells;
    info->pending_ops = (uint32_t)w->n_ops;
    info->event_capacity = std::min(w->fs[w->launch_set].ev_cap, w->fs[w->launch_set].evtmp_cap);
    info->max_slots = w->max_slots;
    info->max_spaces = w->max_spaces;
    return GWAOI_OK;
    });
}

int gwaoi_debug_counters(gwaoi_world *w, gwaoi_debug *out) {
    return gw::api_guard([&]() -> int {
    if (!w || !out) return GWAOI_EINVAL;
    *out = w->dbg;
    out->cells_per_dist = (uint32_t)w->cells_per_dist;
    return GWAOI_OK;
    });
}

int gwaoi_stage_times(gwaoi_world *w, gwaoi_stage_time *out, size_t cap, size_t *n_out) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    size_t k = std::min<size_t>(cap, ST_N);
    for (size_t i = 0; i < k; ++i) {
        std::snprintf(out[i].name, sizeof(out[i].name), "%s", kStageNames[i]);
        out[i].ms = w->stage_ms[i];
        out[i].calls = w->stage_calls[i];
    }
    if (n_out) *n_out = ST_N;
    return GWAOI_OK;
    });
}

int gwaoi_set_stage_timing(gwaoi_world *w, uint32_t stage_mask) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    w->timing_mask = stage_mask & ((1u << ST_N) - 1u);
    return GWAOI_OK;
    });
}

int gwaoi_reset_stage_times(gwaoi_world *w) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    for (int s = 0; s < ST_N; ++s) {
        w->stage_ms[s] = 0;
        w->stage_calls[s] = 0;
    }
    return GWAOI_OK;
    });
}

int gwaoi_sync(gwaoi_world *w) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    HIP_TRY(hipStreamSynchronize(w->stream));
    return GWAOI_OK;
    });
}

void *gwaoi_stream(gwaoi_world *w) {
    if (!w) return nullptr;
    w->gen++;  // the caller may queue work the next flush depends on
    return (void *)w->stream;
}

int gwaoi_stream_after(gwaoi_world *w, void *other) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    HIP_TRY(hipEventRecord(w->order_ev, (hipStream_t)other));
    HIP_TRY(hipStreamWaitEvent(w->stream, w->order_ev, 0));
    w->gen++;  // the next flush's early kernels wait for the other stream too
    return GWAOI_OK;
    });
}

int gwaoi_stream_before(gwaoi_world *w, void *other) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    HIP_TRY(hipEventRecord(w->order_ev, w->stream));
    HIP_TRY(hipStreamWaitEvent((hipStream_t)other, w->order_ev, 0));
    return GWAOI_OK;
    });
}

}  // extern "C"
