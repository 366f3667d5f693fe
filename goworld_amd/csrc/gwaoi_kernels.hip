// gwaoi_kernels.hip -- HIP kernels of the AOI flush for gfx950 (MI355X).
//
// One flush (gwaoi_tick) runs, on one stream:
//   prologue             zero the per-tick counters / ranges
//   copy_state + ops     S' = previous frame, then the queued Enter/Leave/
//                        Moved calls applied last-writer-wins (seq = call
//                        order; only the final state of a slot matters)
//   keygen               cell key per entity (space-major uniform grid), and
//                        the per-tick scalars d_rel (largest "near" move / D)
//                        and bmax (largest |coordinate|)
//   radix sort           stable LSD sort of (key, index), wave64 multisplit
//   gather               new frame (sorted) + previous state in the new order
//   cell_count + scan    cell_start table;  tiles: rows cut into <= 256 entities
//   pairs<2>             combined pass over the new grid: every unordered pair
//                        once, go-aoi's float32 window relation at t and t-1
//                        (last-mover ownership)
//   pairs<1>             leaves of "special" entities (left, changed space,
//                        moved > D/4) over the previous grid
//   reorder + finish     events into deterministic tile order, summary
//   bbox                 per-space bounding box for the next flush's grid
//
// The path is sort/scan/gather/compaction: integer and float32-compare work,
// no dense contraction, so no MFMA.  Compile with -ffp-contract=off: the
// window bounds must be plain float32 sums as in go-aoi (`coord - aoidist`).

#include "gwaoi_internal.h"
#include "gwaoi_device.h"

#include <hip/hip_ext.h>

#include <algorithm>

namespace gw {
namespace {

constexpr int WAVE = 64;

__device__ __forceinline__ uint32_t lane() { return __lane_id(); }
__device__ __forceinline__ unsigned long long lanemask_lt() { return (1ull << lane()) - 1ull; }

inline uint32_t cdiv(size_t a, size_t b) { return (uint32_t)((a + b - 1) / b); }

// ------------------------------------------------------------- prologue ------

// Per-flush start: zero the counters and two ranges, reset the bbox fold,
// and copy the previous frame into S' (n_copy entries).
// The claims of a moves-only flush's first Moved run (k_moves_mark) are stored
// by the same launch (mark.n = 0: none).
__global__ void k_prologue(TickScalars *sc, uint32_t *z0, uint32_t n0, uint32_t *z1, uint32_t n1, int4 *bbox,
                           uint32_t n_spaces, uint32_t n_copy, const Rec16 *__restrict__ p_rec,
                           const SlotSp *__restrict__ p_ss, Rec16 *s_rec, SlotSp *s_ss, MoveRun mark,
                           uint32_t max_slots, SlotTab info, uint32_t tick, uint32_t n_unique) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < mark.n) {
        const uint32_t s = mark.ds[i];
        if (s < max_slots) info.lastop[s] = ((unsigned long long)tick << 32) | (mark.j0 + i);
    }
    if (i < n_copy) {
        reinterpret_cast<uint4 *>(s_rec)[i] = reinterpret_cast<const uint4 *>(p_rec)[i];
        reinterpret_cast<uint2 *>(s_ss)[i] = reinterpret_cast<const uint2 *>(p_ss)[i];
    }
    if (i == 0) {
        sc->err = 0;
        sc->counter = 0;
        sc->d_rel = 0.0f;
        sc->bmax = 0.0f;
        sc->seq_max = 0;
        sc->ncoll = 0;
        sc->ndrop = 0;
        sc->err_apply = 0;
        sc->n_unique = n_unique;
        for (int q = 0; q < (int)DBG_N; ++q) sc->dbg[q] = 0;
    }
    if (i < n0) z0[i] = 0;
    if (i < n1) z1[i] = 0;
    if (i < n_spaces) bbox[i] = make_int4(INT_MAX, INT_MAX, INT_MIN, INT_MIN);
    if (i < EV_SHARDS * 32) (&sc->shard[0][0])[i] = 0;
}

__global__ void k_zero(uint32_t *p, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0;
}

// ------------------------------------------------------------ op apply ------

__global__ void k_init_appended(const uint32_t *__restrict__ new_slots, uint32_t n_app, uint32_t base,
                                Rec16 *s_rec, SlotSp *s_ss, SlotTab info, uint32_t max_slots, TickScalars *sc) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_app) return;
    const uint32_t s = new_slots[i];
    const uint32_t idx = base + i;
    Rec16 r;
    r.x = r.z = 0.0f;
    r.s = 0;
    st_rec(s_rec, idx, r);
    st_ss(s_ss, idx, s, SP_DEAD);  // dead until its Enter applies
    if (s >= max_slots) {
        atomicOr(&sc->err, ERR_BAD_SLOT);
        return;
    }
    // a slot live when the flush began keeps its entry (a device Enter batch breaking the rules)
    if (info.sp[s] != SP_DEAD) {
        atomicOr(&sc->err, ERR_ENTER_LIVE);
        return;
    }
    info.rank[s] = idx;
    info.sp[s] = SP_DEAD;
}

__global__ void k_ops_claim(const uint32_t *__restrict__ slots, uint32_t n, uint32_t j0, uint32_t max_slots,
                            SlotTab info, uint32_t tick, TickScalars *sc) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slots[i];
    if (s == SLOT_NONE) return;  // placeholder of a skipped decoded record
    if (s >= max_slots) {
        atomicOr(&sc->err, ERR_BAD_SLOT);
        return;
    }
    atomicMax(&info.lastop[s], ((unsigned long long)tick << 32) | (j0 + i));
}

// The last op of a slot in this flush determines its state (closed form:
// only the final position and the final seq matter).
// One op of a run, loaded with all its fields at once (coalesced, one round
// trip, independent of the slot's SlotInfo line).
struct OpIn {
    uint32_t slot, sp;  // sp: SP_KEEP = device Moved (keep the slot's space)
    float x, z;
    unsigned long long seq;
};

__device__ __forceinline__ OpIn op_in(const uint32_t *__restrict__ slots, const float *__restrict__ xs,
                                      const float *__restrict__ zs, const uint32_t *__restrict__ sps,
                                      uint32_t sp_def, const unsigned long long *__restrict__ seqs,
                                      unsigned long long seq0, uint32_t i) {
    OpIn o;
    o.slot = slots[i];
    o.x = xs[i];
    o.z = zs[i];
    o.sp = sps ? sps[i] : sp_def;
    o.seq = seqs ? seqs[i] : seq0 + i;
    return o;
}

// The slot's table entry as (lastop lo, lastop hi, rank, sp): both loads issued together (the
// empty asm keeps the compiler from making the rank load wait for the claim compare).
__device__ __forceinline__ uint4 slot_info(SlotTab info, uint32_t s) {
    const unsigned long long lo = info.lastop[s];
    uint4 si = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), info.rank[s], info.sp[s]);
    asm volatile("" : "+v"(si.x), "+v"(si.y), "+v"(si.z), "+v"(si.w));
    return si;
}
// Only the rank (the unique-moves apply compares no claim, and its flush appends no entry, so a
// slot is live exactly when its rank is not 0xFFFFFFFF): one random line per op, from the 4 B-per-
// slot array.  The space word returned is any live space (0) for a live slot, SP_DEAD otherwise.
__device__ __forceinline__ uint4 slot_rank(SlotTab info, uint32_t s) {
    const uint32_t r = info.rank[s];
    return make_uint4(0u, 0u, r, r == 0xFFFFFFFFu ? SP_DEAD : 0u);
}

// The claim and the rank (a claims-path flush that appends no entry and changes no space, i.e.
// virtual S': a slot is live exactly when its rank is not 0xFFFFFFFF, and an op with an explicit
// space moves the slot within it): two random lines per op, not three.
__device__ __forceinline__ uint4 slot_claim_rank(SlotTab info, uint32_t s, uint32_t op_sp) {
    const unsigned long long lo = info.lastop[s];
    const uint32_t r = info.rank[s];
    uint4 si = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), r,
                          r == 0xFFFFFFFFu ? SP_DEAD : op_sp == SP_KEEP ? 0u : op_sp);
    asm volatile("" : "+v"(si.x), "+v"(si.y), "+v"(si.z));
    return si;
}

// Apply op o (index j in the flush) if it is its slot's last op of this flush
// (check_claim; si = the slot's table entry, slot_info); returns its seq (0 if not
// applied) for the seq_max fold.
__device__ __forceinline__ unsigned long long op_apply_one(const OpIn &o, uint32_t j, const uint4 &si,
                                                           SlotTab info, uint32_t tick, uint32_t n_total,
                                                           unsigned long long seq_floor, Rec16 *s_rec, SlotSp *s_ss,
                                                           TickScalars *sc, bool check_claim, uint32_t *errw) {
    const uint32_t s = o.slot;
    if (check_claim && (((unsigned long long)si.y << 32) | si.x) != (((unsigned long long)tick << 32) | j)) return 0;
    const uint32_t idx = si.z, cur_sp = si.w;
    if (idx >= n_total) {
        atomicOr(errw, ERR_MOVE_DEAD);
        return 0;
    }
    uint32_t sp = o.sp;
    Rec16 r;
    r.s = o.seq;
    if (r.s < seq_floor) {  // explicit seq older than an earlier flush: the closed form would be wrong
        atomicOr(errw, ERR_SEQ);
        return 0;
    }
    if (sp == SP_DEAD) {  // Leave: the slot drops out of the next frame
        r.x = r.z = 0.0f;
        st_rec(s_rec, idx, r);
        st_ss(s_ss, idx, s, SP_DEAD);
        info.rank[s] = 0xFFFFFFFFu;
        info.sp[s] = SP_DEAD;
        return r.s;
    }
    const bool keep = sp == SP_KEEP;
    if (keep) {  // device-side Moved
        sp = cur_sp;
        if (sp == SP_DEAD) {
            atomicOr(errw, ERR_MOVE_DEAD);
            return 0;
        }
    }
    r.x = o.x;
    r.z = o.z;
    if (!isfinite(r.x) || !isfinite(r.z)) {
        atomicOr(errw, ERR_NONFINITE);
        return 0;
    }
    st_rec(s_rec, idx, r);
    if (!keep && sp != cur_sp) {
        if (s_ss) st_ss(s_ss, idx, s, sp);
        else atomicOr(errw, ERR_COUNT_MISMATCH);  // moves-only flush (S' spaces = previous frame): bug guard
    }
    return r.s;
}

__global__ void k_ops_apply(const uint32_t *__restrict__ slots, const float *__restrict__ xs,
                            const float *__restrict__ zs, const uint32_t *__restrict__ sps, uint32_t sp_def,
                            uint32_t n, uint32_t j0, uint32_t max_slots, SlotTab info, uint32_t tick,
                            uint32_t n_total, const unsigned long long *__restrict__ seqs, unsigned long long seq0,
                            unsigned long long seq_floor, int track_max, Rec16 *s_rec, SlotSp *s_ss,
                            TickScalars *sc) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long smax = 0;
    if (i < n) {
        OpIn o;
        o.slot = slots[i];
        o.x = xs ? xs[i] : 0.0f;  // a Leave run has no positions
        o.z = zs ? zs[i] : 0.0f;
        o.sp = sps ? sps[i] : sp_def;
        o.seq = seqs ? seqs[i] : seq0 + i;
        if (o.slot < max_slots)
            smax = op_apply_one(o, j0 + i, slot_info(info, o.slot), info, tick, n_total, seq_floor, s_rec, s_ss, sc,
                                true, &sc->err);
    }
    if (track_max) {  // one atomic per wave, not per op
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long v = __shfl_xor(smax, o, WAVE);
            smax = v > smax ? v : smax;
        }
        if (lane() == 0 && smax) atomicMax(&sc->seq_max, smax);
    }
}

// Device Moved batches only (the per-tick position sync), without an atomic
// per move (a device-scope atomic is performed memory-side on gfx950).
// Pass 1 (k_moves_mark) stores every op's claim with a plain 8-byte store:
// ops of one slot race and some claim of this tick survives the kernel
// boundary.  Pass 2 (k_moves_apply_n): the op whose claim survived applies; an
// op that finds another op's claim folds its own in with atomicMax
// (repeated slots only, rare) and lists the slot, so that k_moves_fixup
// re-applies the true last op once this kernel has drained.
__global__ void k_moves_mark(MoveRun R, uint32_t max_slots, SlotTab info, uint32_t tick) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R.n) return;
    const uint32_t s = R.ds[i];
    if (s < max_slots) info.lastop[s] = ((unsigned long long)tick << 32) | (R.j0 + i);
}

#ifndef GWAOI_APPLY_PER
#define GWAOI_APPLY_PER 4  // moves per thread of the single-pass apply (all slot-table lines in flight at once)
#endif
// UNIQUE (GWAOI_F_UNIQUE_MOVES): no op shares its slot with another op of the flush, so every op
// applies without a claim; the ops that write nothing are counted (sc->ndrop, one atomic per wave)
// for keygen's written-entry check.
// VIRT (a flush with virtual S', no Enter/Leave): the claims path loads the claim and the rank only.
template <int PER, bool UNIQUE, bool VIRT>
__global__ __launch_bounds__(256) void k_moves_apply_n(MoveRun R, uint32_t max_slots, SlotTab info, uint32_t tick,
                                                       uint32_t n_total, unsigned long long seq_floor, Rec16 *s_rec,
                                                       SlotSp *s_ss, TickScalars *sc, uint32_t *coll) {
    const uint32_t i0 = blockIdx.x * (256u * PER) + threadIdx.x;
    OpIn o[PER];
    uint4 si[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const uint32_t i = i0 + (uint32_t)u * 256u;
        o[u].slot = SLOT_NONE;
        if (i < R.n) o[u] = op_in(R.ds, R.dx, R.dz, R.dsp, R.sp_def, R.dseq, R.seq0, i);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u)  // every slot-table line in flight at once
        si[u] = o[u].slot >= max_slots ? make_uint4(0, 0, 0, 0)
                : UNIQUE ? slot_rank(info, o[u].slot)
                : VIRT   ? slot_claim_rank(info, o[u].slot, o[u].sp)
                         : slot_info(info, o[u].slot);
    unsigned long long smax = 0;
    uint32_t drop = 0;
    uint32_t *errw = UNIQUE ? &sc->err_apply : &sc->err;  // unique: sc->err is zeroed by keygen, after this
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const uint32_t i = i0 + (uint32_t)u * 256u;
        const uint32_t s = o[u].slot;
        if (i >= R.n) continue;
        if (s == SLOT_NONE) {
            ++drop;
            continue;
        }
        if (s >= max_slots) {
            atomicOr(errw, ERR_BAD_SLOT);
            ++drop;
            continue;
        }
        if (UNIQUE) {
            const unsigned long long q =
                op_apply_one(o[u], R.j0 + i, si[u], info, tick, n_total, seq_floor, s_rec, s_ss, sc, false, errw);
            if (!q) ++drop;
            smax = q > smax ? q : smax;
            continue;
        }
        const unsigned long long mine = ((unsigned long long)tick << 32) | (R.j0 + i);
        const unsigned long long seen = ((unsigned long long)si[u].y << 32) | si[u].x;
        if (seen == mine) {
            const unsigned long long q =
                op_apply_one(o[u], R.j0 + i, si[u], info, tick, n_total, seq_floor, s_rec, s_ss, sc, false, errw);
            smax = q > smax ? q : smax;
        } else {
            atomicMax(&info.lastop[s], mine);
            coll[atomicAdd(&sc->ncoll, 1u)] = s;
        }
    }
    if (UNIQUE) {
        for (int q = 32; q > 0; q >>= 1) drop += __shfl_xor(drop, q, WAVE);
        if (lane() == 0 && drop) atomicAdd(&sc->ndrop, drop);
    }
    if (R.dseq) {
        for (int q = 32; q > 0; q >>= 1) {
            const unsigned long long v = __shfl_xor(smax, q, WAVE);
            smax = v > smax ? v : smax;
        }
        if (lane() == 0 && smax) atomicMax(&sc->seq_max, smax);
    }
}

// The slots moved more than once: the op whose claim survived every atomicMax is applied again.
// A launch of its own: fusing it into the last apply block needed a release fence in every block
// (at agent scope on gfx950, a write-back of the XCD's L2), measured at 162 against 33 us per apply.
__device__ __forceinline__ void moves_fixup(const FixupArgs &F, uint32_t t0, uint32_t stride) {
    const uint32_t nc = F.sc->ncoll;
    for (uint32_t k = t0; k < nc; k += stride) {
        const uint32_t s = F.coll[k];
        const uint4 si = slot_info(F.info, s);
        const uint32_t j = si.x;  // the winner (lastop low word; high word == tick)
        uint32_t q = 0;
        while (q + 1 < F.RS.count && j >= F.RS.r[q + 1].j0) ++q;
        const MoveRun &R = F.RS.r[q];
        // start from the previous state so that a dropped (invalid) winner leaves it unchanged
        if (si.z < F.n_prev) st_rec(F.s_rec, si.z, ld_rec(F.p_rec, si.z));
        const OpIn o = op_in(R.ds, R.dx, R.dz, R.dsp, R.sp_def, R.dseq, R.seq0, j - R.j0);
        op_apply_one(o, j, si, F.info, F.tick, F.n_total, F.seq_floor, F.s_rec, F.s_ss, F.sc, true, &F.sc->err);
    }
}

__global__ void k_moves_fixup(FixupArgs F) { moves_fixup(F, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x); }

// --------------------------------------------------------------- keygen ------

constexpr float FAR_FRAC = 0.25f;  // displacement > FAR_FRAC * D per axis => "special"

// "near" = live at t-1 and at t in the same space and moved at most
// FAR_FRAC*D per axis.  The special pass uses the complement, computed from
// the same operands.
__device__ __forceinline__ bool is_near(float xn, float zn, float xo, float zo, float thr) {
    return (int)(fabsf(xn - xo) <= thr) & (int)(fabsf(zn - zo) <= thr);
}

// Candidate record of the combined pass (k_gather -> k_combined), 16 B per
// frame entry: the exact (x, z) of a "near" entity and its previous-flush
// (x, z); (NaN, NaN, ...) for a jumper -- not near: new in this space,
// changed space, or moved > FAR_FRAC*D on an axis (an absent previous state
// has NaN coordinates and fails is_near).  NaN fails every band compare, so
// the strip filters drop jumper partners without a flag load; the previous
// position lets the filter drop pairs whose relation certainly did not change.
__device__ __forceinline__ uint4 cand_of(const Rec16 &now, const Rec16 &old, float thr) {
    return is_near(now.x, now.z, old.x, old.z, thr)
               ? make_uint4(__float_as_uint(now.x), __float_as_uint(now.z), __float_as_uint(old.x),
                            __float_as_uint(old.z))
               : make_uint4(0x7FC00000u, 0x7FC00000u, 0x7FC00000u, 0x7FC00000u);
}

constexpr int SC_T = 256;
constexpr int SC_I = 16;
constexpr int SC_TILE = SC_T * SC_I;
#ifndef GWAOI_S64_I
#define GWAOI_S64_I 4  // cells per thread of the cell scan (k_scan64); measured (cfg3): 2 -> 10.3 us, 4 -> 8.2, 8 -> 8.7, 16 -> 13.6
#endif
constexpr int S64_I = GWAOI_S64_I;
constexpr uint32_t FG = 256;  // measured (cfg3 k_finish): 128 -> 11.8 us, 256 -> 11.4, 512 -> 11.7
// A pair pass's tile total, also added to its group's total, which follows the entries'
// totals (tile_total[entries + 1 + e / FG], zeroed with them by the prologue).
__device__ __forceinline__ void put_tile_total(uint32_t *tt, uint32_t leave_off, uint32_t e, uint32_t v) {
    tt[e] = v;
    if (v) atomicAdd(tt + 2 * leave_off + 1 + e / FG, v);
}
constexpr int S64_TILE = SC_T * S64_I;

// INCR (the grid is the previous frame's): also count, per cell, the
// entities (low word of cnt64) and the "arrivals" -- entities whose cell
// differs from their previous-frame cell, or new in the frame (high word).
// S' is the previous frame (sorted by the same keys) plus appended entries,
// so equal keys come in runs and one atomic per run and wave suffices.
#ifndef GWAOI_KG_PER
#define GWAOI_KG_PER 2  // S' entries per keygen thread (their operands in flight together)
#endif
constexpr int KG_PER = GWAOI_KG_PER;
static_assert(KG_PER == 1 || KG_PER == 2, "the written-entry count below takes one or two entries per thread");
constexpr uint32_t keygen_blocks(uint32_t n) { return (n + 256u * KG_PER - 1) / (256u * KG_PER); }

template <bool INCR>
__global__ __launch_bounds__(256) void k_keygen(Rec16 *s_rec, const SlotSp *__restrict__ s_ss,
                                                uint32_t n, const SpaceGrid *__restrict__ grid, uint32_t sentinel,
                                                uint32_t *keys, uint32_t *vals, const Rec16 *__restrict__ p_rec,
                                                const SlotSp *__restrict__ p_ss,
                                                const SpaceGrid *__restrict__ p_grid, uint32_t n_prev, float *blk,
                                                const uint32_t *__restrict__ p_key, unsigned long long *cnt64,
                                                unsigned long long seq_base, uint32_t *special, TickZero tz,
                                                unsigned long long *tent) {
    __shared__ float s_m[2][256 / WAVE];
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
    if (tz.sc) {  // the prologue's zeroing (a unique-moves flush without one; see TickZero)
        const uint32_t m = max(max(tz.n1, tz.n_spaces), EV_SHARDS * 32u), stride = gridDim.x * blockDim.x;
        for (uint32_t j = gt; j < m; j += stride) {
            if (j < tz.n1) tz.z1[j] = 0;
            if (j < tz.n_spaces) tz.bbox[j] = make_int4(INT_MAX, INT_MAX, INT_MIN, INT_MIN);
            if (j < EV_SHARDS * 32) (&tz.sc->shard[0][0])[j] = 0;
        }
        if (gt == 0) {
            TickScalars *sc = tz.sc;
            sc->err = 0;
            sc->counter = 0;
            sc->d_rel = 0.0f;
            sc->bmax = 0.0f;
            sc->seq_max = 0;
            sc->ncoll = 0;
            sc->n_unique = tz.n_unique;
            for (int q = 0; q < (int)DBG_N; ++q) sc->dbg[q] = 0;
        }
    }
    // KG_PER entries per thread, 256 apart: entry i_u = base + 256 u is of the special pass's tile
    // KG_PER b + u.  Every operand of every entry first, in one round trip (none depends on
    // another): the S' record and space, the previous frame's record, space and key.
    const uint32_t base = blockIdx.x * (256u * KG_PER) + threadIdx.x;
    uint32_t s[KG_PER], ps[KG_PER], old[KG_PER];
    Rec16 r[KG_PER], p[KG_PER];
#pragma unroll
    for (int u = 0; u < KG_PER; ++u) {
        const uint32_t i = base + 256u * (uint32_t)u;
        const bool in = i < n, inp = i < n_prev;
        s[u] = in ? ld_ss(s_ss, i).sp : SP_DEAD;
        r[u].x = r[u].z = 0.0f;
        r[u].s = 0;
        if (in) r[u] = ld_rec(s_rec, i);
        ps[u] = inp ? ld_ss(p_ss, i).sp : SP_DEAD;
        p[u].x = p[u].z = 0.0f;
        p[u].s = 0;
        if (inp) p[u] = ld_rec(p_rec, i);
        old[u] = INCR && inp ? p_key[i] : sentinel;
    }
    float dr = 0.0f, bm = 0.0f;
    bool near[KG_PER];
    uint32_t kt[KG_PER];  // INCR: the scan tile of each entry's new key (0xFFFFFFFF: no entry)
    uint32_t nwr = 0;  // entries this flush's ops wrote (GWAOI_F_UNIQUE_MOVES: one per op that applied)
#pragma unroll
    for (int u = 0; u < KG_PER; ++u) {
        const uint32_t i = base + 256u * (uint32_t)u;
        const bool inp = i < n_prev;
        near[u] = false;  // live at t-1 and t in the same space, moved <= FAR_FRAC * D per axis
        kt[u] = 0xFFFFFFFFu;
        if (i >= n) continue;
        uint32_t key = sentinel;
        Rec16 rr = r[u];
        if (s[u] != SP_DEAD) {
            nwr += rr.s >= seq_base ? 1u : 0u;
            const bool same = inp && ps[u] == s[u];
            if (same || (inp && rr.s < seq_base)) {
                if (rr.s < seq_base && inp) {  // not written by this flush's ops: the previous state
                    if (rr.x != p[u].x || rr.z != p[u].z || rr.s != p[u].s) st_rec(s_rec, i, p[u]);  // (virtual S')
                    rr = p[u];
                }
                const float D = p_grid[s[u]].D;
                if (same && is_near(rr.x, rr.z, p[u].x, p[u].z, FAR_FRAC * D)) {
                    dr = fmaxf(dr, fmaxf(fabsf(rr.x - p[u].x), fabsf(rr.z - p[u].z)) / D);
                    near[u] = true;
                }
            }
            const SpaceGrid g = grid[s[u]];
            const int cx = cell_of(rr.x, g.ox, g.inv, g.gx);
            const int cz = cell_of(rr.z, g.oz, g.inv, g.gz);
            key = g.base + (uint32_t)cz * g.gx + (uint32_t)cx;
            bm = fmaxf(bm, fmaxf(fabsf(rr.x), fabsf(rr.z)));
        }
        keys[i] = key;
        kt[u] = key / (uint32_t)S64_TILE;
        if (!INCR) vals[i] = i;
        // INCR: only the entities that changed cell count: an arrival in the new cell (low word), a
        // departure from the old one (high word); a cell's stayers are its previous count minus
        // its departures, which k_scan64 takes from the previous cell_start
        if (INCR && key != old[u]) {
            if (key != sentinel) atomicAdd(&cnt64[key], 1ull);
            if (old[u] != sentinel) atomicAdd(&cnt64[old[u]], 1ull << 32);
        }
    }
    // INCR: entries per scan tile of the new keys (dead entries in the sentinel cell's tile).  S'
    // is in the previous frame's order, so a wave's entries almost always share one tile: each
    // wave notes (tile, count) in LDS and thread 0 adds the block's few distinct tiles after the
    // barrier below (an atomic wave-instruction costs ~50 ns of its CU's atomic path whatever its
    // lanes: one per wave made keygen 13 -> 22 us); a wave that spans tiles adds its own.
    // k_scan64 takes a tile's start in the new frame from these counts (no pass over the cell
    // counts before it); k_cell_merge zeroes them again.
    __shared__ uint32_t s_tt[256 / WAVE][KG_PER], s_tc[256 / WAVE][KG_PER];
    if (INCR) {
#pragma unroll
        for (int u = 0; u < KG_PER; ++u) {
            unsigned long long act = __ballot(kt[u] != 0xFFFFFFFFu);
            uint32_t t0 = 0xFFFFFFFFu, c0 = 0u;
            if (act) {
                const uint32_t lead = (uint32_t)__ffsll((long long)act) - 1u;
                t0 = (uint32_t)__builtin_amdgcn_readlane((int)kt[u], (int)lead);
                const unsigned long long m = __ballot(kt[u] == t0);
                c0 = (uint32_t)__popcll(m);
                act &= ~m;
            }
            while (act) {  // rare: the wave's entries span tiles
                const uint32_t lead = (uint32_t)__ffsll((long long)act) - 1u;
                const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)kt[u], (int)lead);
                const unsigned long long m = __ballot(kt[u] == t);
                if (lane() == lead) atomicAdd(&tent[t], (unsigned long long)__popcll(m));
                act &= ~m;
            }
            if (lane() == 0) {
                s_tt[threadIdx.x / WAVE][u] = t0;
                s_tc[threadIdx.x / WAVE][u] = c0;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        dr = fmaxf(dr, __shfl_xor(dr, o));
        bm = fmaxf(bm, __shfl_xor(bm, o));
    }
    if (lane() == 0) {
        s_m[0][threadIdx.x / WAVE] = dr;
        s_m[1][threadIdx.x / WAVE] = bm;
    }
    // the special pass's tiles of this block (previous-frame entries [256 t, 256 t + 256)): does one
    // hold an entity that is not near (left, changed space, jumped)?  k_pairs<1> skips the tiles without
#pragma unroll
    for (int u = 0; u < KG_PER; ++u) {
        const uint32_t t = blockIdx.x * (uint32_t)KG_PER + (uint32_t)u;
        const bool sp_any = __syncthreads_or(base + 256u * (uint32_t)u < n_prev && !near[u]);
        if (special && threadIdx.x == 0 && t * 256u < n_prev) special[t] = sp_any ? 1u : 0u;
    }
    const uint32_t nw = (uint32_t)__syncthreads_count(nwr >= 1) + (KG_PER > 1 ? (uint32_t)__syncthreads_count(nwr >= 2) : 0u);
    if (INCR && threadIdx.x == 0) {  // the block's (tile, count) notes, one add per distinct tile
        uint32_t t = 0xFFFFFFFFu, c = 0u;
        for (int u = 0; u < KG_PER; ++u)  // (entry order: the notes of one tile come together)
            for (int q = 0; q < 256 / WAVE; ++q) {
                const uint32_t tq = s_tt[q][u], cq = s_tc[q][u];
                if (!cq) continue;
                if (tq != t) {
                    if (c) atomicAdd(&tent[t], (unsigned long long)c);
                    t = tq;
                    c = 0u;
                }
                c += cq;
            }
        if (c) atomicAdd(&tent[t], (unsigned long long)c);
    }
    if (threadIdx.x == 0) {
        reinterpret_cast<uint32_t *>(blk)[2 * gridDim.x + blockIdx.x] = nw;
        float a = s_m[0][0], b = s_m[1][0];
        for (int q = 1; q < 256 / WAVE; ++q) {
            a = fmaxf(a, s_m[0][q]);
            b = fmaxf(b, s_m[1][q]);
        }
        blk[2 * blockIdx.x] = a;
        blk[2 * blockIdx.x + 1] = b;
    }
}

// Fold keygen's per-block partials (T threads, one pass): d_rel / bmax into sc, and under
// GWAOI_F_UNIQUE_MOVES the written-entry counts (after the 2 nb float partials): those plus the ops
// that wrote nothing must be the flush's ops; fewer means two ops shared a slot, and which one's
// position the frame holds is then not defined (ERR_DUP_SLOT).
template <int T>
__device__ __forceinline__ void keygen_fold_t(const float *__restrict__ blk, uint32_t nb, TickScalars *sc) {
    __shared__ float s_m[2][T / WAVE];
    __shared__ uint32_t s_c[T / WAVE];
    const uint32_t *cnt = reinterpret_cast<const uint32_t *>(blk) + 2 * nb;
    float a = 0.0f, b = 0.0f;
    uint32_t c = 0;
    for (uint32_t i = threadIdx.x; i < nb; i += T) {
        a = fmaxf(a, blk[2 * i]);
        b = fmaxf(b, blk[2 * i + 1]);
        c += cnt[i];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a = fmaxf(a, __shfl_xor(a, o));
        b = fmaxf(b, __shfl_xor(b, o));
        c += __shfl_xor(c, o);
    }
    if (lane() == 0) {
        s_m[0][threadIdx.x / WAVE] = a;
        s_m[1][threadIdx.x / WAVE] = b;
        s_c[threadIdx.x / WAVE] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < T / WAVE; ++q) {
            a = fmaxf(a, s_m[0][q]);
            b = fmaxf(b, s_m[1][q]);
            c += s_c[q];
        }
        sc->d_rel = a;
        sc->bmax = b;
        const uint32_t want = sc->n_unique, ea = sc->err_apply, nd = sc->ndrop;
        uint32_t e = ea;
        if (want && c + nd != want) e |= ERR_DUP_SLOT;
        if (e) atomicOr(&sc->err, e);
        if (ea) sc->err_apply = 0;  // zero again for the next flush of this set (one without a prologue)
        if (nd) sc->ndrop = 0;
    }
}

__global__ __launch_bounds__(1024) void k_keygen_reduce(const float *__restrict__ blk, uint32_t nb,
                                                        TickScalars *sc) {
    keygen_fold_t<1024>(blk, nb, sc);
}

// ----------------------------------------------------------------- scan ------

constexpr int SC1_T = 1024;  // single-workgroup scan
constexpr int SC1_I = 16;
constexpr size_t SC1_MAX = (size_t)SC1_T * SC1_I * 4;  // loops over chunks of SC1_T*SC1_I

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        uint32_t y = __shfl_up(x, o);
        if ((int)lane() >= o) x += y;
    }
    return x;
}

// exclusive scan of one value per thread over a block of NT threads
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *ws, uint32_t &total) {
    uint32_t x = wave_incl_scan(v);
    const int w = threadIdx.x / WAVE;
    if (lane() == WAVE - 1) ws[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / WAVE; ++i) {
        uint32_t t = ws[i];
        pre += (i < w) ? t : 0u;
        tot += t;
    }
    total = tot;
    return pre + x - v;
}

template <int NI>
__device__ __forceinline__ void loadN(const uint32_t *in, size_t base, size_t n, uint32_t (&v)[NI]) {
    if (base + NI <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(in + base);
#pragma unroll
        for (int q = 0; q < NI / 4; ++q) {
            uint4 t = p[q];
            v[4 * q] = t.x;
            v[4 * q + 1] = t.y;
            v[4 * q + 2] = t.z;
            v[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < NI; ++q) v[q] = (base + q < n) ? in[base + q] : 0u;
    }
}

template <int NI>
__device__ __forceinline__ void storeN_excl(uint32_t *out, size_t base, size_t n, const uint32_t (&v)[NI],
                                            uint32_t run) {
    if (base + NI <= n) {
        uint4 *p = reinterpret_cast<uint4 *>(out + base);
#pragma unroll
        for (int q = 0; q < NI / 4; ++q) {
            uint4 t;
            t.x = run; run += v[4 * q];
            t.y = run; run += v[4 * q + 1];
            t.z = run; run += v[4 * q + 2];
            t.w = run; run += v[4 * q + 3];
            p[q] = t;
        }
    } else {
#pragma unroll
        for (int q = 0; q < NI; ++q)
            if (base + q < n) {
                out[base + q] = run;
                run += v[q];
            }
    }
}

__global__ __launch_bounds__(SC_T) void k_scan_reduce(const uint32_t *__restrict__ in, size_t n, uint32_t *sums) {
    __shared__ uint32_t ws[SC_T / WAVE];
    uint32_t v[SC_I];
    loadN<SC_I>(in, (size_t)blockIdx.x * SC_TILE + (size_t)threadIdx.x * SC_I, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < SC_I; ++q) s += v[q];
    uint32_t tot;
    block_excl_scan<SC_T>(s, ws, tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SC_T) void k_scan_down(const uint32_t *in, uint32_t *out, size_t n,
                                                    const uint32_t *__restrict__ block_off) {
    __shared__ uint32_t ws[SC_T / WAVE];
    const size_t base = (size_t)blockIdx.x * SC_TILE + (size_t)threadIdx.x * SC_I;
    uint32_t v[SC_I];
    loadN<SC_I>(in, base, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < SC_I; ++q) s += v[q];
    uint32_t tot;
    const uint32_t run = block_excl_scan<SC_T>(s, ws, tot) + (block_off ? block_off[blockIdx.x] : 0u);
    storeN_excl<SC_I>(out, base, n, v, run);
}

// one workgroup, chunks of SC1_T*SC1_I with a running carry (small arrays)
__global__ __launch_bounds__(SC1_T) void k_scan_single(const uint32_t *in, uint32_t *out, size_t n) {
    __shared__ uint32_t ws[SC1_T / WAVE];
    uint32_t carry = 0;
    for (size_t c0 = 0; c0 < n; c0 += (size_t)SC1_T * SC1_I) {
        const size_t base = c0 + (size_t)threadIdx.x * SC1_I;
        uint32_t v[SC1_I];
        loadN<SC1_I>(in, base, n, v);
        uint32_t s = 0;
#pragma unroll
        for (int q = 0; q < SC1_I; ++q) s += v[q];
        uint32_t tot;
        const uint32_t run = block_excl_scan<SC1_T>(s, ws, tot) + carry;
        storeN_excl<SC1_I>(out, base, n, v, run);
        carry += tot;
        __syncthreads();
    }
}

// ------------------------------------------------------- bucketed apply ------
// Bucketed form of the moves-only apply (k_moves_*) for large worlds.  The ops
// arrive in the caller's order, which is random against the slot-indexed
// SlotInfo: k_moves_* pay a random 8-B claim store (prologue), a random SlotInfo
// line and the record store per op, plus atomics for repeated slots.  While
// SlotInfo stays in the 256 MB MALL (1M slots: 16 MB) that is the faster form;
// at 16M slots (256 MB) every random line comes from HBM and this one wins
// (cfg5 one strip: 5.9 vs 7.7 ms per tick).
//   k_mv_count    per-workgroup LDS histogram of bucket = slot >> MV_R_LOG,
//                 written bucket-major (hist[b * G + g]); an exclusive scan of it
//                 gives every workgroup its run inside every bucket (no atomics:
//                 a device-scope atomic on one address serialises memory-side);
//   k_mv_scatter  LDS ranks, then {slot, x, z, op index} into the bucket runs;
//   k_mv_apply    one workgroup per bucket (<= MV_R distinct slots: a bucket is
//                 big only through repeated slots): the last op of each slot by
//                 LDS atomicMax on the op index, then the winners apply -- their
//                 SlotInfo lines are one contiguous 64 KB range of the bucket.
// No global claim, no fixup.
constexpr uint32_t MV_R_LOG = 12, MV_R = 1u << MV_R_LOG;  // slots per bucket (LDS claim array: 16 KB)
constexpr int MV_T = 1024;                                 // threads per workgroup (all three kernels)

struct alignas(16) MvOp {
    uint32_t slot;
    float x, z;
    uint32_t j;  // op index in the flush
};

__device__ __forceinline__ uint32_t run_of(const MoveRuns &RS, uint32_t j) {
    uint32_t q = 0;
    while (q + 1 < RS.count && j >= RS.r[q + 1].j0) ++q;
    return q;
}

// Slot of op j (SLOT_NONE: no op; >= max_slots: flagged once, by k_mv_count).
__device__ __forceinline__ uint32_t mv_slot(const MoveRuns &RS, uint32_t j) {
    const MoveRun &R = RS.r[run_of(RS, j)];
    return R.ds[j - R.j0];
}

template <int PER>
__global__ __launch_bounds__(MV_T) void k_mv_count(MoveRuns RS, uint32_t n, uint32_t max_slots, uint32_t nb,
                                                  uint32_t *hist, TickScalars *sc) {
    extern __shared__ uint32_t mv_h[];  // nb
    for (uint32_t b = threadIdx.x; b < nb; b += MV_T) mv_h[b] = 0;
    __syncthreads();
    const uint32_t j0 = blockIdx.x * (uint32_t)(MV_T * PER);
    uint32_t s[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {  // every load first
        const uint32_t j = j0 + (uint32_t)k * MV_T + threadIdx.x;
        s[k] = j < n ? mv_slot(RS, j) : SLOT_NONE;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if (s[k] == SLOT_NONE) continue;  // past the ops, or the placeholder of a skipped decoded record
        if (s[k] >= max_slots) {
            atomicOr(&sc->err, ERR_BAD_SLOT);
            continue;
        }
        atomicAdd(&mv_h[s[k] >> MV_R_LOG], 1u);
    }
    __syncthreads();
    const uint32_t G = gridDim.x;
    for (uint32_t b = threadIdx.x; b < nb; b += MV_T) hist[(size_t)b * G + blockIdx.x] = mv_h[b];
    if (blockIdx.x == 0 && threadIdx.x == 0) hist[(size_t)nb * G] = 0;  // -> total after the scan
}

template <int PER>
__global__ __launch_bounds__(MV_T) void k_mv_scatter(MoveRuns RS, uint32_t n, uint32_t max_slots, uint32_t nb,
                                                    const uint32_t *__restrict__ hist, MvOp *binned) {
    extern __shared__ uint32_t mv_h[];  // nb: ranks, then this workgroup's base in each bucket
    for (uint32_t b = threadIdx.x; b < nb; b += MV_T) mv_h[b] = 0;
    __syncthreads();
    const uint32_t j0 = blockIdx.x * (uint32_t)(MV_T * PER);
    uint32_t bk[PER], rk[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const uint32_t j = j0 + (uint32_t)k * MV_T + threadIdx.x;
        bk[k] = 0xFFFFFFFFu;
        const uint32_t sl = j < n ? mv_slot(RS, j) : SLOT_NONE;
        if (sl < max_slots) {
            bk[k] = sl >> MV_R_LOG;
            rk[k] = atomicAdd(&mv_h[bk[k]], 1u);
        }
    }
    __syncthreads();
    const uint32_t G = gridDim.x;
    for (uint32_t b = threadIdx.x; b < nb; b += MV_T) mv_h[b] = hist[(size_t)b * G + blockIdx.x];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if (bk[k] == 0xFFFFFFFFu) continue;
        const uint32_t j = j0 + (uint32_t)k * MV_T + threadIdx.x;
        const MoveRun &R = RS.r[run_of(RS, j)];
        const uint32_t i = j - R.j0;
        MvOp o;
        o.slot = R.ds[i];
        o.x = R.dx[i];
        o.z = R.dz[i];
        o.j = j;
        binned[mv_h[bk[k]] + rk[k]] = o;
    }
}

// hist: the scanned histogram (bucket b starts at hist[b * G], the last one ends at hist[nb * G]).
__global__ __launch_bounds__(MV_T) void k_mv_apply(MoveRuns RS, const uint32_t *__restrict__ hist, uint32_t G,
                                                  const MvOp *__restrict__ binned, uint32_t n_total,
                                                  unsigned long long seq_floor, Rec16 *s_rec, SlotSp *s_ss,
                                                  SlotTab info, TickScalars *sc, int track_max) {
    __shared__ uint32_t claim[MV_R];
    const uint32_t b = blockIdx.x;
    for (uint32_t i = threadIdx.x; i < MV_R; i += MV_T) claim[i] = 0;
    const uint32_t s0 = hist[(size_t)b * G], s1 = hist[(size_t)(b + 1) * G];
    __syncthreads();
    for (uint32_t i = s0 + threadIdx.x; i < s1; i += MV_T) {
        const MvOp o = binned[i];
        atomicMax(&claim[o.slot & (MV_R - 1)], o.j + 1u);
    }
    __syncthreads();
    unsigned long long smax = 0;
    for (uint32_t i = s0 + threadIdx.x; i < s1; i += MV_T) {
        const MvOp m = binned[i];
        if (claim[m.slot & (MV_R - 1)] != m.j + 1u) continue;  // a later op of this slot wins
        const MoveRun &R = RS.r[run_of(RS, m.j)];
        const uint32_t k = m.j - R.j0;
        OpIn o;
        o.slot = m.slot;
        o.x = m.x;
        o.z = m.z;
        o.sp = R.dsp ? R.dsp[k] : R.sp_def;
        o.seq = R.dseq ? R.dseq[k] : R.seq0 + k;
        const unsigned long long q =
            op_apply_one(o, m.j, slot_info(info, m.slot), info, 0u, n_total, seq_floor, s_rec, s_ss, sc, false, &sc->err);
        smax = q > smax ? q : smax;
    }
    if (track_max) {  // one atomic per wave
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long v = __shfl_xor(smax, o, WAVE);
            smax = v > smax ? v : smax;
        }
        if (lane() == 0 && smax) atomicMax(&sc->seq_max, smax);
    }
}

// ----------------------------------------------------------- radix sort ------
// Tile = 4 waves x RS_I items x 64 lanes.  Element (wave w, item j, lane l)
// is index tile*RS_TILE + w*RS_WSEG + j*64 + l, so processing items in order
// per wave and waves in order keeps the sort stable.

constexpr int RS_T = 256;
constexpr int RS_I = 16;
constexpr int RS_TILE = RS_T * RS_I;
constexpr int RS_WAVES = RS_T / WAVE;
constexpr int RS_WSEG = WAVE * RS_I;
static_assert(RS_T == 256, "the downsweep gives one thread per digit (<= 8-bit digits)");

__global__ __launch_bounds__(RS_T) void k_rs_upsweep(const uint32_t *__restrict__ keys, uint32_t n, int shift,
                                                     int nbits, uint32_t *hist, uint32_t ntiles) {
    __shared__ uint32_t h[RS_WAVES][256];
    const int bins = 1 << nbits;
    const uint32_t mask = (uint32_t)bins - 1u;
    const int w = threadIdx.x / WAVE;
    for (int i = threadIdx.x; i < RS_WAVES * 256; i += RS_T) (&h[0][0])[i] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * RS_TILE;
#pragma unroll 4
    for (int i = 0; i < RS_I; ++i) {
        const size_t idx = base + (size_t)i * RS_T + threadIdx.x;
        const bool valid = idx < n;
        const uint32_t d = valid ? (keys[idx] >> shift) & mask : 0u;
        // wave-aggregated increment: one LDS add per distinct digit of the wave
        unsigned long long peers = __ballot(valid);
        for (int b = 0; b < nbits; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        if (valid && (int)lane() == __ffsll((long long)peers) - 1) h[w][d] += (uint32_t)__popcll(peers);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < bins; d += RS_T)
        hist[(size_t)d * ntiles + blockIdx.x] = h[0][d] + h[1][d] + h[2][d] + h[3][d];
}

// Stable scatter of one tile by digit.  Ranks come from wave multisplits
// (per-wave digit counts in LDS).  With 1 the tile is first
// regrouped by digit in LDS, so that consecutive threads write consecutive
// positions of a digit's run (coalesced stores) instead of scattering every key
// to its own line.
__global__ __launch_bounds__(RS_T) void k_rs_downsweep(const uint32_t *__restrict__ keys_in,
                                                       const uint32_t *__restrict__ vals_in, uint32_t *keys_out,
                                                       uint32_t *vals_out, uint32_t n, int shift, int nbits,
                                                       const uint32_t *__restrict__ hist_scanned, uint32_t ntiles) {
    __shared__ uint32_t wcnt[RS_WAVES][256];
    __shared__ uint32_t lkey[RS_TILE], lval[RS_TILE];
    __shared__ uint32_t dstart[256], dglob[256];
    __shared__ uint32_t s_ws[RS_WAVES];
    const int bins = 1 << nbits;
    const uint32_t mask = (uint32_t)bins - 1u;
    const int w = threadIdx.x / WAVE;
    const int l = lane();
    for (int i = threadIdx.x; i < RS_WAVES * 256; i += RS_T) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const size_t wbase = (size_t)blockIdx.x * RS_TILE + (size_t)w * RS_WSEG;
    const unsigned long long lt = lanemask_lt();
    uint32_t k[RS_I], v[RS_I], rk[RS_I];
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        const size_t idx = wbase + (size_t)j * WAVE + l;
        const bool valid = idx < n;
        k[j] = valid ? keys_in[idx] : 0u;
        v[j] = valid ? vals_in[idx] : 0u;
    }
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        const size_t idx = wbase + (size_t)j * WAVE + l;
        const bool valid = idx < n;
        const uint32_t d = (k[j] >> shift) & mask;
        unsigned long long peers = __ballot(valid);
        for (int b = 0; b < nbits; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const int leader = peers ? (__ffsll((long long)peers) - 1) : 0;
        uint32_t base = 0;
        if (valid && l == leader) {
            base = wcnt[w][d];
            wcnt[w][d] = base + (uint32_t)__popcll(peers);
        }
        base = __shfl(base, leader);
        rk[j] = base + (uint32_t)__popcll(peers & lt);
    }
    __syncthreads();
    // tile-local layout: digit d's run starts at dstart[d]; wave w's keys of digit d follow the
    // lower waves' (stability); the run goes to hist_scanned[d][tile] onwards
    {
        const int d = threadIdx.x;  // RS_T == 256 >= bins
        uint32_t c[RS_WAVES], tot = 0;
#pragma unroll
        for (int ww = 0; ww < RS_WAVES; ++ww) {
            c[ww] = d < bins ? wcnt[ww][d] : 0u;
            tot += c[ww];
        }
        uint32_t x = tot;  // block exclusive scan of the digit totals
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (l >= o) x += y;
        }
        if (l == WAVE - 1) s_ws[w] = x;
        __syncthreads();
        uint32_t pre = x - tot;
        for (int q = 0; q < w; ++q) pre += s_ws[q];
        if (d < bins) {
            dstart[d] = pre;
            dglob[d] = hist_scanned[(size_t)d * ntiles + blockIdx.x];
            uint32_t run = pre;
#pragma unroll
            for (int ww = 0; ww < RS_WAVES; ++ww) {
                wcnt[ww][d] = run;
                run += c[ww];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        const size_t idx = wbase + (size_t)j * WAVE + l;
        if (idx < n) {
            const uint32_t d = (k[j] >> shift) & mask;
            const uint32_t p = wcnt[w][d] + rk[j];
            lkey[p] = k[j];
            lval[p] = v[j];
        }
    }
    __syncthreads();
    const size_t t0 = (size_t)blockIdx.x * RS_TILE;
    const uint32_t tn = (uint32_t)min((size_t)RS_TILE, (size_t)n - t0);
    for (uint32_t t = threadIdx.x; t < tn; t += RS_T) {
        const uint32_t key = lkey[t], d = (key >> shift) & mask;
        const uint32_t pos = dglob[d] + (t - dstart[d]);
        keys_out[pos] = key;
        vals_out[pos] = lval[t];
    }
}

// ------------------------------------------------- incremental frame sort ------
// When the grid is unchanged the new frame is a merge: per cell, the
// entities that stayed (in previous-frame order, i.e. by S' index) and the
// few "arrivals" (moved in from another cell or new), interleaved by S'
// index -- exactly the stable sort of S' by the new keys, without sorting.
//   k_keygen<true>   counts per cell: entities (lo) and arrivals (hi)
//   scan64           exclusive scans -> the new cell_start and arrival offsets
//   k_arrive         arrivals into per-cell lists (atomic order, fixed later)
//   k_cell_merge     one lane per cell: sort its arrivals, merge with the stayers

// ------------------------------------------------------ block offsets ------
// The two scans across blocks (the sort's cell counts, k_finish's tile totals) take a
// block's offset from totals written by an earlier launch -- per scan tile (keygen's entries
// per tile) or per group of FG tile entries (the pair passes' atomics) -- summed by the whole block,
// with no chain between blocks.  Rounds 2-4 used a decoupled look-back instead: its chain
// cost 10 us in the cell scan and 3.5 us in k_finish per cfg3 tick (profiles/archive/r04_variants_scan.log).
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

// Sum of the values of blocks 0..b-1 over NW parallel status arrays
// lb[q * stride + block] (one scan per array; the arrays of one block are
// published together and read as a unit: a block counts as inclusive only
// when all its words are).  Called by all 256 threads of the block: thread t
// reads block j - t of a window, so a walk takes one window per 256 blocks
// (the predecessors' aggregates are published at once, so a window is ready
// after about one poll).  excl is valid in every thread.
__device__ __forceinline__ unsigned long long wave_incl_scan64(unsigned long long x) {
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const unsigned long long y = __shfl_up(x, o);
        if ((int)lane() >= o) x += y;
    }
    return x;
}

template <int NT>
__device__ __forceinline__ unsigned long long block_excl_scan64(unsigned long long v, unsigned long long *ws,
                                                                unsigned long long &total) {
    const unsigned long long x = wave_incl_scan64(v);
    const int w = threadIdx.x / WAVE;
    if (lane() == WAVE - 1) ws[w] = x;
    __syncthreads();
    unsigned long long pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / WAVE; ++i) {
        const unsigned long long t = ws[i];
        pre += (i < w) ? t : 0ull;
        tot += t;
    }
    total = tot;
    return pre + x - v;
}

// LDS tile index with one pad word per 16: a thread's 16 consecutive words
// (stride 17) and a wave's coalesced row (stride 1) are both conflict-free.
__device__ __forceinline__ uint32_t p64(uint32_t i) { return i + (i >> 4); }

// Exclusive scan of the packed (lo = arrivals, hi = departures) cell counts, one
// tile per block, the tile offsets from keygen's entries per tile.  Block 0 (the tiles are blocks 1..nb)
// folds keygen's d_rel / bmax partials.
__device__ __forceinline__ void keygen_fold256(const float *__restrict__ blk, uint32_t nb, TickScalars *sc) {
    keygen_fold_t<SC_T>(blk, nb, sc);
}

// The counts are not cleared here: k_arrive zeroes the two cells of every entity that changed
// cell (the only cells k_keygen<true> counted into), so the next flush's keygen finds them zero
// without a store per cell.  shift[c]: SHIFT_CHANGED for a cell with arrivals or departures, else
// how far its run moved (new start - previous start): k_arrive places such a cell's stayers itself.
constexpr uint32_t SHIFT_CHANGED = 0x80000000u;
__global__ __launch_bounds__(SC_T) void k_scan64(const unsigned long long *__restrict__ in, size_t n, uint32_t nb,
                                                    const unsigned long long *__restrict__ agg, uint32_t *lo, uint32_t *hi,
                                                    const float *__restrict__ blk, uint32_t nbk, TickScalars *sc,
                                                    const uint32_t *__restrict__ p_cs, uint32_t *shift,
                                                    uint32_t *list, unsigned long long *tcnt) {
    if (blockIdx.x == 0) {  // first, so that its serial loop overlaps the tiles
        keygen_fold256(blk, nbk, sc);
        return;
    }
    const uint32_t b = blockIdx.x - 1;
    __shared__ unsigned long long tile[S64_TILE + S64_TILE / 16];
    __shared__ unsigned long long ws[SC_T / WAVE];
    const size_t base = (size_t)b * S64_TILE;
    const uint32_t tid = threadIdx.x;
    // every global operand first, in one round trip: the tile's counts, the previous starts of its
    // cells (for the final write) and this thread's share of the earlier tiles' entries (keygen's
    // per-tile counts of the new keys: their sum is where this tile starts in the new frame)
    unsigned long long pre = 0;
    for (uint32_t q = tid; q < b; q += SC_T) pre += agg[q];
    const uint32_t p_cs0 = p_cs[base];  // where this tile started in the previous frame
    uint32_t pcs[S64_I];
#pragma unroll
    for (int q = 0; q < S64_I; ++q) {
        const uint32_t j = (uint32_t)q * SC_T + tid;
        tile[p64(j)] = base + j < n ? in[base + j] : 0ull;
        pcs[q] = base + j < n ? p_cs[base + j] : 0u;
    }
    __syncthreads();
    unsigned long long v[S64_I];
    unsigned long long s = 0;
#pragma unroll
    for (int q = 0; q < S64_I; ++q) {
        v[q] = tile[p64(tid * S64_I + (uint32_t)q)];
        s += v[q];
    }
    unsigned long long tot;
    unsigned long long run = block_excl_scan64<SC_T>(s, ws, tot);
    {  // the tile's changed cells (not the dead-entry cell n - 1), in cell order, for k_cell_merge
        __shared__ uint32_t ws32[SC_T / WAVE];
        uint32_t nch = 0, t32;
        const size_t c0 = base + (size_t)tid * S64_I;
#pragma unroll
        for (int q = 0; q < S64_I; ++q) nch += (v[q] && c0 + q + 1 < n) ? 1u : 0u;
        uint32_t off = block_excl_scan<SC_T>(nch, ws32, t32);
#pragma unroll
        for (int q = 0; q < S64_I; ++q)
            if (v[q] && c0 + q + 1 < n) list[base + off++] = (uint32_t)(c0 + q);
        if (tid == 0) tcnt[b] = t32;
    }
    // the tile's offset: the sum of the earlier tiles' entries, no look-back chain: a chain
    // serialises ~500 tiles at ~20 ns a hop, the block-wide sum of <= 1k words does not.  Its
    // first cell moves by dt = (new start) - (previous start) = the arrivals minus the departures
    // of every cell before the tile.
    __shared__ unsigned long long s_pre[SC_T / WAVE];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
    if (lane() == 0) s_pre[tid / WAVE] = pre;
    __syncthreads();
    unsigned long long e = 0;
#pragma unroll
    for (int q = 0; q < SC_T / WAVE; ++q) e += s_pre[q];
    const uint32_t dt = (uint32_t)e - p_cs0;
#pragma unroll
    for (int q = 0; q < S64_I; ++q) {  // a thread rewrites only the words it read; bit 31: c changed
        tile[p64(tid * S64_I + (uint32_t)q)] = run | (v[q] ? (unsigned long long)SHIFT_CHANGED : 0ull);
        run += v[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < S64_I; ++q) {
        const uint32_t j = (uint32_t)q * SC_T + tid;
        if (base + j < n) {
            const unsigned long long e = tile[p64(j)];
            // e = (departures before c in the tile) << 32 | (arrivals before c in the tile): cell c
            // starts at its previous start plus the arrivals minus the departures of the cells
            // before it.  Its arrivals are listed from its new start on (k_arrive): a cell has at
            // least as many new entries as arrivals, so the lists of two cells never overlap.
            const uint32_t arr = (uint32_t)e & ~SHIFT_CHANGED, d = dt + arr - (uint32_t)(e >> 32);
            lo[base + j] = pcs[q] + d;
            hi[base + j] = pcs[q] + d;
            shift[base + j] = ((uint32_t)e & SHIFT_CHANGED) ? SHIFT_CHANGED : d;
        }
    }
}

// Arrivals into per-cell lists.  arr_pos[c] starts as the exclusive offset
// of cell c and ends as that of cell c+1.  An entity that changed cell also
// zeroes the counts of both its cells (k_scan64 has read them).  A stayer
// of an unchanged cell (no arrival, no departure) keeps its rank in the run,
// so its frame position is its S' index plus the cell's shift.
__device__ __forceinline__ void arrive_one(const uint32_t i, const uint32_t *__restrict__ keys, uint32_t n, uint32_t n_prev,
                         const uint32_t *__restrict__ p_key, uint32_t sentinel, uint32_t *arr_pos, uint32_t *arr_idx,
                         unsigned long long *cnt64, const uint32_t *__restrict__ shift, uint32_t *perm,
                         uint32_t *skeys) {
    if (i >= n) return;
    const uint32_t key = keys[i];
    const uint32_t old = i < n_prev ? p_key[i] : sentinel;
    if (key == old) {
        if (key == sentinel) return;
        const uint32_t d = shift[key];
        if (d != SHIFT_CHANGED && i + d < n) {  // (the bound only guards against a broken scan)
            perm[i + d] = i;
            skeys[i + d] = key;
        }
        return;
    }
    if (old != sentinel) cnt64[old] = 0ull;
    if (key == sentinel) return;
    cnt64[key] = 0ull;
    const uint32_t pos = atomicAdd(&arr_pos[key], 1u);
    if (pos < n) arr_idx[pos] = i;
}

__global__ void k_arrive(const uint32_t *__restrict__ keys, uint32_t n, uint32_t n_prev,
                         const uint32_t *__restrict__ p_key, uint32_t sentinel, uint32_t *arr_pos, uint32_t *arr_idx,
                         unsigned long long *cnt64, const uint32_t *__restrict__ shift, uint32_t *perm,
                         uint32_t *skeys) {
    arrive_one(blockIdx.x * blockDim.x + threadIdx.x, keys, n, n_prev, p_key, sentinel, arr_pos, arr_idx, cnt64, shift, perm, skeys);
}

// One lane per changed cell c (k_scan64 lists them per scan tile; k_arrive placed the
// others' stayers): the stayers are the entries of c's previous run whose new key is
// still c (S' index order), the arrivals arr_idx[arr_pos[c-1], arr_pos[c])
// are sorted by S' index (insertion sort: a cell rarely gets more than a few)
// and placed around the stayers.  Writes the frame's permutation and keys.
__device__ __forceinline__ void cell_merge_one(uint32_t c, const uint32_t *__restrict__ p_cell_start,
                                               const uint32_t *__restrict__ cell_start,
                                               const uint32_t *__restrict__ keys, const uint32_t *__restrict__ arr_pos,
                                               uint32_t *arr_idx, uint32_t sentinel, uint32_t *perm, uint32_t *skeys,
                                               uint32_t n_total) {
    // the cell's five bounds in one round trip; its arrivals are listed from its new start on
    // (the clamps to n_total only guard the buffers against a broken scan)
    uint32_t o = min(cell_start[c], n_total);
    const uint32_t oe = min(cell_start[c + 1], n_total);
    const uint32_t ab = o, ae = min(arr_pos[c], n_total);
    const uint32_t ps = p_cell_start[c], pe = p_cell_start[c + 1];
    if (o == oe) return;
    for (uint32_t k = ab + 1; k < ae; ++k) {  // insertion sort of the arrivals
        const uint32_t v = arr_idx[k];
        uint32_t j = k;
        while (j > ab && arr_idx[j - 1] > v) {
            arr_idx[j] = arr_idx[j - 1];
            --j;
        }
        arr_idx[j] = v;
    }
    // An arrival is new to c, so its S' index lies outside c's previous run [ps, pe) (which
    // holds exactly the entries whose previous key is c): the cell's order is the arrivals
    // below ps, the stayers in run order, then the arrivals past pe -- no merge.
    uint32_t a = ab;
    for (; a < ae; ++a) {
        const uint32_t v = arr_idx[a];
        if (v >= ps || o >= oe) break;
        perm[o] = v;
        skeys[o] = c;
        ++o;
    }
    constexpr uint32_t MU = 4;  // run keys in flight per step; measured (cfg3 k_cell_merge): 1 -> 11.9 us, 4 -> 10.2, 8 -> 10.1; two-way merge 13.4
    for (uint32_t i = ps; i < pe; i += MU) {
        uint32_t k[MU];
#pragma unroll
        for (uint32_t u = 0; u < MU; ++u) k[u] = i + u < pe ? keys[i + u] : sentinel;
#pragma unroll
        for (uint32_t u = 0; u < MU; ++u)
            if (k[u] == c && o < oe) {
                perm[o] = i + u;
                skeys[o] = c;
                ++o;
            }
    }
    for (; a < ae && o < oe; ++a) {
        perm[o] = arr_idx[a];
        skeys[o] = c;
        ++o;
    }
}

struct MergeArgs {
    const uint32_t *p_cell_start, *cell_start, *keys, *arr_pos;
    uint32_t *arr_idx;
    uint32_t total_cells, n_total, sentinel;
    uint32_t *perm, *skeys;
    const uint32_t *list;
    const unsigned long long *tcnt;
    unsigned long long *tent;
};

// Block b of the merge: scan tile b's changed cells (k_scan64's list), every lane busy (one lane per
// cell of the whole grid, most of them idle: 10.2 against 7.6 us at cfg3).  Dead tail: the entries
// past the device's live count get sentinel keys and no source (so a host count that disagrees
// with the device's -- a device batch breaking its rules -- finds sentinels, not a previous
// flush's values, at [n_new, n_total)); returns that count.
__device__ __forceinline__ uint32_t merge_tile(const MergeArgs &M) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (threadIdx.x == 0) M.tent[blockIdx.x] = 0ull;  // keygen's per-tile entries, read by k_scan64: zero for the next flush
    const uint32_t n_live = M.cell_start[M.total_cells];
    for (uint32_t k = n_live + c; k < M.n_total; k += gridDim.x * blockDim.x) {
        M.skeys[k] = M.sentinel;
        M.perm[k] = 0xFFFFFFFFu;
    }
    const uint32_t nc = (uint32_t)M.tcnt[blockIdx.x];
    const uint32_t *L = M.list + (size_t)blockIdx.x * S64_TILE;
    for (uint32_t k = threadIdx.x; k < nc; k += blockDim.x)
        cell_merge_one(L[k], M.p_cell_start, M.cell_start, M.keys, M.arr_pos, M.arr_idx, M.sentinel, M.perm, M.skeys,
                       M.n_total);
    return n_live;
}

__global__ void k_cell_merge(MergeArgs M) { (void)merge_tile(M); }
// ----------------------------------------------------------------- bbox ------

__device__ __forceinline__ int f2o(float f) {
    int i = __float_as_int(f);
    return i ^ ((i >> 31) & 0x7FFFFFFF);
}

__device__ __forceinline__ void bbox_flush(int4 *bbox, uint32_t ns, uint32_t sp, const int (&v)[4]) {
    if (sp >= ns) return;
    int *p = reinterpret_cast<int *>(bbox + sp);
    atomicMin(p + 0, v[0]);
    atomicMin(p + 1, v[1]);
    atomicMax(p + 2, v[2]);
    atomicMax(p + 3, v[3]);
}

constexpr uint32_t BB_T = 256;

struct BBoxPart {  // one workgroup's fold: space id (SP_DEAD = nothing left) + ordered-int bbox
    uint32_t sp;
    int v[4];
};

// Fold per-thread (space, bbox) over a workgroup: when every thread ends on
// the same space the block reduces to one part; otherwise each thread flushes
// its own run with atomics (only at space boundaries).
__device__ __forceinline__ void bbox_block(uint32_t cur, const int (&own)[4], int4 *bbox, uint32_t ns,
                                           BBoxPart *out) {
    __shared__ uint32_t s_sp[BB_T / WAVE];
    __shared__ int s_v[BB_T / WAVE][4];
    __shared__ int s_uni;
    const uint32_t first = __shfl(cur, 0);
    const bool wuni = __all(cur == first || cur == SP_DEAD);
    int v[4] = {own[0], own[1], own[2], own[3]};
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        v[0] = min(v[0], __shfl_xor(v[0], o));
        v[1] = min(v[1], __shfl_xor(v[1], o));
        v[2] = max(v[2], __shfl_xor(v[2], o));
        v[3] = max(v[3], __shfl_xor(v[3], o));
    }
    const int w = threadIdx.x / WAVE;
    if (threadIdx.x == 0) s_uni = 1;
    __syncthreads();
    if (lane() == 0) {
        s_sp[w] = wuni ? first : SP_KEEP;
        s_v[w][0] = v[0];
        s_v[w][1] = v[1];
        s_v[w][2] = v[2];
        s_v[w][3] = v[3];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t bsp = SP_DEAD;
        int r[4] = {INT_MAX, INT_MAX, INT_MIN, INT_MIN};
        for (int q = 0; q < (int)(BB_T / WAVE); ++q) {
            const uint32_t ws = s_sp[q];
            if (ws == SP_DEAD) continue;
            if (ws == SP_KEEP || (bsp != SP_DEAD && ws != bsp)) {
                s_uni = 0;
                break;
            }
            bsp = ws;
            r[0] = min(r[0], s_v[q][0]);
            r[1] = min(r[1], s_v[q][1]);
            r[2] = max(r[2], s_v[q][2]);
            r[3] = max(r[3], s_v[q][3]);
        }
        out->sp = s_uni ? bsp : SP_DEAD;
        out->v[0] = r[0];
        out->v[1] = r[1];
        out->v[2] = r[2];
        out->v[3] = r[3];
    }
    __syncthreads();
    if (!s_uni && cur != SP_DEAD) bbox_flush(bbox, ns, cur, own);  // mixed spaces: every run flushes
}


// --------------------------------------------------------------- gather ------

__device__ __forceinline__ void gather_one(uint32_t k, const uint32_t *__restrict__ perm, uint32_t n_prev, uint32_t n_new,
                                           const Rec16 *__restrict__ s_rec, const SlotSp *__restrict__ s_ss,
                                           const Rec16 *__restrict__ p_rec, const SlotSp *__restrict__ p_ss,
                                           Rec16 *f_rec, SlotSp *f_ss, Rec16 *o_rec, uint4 *cand,
                                           const SpaceGrid *__restrict__ grid, unsigned long long seq_base,
                                           SlotTab info, const uint32_t *__restrict__ sorted_keys, uint32_t sentinel,
                                           uint32_t n_total, TickScalars *sc, uint32_t *f_key, uint32_t &cur,
                                           int (&bv)[4]);

// Fewer live entries than the host counted (a device Enter / Leave batch broke its rules, or a
// broken permutation): the flush fails and poisons the world, but it must not fault first.  The
// entry becomes an inert placeholder: slot 0 of space 0 at NaN (no relation, no slot-indexed
// write, no bbox).
__device__ __forceinline__ void gather_placeholder(uint32_t k, Rec16 *f_rec, SlotSp *f_ss, Rec16 *o_rec, uint4 *cand,
                                                   TickScalars *sc) {
    atomicOr(&sc->err, ERR_COUNT_MISMATCH);
    Rec16 z;
    z.x = z.z = qnan();
    z.s = 0;
    st_rec(f_rec, k, z);
    st_rec(o_rec, k, z);
    reinterpret_cast<uint2 *>(f_ss)[k] = make_uint2(0u, 0u);
    cand[k] = make_uint4(0x7FC00000u, 0x7FC00000u, 0x7FC00000u, 0x7FC00000u);
}

// Per-cell x bounds of the new frame (k_combined trims the X' rows' end cells by them).  The
// frame is sorted by cell, so a cell's entries are one run: a segmented fold inside the wave,
// then the run's first lane writes.  A run that crosses a wave boundary gets (-inf, +inf) from the
// wave holding its first entry (no trim); an empty cell keeps a stale pair, which trims nothing.

// One thread per new-frame entry; the block also folds its entries' bbox
// (level 1 of the per-space bounding box, k_finish folds level 2).
__global__ __launch_bounds__(256) void k_gather(const uint32_t *__restrict__ perm, uint32_t n_new, uint32_t n_prev,
                         const Rec16 *__restrict__ s_rec, const SlotSp *__restrict__ s_ss,
                         const Rec16 *__restrict__ p_rec, const SlotSp *__restrict__ p_ss, Rec16 *f_rec,
                         SlotSp *f_ss, Rec16 *o_rec, uint4 *cand, const SpaceGrid *__restrict__ grid,
                         unsigned long long seq_base, SlotTab info, const uint32_t *__restrict__ sorted_keys,
                         uint32_t sentinel, uint32_t n_total, TickScalars *sc, uint32_t *f_key, int4 *bbox,
                         uint32_t n_spaces, BBoxPart *parts) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0 && n_new < n_total && sorted_keys[n_new] != sentinel) atomicOr(&sc->err, ERR_COUNT_MISMATCH);
    uint32_t cur = SP_DEAD;
    int bv[4] = {INT_MAX, INT_MAX, INT_MIN, INT_MIN};
    if (k < n_new) gather_one(k, perm, n_prev, n_new, s_rec, s_ss, p_rec, p_ss, f_rec, f_ss, o_rec, cand, grid, seq_base,
                              info, sorted_keys, sentinel, n_total, sc, f_key, cur, bv);
    bbox_block(cur, bv, bbox, n_spaces, &parts[blockIdx.x]);
}

__device__ __forceinline__ void gather_one(uint32_t k, const uint32_t *__restrict__ perm, uint32_t n_prev, uint32_t n_new,
                                           const Rec16 *__restrict__ s_rec, const SlotSp *__restrict__ s_ss,
                                           const Rec16 *__restrict__ p_rec, const SlotSp *__restrict__ p_ss,
                                           Rec16 *f_rec, SlotSp *f_ss, Rec16 *o_rec, uint4 *cand,
                                           const SpaceGrid *__restrict__ grid, unsigned long long seq_base,
                                           SlotTab info, const uint32_t *__restrict__ sorted_keys, uint32_t sentinel,
                                           uint32_t n_total, TickScalars *sc, uint32_t *f_key, uint32_t &cur,
                                           int (&bv)[4]) {
    const uint32_t key = sorted_keys[k];
    if (f_key) f_key[k] = key;  // (nullptr: the sort wrote the frame's keys in place)
    const uint32_t i = perm[k];
    if (key >= sentinel || i >= n_total) {
        gather_placeholder(k, f_rec, f_ss, o_rec, cand, sc);
        return;
    }
    // S' and previous-frame operands of entry i in one round trip (the previous record is loaded
    // before its space is compared, not after)
    const SlotSp ss = ld_ss(s_ss, i);
    const Rec16 now = ld_rec(s_rec, i);
    const bool inp = i < n_prev;
    const uint32_t psp = inp ? ld_ss(p_ss, i).sp : SP_DEAD;
    Rec16 pr;
    pr.x = pr.z = 0.0f;
    pr.s = 0;
    if (inp) pr = ld_rec(p_rec, i);
    st_rec(f_rec, k, now);
    reinterpret_cast<uint2 *>(f_ss)[k] = make_uint2(ss.slot, ss.sp);
    info.rank[ss.slot] = k;
    // the space only when it changed: a slot's sp word holds its space from its Enter or last
    // space change on (and SP_DEAD from its Leave), so an entity in the same space as in the
    // previous frame has it already (a second random store per entity cost the gather 10 us)
    if (!inp || psp != ss.sp) info.sp[ss.slot] = ss.sp;
    // previous state of the same entity, NaN position unless live in the same space then
    Rec16 o;
    o.x = o.z = qnan();
    o.s = 0;
    if (inp && psp == ss.sp) o = pr;
    st_rec(o_rec, k, o);
    const float thr = FAR_FRAC * grid[ss.sp].D;
    const uint4 c = cand_of(now, o, thr);
    (void)n_new;
    cand[k] = c;
    cur = ss.sp;
    bv[0] = bv[2] = f2o(now.x);
    bv[1] = bv[3] = f2o(now.z);
}

// The incremental sort's merge and the gather in one launch (GatherJob): block b merges scan tile
// b's changed cells, then gathers the tile's range of the new frame, [cell_start[b S64_TILE],
// cell_start[(b + 1) S64_TILE]): k_arrive placed the stayers of its unchanged cells and the block
// itself its changed cells, so the permutation it reads is complete with no grid-wide barrier
// (and the launch boundary between the two passes, with the tail of each, is gone).  GU entries
// per thread in flight (every load of the group before its stores); the block folds its entries'
// bbox into part b (a thread's entries are in key order, so its runs of one space are too).
#ifndef GWAOI_MG_GU
#define GWAOI_MG_GU 4
#endif
constexpr int GU = GWAOI_MG_GU;  // entries per thread in flight (k_merge_gather)
__global__ __launch_bounds__(256) void k_merge_gather(MergeArgs M, GatherJob G) {
    const uint32_t n_live = merge_tile(M);
    __syncthreads();  // the block's merged cells before their gather
    const uint32_t b = blockIdx.x, tc = M.total_cells, n_new = G.n_new, sentinel = M.sentinel;
    if (b == 0 && threadIdx.x == 0 && n_live != n_new) atomicOr(&G.sc->err, ERR_COUNT_MISMATCH);
    // entries the host counted but the device did not (placed in no tile's range): placeholders
    for (uint32_t k = n_live + b * blockDim.x + threadIdx.x; k < n_new; k += gridDim.x * blockDim.x)
        gather_placeholder(k, G.f_rec, G.f_ss, G.o_rec, G.cand, G.sc);
    const uint32_t lo = min(M.cell_start[min(b * S64_TILE, tc)], n_new);
    const uint32_t hi = min(M.cell_start[min((b + 1) * S64_TILE, tc)], n_new);
    uint32_t cur = SP_DEAD;
    int bv[4] = {INT_MAX, INT_MAX, INT_MIN, INT_MIN};
    for (uint32_t k0 = lo + threadIdx.x; k0 < hi; k0 += GU * 256) {
        uint32_t key[GU], idx[GU];
        // every load of the group in flight: indices clamped to a valid entry, not branched on (a
        // load under a branch is waited for before the next); the values of the clamped ones unused
#pragma unroll
        for (int u = 0; u < GU; ++u) {
            const uint32_t k = min(k0 + u * 256, hi - 1);
            key[u] = M.skeys[k];
            idx[u] = M.perm[k];
        }
        SlotSp ss[GU];
        Rec16 now[GU], pr[GU];
        uint32_t psp[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) {
            const uint32_t i = idx[u];
            const bool ok = key[u] < sentinel && i < M.n_total, inp = ok && i < G.n_prev;
            const uint32_t ic = ok ? i : 0u, ip = inp ? i : 0u;  // (S' and the previous frame hold >= 1 entry)
            ss[u] = ld_ss(G.s_ss, ic);
            now[u] = ld_rec(G.s_rec, ic);
            psp[u] = ld_ss(G.p_ss, ip).sp;
            pr[u] = ld_rec(G.p_rec, ip);  // (psp / pr are read only for an entry in the previous frame)
        }
#pragma unroll
        for (int u = 0; u < GU; ++u) {
            const uint32_t k = k0 + u * 256, i = idx[u];
            if (k >= hi) continue;
            if (key[u] >= sentinel || i >= M.n_total) {
                gather_placeholder(k, G.f_rec, G.f_ss, G.o_rec, G.cand, G.sc);
                continue;
            }
            const bool inp = i < G.n_prev;
            st_rec(G.f_rec, k, now[u]);
            reinterpret_cast<uint2 *>(G.f_ss)[k] = make_uint2(ss[u].slot, ss[u].sp);
            G.info.rank[ss[u].slot] = k;
            if (!inp || psp[u] != ss[u].sp) G.info.sp[ss[u].slot] = ss[u].sp;  // (as gather_one)
            Rec16 o;
            o.x = o.z = qnan();
            o.s = 0;
            if (inp && psp[u] == ss[u].sp) o = pr[u];
            st_rec(G.o_rec, k, o);
            G.cand[k] = cand_of(now[u], o, FAR_FRAC * G.grid[ss[u].sp].D);
            if (ss[u].sp != cur) {
                if (cur != SP_DEAD) bbox_flush(G.bbox, G.n_spaces, cur, bv);
                cur = ss[u].sp;
                bv[0] = bv[1] = INT_MAX;
                bv[2] = bv[3] = INT_MIN;
            }
            const int fx = f2o(now[u].x), fz = f2o(now[u].z);
            bv[0] = min(bv[0], fx);
            bv[1] = min(bv[1], fz);
            bv[2] = max(bv[2], fx);
            bv[3] = max(bv[3], fz);
        }
    }
    bbox_block(cur, bv, G.bbox, G.n_spaces, reinterpret_cast<BBoxPart *>(G.parts) + b);
}

// Entities per cell from the sorted keys: one atomic per run of equal keys
// per wave.
__global__ void k_cell_count(const uint32_t *__restrict__ keys, uint32_t n, uint32_t *cnt) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = k < n;
    const uint32_t key = valid ? keys[k] : 0u;
    const uint32_t l = lane();
    const bool head = valid && (l == 0 || keys[k - 1] != key);
    const unsigned long long heads = __ballot(head);
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
    if (head) {
        const unsigned long long above = heads & ~((2ull << l) - 1ull);
        const uint32_t next = above ? (uint32_t)(__ffsll((long long)above) - 1) : 64u;
        const uint32_t end = next < nvalid ? next : nvalid;
        atomicAdd(&cnt[key], end - l);
    }
}

// ---------------------------------------------------------------- pairs ------
// A flush's events are the diff of the go-aoi relation N between the
// previous state (t-1) and the new state (t):
//   enter(A,B) = N_t(A,B) && !N_t-1(A,B),   leave(A,B) = N_t-1(A,B) && !N_t(A,B)
// N is symmetric in the pair, so each unordered pair is evaluated once and
// emitted in both directions.
//
// MODE 2 (combined), over the NEW grid.  The member with the lower frame
//   index enumerates (its own cell row from a+1, then the rows above) and
//   keeps the pairs inside the symmetric box |dx|,|dz| <= H + M with
//   H = D(1 + 2 d_rel) and M = (bmax + 3D) 2^-20 (float32 rounding of the
//   window bounds and of the differences).  Every pair with N_t is inside;
//   so is every pair with N_t-1 whose members both moved at most d_rel*D
//   ("near").  Entities not live in this space at t-1 carry NaN old
//   coordinates, which makes N_t-1 false.
// MODE 1 (special), over the PREVIOUS grid, for entities that left, changed
//   space or moved more than D/4: emits the leaves of pairs that the
//   combined pass could not see (box test false at t).  A pair of two
//   specials is emitted by the one with the lower previous-frame index.

constexpr int PT = (int)TILE_A;  // threads per workgroup = entities per tile
constexpr int PCAP = 512;        // candidates staged in LDS per chunk
constexpr int PS = 4;            // events buffered in LDS per thread
constexpr int PMAXR = 32;        // candidate rows a tile may span (else global path)
constexpr uint32_t KIND_LEAVE = 0x80000000u;

struct PairCtx {
    Rec16 now, oth;  // MODE 2: t, t-1 (NaN if absent);  MODE 1: t-1, t (NaN if absent)
    uint32_t a;      // frame index
    float D, HM;     // AOI distance, H + M (combined box half-width)
    unsigned long long seq_base;
    bool chg;
};

// 0: no event, 1: enter, 2: leave.  Branch-free.
template <int MODE>
__device__ __forceinline__ int pair_kind(const PairCtx &A, const Rec16 &bn, const Rec16 &bo, uint32_t b,
                                         float thr) {
    if (MODE == 2) {
        const bool inb = (int)(fabsf(bn.x - A.now.x) <= A.HM) & (int)(fabsf(bn.z - A.now.z) <= A.HM);
        const bool chg = A.chg | (bn.s >= A.seq_base);
        const bool nt = rel(A.now.x, A.now.z, A.now.s, bn.x, bn.z, bn.s, A.D);
        const bool no = rel(A.oth.x, A.oth.z, A.oth.s, bo.x, bo.z, bo.s, A.D);
        const int k = (int)nt + 2 * (int)no;  // 1: nt only (enter), 2: no only (leave)
        return (inb & chg & (nt != no)) ? k : 0;
    } else {
        const bool was = rel(A.now.x, A.now.z, A.now.s, bn.x, bn.z, bn.s, A.D);
        const bool is = rel(A.oth.x, A.oth.z, A.oth.s, bo.x, bo.z, bo.s, A.D);
        const bool seen = (int)(fabsf(bo.x - A.oth.x) <= A.HM) & (int)(fabsf(bo.z - A.oth.z) <= A.HM);
        const bool b_special = !is_near(bo.x, bo.z, bn.x, bn.z, thr);
        const bool mine = !(b_special && b < A.a);
        return (was & !is & !seen & mine) ? 2 : 0;
    }
}

// other-time record of frame entry j (MODE 1 derives validity from O_ss)
template <int MODE>
__device__ __forceinline__ Rec16 other_rec(const FrameView &F, const Rec16 *O_rec, const SlotSp *O_ss, uint32_t j) {
    Rec16 o = ld_rec(O_rec, j);
    if (MODE == 1 && ld_ss(O_ss, j).sp != ld_ss(F.ss, j).sp) o.x = o.z = qnan();
    return o;
}

// Row-major enumeration of A's partners straight from HBM/L2 (fallback and
// overflow path; same order and predicate as the LDS path).  Counts events
// per kind; when WRITE, writes (A,B),(B,A) for events number >= skip.
template <int MODE, bool WRITE>
__device__ void enum_global(const FrameView &F, const Rec16 *O_rec, const SlotSp *O_ss, const SpaceGrid &g,
                            const PairCtx &A, float thr, int cx0, int cx1, int cz0, int cz1, uint32_t skip, uint2 *out,
                            unsigned long long pe, unsigned long long pl, uint64_t cap, uint32_t &ne, uint32_t &nl) {
    const uint32_t slot_a = WRITE ? ld_ss(F.ss, A.a).slot : 0u;
    uint32_t k = 0;
    for (int cz = cz0; cz <= cz1; ++cz) {
        const uint32_t row = g.base + (uint32_t)cz * g.gx;
        uint32_t jb = F.cell_start[row + (uint32_t)cx0];
        const uint32_t je = F.cell_start[row + (uint32_t)cx1 + 1u];
        if (MODE == 2 && cz == cz0) jb = A.a + 1;
        for (uint32_t b = jb; b < je; ++b) {
            if (MODE == 1 && b == A.a) continue;
            const Rec16 bn = ld_rec(F.rec, b);
            const Rec16 bo = other_rec<MODE>(F, O_rec, O_ss, b);
            const int kind = pair_kind<MODE>(A, bn, bo, b, thr);
            if (!kind) continue;
            if (WRITE && k >= skip) {
                const uint32_t slot_b = ld_ss(F.ss, b).slot;
                ev_put2(out, cap, kind == 1 ? pe + 2ull * ne : pl + 2ull * nl, slot_a, slot_b);
            }
            if (!WRITE || k >= skip) {
                ne += (uint32_t)(kind == 1);
                nl += (uint32_t)(kind == 2);
            }
            ++k;
        }
    }
}

template <int MODE>
__device__ __forceinline__ void pairs_tile(const uint32_t t, FrameView F, const Rec16 *__restrict__ O_rec,
                           const SlotSp *__restrict__ O_ss, unsigned long long seq_base, const TickScalars *__restrict__ sc,
                           TickScalars *scw, uint2 *tmp, uint64_t cap,
                           uint32_t *tile_total, unsigned long long *tile_base, uint32_t tile_off,
                           uint32_t leave_off, uint32_t *dbg) {
    __shared__ uint4 s_now[PCAP];
    __shared__ uint4 s_oth[PCAP];
    __shared__ uint32_t s_slot[PCAP];
    __shared__ uint32_t s_ev[PS * PT];
    __shared__ int s_box[4];
    __shared__ uint32_t s_seg[PMAXR];
    __shared__ uint32_t s_pre[PMAXR + 1];
    __shared__ uint32_t s_ws[PT / WAVE];
    __shared__ unsigned long long s_base;

    __shared__ uint32_t s_spr[2];  // smallest / largest space among the active lanes
    __shared__ uint32_t s_nglob;   // lanes taking the global write path (DBG_SPECIAL_GLOBAL)
    // tile t: entries [t*PT, t*PT + PT) of the frame
    const uint32_t tid = threadIdx.x;
    PairCtx A;
    A.seq_base = seq_base;
    A.a = t * PT + tid;
    bool active = A.a < F.n;
    const uint32_t my_sp = active ? ld_ss(F.ss, A.a).sp : SP_DEAD;
    SpaceGrid g{};
    float M = 0.0f, thr = 0.0f;
    int cx0 = 0, cx1 = -1, cz0 = 0, cz1 = -1;
    if (active) {
        g = F.grid[my_sp];
        M = (sc->bmax + 3.0f * g.D) * 0x1p-20f;
        thr = FAR_FRAC * g.D;
        A.D = g.D;
        A.HM = g.D * (1.0f + 2.0f * sc->d_rel) + M;
        A.now = ld_rec(F.rec, A.a);
        A.oth = other_rec<MODE>(F, O_rec, O_ss, A.a);
        if (MODE == 2) {
            A.chg = A.now.s >= seq_base;
            const float r = A.HM + M;
            cx0 = cell_of(A.now.x - r, g.ox, g.inv, g.gx);
            cx1 = cell_of(A.now.x + r, g.ox, g.inv, g.gx);
            cz0 = cell_of(A.now.z, g.oz, g.inv, g.gz);  // own row (the tile's row)
            cz1 = cell_of(A.now.z + r, g.oz, g.inv, g.gz);
        } else {
            A.chg = true;
            active = !is_near(A.oth.x, A.oth.z, A.now.x, A.now.z, thr);
            // every partner with N_t-1: |dx| <= D + (|x| + 2D) 2^-24
            const float mx = (fabsf(A.now.x) + 3.0f * A.D) * 0x1p-20f;
            const float mz = (fabsf(A.now.z) + 3.0f * A.D) * 0x1p-20f;
            cx0 = cell_of(A.now.x - A.D - mx, g.ox, g.inv, g.gx);
            cx1 = cell_of(A.now.x + A.D + mx, g.ox, g.inv, g.gx);
            cz0 = cell_of(A.now.z - A.D - mz, g.oz, g.inv, g.gz);
            cz1 = cell_of(A.now.z + A.D + mz, g.oz, g.inv, g.gz);
        }
    }
    if (MODE == 1 && !__syncthreads_or(active)) return;  // no special entity: totals stay 0
    if (tid == 0) {
        s_spr[0] = 0xFFFFFFFFu;
        s_spr[1] = 0u;
        s_nglob = 0u;
    }
    __syncthreads();
    if (active) {
        atomicMin(&s_spr[0], my_sp);
        atomicMax(&s_spr[1], my_sp);
    }
    // tile box = union of the active entities' query cells
    {
        int v0 = active ? cx0 : INT_MAX, v1 = active ? cx1 : INT_MIN;
        int v2 = active ? cz0 : INT_MAX, v3 = active ? cz1 : INT_MIN;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            v0 = min(v0, __shfl_xor(v0, o));
            v1 = max(v1, __shfl_xor(v1, o));
            v2 = min(v2, __shfl_xor(v2, o));
            v3 = max(v3, __shfl_xor(v3, o));
        }
        if (tid == 0) {
            s_box[0] = INT_MAX;
            s_box[1] = INT_MIN;
            s_box[2] = INT_MAX;
            s_box[3] = INT_MIN;
        }
        __syncthreads();
        if (lane() == 0) {
            atomicMin(&s_box[0], v0);
            atomicMax(&s_box[1], v1);
            atomicMin(&s_box[2], v2);
            atomicMax(&s_box[3], v3);
        }
        __syncthreads();
    }
    const int CX0 = s_box[0], CX1 = s_box[1], CZ0 = s_box[2], CZ1 = s_box[3];
    const int nrows = CZ1 - CZ0 + 1;
    // the LDS path indexes the rows of one grid: all active lanes in one space
    const bool one_space = s_spr[0] == s_spr[1];
    const SpaceGrid gb = F.grid[one_space ? s_spr[0] : 0u];
    const bool staged = one_space && nrows <= PMAXR;
    uint32_t ne = 0, nl = 0, nk = 0;  // enters, leaves, buffered
    if (staged) {
        if ((int)tid < nrows) {
            const uint32_t row = gb.base + (uint32_t)(CZ0 + (int)tid) * gb.gx;
            const uint32_t b = F.cell_start[row + (uint32_t)CX0];
            s_seg[tid] = b;
            s_pre[tid + 1] = F.cell_start[row + (uint32_t)CX1 + 1u] - b;
        }
        __syncthreads();
        if (tid == 0) {
            s_pre[0] = 0;
            for (int r = 0; r < nrows; ++r) s_pre[r + 1] += s_pre[r];
        }
        __syncthreads();
        const uint32_t L = s_pre[nrows];
        for (uint32_t base = 0; base < L; base += PCAP) {
            const uint32_t lim = min(L - base, (uint32_t)PCAP);
            int r = 0;
            for (uint32_t i = tid; i < lim; i += PT) {  // stage candidates [base, base+lim)
                const uint32_t v = base + i;
                while (v >= s_pre[r + 1]) ++r;
                const uint32_t j = s_seg[r] + (v - s_pre[r]);
                s_now[i] = reinterpret_cast<const uint4 *>(F.rec)[j];
                const Rec16 o = other_rec<MODE>(F, O_rec, O_ss, j);
                s_oth[i] = make_uint4(__float_as_uint(o.x), __float_as_uint(o.z), (uint32_t)o.s,
                                      (uint32_t)(o.s >> 32));
                s_slot[i] = ld_ss(F.ss, j).slot;
            }
            __syncthreads();
            if (active) {
                for (int cz = cz0; cz <= cz1; ++cz) {
                    const int rr = cz - CZ0;
                    const uint32_t row = g.base + (uint32_t)cz * g.gx;
                    uint32_t jb = F.cell_start[row + (uint32_t)cx0];
                    const uint32_t je = F.cell_start[row + (uint32_t)cx1 + 1u];
                    if (MODE == 2 && cz == cz0) jb = A.a + 1;
                    if (jb >= je) continue;
                    const uint32_t vb = s_pre[rr] + (jb - s_seg[rr]);
                    const uint32_t lo = max(vb, base), hi = min(vb + (je - jb), base + lim);
                    for (uint32_t v = lo; v < hi; ++v) {
                        const uint32_t i = v - base;
                        const uint32_t b = jb + (v - vb);
                        const uint4 qn = s_now[i], qo = s_oth[i];
                        Rec16 bn, bo;
                        bn.x = __uint_as_float(qn.x);
                        bn.z = __uint_as_float(qn.y);
                        bn.s = ((unsigned long long)qn.w << 32) | qn.z;
                        bo.x = __uint_as_float(qo.x);
                        bo.z = __uint_as_float(qo.y);
                        bo.s = ((unsigned long long)qo.w << 32) | qo.z;
                        int kind = pair_kind<MODE>(A, bn, bo, b, thr);
                        if (MODE == 1 && b == A.a) kind = 0;
                        if (kind) {
                            if (nk < PS) s_ev[nk * PT + tid] = s_slot[i] | (kind == 2 ? KIND_LEAVE : 0u);
                            ++nk;
                            ne += (uint32_t)(kind == 1);
                            nl += (uint32_t)(kind == 2);
                        }
                    }
                }
            }
            __syncthreads();
        }
    } else if (active) {
        enum_global<MODE, false>(F, O_rec, O_ss, g, A, thr, cx0, cx1, cz0, cz1, 0, nullptr, 0, 0, 0, ne, nl);
    }
    // offsets: directed pairs = 2 per event, the tile's enters then its leaves
    uint32_t te, tl;
    const uint32_t oe = block_excl_scan<PT>(2 * ne, s_ws, te);
    __syncthreads();
    const uint32_t ol = block_excl_scan<PT>(2 * nl, s_ws, tl);
    if (tid == 0) {
        const uint32_t tot = te + tl, q = xcc_id();
        const unsigned long long b = tot ? ev_alloc(scw, q, tot) : ev_enc(q, 0ull);
        s_base = b;
        put_tile_total(tile_total, leave_off, tile_off + t, te);
        tile_base[tile_off + t] = b;
        put_tile_total(tile_total, leave_off, leave_off + tile_off + t, tl);
        tile_base[leave_off + tile_off + t] = b + te;
    }
    __syncthreads();
    if (active && (ne | nl)) {
        const unsigned long long pe = s_base + oe, pl = s_base + te + ol;
        if (staged) {
            const uint32_t slot_a = ld_ss(F.ss, A.a).slot;
            const uint32_t k = min(nk, (uint32_t)PS);
            uint32_t ie = 0, il = 0;
            for (uint32_t q = 0; q < k; ++q) {
                const uint32_t e = s_ev[q * PT + tid];
                const uint32_t slot_b = e & ~KIND_LEAVE;
                const bool lv = (e & KIND_LEAVE) != 0u;
                const unsigned long long p = lv ? pl + 2ull * il : pe + 2ull * ie;
                il += (uint32_t)lv;
                ie += (uint32_t)!lv;
                ev_put2(tmp, cap, p, slot_a, slot_b);
            }
            if (nk > PS) {
                atomicAdd(&s_nglob, 1u);
                uint32_t we = 0, wl = 0;  // continue after the buffered events, in order
                enum_global<MODE, true>(F, O_rec, O_ss, g, A, thr, cx0, cx1, cz0, cz1, PS, tmp, pe + 2ull * ie,
                                        pl + 2ull * il, cap, we, wl);
            }
        } else {
            uint32_t we = 0, wl = 0;
            enum_global<MODE, true>(F, O_rec, O_ss, g, A, thr, cx0, cx1, cz0, cz1, 0, tmp, pe, pl, cap, we, wl);
        }
    }
    __syncthreads();
    if (tid == 0 && s_nglob) atomicAdd(dbg + DBG_SPECIAL_GLOBAL, s_nglob);
}

template <int MODE>
__global__ __launch_bounds__(PT) void k_pairs(FrameView F, const Rec16 *__restrict__ O_rec,
                                              const SlotSp *__restrict__ O_ss, unsigned long long seq_base, const TickScalars *__restrict__ sc,
                                              TickScalars *scw, uint2 *tmp, uint64_t cap,
                                              uint32_t *tile_total, unsigned long long *tile_base, uint32_t tile_off,
                                              uint32_t leave_off, uint32_t *dbg, const uint32_t *__restrict__ special) {
    if (MODE == 1 && special && !special[blockIdx.x]) return;  // keygen saw no special entity in this tile
    pairs_tile<MODE>(blockIdx.x, F, O_rec, O_ss, seq_base, sc, scw, tmp, cap, tile_total, tile_base, tile_off,
                     leave_off, dbg);
}

// k_arrive with the special pass behind it (the steady incremental flush): the first cdiv(n, PT)
// workgroups run k_arrive, workgroup na + t is the special pass's tile t (it leaves at once unless
// keygen flagged the tile).  The special pass needs only keygen and its fold (k_scan64), so it
// rides on this launch instead of one of its own: a launch costs ~4.5 us on this chip however
// little it does, and a steady config-3 flush flags no tile.  Same tiles, same events, same
// per-tile totals as k_pairs<1>; an overflow re-run still launches k_pairs<1>.
__global__ __launch_bounds__(PT) void k_arrive_special(SpecialJob J, const uint32_t *__restrict__ keys, uint32_t n,
                                                       uint32_t n_prev, const uint32_t *__restrict__ p_key,
                                                       uint32_t sentinel, uint32_t *arr_pos, uint32_t *arr_idx,
                                                       unsigned long long *cnt64, const uint32_t *__restrict__ shift,
                                                       uint32_t *perm, uint32_t *skeys) {
    const uint32_t na = (n + PT - 1) / PT;  // the arrival workgroups first, the special pass's after them
    if (blockIdx.x < na) {
        arrive_one(blockIdx.x * PT + threadIdx.x, keys, n, n_prev, p_key, sentinel, arr_pos, arr_idx, cnt64, shift,
                   perm, skeys);
        return;
    }
    const uint32_t t = blockIdx.x - na;
    if (!J.special[t]) return;  // keygen saw no special entity in this tile
    pairs_tile<1>(t, J.F, J.O_rec, J.O_ss, J.seq_base, J.sc, J.sc, J.tmp, J.cap, J.tile_total, J.tile_base,
                  J.tile_off, J.leave_off, J.sc->dbg);
}

// ------------------------------------------------------- combined pass ------
// Every unordered pair that can have an event this flush is visited once,
// by one of its members A, in the new frame (sorted by cell).  One lane per A,
// fixed blocks of 256 consecutive frame entries.
//
// Both members "near" (not a jumper: live in the same space at t-1 and moved
// at most d_rel*D <= D/4 per axis): N_t != N_t-1 needs the pair in the band
// (BW = 2 d_rel D + M covers both displacements plus the float32 rounding of
// the window bounds; lo = D - BW, hi = D + BW, all differences fl(b - a)):
//   Z : dz in [lo, hi] and |dx| <= hi      (B above A)
//   X': dx in [lo, hi] and |dz| <  lo      (B right of A, not in Z either way)
// Z and X' are disjoint and every band pair is in exactly one of them from
// exactly one side, so A queries two thin strips of cells instead of the
// whole window.  Pairs where neither member changed yield no event.
// A "jumper" A (new, changed space, moved > D/4) tests its whole window
// (|d| <= hi + M) instead; a pair of two jumpers is visited by the lower
// frame index, and near entities skip jumper partners.
// Survivors of the cheap filter go to a per-wave LDS queue and get the full
// go-aoi test (pair_kind<2>) with lanes over queue entries.  Events are
// buffered per wave in processing order (deterministic); a wave whose buffer
// overflows replays its sweep and writes the rest straight to the output.

constexpr int CT = (int)COMBINED_TILE;
constexpr int CW = CT / WAVE;  // waves per k_combined workgroup
#ifndef GWAOI_QCAP
#define GWAOI_QCAP 384
#endif
#ifndef GWAOI_EVW
#define GWAOI_EVW 192
#endif
#ifndef GWAOI_SW_U
#define GWAOI_SW_U 4  // candidates per lane per sweep iteration on long rows
#endif
#ifndef GWAOI_FLAT_U
#define GWAOI_FLAT_U 2  // flat sweep: 64-candidate chunks per iteration
#endif
constexpr int QCAP = GWAOI_QCAP;  // per-wave queue of filter survivors (>= one sweep iteration + a drain batch)
constexpr int EVW = GWAOI_EVW;    // events buffered per wave
static_assert(QCAP >= GWAOI_SW_U * WAVE, "queue must hold one sweep iteration");

// A queued pair is (A, B): A is one of the block's own entries, so it is kept
// as its offset in the block (1 B) next to B's frame index (4 B).  5 B per
// entry keeps the block under 20 KB of LDS (8 blocks per CU).
constexpr int NCLS = 14;  // lane work classes of k_combined

struct CombinedLds {
    uint32_t ndrain[CW];    // mid-sweep queue drains of each wave (DBG_COMBINED_DRAIN)
    uint16_t ccnt[NCLS][CW];  // entities per work class and wave
    uint8_t perm[CT];         // the block's entries regrouped by work class
    uint32_t qb[CW][QCAP];  // queued pairs of a wave: B frame index
    uint8_t qa[CW][QCAP];   //   ... A frame index - block start
    uint2 ev[CW][EVW];      // buffered events of a wave: (A slot, B slot | KIND_LEAVE)
    uint4 seg[CW][WAVE];                   // flat sweep: a lane's row ranges of the current group (sweep_flat)
    float4 atab[CW][WAVE];                 //   ... the lanes' own positions (x, z, old x, old z)
    uint8_t mark[CW][WAVE * GWAOI_FLAT_U];  //   ... lane + 1 at the flat position where its items start
    uint32_t wcnt[CW][2];
    uint32_t wwork[CW];  // flat sweep: candidates dealt out by each wave (the tile's work, for the next flush's order)
    unsigned long long base;
    uint32_t te, tl;
    int overflow;
};

struct CombinedCtx {  // block-uniform
    uint32_t *dbg;  // TickScalars::dbg (rare-path counters)
    SpaceGrid g;
    PairCtx proto;
    float thr, lo, hi, lo_in, M;
    float in_max, out_min;  // Chebyshev distance certainly inside (<=) / outside (>) every owner's window
    bool band_ok;  // lo > 0 (else every lane sweeps its whole window)
};

struct LaneA {
    uint32_t a;  // frame index
    float x, z;
    float xo, zo;  // previous-flush position (near lanes)
    bool valid, jump;
};

[[maybe_unused]] __device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

// Full test of the queued pairs of wave w; appends events (deterministic order).
// replay: count only, and write events number >= EVW straight to the output.
__device__ __forceinline__ void drain_queue(const uint32_t *qb, const uint8_t *qa, uint2 *evb, uint32_t qn, uint32_t e0,
                                         const FrameView &F, const Rec16 *__restrict__ O_rec, const PairCtx &proto,
                                         float thr, uint32_t &ne, uint32_t &nl, uint2 *out, uint64_t cap,
                                         unsigned long long pe, unsigned long long pl, bool replay) {
    const uint32_t ln = lane();
    for (uint32_t q0 = 0; q0 < qn; q0 += WAVE) {
        const uint32_t e = q0 + ln;
        int kind = 0;
        uint32_t a = 0, b = 0;
        if (e < qn) {
            a = e0 + (uint32_t)qa[e];
            b = qb[e];
            PairCtx A = proto;
            A.a = a;
            A.now = ld_rec(F.rec, a);
            A.oth = ld_rec(O_rec, a);
            A.chg = A.now.s >= proto.seq_base;
            const Rec16 bn = ld_rec(F.rec, b), bo = ld_rec(O_rec, b);
            kind = pair_kind<2>(A, bn, bo, b, thr);
        }
        const unsigned long long em = __ballot(kind == 1), lm = __ballot(kind == 2);
        const uint32_t pos = ne + nl + (uint32_t)__popcll((em | lm) & lanemask_lt());
        if (kind) {
            const uint32_t a_slot = ld_ss(F.ss, a).slot, b_slot = ld_ss(F.ss, b).slot;
            if (!replay) {
                if (pos < EVW) evb[pos] = make_uint2(a_slot, b_slot | (kind == 2 ? KIND_LEAVE : 0u));
            } else if (pos >= EVW) {
                const uint32_t kidx = kind == 1 ? ne + (uint32_t)__popcll(em & lanemask_lt())
                                                : nl + (uint32_t)__popcll(lm & lanemask_lt());
                ev_put2(out, cap, (kind == 1 ? pe : pl) + 2ull * kidx, a_slot, b_slot);
            }
        }
        ne += (uint32_t)__popcll(em);
        nl += (uint32_t)__popcll(lm);
    }
}

// First frame entry of A's block, as a scalar (blocks are CT-aligned).
__device__ __forceinline__ uint32_t block_start(const LaneA &A) {
    return __builtin_amdgcn_readfirstlane(A.a & ~(uint32_t)(CT - 1));
}

__device__ __forceinline__ float uniform_f32(float v) {
    return __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(v)));
}

__device__ __forceinline__ unsigned long long uniform_u64(unsigned long long v) {
    return ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           (unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

struct WaveQueue {
    uint32_t qn;
    uint32_t ne, nl;
    uint32_t lw;  // per lane: candidates of this lane's ranges (flat sweep; the next flush's deal)
};

// Append (a, b) for the lanes with keep set.  Wave-uniform.
// a_off = A's offset in its block (the block's first frame entry is e0).
__device__ __forceinline__ void qpush(uint32_t *qb, uint8_t *qa, WaveQueue &Q, bool keep, uint32_t a_off, uint32_t b) {
    // the lane predicate stays an SGPR mask: the i1 ballot builtin, and the lane's rank by
    // v_mbcnt on the mask's halves (an SGPR operand) instead of an AND with a VGPR lane mask
    const unsigned long long m = __builtin_amdgcn_ballot_w64(keep);
    if (keep) {
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint32_t i = Q.qn + r;
        qb[i] = b;
        qa[i] = (uint8_t)a_off;
    }
    Q.qn += (uint32_t)__popcll(m);
}

// Cheap filter of candidate b (k = cand[b]: x, z, old x, old z; NaN for a
// jumper) for lane A.  MODE 0: Z strip, 1: X' strip (jumper partners fail
// the NaN compares), 2: whole window of a jumper A -- a jumper partner is kept
// unfiltered by the lower frame index (the full test in drain_queue has the
// window box).
// The strips also drop a pair whose relation certainly did not change: with
// both members near, the pair is related at t-1 and at t when its Chebyshev
// distance is <= D - M both times, and unrelated both times when it is
// > D + M both times, whichever member owns the window (M covers the float32
// rounding of the window bounds and of the differences).

typedef float f32x2_t __attribute__((ext_vector_type(2)));

template <int MODE>
__device__ __forceinline__ bool band_keep(const LaneA &A, const CombinedCtx &C, const uint4 &k, uint32_t b) {
    const float lo = C.lo, hi = C.hi;
    const float dx = __uint_as_float(k.x) - A.x, dz = __uint_as_float(k.y) - A.z;
    if (MODE == 2) {
        const bool b_jump = __uint_as_float(k.x) != __uint_as_float(k.x);
        return (int)(b != A.a) & (b_jump ? (int)(A.a < b) : (int)(fabsf(dx) <= hi) & (int)(fabsf(dz) <= hi));
    }
    // Only the lower bounds that split the band between the Z and X' strips: a pair past the
    // band's outer bound (dz or dx > hi = D + 2 d_rel D + M) has Chebyshev distance > D + M at t
    // and at t-1 (both members near: each moved <= d_rel D per axis), so the unchanged-relation
    // test below drops it anyway.
    (void)hi;
    const bool bz = (int)(dz >= lo), bx = (int)(dx >= lo) & (int)(fabsf(dz) <= C.lo_in);
    // MODE 3: the rows of both strips in one sweep, either band (the strips stay disjoint)
    const bool band = MODE == 0 ? bz : MODE == 1 ? bx : (bool)((int)bz | (int)bx);
    const float dn = fmaxf(fabsf(dx), fabsf(dz));
    const float dxo = __uint_as_float(k.z) - A.xo, dzo = __uint_as_float(k.w) - A.zo;
    const float dold = fmaxf(fabsf(dxo), fabsf(dzo));
    // (dn <= in_max && dold <= in_max) || (dn > out_min && dold > out_min), as one max and one min
    // (a band hit is near at t and t-1: finite positions, no NaN operand)
    const bool same = (int)(fmaxf(dn, dold) <= C.in_max) | (int)(fminf(dn, dold) > C.out_min);
    return band & !same;
}

// Sweep candidates [jb, jb + len) of one grid row for every lane (ranges are
// per lane; the loop runs to the wave maximum mx).  MODE 0: Z strip, 1: X'
// strip, 2: whole window of a jumper.  U candidates (16-B records) per lane
// per iteration, all U loads issued before the first is used.
template <int MODE, int U>
__device__ __forceinline__ void sweep_range(CombinedLds &L, int w, WaveQueue &Q, const LaneA &A, uint32_t jb,
                                            uint32_t len, uint32_t mx, const uint4 *__restrict__ cand,
                                            const FrameView &F, const Rec16 *__restrict__ O_rec, const CombinedCtx &C,
                                            uint2 *out, uint64_t cap, unsigned long long pe, unsigned long long pl,
                                            bool replay) {
    (void)mx;
    for (uint32_t t = 0; __ballot(t < len); t += U) {  // to the wave's longest range (scalar mask test)
        if (Q.qn > QCAP - U * WAVE) {  // room for this iteration's pushes (any earlier sweep may have filled it)
            if (!replay && lane() == 0) atomicAdd(&L.ndrain[w], 1u);  // LDS; one global add per block
            __builtin_amdgcn_wave_barrier();
            drain_queue(L.qb[w], L.qa[w], L.ev[w], Q.qn, block_start(A), F, O_rec, C.proto, C.thr, Q.ne, Q.nl, out,
                        cap, pe, pl, replay);
            Q.qn = 0;
        }
        uint4 k[U];
#pragma unroll
        for (int u = 0; u < U; ++u) k[u] = cand[t + (uint32_t)u < len ? jb + t + (uint32_t)u : 0u];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t b = jb + t + (uint32_t)u;
            const bool keep = band_keep<MODE>(A, C, k[u], b) & (t + (uint32_t)u < len);
            qpush(L.qb[w], L.qa[w], Q, keep, A.a & (uint32_t)(CT - 1), b);
        }
    }
}

// sweep_range over P row ranges of a lane taken as one sequence (index select per candidate):
// the short X' rows share sweep iterations instead of paying one each.
template <int MODE, int U, int P>
__device__ __forceinline__ void sweep_segs(CombinedLds &L, int w, WaveQueue &Q, const LaneA &A,
                                           const uint32_t (&jb)[P], const uint32_t (&ln)[P],
                                           const uint4 *__restrict__ cand, const FrameView &F,
                                           const Rec16 *__restrict__ O_rec, const CombinedCtx &C, uint2 *out,
                                           uint64_t cap, unsigned long long pe, unsigned long long pl, bool replay) {
    uint32_t cum[P], tot = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        tot += ln[q];
        cum[q] = tot;
    }
    for (uint32_t t = 0; __ballot(t < tot); t += U) {
        if (Q.qn > QCAP - U * WAVE) {
            if (!replay && lane() == 0) atomicAdd(&L.ndrain[w], 1u);
            __builtin_amdgcn_wave_barrier();
            drain_queue(L.qb[w], L.qa[w], L.ev[w], Q.qn, block_start(A), F, O_rec, C.proto, C.thr, Q.ne, Q.nl, out,
                        cap, pe, pl, replay);
            Q.qn = 0;
        }
        uint4 k[U];
        uint32_t bi[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t v = t + (uint32_t)u;
            uint32_t idx = jb[0] + v;
#pragma unroll
            for (int q = 1; q < P; ++q)
                if (v >= cum[q - 1]) idx = jb[q] + (v - cum[q - 1]);
            bi[u] = v < tot ? idx : 0u;
            k[u] = cand[bi[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool keep = band_keep<MODE>(A, C, k[u], bi[u]) & (t + (uint32_t)u < tot);
            qpush(L.qb[w], L.qa[w], Q, keep, A.a & (uint32_t)(CT - 1), bi[u]);
        }
    }
}

// The candidates of P row ranges per lane, dealt out evenly: the wave's lanes
// lay their ranges end to end (lane order, then row order) and every lane
// takes one position of each 64-position chunk.  A position's owner is the
// last lane whose items start at or before it: each lane with items marks its
// start (lane + 1) in LDS, and a max-scan over the chunk fills the gaps.  The
// owner's ranges and its offset come from the wave's table in LDS, its
// position by ds_bpermute.  Lock-step sweeps pay for the busiest lane of every
// row (29% of the loaded slots were a lane's own candidates at config 3);
// here only the last chunk of a group is partial.
template <int MODE, int P>
__device__ __forceinline__ void sweep_flat(CombinedLds &L, int w, WaveQueue &Q, const LaneA &A,
                                           const uint32_t (&jb)[P], const uint32_t (&ln)[P],
                                           const uint4 *__restrict__ cand, const FrameView &F,
                                           const Rec16 *__restrict__ O_rec, const CombinedCtx &C, uint2 *out,
                                           uint64_t cap, unsigned long long pe, unsigned long long pl, bool replay) {
    static_assert(P == 1 || P == 2, "one or two row ranges per lane");
    constexpr int U = GWAOI_FLAT_U;
    const uint32_t me = lane();
    uint32_t cum[P], tot = 0;  // items before row q of this lane
#pragma unroll
    for (int q = 0; q < P; ++q) {
        cum[q] = tot;
        tot += ln[q];
    }
    const uint32_t inc = wave_scan_add(tot);
    const uint32_t T = __builtin_amdgcn_readlane(inc, WAVE - 1);
    if (T == 0) return;
    if (me == 0 && !replay) L.wwork[w] += T;
    Q.lw += tot;
    const uint32_t off = inc - tot;
    const uint32_t offa = off | ((A.a & (uint32_t)(CT - 1)) << 24);
    // row q's candidate of lane-local item kk is (jb[q] - cum[q]) + kk, for the last q with cum[q] <= kk
    L.seg[w][me] = make_uint4(jb[0], P == 2 ? jb[P - 1] - cum[P - 1] : 0u, P == 2 ? cum[P - 1] : 0xFFFFFFFFu, offa);
    L.atab[w][me] = make_float4(A.x, A.z, A.xo, A.zo);
    uint8_t *mk = L.mark[w];
    uint32_t carry = 0;  // owner + 1 of the position before this chunk
    for (uint32_t g0 = 0; g0 < T; g0 += U * WAVE) {
        if (Q.qn > QCAP - U * WAVE) {
            if (!replay && me == 0) atomicAdd(&L.ndrain[w], 1u);
            __builtin_amdgcn_wave_barrier();
            drain_queue(L.qb[w], L.qa[w], L.ev[w], Q.qn, block_start(A), F, O_rec, C.proto, C.thr, Q.ne, Q.nl, out,
                        cap, pe, pl, replay);
            Q.qn = 0;
        }
        if (me < (uint32_t)(U * WAVE / 4)) reinterpret_cast<uint32_t *>(mk)[me] = 0u;
        if (tot != 0 && off >= g0 && off < g0 + (uint32_t)(U * WAVE)) mk[off - g0] = (uint8_t)(me + 1u);
        __builtin_amdgcn_wave_barrier();
        uint32_t own[U];
#pragma unroll
        for (int u = 0; u < U; ++u) own[u] = wave_scan_max(mk[u * WAVE + me]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            own[u] = max(own[u], carry);
            carry = __builtin_amdgcn_readlane(own[u], WAVE - 1);
        }
        __builtin_amdgcn_wave_barrier();  // the marks are read before the next chunk clears them
        uint4 k[U];
        uint32_t bi[U], ao[U];
        float ax[U], az[U], axo[U], azo[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t p = g0 + (uint32_t)(u * WAVE) + me;
            const uint32_t o = (own[u] - 1u) & (uint32_t)(WAVE - 1);
            const uint4 s = L.seg[w][o];
            const uint32_t kk = p - (s.w & 0xFFFFFFu);
            const uint32_t idx = (kk >= s.z ? s.y : s.x) + kk;
            ao[u] = s.w >> 24;
            bi[u] = p < T ? idx : 0u;
            // (from an LDS table: the owner's registers by ds_bpermute, 4 per position, cost 81.7
            // against 78.0 us at config 3, and 87.0 with the freed LDS spent on an 8th wave per SIMD)
            const float4 ap = L.atab[w][o];
            ax[u] = ap.x;
            az[u] = ap.y;
            axo[u] = ap.z;
            azo[u] = ap.w;
            k[u] = cand[bi[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            LaneA B;
            B.a = 0;
            B.x = ax[u];
            B.z = az[u];
            B.xo = axo[u];
            B.zo = azo[u];
            const bool keep = band_keep<MODE>(B, C, k[u], bi[u]) & (g0 + (uint32_t)(u * WAVE) + me < T);
            qpush(L.qb[w], L.qa[w], Q, keep, ao[u], bi[u]);
        }
    }
}

// Rows r0..r1 (per lane; `on` = the lane takes part), cells c0..c1 of each row.
// The next row's candidate range is loaded while the current one is swept.
template <int MODE>
__device__ __forceinline__ void sweep_rows(CombinedLds &L, int w, WaveQueue &Q, const LaneA &A, bool on, int r0,
                                           int r1, int c0, int c1, const uint4 *__restrict__ cand, const FrameView &F,
                                           const Rec16 *__restrict__ O_rec, const CombinedCtx &C, uint2 *out,
                                           uint64_t cap, unsigned long long pe, unsigned long long pl, bool replay) {
    const uint32_t nr = on ? (uint32_t)(r1 - r0 + 1) : 0u;
    const uint32_t *cs = F.cell_start;
    const uint32_t rb0 = C.g.base + (uint32_t)c0, gx = C.g.gx, span = on ? (uint32_t)(c1 - c0) + 1u : 0u;
    uint32_t jb = 0, je = 0;
    if (nr) {
        const uint32_t rb = rb0 + (uint32_t)r0 * gx;
        jb = cs[rb];
        je = cs[rb + span];
    }
    for (uint32_t k = 0; __ballot(k < nr); ++k) {
        uint32_t nb = 0, ne = 0;
        if (k + 1 < nr) {  // prefetch the next row's range
            const uint32_t rb = rb0 + (uint32_t)(r0 + (int)k + 1) * gx;
            nb = cs[rb];
            ne = cs[rb + span];
        }
        const uint32_t len = je - jb;
        const uint32_t mx = 0;
        if (MODE != 2 && __ballot(len > 2))
            sweep_range<MODE, GWAOI_SW_U>(L, w, Q, A, jb, len, mx, cand, F, O_rec, C, out, cap, pe, pl, replay);
        else if (__ballot(len != 0))
            sweep_range<MODE, 2>(L, w, Q, A, jb, len, mx, cand, F, O_rec, C, out, cap, pe, pl, replay);
        jb = nb;
        je = ne;
    }
}

// Both strips as one list of rows per lane, swept flat P rows at a time with the union band
// (MODE 3): the X' rows below the Z strip's first row, then the Z rows.  The row the two strips
// share is swept once, over the Z strip's wider cells, where the union band finds both kinds.
template <int P>
__device__ __forceinline__ void sweep_rows_merged(CombinedLds &L, int w, WaveQueue &Q, const LaneA &A, bool on,
                                                  int zr0, int zr1, int zc0, int zc1, int xr0, int xr1, int xc0,
                                                  int xc1, const uint4 *__restrict__ cand, const FrameView &F,
                                                  const Rec16 *__restrict__ O_rec, const CombinedCtx &C, uint2 *out,
                                                  uint64_t cap, unsigned long long pe, unsigned long long pl,
                                                  bool replay) {
    const int xe = min(xr1, zr0 - 1);
    const uint32_t nx = on && xe >= xr0 ? (uint32_t)(xe - xr0 + 1) : 0u;
    const uint32_t nr = on ? nx + (uint32_t)(zr1 - zr0 + 1) : 0u;
    const uint32_t *cs = F.cell_start;
    const uint32_t gx = C.g.gx;
    const uint32_t xb = C.g.base + (uint32_t)xr0 * gx + (uint32_t)xc0, xs = (uint32_t)(xc1 - xc0) + 1u;
    const uint32_t zb = C.g.base + (uint32_t)zr0 * gx + (uint32_t)zc0, zs = (uint32_t)(zc1 - zc0) + 1u;
    // (both bounds loaded whatever q, cell 0 past the lane's rows: under a per-lane branch each
    // load was waited for on its own, and the next group's ranges were not in flight during the
    // current group's sweep)
    auto range = [&](uint32_t q, uint32_t &b, uint32_t &l) {
        const bool v = q < nr;
        const uint32_t rb = !v ? 0u : q < nx ? xb + q * gx : zb + (q - nx) * gx;
        const uint32_t re = !v ? 0u : rb + (q < nx ? xs : zs);
        const uint32_t b0 = cs[rb], e0 = cs[re];
        b = v ? b0 : 0u;
        l = v ? e0 - b0 : 0u;
    };
    uint32_t jb[P], ln[P];
#pragma unroll
    for (int q = 0; q < P; ++q) range((uint32_t)q, jb[q], ln[q]);
    for (uint32_t k = 0; __ballot(k < nr); k += P) {
        uint32_t nb[P], nl[P];
#pragma unroll
        for (int q = 0; q < P; ++q) range(k + P + (uint32_t)q, nb[q], nl[q]);  // the next group's ranges
        sweep_flat<3, P>(L, w, Q, A, jb, ln, cand, F, O_rec, C, out, cap, pe, pl, replay);
#pragma unroll
        for (int q = 0; q < P; ++q) {
            jb[q] = nb[q];
            ln[q] = nl[q];
        }
    }
}

// The wave's index in its block as a scalar (an SGPR: the per-wave LDS bases then cost no VGPR).
__device__ __forceinline__ int wave_id() { return (int)__builtin_amdgcn_readfirstlane(threadIdx.x / WAVE); }

__device__ void combined_sweep(CombinedLds &L, const int w, const LaneA &A, const uint4 *__restrict__ cand,
                               const FrameView &F, const Rec16 *__restrict__ O_rec, const CombinedCtx &C, uint32_t &ne,
                               uint32_t &nl, uint32_t &lw, uint2 *out, uint64_t cap, unsigned long long pe,
                               unsigned long long pl, bool replay) {
    const SpaceGrid &g = C.g;
    WaveQueue Q{0u, ne, nl, lw};
    const float lo = C.lo, hi = C.hi, M = C.M;
    const bool strip = A.valid && !A.jump && C.band_ok;
    const bool whole = A.valid && (A.jump || !C.band_ok);
    if (__ballot(strip)) {
        int zr0 = 0, zr1 = -1, zc0 = 0, zc1 = -1, xr0 = 0, xr1 = -1, xc0 = 0, xc1 = -1;
        if (strip) {
            zr0 = cell_of(A.z + lo - M, g.oz, g.inv, g.gz);
            zr1 = cell_of(A.z + hi + M, g.oz, g.inv, g.gz);
            zc0 = cell_of(A.x - hi - M, g.ox, g.inv, g.gx);
            zc1 = cell_of(A.x + hi + M, g.ox, g.inv, g.gx);
            xr0 = cell_of(A.z - lo - M, g.oz, g.inv, g.gz);
            xr1 = cell_of(A.z + lo + M, g.oz, g.inv, g.gz);
            xc0 = cell_of(A.x + lo - M, g.ox, g.inv, g.gx);
            xc1 = cell_of(A.x + hi + M, g.ox, g.inv, g.gx);
        }
        sweep_rows_merged<2>(L, w, Q, A, strip, zr0, zr1, zc0, zc1, xr0, xr1, xc0, xc1, cand, F, O_rec, C,
                                       out, cap, pe, pl, replay);
    }
    if (__ballot(whole)) {
        const float r = hi + M;
        int r0 = 0, r1 = -1, c0 = 0, c1 = -1;
        if (whole) {
            r0 = cell_of(A.z - r, g.oz, g.inv, g.gz);
            r1 = cell_of(A.z + r, g.oz, g.inv, g.gz);
            c0 = cell_of(A.x - r, g.ox, g.inv, g.gx);
            c1 = cell_of(A.x + r, g.ox, g.inv, g.gx);
        }
        sweep_rows<2>(L, w, Q, A, whole, r0, r1, c0, c1, cand, F, O_rec, C, out, cap, pe, pl, replay);
    }
    if (Q.qn) {
        __builtin_amdgcn_wave_barrier();
        drain_queue(L.qb[w], L.qa[w], L.ev[w], Q.qn, block_start(A), F, O_rec, C.proto, C.thr, Q.ne, Q.nl, out, cap,
                    pe, pl, replay);
    }
    ne = Q.ne;
    nl = Q.nl;
    lw = Q.lw;
}

// One block = frame entries [256 t, 256 t + 256).  A block that straddles
// spaces (small spaces) sweeps once per distinct space among a wave's lanes.
#ifndef GWAOI_COMBINED_WPE
#define GWAOI_COMBINED_WPE 7  // 68 VGPRs without spills
#endif
#if GWAOI_COMBINED_WPE
#define COMBINED_ATTR __attribute__((amdgpu_waves_per_eu(GWAOI_COMBINED_WPE)))
#else
#define COMBINED_ATTR
#endif
#ifdef GWAOI_EXP_BLOCKTIME
constexpr uint32_t BT_MAX = 65536;
__device__ unsigned long long gw_blocktime[3 * BT_MAX];
constexpr uint32_t BT_FIN = 40000;  // k_finish's blocks (k_combined's units stay below it at config 3)
#define BT_STAMP(slot) \
    do { \
        if (threadIdx.x == 0) gw_blocktime[3 * (BT_FIN + 2000) + (slot)] = wall_clock64(); \
    } while (0)
#define BT_OSTAMP(slot) \
    do { \
        if (threadIdx.x == 0 && blockIdx.x == 0) gw_blocktime[3 * (BT_FIN + 2004) + (slot)] = wall_clock64(); \
    } while (0)
#else
#define BT_STAMP(slot) \
    do { \
    } while (0)
#define BT_OSTAMP(slot) \
    do { \
    } while (0)
#endif
// The schedule (tile_order, built by k_finish for the next flush from this flush's measured time
// per tile; any schedule gives the same events): each XCD x gets a contiguous range of tiles, cut
// where the cumulative time crosses x/8 of the total (the XCDs end together: an even split by
// count left them 65-88 us apart at config 3), run heaviest first; workgroup b runs on XCD b % 8
// (the round-robin dispatch, for speed only) as that range's (b / 8)-th tile, and the workgroups
// past a range's end leave at once.
__host__ __device__ inline uint32_t range_max(uint32_t n_tiles) {
    const uint32_t even = (n_tiles + N_XCD - 1) / N_XCD;
    return even + even / 4 + 64;
}
__host__ __device__ inline uint32_t order_meta(uint32_t n_tiles) { return 1 + n_tiles; }

__global__ __launch_bounds__(CT) COMBINED_ATTR void k_combined(FrameView F, const uint4 *__restrict__ cand,
                                                 const Rec16 *__restrict__ O_rec, unsigned long long seq_base,
                                                 const TickScalars *__restrict__ sc, TickScalars *scw,
                                                 uint2 *out, uint64_t cap, uint32_t *tile_total,
                                                 unsigned long long *tile_base, uint32_t leave_off, uint32_t *dbg,
                                                 const uint32_t *__restrict__ tile_order, uint32_t *tile_work,
                                                 uint8_t *ework, uint32_t n_tiles) {
    __shared__ CombinedLds L;
    uint32_t t;
    {
        const uint32_t x = blockIdx.x % N_XCD, k = blockIdx.x / N_XCD;
        const bool ordered = tile_order && tile_order[0] == n_tiles;
        uint32_t lo, hi;
        if (ordered) {
            lo = tile_order[order_meta(n_tiles) + x];
            hi = tile_order[order_meta(n_tiles) + x + 1];
        } else {
            const uint32_t q = n_tiles / N_XCD, r = n_tiles % N_XCD;
            lo = x * q + min(x, r);
            hi = lo + q + (x < r ? 1u : 0u);
        }
        if (lo + k >= hi) return;  // past this XCD's range (block-uniform: before any barrier)
        t = ordered ? tile_order[1 + lo + k] : lo + k;
    }
    const unsigned long long t_start = wall_clock64();
#ifdef GWAOI_EXP_BLOCKTIME
    const unsigned long long bt0 = t_start;
#endif
    const uint32_t tid = threadIdx.x, ln = lane();
    const int w = wave_id();
    const uint32_t e0 = t * CT;
    if (tid < CW) L.wwork[tid] = L.ndrain[tid] = 0;
    if (tid == 0) L.overflow = 0;
    __syncthreads();

    // A block holds its LDS until its slowest wave ends, so the waves get equal
    // work: the block's entries are ranked by the candidates their lanes swept
    // last flush (stable, by ballots over log2 classes) and dealt round-robin,
    // rank r to wave r mod 4; lane tid takes entry e0 + perm[tid].
    uint32_t off = tid;
    {
        const uint32_t a = e0 + tid;
        uint32_t cls = NCLS - 1;  // past the frame
        // by the work this entry's lane had last flush (the frame index then held about the same
        // entity), heaviest first, dealt round-robin to the waves below
        if (a < F.n) {
            const uint32_t lg = ework ? ework[a] : 0u;  // log2 of the candidates, one byte per entry
            cls = (uint32_t)(NCLS - 2) - min((uint32_t)(NCLS - 2), lg);
        }
        unsigned long long mine = 0;
#pragma unroll
        for (int c = 0; c < NCLS; ++c) {
            const unsigned long long m = __ballot(cls == (uint32_t)c);
            if ((uint32_t)c == cls) mine = m;
            if (ln == 0) L.ccnt[c][w] = (uint16_t)__popcll(m);
        }
        __syncthreads();
        uint32_t pos = (uint32_t)__popcll(mine & lanemask_lt());
        for (int c = 0; c < NCLS; ++c)
            for (int q = 0; q < CW; ++q)
                if ((uint32_t)c < cls || ((uint32_t)c == cls && q < w)) pos += L.ccnt[c][q];
        pos = (pos & (uint32_t)(CW - 1)) * WAVE + pos / CW;  // rank r goes to wave r mod CW
        L.perm[pos] = (uint8_t)tid;
        __syncthreads();
        off = L.perm[tid];  // (measured: combined 0.135 ms vs 0.148 in frame order)
    }
    LaneA A;
    A.a = e0 + off;
    A.valid = A.a < F.n;
    const uint32_t ia = A.valid ? A.a : 0u;
    const uint4 ca = cand[ia];
    const Rec16 ra = ld_rec(F.rec, ia);  // exact position (a jumper's candidate record is NaN)
    A.x = ra.x;
    A.z = ra.z;
    A.xo = __uint_as_float(ca.z);
    A.zo = __uint_as_float(ca.w);
    A.jump = __uint_as_float(ca.x) != __uint_as_float(ca.x);
    const uint32_t my_sp = ld_ss(F.ss, ia).sp;

    uint32_t ne = 0, nl = 0;  // wave totals (wave-uniform)
    uint32_t lw = 0;          // this lane's candidates
    // sweep once per distinct space in this wave (almost always one)
    auto run = [&](bool replay, uint2 *o, unsigned long long pe, unsigned long long pl, uint32_t &e,
                   uint32_t &l) {
        unsigned long long pending = __ballot(A.valid);
        while (pending) {
            const uint32_t lead = (uint32_t)__ffsll((long long)pending) - 1u;
            const uint32_t sp = __builtin_amdgcn_readfirstlane(__shfl(my_sp, (int)lead));  // wave-uniform: scalar grid loads
            const bool mine = A.valid && my_sp == sp;
            pending &= ~__ballot(mine);
            CombinedCtx C;
            C.dbg = dbg;
            C.g = F.grid[sp];
            C.M = (sc->bmax + 3.0f * C.g.D) * 0x1p-20f;
            C.thr = FAR_FRAC * C.g.D;
            const float BW = 2.0f * sc->d_rel * C.g.D + C.M;
            C.lo = C.g.D - BW;
            C.hi = C.g.D + BW;
            C.lo_in = C.lo > 0.f ? __uint_as_float(__float_as_uint(C.lo) - 1u) : 0.f;
            C.band_ok = C.lo > 0.f;
            C.in_max = C.g.D - C.M;
            C.out_min = C.g.D + C.M;
            // wave-uniform by construction: keep them in SGPRs (they were VALU results in VGPRs)
            C.M = uniform_f32(C.M);
            C.thr = uniform_f32(C.thr);
            C.lo = uniform_f32(C.lo);
            C.hi = uniform_f32(C.hi);
            C.lo_in = uniform_f32(C.lo_in);
            C.in_max = uniform_f32(C.in_max);
            C.out_min = uniform_f32(C.out_min);
            C.proto.D = C.g.D;
            C.proto.HM = C.hi;
            C.proto.seq_base = seq_base;
            C.proto.a = 0;
            C.proto.chg = false;
            LaneA B = A;
            B.valid = mine;
            combined_sweep(L, w, B, cand, F, O_rec, C, e, l, lw, o, cap, pe, pl, replay);
        }
    };
    run(false, nullptr, 0ull, 0ull, ne, nl);
    if (ework && A.valid) ework[A.a] = (uint8_t)(31 - __clz((int)(lw | 1u)));
    if (ln == 0) {
        L.wcnt[w][0] = ne;
        L.wcnt[w][1] = nl;
        if (ne + nl > (uint32_t)EVW) atomicAdd(dbg + DBG_COMBINED_REPLAY, 1u);
    }
    // ---- offsets: 2 directed pairs per event; the block's enters, then its leaves
    __syncthreads();
    if (tid == 0) {
        uint32_t se = 0, sl = 0;
        for (int q = 0; q < CW; ++q) {
            const uint32_t e = L.wcnt[q][0], l = L.wcnt[q][1];
            L.wcnt[q][0] = se;
            L.wcnt[q][1] = sl;
            se += e;
            sl += l;
            if (e + l > (uint32_t)EVW) L.overflow = 1;
        }
        L.te = se;
        L.tl = sl;
        uint32_t nd = 0;
        for (int q = 0; q < CW; ++q) nd += L.ndrain[q];
        if (nd) atomicAdd(dbg + DBG_COMBINED_DRAIN, nd);
        const uint32_t tot = 2 * (se + sl), q = xcc_id();
        const unsigned long long b = tot ? ev_alloc(scw, q, tot) : ev_enc(q, 0ull);
        L.base = b;
        put_tile_total(tile_total, leave_off, t, 2 * se);
        tile_base[t] = b;
        put_tile_total(tile_total, leave_off, leave_off + t, 2 * sl);
        tile_base[leave_off + t] = b + 2ull * se;
    }
    __syncthreads();
    const uint32_t pre_e = L.wcnt[w][0], pre_l = L.wcnt[w][1];
    const unsigned long long pe = uniform_u64(L.base + 2ull * pre_e),
                             pl = uniform_u64(L.base + 2ull * L.te + 2ull * pre_l);
    // buffered events of this wave, in order, split by kind
    const uint32_t nbuf = min(ne + nl, (uint32_t)EVW);
    uint32_t ie = 0, il = 0;
    for (uint32_t c = 0; c < nbuf; c += WAVE) {
        const uint32_t e = c + ln;
        const uint2 ev = e < nbuf ? L.ev[w][e] : make_uint2(0, 0);
        const bool valid = e < nbuf;
        const bool lv = (ev.y & KIND_LEAVE) != 0u;
        const unsigned long long lm = __ballot(valid && lv), em = __ballot(valid && !lv);
        if (valid) {
            const uint32_t b_slot = ev.y & ~KIND_LEAVE;
            const unsigned long long p = lv ? pl + 2ull * (il + (uint32_t)__popcll(lm & lanemask_lt()))
                                            : pe + 2ull * (ie + (uint32_t)__popcll(em & lanemask_lt()));
            ev_put2(out, cap, p, ev.x, b_slot);
        }
        ie += (uint32_t)__popcll(em);
        il += (uint32_t)__popcll(lm);
    }
    if (ne + nl > (uint32_t)EVW) {  // replay: this wave writes the events past its buffer directly
        uint32_t re = 0, rl = 0;
        run(true, out, pe, pl, re, rl);
    }
    // the tile's cost for the next flush's schedule: its measured time (100 MHz ticks), which the
    // candidate count predicted poorly (crowd tiles take longer per candidate)
    __syncthreads();
#ifndef GWAOI_TILE_TIME
#define GWAOI_TILE_TIME 1
#endif
    if (tile_work && tid == 0) {
        uint32_t wk = CT;
        for (int q = 0; q < CW; ++q) wk += L.wwork[q];
#if GWAOI_TILE_TIME
        tile_work[t] = max(1u, (uint32_t)min(wall_clock64() - t_start, 0xFFFFFFFFull));
#else
        tile_work[t] = wk;
#endif
        tile_work[n_tiles + t] = wk;  // its candidates: how uneven a range's work is (order_range)
    }
#ifdef GWAOI_EXP_BLOCKTIME  // diagnostics build only: per-block start/end (wall clock) and hardware ids
    if (tid == 0 && t < BT_MAX) {
        gw_blocktime[3 * t] = bt0;
        gw_blocktime[3 * t + 1] = wall_clock64();
        gw_blocktime[3 * t + 2] = (unsigned long long)__smid() | ((unsigned long long)__builtin_amdgcn_s_getreg(6164) << 32) |
                                  ((unsigned long long)blockIdx.x << 40);
    }
#endif
}



// ------------------------------------------------------------- finish ------
// The flush's tail in one launch (it was three: a scan of the tile totals,
// the tile copy and the bbox fold).  Blocks 0..R-1 take FT consecutive tile
// entries each; a block's output offset is the sum of the tile totals before
// it: the group totals (FG entries each) before its group, added by the pair
// passes, then its own group's entries before it.  Block R
// folds the bbox parts and writes the scalars of TickOut.
#ifndef GWAOI_FT
#define GWAOI_FT 16  // measured (cfg3, group totals): 8 -> 12.4 us, 16 -> 11.4, 32 -> 13.7
#endif
constexpr int FT = GWAOI_FT;  // tile entries per finish block (<= 64: one wave scans them)
static_assert(FT <= WAVE, "one wave scans a finish block's tile totals");

// The next flush's k_combined schedule is built by the finish from this flush's work per tile:
// within each XCD's range, heaviest first, as a counting sort over 64 log-spaced work classes.
// Only the schedule changes; k_combined's events do not depend on it.
// Bands (GWAOI_ORDER_BANDS): the range is cut into that many consecutive bands, run one after the
// other, heaviest first within each -- the tail of the launch gets the light units of the last
// band, and the units in flight stay near one another in the frame.
#ifndef GWAOI_ORDER_BANDS
#define GWAOI_ORDER_BANDS 1
#endif
#ifndef GWAOI_ORDER_SKEW
#define GWAOI_ORDER_SKEW 4  // even ranges (top percentile within this many work classes of the median) keep frame order; 0: off
#endif
#ifndef GWAOI_ORDER_TOP
#define GWAOI_ORDER_TOP 2  // ... the percentile, from the heaviest
#endif
constexpr int TO_NB = 64;
constexpr int TO_BANDS = GWAOI_ORDER_BANDS;
static_assert(TO_NB * TO_BANDS <= 256, "one histogram bin per thread");

// Counting sort of range [lo, hi) of tiles by (band, descending work class) into tile_order[1 + ...].
// wt(i), wc(i): tile i's measured time and candidate count (tile_work's two halves, 16-bit).
template <class WT, class WC>
__device__ void order_range(WT wt, WC wc, uint32_t lo, uint32_t hi, uint32_t *tile_order) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t ws[256 / WAVE];
    const uint32_t len = hi - lo;
    uint32_t *dst = tile_order + 1;
    // descending: 0 = heaviest; 8 classes per factor 2 from 2^(off/8): the measured times (100 MHz
    // ticks: 30 us = 3000) from 2^5, the candidate counts (256 entities x ~27 = 7000) from 2^8
    auto wcls = [](uint32_t v, int off) {
        const int c = (int)(8.0f * __log2f((float)v + 1.0f)) - off;
        return (uint32_t)(TO_NB - 1 - min(max(c, 0), TO_NB - 1));
    };
#if GWAOI_ORDER_SKEW
    // An even range -- its heaviest GWAOI_ORDER_TOP percent of tiles within GWAOI_ORDER_SKEW
    // classes of its median by candidate count (deterministic, unlike the measured time) -- runs in
    // frame order: reordering only scatters the tiles in flight (their candidate rows no longer
    // shared in L2), and nothing in it makes a tail.  Uniform worlds (config 5) take this; crowd
    // hotspots (config 3, tiles 14x apart) are ordered heaviest first.
    {
        __shared__ uint32_t s_top, s_p50;
        hist[threadIdx.x] = 0;
        if (threadIdx.x == 0) s_top = s_p50 = 0;
        __syncthreads();
        for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&hist[wcls(wc(i), 64)], 1u);
        __syncthreads();
        uint32_t total;
        const uint32_t ex = block_excl_scan<256>(hist[threadIdx.x], ws, total);
        const uint32_t incl = ex + hist[threadIdx.x];
        if (hist[threadIdx.x]) {
            if (ex * 100 <= len * GWAOI_ORDER_TOP && incl * 100 > len * GWAOI_ORDER_TOP) s_top = threadIdx.x;
            if (ex * 2 <= len && incl * 2 > len) s_p50 = threadIdx.x;
        }
        __syncthreads();
        if (TO_BANDS == 1 && s_p50 - s_top <= (uint32_t)GWAOI_ORDER_SKEW) {
            for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) dst[i] = i;
            return;
        }
        __syncthreads();
    }
#endif
    hist[threadIdx.x] = 0;
    __syncthreads();
    auto cls = [&](uint32_t i) {  // band-major, then descending work: bin 0 = heaviest of band 0
        // (one band: no 64-bit division per tile)
        const uint32_t band =
            TO_BANDS == 1 ? 0u : (uint32_t)(((unsigned long long)(i - lo) * TO_BANDS) / max(len, 1u));
        return band * TO_NB + wcls(wt(i), 40);
    };
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&hist[cls(i)], 1u);
    __syncthreads();
    uint32_t total;
    const uint32_t ex = block_excl_scan<256>(hist[threadIdx.x], ws, total);
    __syncthreads();
    hist[threadIdx.x] = ex;
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) dst[lo + atomicAdd(&hist[cls(i)], 1u)] = i;
}


// The next flush's tile schedule (k_finish's last N_XCD blocks, block x for XCD x; see k_combined):
// the eight ranges cut at the eighths of the cumulative measured time (every block computes the
// same cuts; each thread sums a contiguous segment, so one scan finds them), at most range_max
// long; range x heaviest first; the cuts at tile_order[order_meta .. order_meta + 8].
// Tiles whose times and counts the block stages in LDS (2 x 16 KB), as 16-bit values: 655 us of
// measured time or 65535 candidates saturate, above every work class's top (and no tile of a launch
// takes that long), so the schedule is the same from either copy.
constexpr uint32_t TO_LDS = 8192;
__device__ void tile_order_block(uint32_t x, const uint32_t *__restrict__ tile_work, uint32_t nb, uint32_t *tile_order) {
    __shared__ uint32_t s_cut[N_XCD + 1];
    __shared__ unsigned long long s_sum[256];
    __shared__ __attribute__((aligned(16))) uint16_t s_t[TO_LDS];
    __shared__ uint16_t s_c[TO_LDS];
    const uint32_t tid = threadIdx.x;
    // both halves into LDS with coalesced loads (TO_U of each in flight per thread), then every pass
    // reads LDS: a thread's contiguous segment read from global memory touched a line per lane per
    // load, and the range's counts were a round trip of their own (12 us at config 3)
    const bool lds = nb <= TO_LDS;
    // segments of seg contiguous tiles per thread; in LDS a multiple of 8 (16-B reads), the tail
    // past nb zero
    const uint32_t seg = lds ? ((nb + 255) / 256 + 7) & ~7u : (nb + 255) / 256;
    if (lds) {
        for (uint32_t i = nb + tid; i < 256 * seg; i += 256) s_t[i] = 0;
        constexpr uint32_t TO_U = 8;
        for (uint32_t i0 = tid; i0 < nb; i0 += TO_U * 256) {
            uint32_t t[TO_U], c[TO_U];
#pragma unroll
            for (uint32_t u = 0; u < TO_U; ++u) {  // (clamped, not branched: a load under a branch
                const uint32_t i = min(i0 + u * 256, nb - 1);  // waits for itself before the next)
                t[u] = tile_work[i];
                c[u] = tile_work[nb + i];
            }
#pragma unroll
            for (uint32_t u = 0; u < TO_U; ++u) {
                const uint32_t i = i0 + u * 256;
                if (i < nb) {
                    s_t[i] = (uint16_t)min(t[u], 65535u);
                    s_c[i] = (uint16_t)min(c[u], 65535u);
                }
            }
        }
        __syncthreads();
    }
    auto wt = [&](uint32_t i) -> uint32_t { return lds ? (uint32_t)s_t[i] : min(tile_work[i], 65535u); };
    auto wc = [&](uint32_t i) -> uint32_t { return lds ? (uint32_t)s_c[i] : min(tile_work[nb + i], 65535u); };
    BT_OSTAMP(0);
    const uint32_t s0 = min(nb, tid * seg), s1 = min(nb, s0 + seg);
    unsigned long long my = 0;
    if (lds) {
        const uint4 *p = reinterpret_cast<const uint4 *>(s_t + tid * seg);
        for (uint32_t r = 0; r < seg / 8; ++r) {
            const uint4 q = p[r];
            my += (q.x & 0xFFFFu) + (q.x >> 16) + (q.y & 0xFFFFu) + (q.y >> 16) + (q.z & 0xFFFFu) + (q.z >> 16) +
                  (q.w & 0xFFFFu) + (q.w >> 16);
        }
    } else {
        for (uint32_t i = s0; i < s1; ++i) my += wt(i);
    }
    s_sum[tid] = my;
    if (tid <= N_XCD) s_cut[tid] = tid == N_XCD ? nb : 0u;
    __shared__ uint32_t s_own[N_XCD];
    if (tid < N_XCD) s_own[tid] = 0xFFFFFFFFu;
    __syncthreads();
    if (tid < WAVE) {  // inclusive scan of the 256 segment sums by one wave (4 per lane)
        unsigned long long v[4], tt = 0;
        for (int q = 0; q < 4; ++q) {
            tt += s_sum[4 * tid + q];
            v[q] = tt;
        }
        unsigned long long incl = tt;
        for (int o = 1; o < WAVE; o <<= 1) {
            const unsigned long long y = __shfl_up(incl, o);
            if ((int)tid >= o) incl += y;
        }
        const unsigned long long ex = incl - tt;
        for (int q = 0; q < 4; ++q) s_sum[4 * tid + q] = ex + v[q];
    }
    __syncthreads();
    BT_OSTAMP(1);
    // cut q: the first tile whose exclusive prefix reaches q W / 8.  The one segment whose prefixes
    // cross q W / 8 holds it; then one wave scans that segment's tiles, a lane each (a serial walk
    // or every thread testing every cut on every tile of its segment cost 4 us of VALU at config 3)
    const unsigned long long W = s_sum[255];
    {
        const unsigned long long e0 = tid ? s_sum[tid - 1] : 0ull, e1 = s_sum[tid];
        for (uint32_t q = 1; q < N_XCD; ++q) {
            const unsigned long long T = (W * q) / N_XCD;
            if (e0 < T && e1 >= T) s_own[q] = tid;
        }
    }
    __syncthreads();
    if (seg <= WAVE) {
        for (uint32_t q = tid / WAVE + 1; q < N_XCD; q += 256 / WAVE) {
            const uint32_t sg = s_own[q];
            if (sg == 0xFFFFFFFFu) continue;
            const uint32_t a0 = min(nb, sg * seg), a1 = min(nb, a0 + seg), i = a0 + lane();
            const uint32_t val = i < a1 ? wt(min(i, nb - 1)) : 0u;
            const uint32_t inc = wave_incl_scan(val);  // (a segment's sum fits: <= 64 x 65535)
            const unsigned long long base = sg ? s_sum[sg - 1] : 0ull, T = (W * q) / N_XCD;
            const unsigned long long hits = __ballot(i < a1 && base + (inc - val) < T && base + inc >= T);
            if (hits && lane() == 0) s_cut[q] = a0 + (uint32_t)__ffsll((long long)hits);
        }
    } else {  // (segments wider than a wave: their owners walk them)
        unsigned long long e = tid ? s_sum[tid - 1] : 0ull;
        for (uint32_t i = s0; i < s1; ++i) {
            const unsigned long long in = e + wt(i);
            for (uint32_t q = 1; q < N_XCD; ++q) {
                const unsigned long long T = (W * q) / N_XCD;
                if (e < T && in >= T) s_cut[q] = i + 1;
            }
            e = in;
        }
    }
    __syncthreads();
    if (tid == 0) {  // at most range_max per range (the launch grid's bound), in order
        const uint32_t Lmax = range_max(nb);
        for (uint32_t q = 1; q < N_XCD; ++q) {
            const unsigned long long rest = (unsigned long long)(N_XCD - q) * Lmax;
            uint32_t lo_b = s_cut[q - 1];
            if (nb > rest) lo_b = max(lo_b, (uint32_t)(nb - rest));
            const uint32_t hi_b = (uint32_t)min((unsigned long long)nb, (unsigned long long)s_cut[q - 1] + Lmax);
            s_cut[q] = min(max(s_cut[q], lo_b), hi_b);
        }
    }
    __syncthreads();
    BT_OSTAMP(2);
    order_range(wt, wc, s_cut[x], s_cut[x + 1], tile_order);
    BT_OSTAMP(3);
    if (x == 0 && tid <= N_XCD) tile_order[order_meta(nb) + tid] = s_cut[tid];
    if (x == 0 && tid == 0) tile_order[0] = nb;
}


__global__ __launch_bounds__(256) void k_finish(const uint32_t *__restrict__ tile_total,
                                                const unsigned long long *__restrict__ tile_base, uint32_t n_entries,
                                                uint32_t n_enter_entries,
                                                const uint2 *__restrict__ tmp, uint2 *out, uint64_t cap_tmp,
                                                uint64_t cap_out, const TickScalars *__restrict__ sc, TickOut *res,
                                                const BBoxPart *__restrict__ parts, uint32_t np, int4 *bbox,
                                                uint32_t ns, int4 *hbbox, const uint32_t *__restrict__ tile_work,
                                                uint32_t n_tiles, uint32_t *tile_order, uint32_t *dcnt) {
#ifdef GWAOI_EXP_BLOCKTIME  // diagnostics build only: thread 0's start / return per block, from BT_FIN on
    struct BtFin {
        unsigned long long t0 = wall_clock64();
        __device__ ~BtFin() {
            const uint32_t t = BT_FIN + blockIdx.x;
            if (threadIdx.x == 0 && t < BT_MAX) {
                gw_blocktime[3 * t] = t0;
                gw_blocktime[3 * t + 1] = wall_clock64();
                gw_blocktime[3 * t + 2] = (unsigned long long)__smid() |
                                          ((unsigned long long)__builtin_amdgcn_s_getreg(6164) << 32);
            }
        }
    } bt_fin;
#endif
    // blocks [0, nx): the next flush's tile order; block nx: the summary; then R copy blocks.  The
    // two serial kinds go first so that they overlap the copies instead of trailing them.
    const uint32_t nx = tile_order ? N_XCD : 0u, R = gridDim.x - 1 - nx;
    if (blockIdx.x < nx) {
        tile_order_block(blockIdx.x, tile_work, n_tiles, tile_order);
        return;
    }
    const uint32_t b = blockIdx.x - nx;
    if (blockIdx.x == gridDim.x - 1) {  // scalars + bbox fold (level 2 of the per-space bounding box)
        BT_STAMP(0);
        // thread t folds parts t, t + 256, ... (coalesced; the parts are in space order, so a
        // thread's spaces only move forward and it flushes a run when its space changes).  Read
        // thread-contiguous (t: parts 5t .. 5t + 4), each 20-B load instruction touched 64 lines
        // and held every block on this block's CU for up to 13 us at config 3.
        uint32_t cur = SP_DEAD;
        int v[4] = {INT_MAX, INT_MAX, INT_MIN, INT_MIN};
        constexpr uint32_t PF = 8;  // parts in flight per thread (the loads of a group before its fold)
        for (uint32_t pb = threadIdx.x; pb < np; pb += PF * BB_T) {
            BBoxPart q[PF];
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) {  // (clamped, not branched: every load in flight)
                q[u] = parts[min(pb + u * BB_T, np - 1)];
                if (pb + u * BB_T >= np) q[u].sp = SP_DEAD;
            }
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) {
                if (q[u].sp == SP_DEAD) continue;
                if (q[u].sp != cur) {
                    if (cur != SP_DEAD) bbox_flush(bbox, ns, cur, v);
                    cur = q[u].sp;
                    v[0] = v[1] = INT_MAX;
                    v[2] = v[3] = INT_MIN;
                }
                v[0] = min(v[0], q[u].v[0]);
                v[1] = min(v[1], q[u].v[1]);
                v[2] = max(v[2], q[u].v[2]);
                v[3] = max(v[3], q[u].v[3]);
            }
        }
        BT_STAMP(1);
        __shared__ BBoxPart s_fold;
        bbox_block(cur, v, bbox, ns, &s_fold);
        // The boxes: what the runs of mixed spaces flushed into bbox (the gather's atomics, and this
        // block's, complete before the barrier: each wave waits for its own) plus the fold, straight
        // into the host's summary.  bbox only accumulates one flush, so the fold need not be added
        // to it first (four atomics and a fence less on the launch's serial path).
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        BT_STAMP(2);
        const BBoxPart F = s_fold;
        if (hbbox) {
            for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
                const int *q = reinterpret_cast<const int *>(bbox + i);
                int4 r = make_int4(__hip_atomic_load(q + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                   __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                   __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                   __hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (F.sp == i) {
                    r.x = min(r.x, F.v[0]);
                    r.y = min(r.y, F.v[1]);
                    r.z = max(r.z, F.v[2]);
                    r.w = max(r.w, F.v[3]);
                }
                hbbox[i] = r;
            }
        } else if (threadIdx.x == 0 && F.sp != SP_DEAD) {
            bbox_flush(bbox, ns, F.sp, F.v);
        }
        // the scalars
        if (threadIdx.x == 0) {
            res->err = sc->err;
            // the events (the streams' lengths) and the scratch extent the pair passes needed (each
            // stream's last chunk): against the set's and the scratch's capacity
            unsigned long long ext = 0, tot = 0;
            for (uint32_t q = 0; q < EV_SHARDS; ++q) {
                const unsigned long long len = *reinterpret_cast<const unsigned long long *>(&sc->shard[q][2]);
                if (len) ext = max(ext, ev_phys(ev_enc(q, len - 1)) + 1);
                tot += len;
            }
            res->total64 = tot;
            res->ext64 = ext;
            res->seq_max = sc->seq_max;
            for (int q = 0; q < (int)DBG_N; ++q) res->dbg[q] = sc->dbg[q];
            if (n_entries == 0) {
                res->n_enter = res->n_total = 0;
                if (dcnt) dcnt[0] = dcnt[1] = 0;
            }
        }
        BT_STAMP(4);
        return;
    }
    __shared__ uint32_t s_off[FT + 1];
    __shared__ unsigned long long s_src[FT];
    const uint32_t e0 = b * FT;
    __shared__ uint32_t s_agg;
    uint32_t cnt = 0, incl = 0;
    unsigned long long src = 0;  // the tile's stream position, loaded with its total (one round trip)
    // the offset: the totals of the groups before e0's, then its group's entries before e0 (their
    // loads issued before wave 0's own scan)
    __shared__ uint32_t s_pw[256 / WAVE];
    uint32_t gsum = 0;
    {
        const uint32_t *grp = tile_total + n_entries + 1, g = e0 / FG;
        for (uint32_t q = threadIdx.x; q < g; q += blockDim.x) gsum += grp[q];
        for (uint32_t e = g * FG + threadIdx.x; e < e0; e += blockDim.x) gsum += tile_total[e];
    }
    if (threadIdx.x < WAVE) {
        const uint32_t l = lane(), e = e0 + l;
        const bool own = l < (uint32_t)FT && e < n_entries;
        cnt = own ? tile_total[e] : 0u;
        src = own ? tile_base[e] : 0ull;
        incl = wave_incl_scan(cnt);
        const uint32_t agg = __shfl(incl, WAVE - 1);
        if (l == 0) s_agg = agg;
    }
    gsum = wave_sum_u32(gsum);
    if (lane() == 0) s_pw[threadIdx.x / WAVE] = gsum;
    __syncthreads();
    uint32_t excl = 0;
    for (uint32_t q = 0; q < blockDim.x / WAVE; ++q) excl += s_pw[q];
    const uint32_t agg = s_agg;
    if (threadIdx.x < WAVE) {
        const uint32_t l = lane(), e = e0 + l;
        const uint32_t off = excl + incl - cnt;
        if (l < (uint32_t)FT) {
            s_off[l] = off;
            s_src[l] = src;
            if (e == n_enter_entries) {
                res->n_enter = off;
                if (dcnt) dcnt[0] = off;  // device copy of the counts (events read on the device before the host)
            }
        }
        if (l == 0) s_off[FT] = excl + agg;
        if (b == R - 1 && l == 0) {
            res->n_total = excl + agg;
            if (dcnt) dcnt[1] = excl + agg;
        }
    }
    __syncthreads();
    // the block's tiles fill one contiguous output range: every thread takes
    // positions tid, tid + 256, ... (increasing, so its tile index only moves
    // forward); FU positions per thread in flight: the loads before the stores
    constexpr int FU = 8;
    const uint32_t o0 = s_off[0], o1 = s_off[FT];
    uint32_t t = 0;
    // (the loads take clamped positions instead of a branch each: a load under a branch is waited
    // for before the next one issues)
    for (uint32_t p0 = o0 + threadIdx.x; p0 < o1 && cap_tmp; p0 += FU * blockDim.x) {
        unsigned long long src[FU];
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const uint32_t p = p0 + (uint32_t)u * blockDim.x;
            src[u] = cap_tmp;
            if (p < o1) {
                while (s_off[t + 1] <= p) ++t;  // last tile t with s_off[t] <= p (s_off[FT] = o1 > p)
                src[u] = ev_phys(s_src[t] + (p - s_off[t]));
            }
        }
        uint2 v[FU];
#pragma unroll
        for (int u = 0; u < FU; ++u) v[u] = tmp[src[u] < cap_tmp ? src[u] : 0ull];
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const uint32_t p = p0 + (uint32_t)u * blockDim.x;
            if (p < o1 && p < cap_out) out[p] = src[u] < cap_tmp ? v[u] : make_uint2(0u, 0u);
        }
    }
    for (uint32_t p = o0 + threadIdx.x; p < o1 && !cap_tmp; p += blockDim.x)  // (no scratch: zeros, as ever)
        if (p < cap_out) out[p] = make_uint2(0u, 0u);
}

// ------------------------------------------------------------ neighbors ------

__global__ __launch_bounds__(256) void k_neighbors(FrameView F, SlotTab info, uint32_t slot,
                                                   uint32_t *out, uint32_t cap, uint32_t *count) {
    const uint32_t a = info.rank[slot];
    if (a >= F.n || ld_ss(F.ss, a).slot != slot) return;
    const Rec16 A = ld_rec(F.rec, a);
    const SpaceGrid g = F.grid[ld_ss(F.ss, a).sp];
    const float D = g.D;
    const float mx = (fabsf(A.x) + 3.0f * D) * 0x1p-20f, mz = (fabsf(A.z) + 3.0f * D) * 0x1p-20f;
    const int cx0 = cell_of(A.x - D - mx, g.ox, g.inv, g.gx), cx1 = cell_of(A.x + D + mx, g.ox, g.inv, g.gx);
    const int cz0 = cell_of(A.z - D - mz, g.oz, g.inv, g.gz), cz1 = cell_of(A.z + D + mz, g.oz, g.inv, g.gz);
    for (int cz = cz0; cz <= cz1; ++cz) {
        const uint32_t row = g.base + (uint32_t)cz * g.gx;
        const uint32_t jb = F.cell_start[row + (uint32_t)cx0], je = F.cell_start[row + (uint32_t)cx1 + 1u];
        for (uint32_t b = jb + threadIdx.x; b < je; b += blockDim.x) {
            if (b == a) continue;
            const Rec16 B = ld_rec(F.rec, b);
            if (rel(A.x, A.z, A.s, B.x, B.z, B.s, D)) {
                const uint32_t p = atomicAdd(count, 1u);
                if (p < cap) out[p] = ld_ss(F.ss, b).slot;
            }
        }
    }
}

// ------------------------------------------------------------ event CSR ------
// The flush's directed events regrouped by their first entity (gwaoi_events_csr):
// row a = items[off[a] .. off[a+1]), an item is b (leave) or b | CSR_ENTER
// (enter), so sorting a row puts its leaves first, each part by b.
constexpr uint32_t CSR_ENTER = 0x80000000u;

__global__ void k_csr_count(const uint2 *__restrict__ ev, uint32_t n_total, uint32_t *cnt) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n_total) atomicAdd(&cnt[ev[e].x], 1u);
}

__global__ void k_csr_fill(const uint2 *__restrict__ ev, uint32_t n_enter, uint32_t n_total,
                           const uint32_t *__restrict__ off, uint32_t *cur, uint32_t *items) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_total) return;
    const uint2 p = ev[e];
    items[off[p.x] + atomicAdd(&cur[p.x], 1u)] = p.y | (e < n_enter ? CSR_ENTER : 0u);
}

// Rows are short in a steady tick (about one event per entity): one lane sorts
// a row of up to CSR_SHORT items by insertion.  Longer rows (a populate or
// teleport burst: 85-460 items at config 3, the whole crowd for co-located
// entities) are listed and sorted by a block each (k_csr_sort_long).
constexpr uint32_t CSR_SHORT = 32;
constexpr uint32_t CSR_LDS = 4096;  // items a block sorts in LDS at once (16 KB)

__global__ void k_csr_sort(const uint32_t *__restrict__ off, uint32_t n_rows, uint32_t *items, uint32_t *long_rows,
                           uint32_t *n_long) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const uint32_t b = off[r], e = off[r + 1];
    if (e - b > CSR_SHORT) {
        long_rows[atomicAdd(n_long, 1u)] = r;
        return;
    }
    for (uint32_t k = b + 1; k < e; ++k) {
        const uint32_t v = items[k];
        uint32_t j = k;
        while (j > b && items[j - 1] > v) {
            items[j] = items[j - 1];
            --j;
        }
        items[j] = v;
    }
}

// Block-wide merge of the sorted runs a[0, na) and b[0, nb) into out: thread t
// writes outputs [t * per, (t + 1) * per), its split found on the merge path.
__device__ void block_merge(const uint32_t *__restrict__ a, uint32_t na, const uint32_t *__restrict__ b, uint32_t nb,
                            uint32_t *__restrict__ out) {
    const uint32_t n = na + nb, per = (n + blockDim.x - 1) / blockDim.x;
    const uint32_t d0 = min(threadIdx.x * per, n), d1 = min(d0 + per, n);
    if (d0 >= d1) return;
    // i = items taken from a among the first d0 outputs (a wins ties: stable)
    uint32_t lo = d0 > nb ? d0 - nb : 0u, hi = min(d0, na);
    while (lo < hi) {
        const uint32_t i = (lo + hi) / 2;
        if (a[i] <= b[d0 - i - 1]) lo = i + 1;
        else hi = i;
    }
    uint32_t i = lo, j = d0 - lo;
    for (uint32_t d = d0; d < d1; ++d) out[d] = (j >= nb || (i < na && a[i] <= b[j])) ? a[i++] : b[j++];
}

__global__ __launch_bounds__(256) void k_csr_sort_long(const uint32_t *__restrict__ off, uint32_t *items,
                                                       uint32_t *scratch, const uint32_t *__restrict__ long_rows,
                                                       const uint32_t *__restrict__ n_long) {
    __shared__ uint32_t s[CSR_LDS];
    const uint32_t nl = *n_long, tid = threadIdx.x, T = blockDim.x;
    for (uint32_t q = blockIdx.x; q < nl; q += gridDim.x) {
        const uint32_t r = long_rows[q], b = off[r], len = off[r + 1] - b;
        // runs of CSR_LDS sorted in LDS (bitonic over the next power of two, padded with ~0)
        for (uint32_t c0 = 0; c0 < len; c0 += CSR_LDS) {
            const uint32_t m = min(CSR_LDS, len - c0);
            uint32_t p = 1;
            while (p < m) p <<= 1;
            for (uint32_t i = tid; i < p; i += T) s[i] = i < m ? items[b + c0 + i] : 0xFFFFFFFFu;
            __syncthreads();
            for (uint32_t k = 2; k <= p; k <<= 1)
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    for (uint32_t i = tid; i < p; i += T) {
                        const uint32_t ixj = i ^ j;
                        if (ixj > i) {
                            const uint32_t x = s[i], y = s[ixj];
                            if ((x > y) == ((i & k) == 0)) {
                                s[i] = y;
                                s[ixj] = x;
                            }
                        }
                    }
                    __syncthreads();
                }
            for (uint32_t i = tid; i < m; i += T) items[b + c0 + i] = s[i];
            __syncthreads();
        }
        // merge passes, ping-pong with the scratch
        uint32_t *src = items + b, *dst = scratch + b;
        for (uint32_t w = CSR_LDS; w < len; w <<= 1) {
            for (uint32_t lo = 0; lo < len; lo += 2 * w) {
                const uint32_t na = min(w, len - lo), nb = len - lo > w ? min(w, len - lo - w) : 0u;
                block_merge(src + lo, na, src + lo + na, nb, dst + lo);
            }
            __syncthreads();
            uint32_t *t = src;
            src = dst;
            dst = t;
        }
        if (src != items + b) {
            for (uint32_t i = tid; i < len; i += T) items[b + i] = src[i];
        }
        __syncthreads();
    }
}

}  // namespace

// ============================================================ launchers ======

void launch_events_csr(const uint32_t *ev_pairs, uint64_t n_enter, uint64_t n_total, uint32_t n_rows, uint32_t *cnt,
                       uint32_t *off, uint32_t *scan_tmp, uint32_t *items, uint32_t *scratch, uint32_t *long_rows,
                       hipStream_t st) {
    const uint2 *ev = reinterpret_cast<const uint2 *>(ev_pairs);
    k_zero<<<cdiv((size_t)n_rows + 1, 256), 256, 0, st>>>(cnt, (size_t)n_rows + 1);
    if (n_total) k_csr_count<<<cdiv(n_total, 256), 256, 0, st>>>(ev, (uint32_t)n_total, cnt);
    scan_exclusive(cnt, off, (size_t)n_rows + 1, scan_tmp, st);
    if (!n_total) return;
    k_zero<<<cdiv((size_t)n_rows + 1, 256), 256, 0, st>>>(cnt, (size_t)n_rows + 1);  // cursors + long-row count
    k_csr_fill<<<cdiv(n_total, 256), 256, 0, st>>>(ev, (uint32_t)n_enter, (uint32_t)n_total, off, cnt, items);
    k_csr_sort<<<cdiv(n_rows, 256), 256, 0, st>>>(off, n_rows, items, long_rows, cnt + n_rows);
    k_csr_sort_long<<<512, 256, 0, st>>>(off, items, scratch, long_rows, cnt + n_rows);
}

void launch_prologue(TickScalars *sc, uint32_t *z0, size_t n0, uint32_t *z1, size_t n1, int4 *bbox,
                     uint32_t n_spaces, uint32_t n_copy, const Rec16 *p_rec, const SlotSp *p_ss, Rec16 *s_rec,
                     SlotSp *s_ss, const MoveRun *mark, uint32_t max_slots, SlotTab info, uint32_t tick_id,
                     uint32_t n_unique, hipStream_t st) {
    MoveRun mk{};
    if (mark) mk = *mark;
    const size_t m = std::max<size_t>({n0, n1, (size_t)n_spaces, (size_t)n_copy, (size_t)mk.n, (size_t)EV_SHARDS * 32});
    k_prologue<<<cdiv(m, 256), 256, 0, st>>>(sc, z0, (uint32_t)n0, z1, (uint32_t)n1, bbox, n_spaces, n_copy, p_rec,
                                             p_ss, s_rec, s_ss, mk, max_slots, info, tick_id, n_unique);
}

void launch_zero(uint32_t *p, size_t n, hipStream_t st) {
    if (n) k_zero<<<cdiv(n, 256), 256, 0, st>>>(p, n);
}

void launch_init_appended(const uint32_t *new_slots, uint32_t n_app, uint32_t base, Rec16 *s_rec, SlotSp *s_ss,
                          SlotTab info, uint32_t max_slots, TickScalars *sc, hipStream_t st) {
    if (!n_app) return;
    k_init_appended<<<cdiv(n_app, 256), 256, 0, st>>>(new_slots, n_app, base, s_rec, s_ss, info, max_slots, sc);
}

void launch_moves(const MoveRuns &RS, uint32_t max_slots, SlotTab info, uint32_t tick_id, uint32_t n_total,
                  uint64_t seq_floor, Rec16 *s_rec, SlotSp *s_ss, const Rec16 *p_rec, uint32_t n_prev,
                  TickScalars *sc, uint32_t *coll, uint32_t n_marked, bool unique, hipStream_t st) {
    if (unique) {  // no claims, no fixup
        for (uint32_t q = 0; q < RS.count; ++q)
            if (RS.r[q].n)
                k_moves_apply_n<GWAOI_APPLY_PER, true, true><<<cdiv(RS.r[q].n, 256 * GWAOI_APPLY_PER), 256, 0, st>>>(
                    RS.r[q], max_slots, info, tick_id, n_total, seq_floor, s_rec, s_ss, sc, coll);
        return;
    }
    for (uint32_t q = n_marked; q < RS.count; ++q)  // every run's claims before any apply
        if (RS.r[q].n) k_moves_mark<<<cdiv(RS.r[q].n, 256), 256, 0, st>>>(RS.r[q], max_slots, info, tick_id);
    for (uint32_t q = 0; q < RS.count; ++q) {
        if (!RS.r[q].n) continue;
        if (!s_ss)  // virtual S'
            k_moves_apply_n<GWAOI_APPLY_PER, false, true><<<cdiv(RS.r[q].n, 256 * GWAOI_APPLY_PER), 256, 0, st>>>(
                RS.r[q], max_slots, info, tick_id, n_total, seq_floor, s_rec, s_ss, sc, coll);
        else
            k_moves_apply_n<GWAOI_APPLY_PER, false, false><<<cdiv(RS.r[q].n, 256 * GWAOI_APPLY_PER), 256, 0, st>>>(
                RS.r[q], max_slots, info, tick_id, n_total, seq_floor, s_rec, s_ss, sc, coll);
    }
    {
        FixupArgs F;
        F.RS = RS;
        F.max_slots = max_slots;
        F.tick = tick_id;
        F.n_total = n_total;
        F.n_prev = n_prev;
        F.seq_floor = seq_floor;
        F.info = info;
        F.s_rec = s_rec;
        F.s_ss = s_ss;
        F.p_rec = p_rec;
        F.sc = sc;
        F.coll = coll;
        k_moves_fixup<<<64, 256, 0, st>>>(F);
    }
}

uint32_t moves_buckets(uint32_t max_slots) { return cdiv(max_slots, MV_R); }

// ops per workgroup of k_mv_count / k_mv_scatter: 4 per thread, 16 once the bucket-major
// histogram (buckets x workgroups) would pass 2^20 entries
static int mv_per(uint32_t n, uint32_t nb) {
    return (size_t)nb * cdiv(std::max(n, 1u), (size_t)MV_T * 4) > (1u << 20) ? 16 : 4;
}

size_t moves_hist_elems(uint32_t n, uint32_t max_slots) {
    const uint32_t nb = moves_buckets(max_slots);
    return (size_t)nb * cdiv(std::max(n, 1u), (size_t)MV_T * mv_per(n, nb)) + 1;
}

void launch_moves_bucketed(const MoveRuns &RS, uint32_t max_slots, SlotTab info, uint32_t n_total,
                           uint64_t seq_floor, Rec16 *s_rec, SlotSp *s_ss, TickScalars *sc, uint32_t *hist,
                           uint32_t *scan_tmp, void *binned, hipStream_t st) {
    const uint32_t n = RS.count ? RS.r[RS.count - 1].j0 + RS.r[RS.count - 1].n : 0u;
    if (!n) return;
    const uint32_t nb = moves_buckets(max_slots);
    bool track = false;
    for (uint32_t q = 0; q < RS.count; ++q) track |= RS.r[q].dseq != nullptr;
    MvOp *bo = reinterpret_cast<MvOp *>(binned);
    const int per = mv_per(n, nb);
    const uint32_t G = cdiv(n, (size_t)MV_T * per);
    const size_t lds = nb * sizeof(uint32_t);
    if (per == 4) k_mv_count<4><<<G, MV_T, lds, st>>>(RS, n, max_slots, nb, hist, sc);
    else k_mv_count<16><<<G, MV_T, lds, st>>>(RS, n, max_slots, nb, hist, sc);
    scan_exclusive(hist, hist, (size_t)nb * G + 1, scan_tmp, st);
    if (per == 4) k_mv_scatter<4><<<G, MV_T, lds, st>>>(RS, n, max_slots, nb, hist, bo);
    else k_mv_scatter<16><<<G, MV_T, lds, st>>>(RS, n, max_slots, nb, hist, bo);
    k_mv_apply<<<nb, MV_T, 0, st>>>(RS, hist, G, bo, n_total, seq_floor, s_rec, s_ss, info, sc, track ? 1 : 0);
}

void launch_ops_claim(const uint32_t *slots, uint32_t n, uint32_t j0, uint32_t max_slots, SlotTab info,
                      uint32_t tick_id, TickScalars *sc, hipStream_t st) {
    if (!n) return;
    k_ops_claim<<<cdiv(n, 256), 256, 0, st>>>(slots, n, j0, max_slots, info, tick_id, sc);
}

void launch_ops_apply(const uint32_t *slots, const float *x, const float *z, const uint32_t *sp, uint32_t sp_def,
                      uint32_t n, uint32_t j0, uint32_t max_slots, SlotTab info, uint32_t tick_id, uint32_t n_total,
                      const unsigned long long *seqs, uint64_t seq0, uint64_t seq_floor, bool track_max,
                      Rec16 *s_rec, SlotSp *s_ss, TickScalars *sc, hipStream_t st) {
    if (!n) return;
    k_ops_apply<<<cdiv(n, 256), 256, 0, st>>>(slots, x, z, sp, sp_def, n, j0, max_slots, info, tick_id, n_total, seqs,
                                              seq0, seq_floor, track_max ? 1 : 0, s_rec, s_ss, sc);
}

void launch_keygen(Rec16 *s_rec, const SlotSp *s_ss, uint32_t n_total, const SpaceGrid *grid,
                   uint32_t sentinel, uint32_t *keys, uint32_t *vals, const Rec16 *p_rec, const SlotSp *p_ss,
                   const SpaceGrid *p_grid, uint32_t n_prev, float *blk, TickScalars *sc, const uint32_t *p_key,
                   unsigned long long *cnt64, uint64_t seq_base, uint32_t *special, const TickZero &tz,
                   unsigned long long *tent, hipStream_t st) {
    if (!n_total) {  // no entry: only the fold (d_rel = bmax = 0; a unique-moves apply's dropped ops and
                     // errors reach sc->err, and its error word and drop count are reset for the next flush)
        k_keygen_reduce<<<1, 1024, 0, st>>>(blk, 0u, sc);
        return;
    }
    const uint32_t nb = keygen_blocks(n_total);
    if (cnt64)
        k_keygen<true><<<nb, 256, 0, st>>>(s_rec, s_ss, n_total, grid, sentinel, keys, vals, p_rec, p_ss, p_grid,
                                           n_prev, blk, p_key, cnt64, seq_base, special, tz, tent);  // folded by incremental_sort
    else {
        k_keygen<false><<<nb, 256, 0, st>>>(s_rec, s_ss, n_total, grid, sentinel, keys, vals, p_rec, p_ss, p_grid,
                                            n_prev, blk, nullptr, nullptr, seq_base, special, tz, nullptr);
        k_keygen_reduce<<<1, 1024, 0, st>>>(blk, nb, sc);
    }
}

// k_arrive re-zeroes the counted cells (no clearing pass over cnt64)
bool scan_rezeroes_counts() { return true; }

size_t incr_sort_tmp_elems(size_t cells) { return 2 * ((size_t)cdiv(cells + 1, S64_TILE) + 1); }  // tile totals, counts

void incremental_sort(const uint32_t *keys, uint32_t n_total, uint32_t n_prev, const uint32_t *p_key,
                      const uint32_t *p_cell_start, unsigned long long *cnt64, uint32_t total_cells,
                      uint32_t sentinel, uint32_t *cell_start, uint32_t *arr_pos, uint32_t *arr_idx,
                      unsigned long long *tmp, uint32_t *perm, uint32_t *skeys, const float *blk,
                      TickScalars *sc, const SpecialJob *sp, const GatherJob *gj, hipStream_t st) {
    const size_t m = (size_t)total_cells + 1;
    const uint32_t nb = cdiv(m, S64_TILE);
    uint32_t *shift = arr_pos + m;  // the caller allocates arr_pos with 3 (total_cells + 1) words
    uint32_t *list = shift + m;  // the changed cells, per scan tile
    unsigned long long *tcnt = tmp + nb;
    unsigned long long *tent = tmp;  // keygen's entries per tile (incr_keygen_tiles)
    k_scan64<<<nb + 1, SC_T, 0, st>>>(cnt64, m, nb, tent, cell_start, arr_pos, blk,
                                      keygen_blocks(n_total), sc, p_cell_start, shift, list, tcnt);
    if (sp && sp->n_tiles) {
        const SpecialJob &J = *sp;
        k_arrive_special<<<J.n_tiles + cdiv(n_total, PT), PT, 0, st>>>(J, keys, n_total, n_prev, p_key, sentinel, arr_pos,
                                                                 arr_idx, cnt64, shift, perm, skeys);
    } else if (n_total) {
        k_arrive<<<cdiv(n_total, 256), 256, 0, st>>>(keys, n_total, n_prev, p_key, sentinel, arr_pos, arr_idx, cnt64,
                                                     shift, perm, skeys);
    }
    const MergeArgs M{p_cell_start, cell_start, keys, arr_pos, arr_idx, total_cells, n_total, sentinel,
                      perm, skeys, list, tcnt, tent};
    if (gj) k_merge_gather<<<nb, 256, 0, st>>>(M, *gj);
    else k_cell_merge<<<nb, 256, 0, st>>>(M);
}

uint32_t incr_sort_tiles(uint32_t total_cells) { return cdiv((size_t)total_cells + 1, S64_TILE); }

size_t scan_tmp_elems(size_t n) {
    if (n <= SC1_MAX) return 0;
    const size_t nb = cdiv(n, SC_TILE);
    return ((nb + 3) & ~(size_t)3) + scan_tmp_elems(nb);
}

void scan_exclusive(const uint32_t *in, uint32_t *out, size_t n, uint32_t *tmp, hipStream_t st) {
    if (!n) return;
    if (n <= SC1_MAX) {
        k_scan_single<<<1, SC1_T, 0, st>>>(in, out, n);
        return;
    }
    const size_t nb = cdiv(n, SC_TILE);
    uint32_t *sums = tmp;
    uint32_t *rest = tmp + ((nb + 3) & ~(size_t)3);
    k_scan_reduce<<<(uint32_t)nb, SC_T, 0, st>>>(in, n, sums);
    scan_exclusive(sums, sums, nb, rest, st);
    k_scan_down<<<(uint32_t)nb, SC_T, 0, st>>>(in, out, n, sums);
}

size_t radix_hist_elems(uint32_t n) { return (size_t)256 * std::max<uint32_t>(1u, cdiv(n, RS_TILE)); }

int radix_sort(SortBuffers &b, uint32_t n, int bits, hipStream_t st) {
    int cur = 0;
    if (n <= 1 || bits <= 0) return cur;
    const int passes = (bits + 7) / 8;
    const int per = (bits + passes - 1) / passes;
    const uint32_t ntiles = cdiv(n, RS_TILE);
    int shift = 0;
    for (int p = 0; p < passes; ++p) {
        const int nb = std::min(per, bits - shift);
        const size_t nh = (size_t)(1u << nb) * ntiles;
        k_rs_upsweep<<<ntiles, RS_T, 0, st>>>(b.keys[cur], n, shift, nb, b.hist, ntiles);
        scan_exclusive(b.hist, b.hist, nh, b.scan_tmp, st);
        k_rs_downsweep<<<ntiles, RS_T, 0, st>>>(b.keys[cur], b.vals[cur], b.keys[cur ^ 1], b.vals[cur ^ 1], n,
                                                shift, nb, b.hist, ntiles);
        cur ^= 1;
        shift += nb;
    }
    return cur;
}

void launch_gather(const uint32_t *perm, uint32_t n_new, uint32_t n_prev, const Rec16 *s_rec, const SlotSp *s_ss,
                   const Rec16 *p_rec, const SlotSp *p_ss, Rec16 *f_rec, SlotSp *f_ss, Rec16 *o_rec, uint4 *cand,
                   const SpaceGrid *grid, uint64_t seq_base, SlotTab info, const uint32_t *sorted_keys,
                   uint32_t sentinel, uint32_t n_total, TickScalars *sc, uint32_t *f_key, int4 *bbox,
                   uint32_t n_spaces, void *bbox_parts, hipStream_t st) {
    const uint32_t nt = std::max<uint32_t>(n_new, 1u);
    k_gather<<<cdiv(nt, 256), 256, 0, st>>>(perm, n_new, n_prev, s_rec, s_ss, p_rec, p_ss, f_rec, f_ss, o_rec, cand,
                                            grid, seq_base, info, sorted_keys, sentinel, n_total, sc, f_key, bbox,
                                            n_spaces, reinterpret_cast<BBoxPart *>(bbox_parts));
}

void launch_cell_count(const uint32_t *sorted_keys, uint32_t n, uint32_t *cnt, hipStream_t st) {
    if (!n) return;
    k_cell_count<<<cdiv(n, 256), 256, 0, st>>>(sorted_keys, n, cnt);
}

void launch_pairs(FrameView F, const Rec16 *O_rec, const SlotSp *O_ss, uint64_t seq_base, TickScalars *sc,
                  uint32_t *tmp_pairs, uint64_t cap, uint32_t *tile_total, unsigned long long *tile_base,
                  uint32_t tile_off, uint32_t leave_off, const uint32_t *special, hipStream_t st) {
    if (!F.n) return;
    uint2 *tmp = reinterpret_cast<uint2 *>(tmp_pairs);
    k_pairs<1><<<combined_blocks(F.n), PT, 0, st>>>(F, O_rec, O_ss, seq_base, sc, sc, tmp, cap, tile_total,
                                                    tile_base, tile_off, leave_off, sc->dbg, special);
}

void launch_combined(FrameView F, const uint4 *cand, const Rec16 *O_rec, uint64_t seq_base, TickScalars *sc,
                     uint32_t *tmp_pairs, uint64_t cap, uint32_t *tile_total, unsigned long long *tile_base,
                     uint32_t leave_off, const uint32_t *tile_order, uint32_t *tile_work, uint8_t *ework,
                     hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
    if (!F.n) return;
    // hipExtLaunchKernelGGL records the events at the kernel's own start and
    // end: no marker packets between kernels when the stage is timed
    const uint32_t tiles = combined_tiles(F.n);
    hipExtLaunchKernelGGL(k_combined, dim3(N_XCD * range_max(tiles)),
                          dim3(CT), 0, st, ev0, ev1, 0, F, cand, O_rec,
                          (unsigned long long)seq_base, (const TickScalars *)sc, sc,
                          reinterpret_cast<uint2 *>(tmp_pairs), cap, tile_total, tile_base, leave_off, sc->dbg,
                          tile_order, tile_work, ework, tiles);
}

// One event of each mirrored pair ((a,b) at an even index, (b,a) after it) into pinned host memory:
// dst[k] = ev[2k], half the bytes of the directed list over PCIe.
__global__ __launch_bounds__(256) void k_pairs_out(const uint4 *__restrict__ ev4, uint64_t n2, uint4 *dst4,
                                                   const uint2 *__restrict__ ev2, uint2 *dst2, uint64_t n_pairs) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n2; k += stride) {
        const uint4 a = ev4[2 * k], b = ev4[2 * k + 1];  // ev[4k .. 4k+3]: two pairs
        dst4[k] = make_uint4(a.x, a.y, b.x, b.y);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && (n_pairs & 1u)) dst2[n_pairs - 1] = ev2[2 * (n_pairs - 1)];
}

void launch_pairs_out(const void *events, uint64_t n_pairs, void *dst, hipStream_t st) {
    if (!n_pairs) return;
    const uint64_t n2 = n_pairs / 2;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(cdiv(n2, 256 * 8), 1), 64);
    k_pairs_out<<<blocks, 256, 0, st>>>(static_cast<const uint4 *>(events), n2, static_cast<uint4 *>(dst),
                                        static_cast<const uint2 *>(events), static_cast<uint2 *>(dst), n_pairs);
}

size_t tile_total_elems(size_t n_entries) { return n_entries + 1 + cdiv(n_entries, FG); }

void launch_finish(const uint32_t *tile_total, const unsigned long long *tile_base, uint32_t n_entries,
                   uint32_t n_enter_entries, const uint32_t *tmp_pairs,
                   uint32_t *out_pairs, uint64_t cap_tmp, uint64_t cap_out, const TickScalars *sc, TickOut *out,
                   uint32_t n_new, int4 *bbox, uint32_t n_spaces, void *parts_mem, uint32_t np, int4 *hbbox,
                   const uint32_t *tile_work, uint32_t *tile_order, uint32_t *dcount, hipStream_t st) {
    const uint32_t R = cdiv(n_entries, FT);
    if (!n_new) tile_order = nullptr;
    k_finish<<<R + 1 + (tile_order ? N_XCD : 0u), 256, 0, st>>>(
        tile_total, tile_base, n_entries, n_enter_entries, reinterpret_cast<const uint2 *>(tmp_pairs),
        reinterpret_cast<uint2 *>(out_pairs), cap_tmp, cap_out, sc, out, reinterpret_cast<const BBoxPart *>(parts_mem),
        np, bbox,
        n_spaces, hbbox, tile_work, combined_tiles(n_new), tile_order, dcount);
}

size_t bbox_part_bytes(uint32_t n) { return sizeof(BBoxPart) * ((size_t)gather_parts(n) + 2); }
uint32_t gather_parts(uint32_t n) { return cdiv(std::max(n, 1u), 256); }  // k_gather's blocks

void launch_neighbors(FrameView F, SlotTab info, uint32_t slot, uint32_t *out, uint32_t cap,
                      uint32_t *count, hipStream_t st) {
    k_neighbors<<<1, 256, 0, st>>>(F, info, slot, out, cap, count);
}

}  // namespace gw

#ifdef GWAOI_EXP_BLOCKTIME
extern "C" __attribute__((visibility("default"))) int gwaoi_debug_blocktime(unsigned long long *host, size_t n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(gw::gw_blocktime), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif
