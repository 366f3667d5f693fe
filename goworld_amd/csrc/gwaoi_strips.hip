// gwaoi_strips.hip -- strip tiling of one oversized space over several GPUs
// (include/gwaoi_strips.h; BASELINE config 5).
//
// A strip rank keeps, per global slot, the entity's state as this rank last
// saw it (cur) and, for the tick in progress, the state before it (prv,
// valid when ptick == tick).  "Present" = inside this rank's region
// [edge_lo - H, edge_hi + H) and in the space; absent records have NaN x.
//
// Kernels (all one-lane-per-record, 256-thread blocks, stable block-scan
// compaction so that every output order is deterministic):
//   k_route      owner side: op -> halo records per destination + teleports,
//                plus the ENTER / LEAVE counts and Enter box per destination
//   k_recv       receiver side: records -> world ops [moves | enters | leaves]
//                (device batches) + per-slot state update
//   k_tele_mark  mark this tick's teleporters
//   k_filter     keep the world events this strip owns (count read on the
//                device, so it is queued behind the world's flush)
//   k_tele_pairs teleporter x teleporter pairs decided from before/after states
// The exchange between ranks is the caller's (goworld_amd/strips.py: counts
// on the host, records point to point over RCCL).
//
// Host waits: one per tick.  gwaoi_strips_route waits for its counts, and the
// same wait completes the previous tick (queued by gwaoi_strips_tick_async:
// the receive, the world's device Enter/Leave/Moved batches, its flush, the
// filter), whose results are then read from pinned memory.

#include "gwaoi_internal.h"
#include "../../include/gwaoi_strips.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <vector>

using gw::Rec16;

namespace {

constexpr int BT = 256;
constexpr int WV = 64;
constexpr int NW = BT / WV;

constexpr uint32_t SE_STATE = 1u;     // op for an entity this strip does not own / record for a slot in the wrong state
constexpr uint32_t SE_NONFINITE = 2u;
constexpr uint32_t SE_BADSLOT = 4u;
constexpr uint32_t SE_KIND = 8u;
constexpr uint32_t SE_COUNT = 16u;    // the records' kinds disagree with the announced counts

struct StripGeo {
    uint32_t S, rank;
    float H, tele, D;
    uint32_t max_slots;
    float edge[GWAOI_MAX_STRIPS];  // S-1 interior edges
    float rlo[GWAOI_MAX_STRIPS];   // region of strip q: [rlo[q], rhi[q])
    float rhi[GWAOI_MAX_STRIPS];
};

__device__ __forceinline__ uint32_t strip_of(const StripGeo &g, float x) {
    uint32_t q = 0;
    for (uint32_t i = 0; i + 1 < g.S; ++i) q += (x >= g.edge[i]) ? 1u : 0u;
    return q;
}

__device__ __forceinline__ unsigned long long region_mask(const StripGeo &g, float x) {
    unsigned long long m = 0;
    for (uint32_t q = 0; q < g.S; ++q)
        if (x >= g.rlo[q] && x < g.rhi[q]) m |= 1ull << q;
    return m;
}

__device__ __forceinline__ bool present(const Rec16 &r) { return !isnan(r.x); }

__device__ __forceinline__ Rec16 ld16(const Rec16 *p, uint32_t i) {
    const uint4 q = reinterpret_cast<const uint4 *>(p)[i];
    Rec16 r;
    r.x = __uint_as_float(q.x);
    r.z = __uint_as_float(q.y);
    r.s = ((unsigned long long)q.w << 32) | q.z;
    return r;
}
__device__ __forceinline__ void st16(Rec16 *p, uint32_t i, const Rec16 &r) {
    reinterpret_cast<uint4 *>(p)[i] =
        make_uint4(__float_as_uint(r.x), __float_as_uint(r.z), (uint32_t)r.s, (uint32_t)(r.s >> 32));
}
__device__ __forceinline__ Rec16 absent_rec() {
    Rec16 r;
    r.x = r.z = __int_as_float(0x7FC00000);
    r.s = 0;
    return r;
}

// go-aoi window test of the closed form (same operand
// order as the world kernels): W = the one whose Enter/Moved came last.
__device__ __forceinline__ bool rel(const Rec16 &a, const Rec16 &b, float D) {
    const bool own = a.s > b.s;
    const float wx = own ? a.x : b.x, wz = own ? a.z : b.z;
    const float px = own ? b.x : a.x, pz = own ? b.z : a.z;
    return (int)(px >= wx - D) & (int)(px <= wx + D) & (int)(pz >= wz - D) & (int)(pz <= wz + D);
}

__device__ __forceinline__ unsigned long long lanemask_lt() { return (1ull << __lane_id()) - 1ull; }

// Block-level stable multi-split: every lane holds a destination mask over K
// classes (K <= 65); class extra_q takes its bit from `extra`.  Phase 0 writes the block's per-class counts to
// counts[q*nb + blk]; phase 1 returns, through `pos`, each lane's output
// index for class q (offs = exclusive scan of counts) via the callback.
template <class Emit>
__device__ __forceinline__ void multisplit(int phase, unsigned long long mask, bool extra, uint32_t extra_q, uint32_t K,
                                           uint32_t *counts, const uint32_t *offs, uint32_t nb, Emit emit) {
    __shared__ uint32_t cnt[GWAOI_MAX_STRIPS + 1][NW];
    const uint32_t w = threadIdx.x / WV;
    for (uint32_t q = 0; q < K; ++q) {
        const bool in = q == extra_q ? extra : (bool)((mask >> q) & 1ull);
        const unsigned long long b = __ballot(in);
        if (__lane_id() == 0) cnt[q][w] = (uint32_t)__popcll(b);
    }
    __syncthreads();
    if (phase == 0) {
        for (uint32_t q = threadIdx.x; q < K; q += BT) {
            uint32_t t = 0;
            for (int k = 0; k < NW; ++k) t += cnt[q][k];
            counts[(size_t)q * nb + blockIdx.x] = t;
        }
        return;
    }
    for (uint32_t q = 0; q < K; ++q) {
        const bool in = q == extra_q ? extra : (bool)((mask >> q) & 1ull);
        const unsigned long long b = __ballot(in);
        if (!in) continue;
        uint32_t base = offs[(size_t)q * nb + blockIdx.x];
        for (uint32_t k = 0; k < w; ++k) base += cnt[q][k];
        emit(q, base + (uint32_t)__popcll(b & lanemask_lt()));
    }
}

// Per-destination kind statistics of a route (and of a receiver's records): the
// ENTER and LEAVE records and the box of the ENTER positions.  The host needs
// them to queue its world's device Enter / Leave batches without reading the
// records back (gwaoi_enter_batch_device sizes the grid from the box).
constexpr int KS = 6;  // enters, leaves, box x0, z0, x1, z1 (ordered ints)

__device__ __forceinline__ int f2o(float f) {
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7FFFFFFF;
}

__global__ void k_kstat_init(int *ks, uint32_t n) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    int *k = ks + (size_t)q * KS;
    k[0] = k[1] = 0;
    k[2] = k[3] = INT_MAX;
    k[4] = k[5] = INT_MIN;
}

// Block-level accumulation of kind statistics over up to GWAOI_MAX_STRIPS classes: every lane
// adds its few ENTER / LEAVE records (rare: entities crossing a region boundary) in LDS, then
// one thread per class folds the block's figures into the global ones.
struct KindLds {
    int k[GWAOI_MAX_STRIPS][KS];
};
__device__ __forceinline__ void kind_init(KindLds &L, uint32_t K) {
    for (uint32_t i = threadIdx.x; i < K * KS; i += blockDim.x) {
        const uint32_t c = i % KS;
        L.k[i / KS][c] = c < 2 ? 0 : (c < 4 ? INT_MAX : INT_MIN);
    }
}
__device__ __forceinline__ void kind_add(KindLds &L, unsigned long long ent, unsigned long long lev, float x, float z) {
    while (ent) {
        const int q = __ffsll((long long)ent) - 1;
        ent &= ent - 1;
        atomicAdd(&L.k[q][0], 1);
        atomicMin(&L.k[q][2], f2o(x));
        atomicMin(&L.k[q][3], f2o(z));
        atomicMax(&L.k[q][4], f2o(x));
        atomicMax(&L.k[q][5], f2o(z));
    }
    while (lev) {
        const int q = __ffsll((long long)lev) - 1;
        lev &= lev - 1;
        atomicAdd(&L.k[q][1], 1);
    }
}
__device__ __forceinline__ void kind_flush(const KindLds &L, uint32_t K, int *ks) {
    for (uint32_t q = threadIdx.x; q < K; q += blockDim.x) {
        if (!L.k[q][0] && !L.k[q][1]) continue;
        int *g = ks + (size_t)q * KS;
        if (L.k[q][0]) {
            atomicAdd(g + 0, L.k[q][0]);
            atomicMin(g + 2, L.k[q][2]);
            atomicMin(g + 3, L.k[q][3]);
            atomicMax(g + 4, L.k[q][4]);
            atomicMax(g + 5, L.k[q][5]);
        }
        if (L.k[q][1]) atomicAdd(g + 1, L.k[q][1]);
    }
}

// ---- owner side: classes 0..S-1 = destination ranks, S = teleports.  Phase 0 also gathers the
// kind statistics per destination (ks).
__global__ void __launch_bounds__(BT) k_route(int phase, const gwaoi_halo_rec *__restrict__ ops, uint32_t n,
                                              const Rec16 *__restrict__ cur, StripGeo g, uint32_t *counts,
                                              const uint32_t *__restrict__ offs, uint32_t nb, uint32_t *err,
                                              gwaoi_halo_rec *send, gwaoi_tele_rec *tele, int *ks) {
    __shared__ KindLds KL;
    if (phase == 0) kind_init(KL, g.S);
    const uint32_t i = blockIdx.x * BT + threadIdx.x;
    unsigned long long mP = 0, mN = 0;
    bool tp = false;
    gwaoi_halo_rec op{};
    Rec16 pv = absent_rec(), nw = absent_rec();
    if (i < n) {
        op = ops[i];
        uint32_t e = 0;
        if (op.slot >= g.max_slots) {
            e = SE_BADSLOT;
        } else {
            pv = ld16(cur, op.slot);
            const bool have = present(pv);
            const bool mine = have && strip_of(g, pv.x) == g.rank;
            if (op.kind == GWAOI_HALO_MOVE || op.kind == GWAOI_HALO_ENTER) {
                nw.x = op.x;
                nw.z = op.z;
                nw.s = op.seq;
                if (!isfinite(op.x) || !isfinite(op.z)) e = SE_NONFINITE;
                else if (op.kind == GWAOI_HALO_MOVE ? !mine : (have || strip_of(g, op.x) != g.rank)) e = SE_STATE;
            } else if (op.kind == GWAOI_HALO_LEAVE) {
                if (!mine) e = SE_STATE;
            } else {
                e = SE_KIND;
            }
        }
        if (e) {
            if (phase == 0) atomicOr(err, e);
        } else {
            if (op.kind != GWAOI_HALO_ENTER) mP = region_mask(g, pv.x);
            if (op.kind != GWAOI_HALO_LEAVE) mN = region_mask(g, nw.x);
            tp = op.kind == GWAOI_HALO_MOVE && fabsf(nw.x - pv.x) > g.tele;
        }
    }
    if (phase == 0) {
        __syncthreads();  // KL initialised
        kind_add(KL, mN & ~mP, mP & ~mN, nw.x, nw.z);
    }
    if (phase == 0 && i == 0) counts[(size_t)(g.S + 1) * nb] = 0;
    multisplit(phase, mP | mN, tp, g.S, g.S + 1, counts, offs, nb, [&](uint32_t q, uint32_t pos) {
        if (q < g.S) {
            const bool inP = (mP >> q) & 1ull, inN = (mN >> q) & 1ull;
            gwaoi_halo_rec r;
            r.slot = op.slot;
            r.kind = inP && inN ? GWAOI_HALO_MOVE : (inN ? GWAOI_HALO_ENTER : GWAOI_HALO_LEAVE);
            const Rec16 &src = inN ? nw : pv;
            r.x = src.x;
            r.z = src.z;
            r.seq = src.s;
            send[pos] = r;
        } else {
            gwaoi_tele_rec t;
            t.slot = op.slot;
            t.flags = 3u;
            t.px = pv.x;
            t.pz = pv.z;
            t.pseq = pv.s;
            t.x = nw.x;
            t.z = nw.z;
            t.seq = nw.s;
            tele[pos - offs[(size_t)g.S * nb]] = t;
        }
    });
    if (phase == 0) {
        __syncthreads();  // (multisplit's barrier orders the adds too; explicit for clarity)
        kind_flush(KL, g.S, ks);
    }
}

// ---- receiver side: classes 0 = world device moves, 1 = enters, 2 = leaves.  Every record is
// emitted by its kind, so that the classes have exactly the sizes the senders' kind statistics
// announced (the host queued the world batches with them); a record in the wrong state is
// flagged (err), never dropped.  Output: one SoA array set [moves | enters | leaves].  Phase 0
// also gathers the kind statistics (ks: one class) for gwaoi_strips_tick, which has no announced
// counts.
__global__ void __launch_bounds__(BT) k_recv(int phase, const gwaoi_halo_rec *__restrict__ lv, uint32_t n_local,
                                             const gwaoi_halo_rec *__restrict__ rv, uint32_t n, Rec16 *cur,
                                             Rec16 *prv, uint32_t *ptick, uint32_t tick, uint32_t max_slots,
                                             uint32_t *counts, const uint32_t *__restrict__ offs, uint32_t nb,
                                             uint32_t *err, uint32_t *m_slot, float *m_x, float *m_z,
                                             unsigned long long *m_seq, int *ks) {
    __shared__ KindLds KL;
    if (phase == 0 && ks) kind_init(KL, 1);
    const uint32_t i = blockIdx.x * BT + threadIdx.x;
    unsigned long long m = 0;
    gwaoi_halo_rec r{};
    if (i < n) {  // this rank's own records first, then the received ones
        r = i < n_local ? lv[i] : rv[i - n_local];
        uint32_t e = 0;
        if (r.slot >= max_slots) {
            e = SE_BADSLOT;
        } else if (r.kind > GWAOI_HALO_LEAVE) {
            e = SE_KIND;
        } else {
            const Rec16 c = ld16(cur, r.slot);
            if ((r.kind == GWAOI_HALO_ENTER) == present(c)) e = SE_STATE;  // a sender sends one record per slot
            if (phase == 1 && !e) {
                prv[r.slot] = c;
                ptick[r.slot] = tick;
                Rec16 nw = absent_rec();
                if (r.kind != GWAOI_HALO_LEAVE) {
                    nw.x = r.x;
                    nw.z = r.z;
                    nw.s = r.seq;
                }
                st16(cur, r.slot, nw);
            }
        }
        if (e && phase == 0) atomicOr(err, e);
        // a record of no known kind counts as a move on the host (n_move = all - enters - leaves):
        // it goes into class 0 as a no-op placeholder (SLOT_NONE), so the world's move batch never
        // reads a word this tick did not write
        if (r.kind <= GWAOI_HALO_LEAVE) m = 1ull << r.kind;
        else {
            m = 1ull;
            r.slot = gw::SLOT_NONE;
        }
    }
    if (phase == 0 && ks) {
        __syncthreads();
        kind_add(KL, m >> 1 & 1ull, m >> 2 & 1ull, r.x, r.z);
    }
    if (phase == 0 && i == 0) counts[3 * nb] = 0;
    multisplit(phase, m, false, 0xFFFFFFFFu, 3, counts, offs, nb, [&](uint32_t, uint32_t pos) {
        m_slot[pos] = r.slot;
        m_x[pos] = r.x;
        m_z[pos] = r.z;
        m_seq[pos] = r.seq;
    });
    if (phase == 0 && ks) {
        __syncthreads();
        kind_flush(KL, 1, ks);
    }
}

// The receiver's class sizes against the counts the host queued the world batches with.
__global__ void k_recv_check(const uint32_t *__restrict__ offs, uint32_t nb, uint32_t n_move, uint32_t n_ent,
                             uint32_t n_lev, uint32_t *err) {
    if (threadIdx.x == 0 && (offs[nb] != n_move || offs[2 * nb] - offs[nb] != n_ent ||
                             offs[3 * nb] - offs[2 * nb] != n_lev))
        atomicOr(err, SE_COUNT);
}

__global__ void k_tele_mark(const gwaoi_tele_rec *__restrict__ t, uint32_t n, uint32_t *ttick, uint32_t tick,
                            uint32_t max_slots) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && t[i].slot < max_slots) ttick[t[i].slot] = tick;
}

__device__ __forceinline__ Rec16 before(const Rec16 *cur, const Rec16 *prv, const uint32_t *ptick, uint32_t s,
                                        uint32_t tick) {
    return ptick[s] == tick ? ld16(prv, s) : ld16(cur, s);
}

// ---- keep the world events this strip owns: class 0 enters (owner after the
// tick), class 1 leaves (owner before the tick); teleporter pairs are dropped
// here and decided by k_tele_pairs.  The event count is read on the device
// (dcnt = {n_enter, n_total}, written by the world flush's k_finish, clipped to
// cap): the filter is queued behind the flush without a host round trip.  Block
// b takes one contiguous chunk of the events, BT at a time; phase 0 counts per
// class, phase 1 writes at the scanned offsets (counts[q * G + b]).
__global__ void __launch_bounds__(BT) k_filter(int phase, const uint2 *__restrict__ ev,
                                               const uint32_t *__restrict__ dcnt, uint64_t cap,
                                               const Rec16 *__restrict__ cur, const Rec16 *__restrict__ prv,
                                               const uint32_t *__restrict__ ptick, const uint32_t *__restrict__ ttick,
                                               uint32_t tick, StripGeo g, uint32_t *counts,
                                               const uint32_t *__restrict__ offs,
                                               const unsigned long long *__restrict__ tcnt, uint2 *out, uint64_t ocap) {
    __shared__ uint32_t cnt[2][NW];
    const uint32_t G = gridDim.x, b = blockIdx.x, w = threadIdx.x / WV;
    const uint32_t n = (uint32_t)min((uint64_t)dcnt[1], cap), ne = min(dcnt[0], n);
    const uint32_t per = (uint32_t)(((uint64_t)n + (uint64_t)G * BT - 1) / ((uint64_t)G * BT)) * BT;
    const uint32_t lo = (uint32_t)min((uint64_t)b * per, (uint64_t)n), hi = (uint32_t)min((uint64_t)lo + per, (uint64_t)n);
    // phase 1: the teleporter enters go between the filter's enters and leaves
    const uint32_t gap = phase == 1 && tcnt ? (uint32_t)tcnt[0] : 0u;
    uint32_t base0 = phase == 1 ? offs[b] : 0u, base1 = phase == 1 ? offs[G + b] + gap : 0u;
    for (uint32_t i0 = lo; i0 < hi; i0 += BT) {
        const uint32_t i = i0 + threadIdx.x;
        bool k0 = false, k1 = false;
        uint2 p = make_uint2(0, 0);
        if (i < hi) {
            p = ev[i];
            const bool is_enter = i < ne;
            const bool tt = ttick[p.x] == tick && ttick[p.y] == tick;
            if (!tt) {
                const Rec16 a = is_enter ? ld16(cur, p.x) : before(cur, prv, ptick, p.x, tick);
                const bool own = present(a) && strip_of(g, a.x) == g.rank;
                k0 = own && is_enter;
                k1 = own && !is_enter;
            }
        }
        const unsigned long long b0 = __ballot(k0), b1 = __ballot(k1);
        if (__lane_id() == 0) {
            cnt[0][w] = (uint32_t)__popcll(b0);
            cnt[1][w] = (uint32_t)__popcll(b1);
        }
        __syncthreads();
        uint32_t t0 = 0, t1 = 0, p0 = 0, p1 = 0;
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)NW; ++k) {
            if (k < w) {
                p0 += cnt[0][k];
                p1 += cnt[1][k];
            }
            t0 += cnt[0][k];
            t1 += cnt[1][k];
        }
        if (phase == 1) {  // (past ocap: counted, not written; the host re-runs the filter with room)
            const uint64_t q0 = (uint64_t)base0 + p0 + (uint32_t)__popcll(b0 & lanemask_lt());
            const uint64_t q1 = (uint64_t)base1 + p1 + (uint32_t)__popcll(b1 & lanemask_lt());
            if (k0 && q0 < ocap) out[q0] = p;
            if (k1 && q1 < ocap) out[q1] = p;
        }
        base0 += t0;
        base1 += t1;
        __syncthreads();  // cnt is rewritten by the next step
    }
    if (phase == 0 && threadIdx.x == 0) {
        counts[b] = base0;
        counts[G + b] = base1;
        if (b == 0) counts[2 * G] = 0;
    }
}

// ---- teleporter x teleporter: phase 0 counts, phase 1 writes (atomic slots;
// the pairs are few and their order is not part of the contract).
__global__ void k_tele_pairs(int phase, const gwaoi_tele_rec *__restrict__ t, uint32_t n, StripGeo g,
                             unsigned long long *cnt, uint2 *ent, uint2 *lev, unsigned long long cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const gwaoi_tele_rec A = t[i];
    Rec16 ap, an;
    ap.x = A.px; ap.z = A.pz; ap.s = A.pseq;
    an.x = A.x; an.z = A.z; an.s = A.seq;
    const bool own_now = (A.flags & 2u) && strip_of(g, an.x) == g.rank;
    const bool own_before = (A.flags & 1u) && strip_of(g, ap.x) == g.rank;
    if (!own_now && !own_before) return;
    uint32_t ce = 0, cl = 0;
    for (uint32_t j = 0; j < n; ++j) {
        if (j == i) continue;
        const gwaoi_tele_rec B = t[j];
        Rec16 bp, bn;
        bp.x = B.px; bp.z = B.pz; bp.s = B.pseq;
        bn.x = B.x; bn.z = B.z; bn.s = B.seq;
        const bool was = (A.flags & 1u) && (B.flags & 1u) && rel(ap, bp, g.D);
        const bool is = (A.flags & 2u) && (B.flags & 2u) && rel(an, bn, g.D);
        if (own_now && is && !was) {
            if (phase == 1) {
                const unsigned long long k = atomicAdd(&cnt[0], 1ull);
                if (k < cap) ent[k] = make_uint2(A.slot, B.slot);
            }
            else ++ce;
        }
        if (own_before && was && !is) {
            if (phase == 1) {
                const unsigned long long k = atomicAdd(&cnt[1], 1ull);
                if (k < cap) lev[k] = make_uint2(A.slot, B.slot);
            }
            else ++cl;
        }
    }
    if (phase == 0) {
        if (ce) atomicAdd(&cnt[0], (unsigned long long)ce);
        if (cl) atomicAdd(&cnt[1], (unsigned long long)cl);
    }
}

// The teleporter pairs next to the filtered events, all offsets read on the device:
// out = [filter enters (fe) | tele enters (te) | filter leaves (fl) | tele leaves (tl)],
// fe = offs[nb], fe + fl = offs[2 nb] (the filter's scanned counts).
__global__ void k_tele_place(const uint32_t *__restrict__ offs, uint32_t nb, const unsigned long long *__restrict__ tcnt,
                             const uint2 *__restrict__ tent, const uint2 *__restrict__ tlev, uint2 *out, uint64_t ocap) {
    const uint32_t fe = offs[nb], fl = offs[2 * nb] - fe;
    const uint32_t te = (uint32_t)tcnt[0], tl = (uint32_t)tcnt[1];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < max(te, tl); i += gridDim.x * blockDim.x) {
        if (i < te && (uint64_t)fe + i < ocap) out[fe + i] = tent[i];
        if (i < tl && (uint64_t)fe + te + fl + i < ocap) out[fe + te + fl + i] = tlev[i];
    }
}

// The tick's result for the host: small[0] = filter enters, [1] = filter leaves,
// [2] = tele enters, [3] = tele leaves, [4] = err.
__global__ void k_tick_totals(const uint32_t *__restrict__ offs, uint32_t nb, const unsigned long long *__restrict__ tcnt,
                              const uint32_t *__restrict__ err, uint32_t *small) {
    if (threadIdx.x == 0) {
        small[0] = offs[nb];
        small[1] = offs[2 * nb] - offs[nb];
        small[2] = (uint32_t)tcnt[0];
        small[3] = (uint32_t)tcnt[1];
        small[4] = *err;
    }
}

// totals of a K-class multisplit: small[q] = offs[q*nb] for q = 0..K, small[K+1] = err
__global__ void k_totals(const uint32_t *offs, uint32_t K, uint32_t nb, const uint32_t *err, uint32_t *small) {
    const uint32_t q = threadIdx.x;
    if (q <= K) small[q] = offs[(size_t)q * nb];
    if (q == 0) small[K + 1] = *err;
}

inline uint32_t cdivu(size_t a, size_t b) { return (uint32_t)((a + b - 1) / b); }

// This strip's count row (gwaoi_strips_route_begin): [records to each strip (S) | teleports |
// per destination: ENTER, LEAVE, ENTER box x0 z0 x1 z1 (KS ints each) | route error word].
inline uint32_t row_words(uint32_t S) { return S + 1 + S * 6 + 1; }
__global__ void k_route_row(const uint32_t *__restrict__ small, const int *__restrict__ kstat, uint32_t S,
                            uint32_t *row) {
    const uint32_t K = S + 1, words = K + S * 6 + 1;
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) {
        if (i < K) row[i] = small[i + 1] - small[i];
        else if (i < K + S * 6) row[i] = (uint32_t)kstat[i - K];
        else row[i] = small[K + 1];
    }
}

float o2f(int i) {
    const int b = i >= 0 ? i : i ^ 0x7FFFFFFF;
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}

constexpr uint64_t TELE_PAIRS_MAX = 1ull << 22;  // bound n (n-1) per kind sized without a count (n_tele <= 2048)
constexpr uint32_t FILTER_BLOCKS = 1024;         // k_filter's grid (chunks of the world's events)
// pinned / device scalar regions (uint32 words)
constexpr size_t SM_ROUTE = 0;                                  // route totals: K + 2
constexpr size_t SM_KIND = 128;                                 // route kind statistics: KS per destination
constexpr size_t SM_TICK = SM_KIND + KS * GWAOI_MAX_STRIPS;     // the tick's result (k_tick_totals): 5
constexpr size_t SM_RECV = SM_TICK + 8;                         // gwaoi_strips_tick: receive totals 4 + kinds KS
constexpr size_t SM_WORDS = SM_RECV + 16;

}  // namespace

struct gwaoi_strips {
    gwaoi_world *w = nullptr;
    bool broken = false;  // a failed asynchronous tick (complete_or_break)
    std::string broken_msg;
    uint32_t space = 0;
    hipStream_t st = nullptr;
    StripGeo geo{};
    uint32_t max_slots = 0;
    Rec16 *cur = nullptr, *prv = nullptr;
    uint32_t *ptick = nullptr, *ttick = nullptr;
    uint32_t tick = 0;
    // multisplit scratch
    uint32_t *counts = nullptr, *scan_tmp = nullptr, *err = nullptr, *small_d = nullptr;
    size_t counts_cap = 0, scan_cap = 0;
    // the filter's own multisplit scratch and the tick's error word: a filter re-run (after the
    // world regrew its events) happens inside the next route, whose counts and error word it
    // must leave alone
    uint32_t *fcounts = nullptr, *fscan_tmp = nullptr, *terr = nullptr;
    size_t fcounts_cap = 0, fscan_cap = 0;
    uint32_t *small_h = nullptr;  // pinned, SM_WORDS
    int *kstat = nullptr;         // device kind statistics: route (GWAOI_MAX_STRIPS x KS), receive (KS)
    // route state
    const gwaoi_halo_rec *r_ops = nullptr;
    uint32_t r_n = 0, r_nb = 0;
    bool routed = false;
    bool kinds_valid = false;
    bool row_pending = false;     // gwaoi_strips_route_begin queued, its _end not called yet
    uint32_t *row_h = nullptr;    // pinned: every strip's count row (gwaoi_strips_route_end)
    // received records as world ops, SoA [moves | enters | leaves]
    uint32_t *m_slot = nullptr;
    float *m_x = nullptr, *m_z = nullptr;
    unsigned long long *m_seq = nullptr;
    size_t m_cap = 0;
    // teleporter pairs
    unsigned long long *tcnt = nullptr;
    uint2 *tpairs = nullptr;
    size_t tpairs_cap = 0;
    // this strip's events
    uint2 *out = nullptr;
    size_t out_cap = 0;
    uint64_t n_enter = 0, n_leave = 0;
    uint32_t *h_events = nullptr;
    size_t h_cap = 0;
    // a tick queued by gwaoi_strips_tick_async, completed by the next host wait
    bool pending = false;
    uint64_t pend_tcap = 0;     // its teleporter-pair buffers (for a filter re-run)
    uint64_t pend_regrows = 0;  // the world's event regrows before its flush
    uint64_t pend_ocap = 0;     // the output capacity its filter was launched with
    uint64_t last_kept = 0;     // events the last completed tick kept (sizes the output)
    uint64_t waits = 0;         // host waits (stream synchronisations) so far
    std::string last_error;
};

namespace {

#define S_TRY(expr)                                                          \
    do {                                                                     \
        hipError_t e_ = (expr);                                              \
        if (e_ != hipSuccess) {                                              \
            s->last_error = std::string(#expr) + ": " + hipGetErrorString(e_); \
            return GWAOI_EDEVICE;                                            \
        }                                                                    \
    } while (0)

int wait(gwaoi_strips *s) {
    s->waits++;
    S_TRY(hipStreamSynchronize(s->st));
    return GWAOI_OK;
}

template <class T>
int grow(gwaoi_strips *s, T **p, size_t &cap, size_t need) {
    if (need <= cap && *p) return GWAOI_OK;
    const size_t c = std::max<size_t>({need + need / 4, cap * 2, 256});
    if (int rc = wait(s)) return rc;  // nothing queued may still use the old buffer
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc((void **)p, c * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        s->last_error = std::string("hipMalloc: ") + hipGetErrorString(e);
        return e == hipErrorOutOfMemory ? GWAOI_ENOMEM : GWAOI_EDEVICE;
    }
    cap = c;
    return GWAOI_OK;
}

int ensure_split(gwaoi_strips *s, uint32_t K, uint32_t nb) {
    const size_t n = (size_t)K * nb + 1;
    if (int rc = grow(s, &s->counts, s->counts_cap, n)) return rc;
    if (int rc = grow(s, &s->scan_tmp, s->scan_cap, gw::scan_tmp_elems(n) + 16)) return rc;
    return GWAOI_OK;
}

int ensure_fsplit(gwaoi_strips *s, uint32_t G) {
    const size_t n = (size_t)2 * G + 1;
    if (int rc = grow(s, &s->fcounts, s->fcounts_cap, n)) return rc;
    if (int rc = grow(s, &s->fscan_tmp, s->fscan_cap, gw::scan_tmp_elems(n) + 16)) return rc;
    return GWAOI_OK;
}

int ensure_moves(gwaoi_strips *s, size_t n) {
    if (n <= s->m_cap && s->m_slot) return GWAOI_OK;
    size_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    const size_t need = std::max<size_t>(n, s->m_cap * 2);
    int rc;
    if ((rc = grow(s, &s->m_slot, c0, need)) || (rc = grow(s, &s->m_x, c1, need)) ||
        (rc = grow(s, &s->m_z, c2, need)) || (rc = grow(s, &s->m_seq, c3, need))) {
        s->m_cap = 0;
        return rc;
    }
    s->m_cap = std::min({c0, c1, c2, c3});
    return GWAOI_OK;
}

int strip_err(gwaoi_strips *s, uint32_t e, const char *where) {
    if (!e) return GWAOI_OK;
    s->last_error = std::string(where) + ": " +
                    ((e & SE_BADSLOT) ? "slot out of range" :
                     (e & SE_KIND) ? "bad record kind" :
                     (e & SE_NONFINITE) ? "non-finite coordinate" :
                     (e & SE_COUNT) ? "received records disagree with the announced enter / leave counts" :
                                          "entity not owned by / in the wrong state for this strip");
    return (e & SE_BADSLOT) ? GWAOI_EBADSLOT : (e & SE_NONFINITE) ? GWAOI_ENONFINITE :
           (e & SE_KIND) ? GWAOI_EINVAL : (e & SE_COUNT) ? GWAOI_EDEVICE : GWAOI_ESTATE;
}

// The filter of the world flush's events (in flight, or committed after a regrow), the teleporter
// placement and the tick's totals (copied into small_h[SM_TICK..]), all queued on the stream.
// The output is sized by the events the last tick kept (+ room for every teleporter pair): a tick
// that keeps more is counted, completed by a re-run with room (complete), and no reallocation --
// a wait on the stream -- falls into the steady tick.
int launch_filter(gwaoi_strips *s, uint64_t tcap) {
    const uint32_t *wev = nullptr, *dcnt = nullptr;
    uint64_t cap = 0;
    gw::world_flush_events(s->w, &wev, &dcnt, &cap);
    const uint64_t need = s->last_kept + s->last_kept / 8 + 2 * tcap + 65536;
    if (s->out_cap < need)
        if (int rc = grow(s, &s->out, s->out_cap, need)) return rc;
    s->pend_ocap = s->out_cap;
    const uint32_t G = std::max(1u, std::min<uint32_t>(FILTER_BLOCKS, cdivu(std::max<uint64_t>(cap, 1), BT)));
    if (int rc = ensure_fsplit(s, G)) return rc;
    hipStream_t st = s->st;
    const uint2 *ev = reinterpret_cast<const uint2 *>(wev);
    k_filter<<<G, BT, 0, st>>>(0, ev, dcnt, cap, s->cur, s->prv, s->ptick, s->ttick, s->tick, s->geo, s->fcounts,
                               nullptr, nullptr, nullptr, 0);
    gw::scan_exclusive(s->fcounts, s->fcounts, (size_t)2 * G + 1, s->fscan_tmp, st);
    k_filter<<<G, BT, 0, st>>>(1, ev, dcnt, cap, s->cur, s->prv, s->ptick, s->ttick, s->tick, s->geo, s->fcounts,
                               s->fcounts, s->tcnt, s->out, s->out_cap);
    k_tele_place<<<64, 256, 0, st>>>(s->fcounts, G, s->tcnt, s->tpairs, s->tpairs + tcap, s->out, s->out_cap);
    k_tick_totals<<<1, 64, 0, st>>>(s->fcounts, G, s->tcnt, s->terr, s->small_d + SM_TICK);
    S_TRY(hipGetLastError());
    S_TRY(hipMemcpyAsync(s->small_h + SM_TICK, s->small_d + SM_TICK, 5 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    return GWAOI_OK;
}

// Complete the tick queued by gwaoi_strips_tick_async.  synced: the caller has just waited for
// the stream (everything queued before has finished), so this adds no wait.  The world's flush
// is committed (its summary is in pinned memory already); if it overflowed its event buffer,
// it re-ran its pair passes on commit, and the filter runs again on the complete events.
int complete(gwaoi_strips *s, bool synced) {
    if (!s->pending) return GWAOI_OK;
    if (!synced)
        if (int rc = wait(s)) return rc;
    s->pending = false;
    uint64_t wne = 0, wnl = 0;
    if (int rc = gwaoi_tick_finish(s->w, 0u, &wne, &wnl)) {
        s->last_error = std::string("world tick: ") + gwaoi_last_error(s->w);
        return rc;
    }
    gwaoi_debug dbg{};
    (void)gwaoi_debug_counters(s->w, &dbg);
    const uint32_t *t = s->small_h + SM_TICK;
    s->last_kept = (uint64_t)t[0] + t[1] + t[2] + t[3];
    // the world re-ran its pair passes (its event buffer grew), or this strip kept more events than
    // its output held: the filter again, on the complete events, with room
    if (dbg.event_regrows != s->pend_regrows || s->last_kept > s->pend_ocap) {
        if (int rc = launch_filter(s, s->pend_tcap)) return rc;
        if (int rc = wait(s)) return rc;
        s->last_kept = (uint64_t)t[0] + t[1] + t[2] + t[3];
    }
    s->n_enter = (uint64_t)t[0] + t[2];
    s->n_leave = (uint64_t)t[1] + t[3];
    if (wne + wnl > 0x7FFFFFFFull) return GWAOI_ECAPACITY;
    return strip_err(s, t[4], "recv");
}

// An asynchronous tick that fails on completion has already changed the strip's per-slot state
// and fed its world (which a record in the wrong state poisons): the strip is unusable from then
// on, and every later call says so (gwaoi_strips.h).
int complete_or_break(gwaoi_strips *s, bool synced) {
    if (s->broken) {
        s->last_error = s->broken_msg;
        return GWAOI_ESTATE;
    }
    const int rc = complete(s, synced);
    if (rc) {
        s->broken = true;
        s->broken_msg = "strip unusable after a failed tick: " + s->last_error;
    }
    return rc;
}

}  // namespace

extern "C" {

int gwaoi_strips_destroy(gwaoi_strips *s) {
    return gw::api_guard([&]() -> int {
    if (!s) return GWAOI_EINVAL;
    if (s->pending) (void)complete(s, false);
    if (s->st) (void)hipStreamSynchronize(s->st);
    void *dev[] = {s->cur, s->prv, s->ptick, s->ttick, s->counts, s->scan_tmp, s->err, s->small_d, s->kstat,
                   s->m_slot, s->m_x, s->m_z, s->m_seq, s->tcnt, s->tpairs, s->out, s->fcounts, s->fscan_tmp,
                   s->terr};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    if (s->small_h) (void)hipHostFree(s->small_h);
    if (s->row_h) (void)hipHostFree(s->row_h);
    if (s->h_events) (void)hipHostFree(s->h_events);
    delete s;
    return GWAOI_OK;
    });
}

int gwaoi_strips_create(gwaoi_world *w, uint32_t space, const gwaoi_strips_config *cfg, gwaoi_strips **out) {
    return gw::api_guard([&]() -> int {
    if (!w || !cfg || !out || cfg->n_strips == 0 || cfg->n_strips > GWAOI_MAX_STRIPS || cfg->rank >= cfg->n_strips ||
        (cfg->n_strips > 1 && !cfg->edges) || !(cfg->aoi_distance > 0.f) || !std::isfinite(cfg->aoi_distance))
        return GWAOI_EINVAL;
    *out = nullptr;
    for (uint32_t i = 0; i + 2 < cfg->n_strips; ++i)
        if (!(cfg->edges[i] < cfg->edges[i + 1])) return GWAOI_EINVAL;
    for (uint32_t i = 0; i + 1 < cfg->n_strips; ++i)
        if (!std::isfinite(cfg->edges[i])) return GWAOI_EINVAL;
    gwaoi_info info;
    if (int rc = gwaoi_world_info(w, &info)) return rc;
    gwaoi_strips *s = new (std::nothrow) gwaoi_strips();
    if (!s) return GWAOI_ENOMEM;
    s->w = w;
    s->space = space;
    s->st = (hipStream_t)gwaoi_stream(w);
    s->max_slots = info.max_slots;
    StripGeo &g = s->geo;
    g.S = cfg->n_strips;
    g.rank = cfg->rank;
    g.D = cfg->aoi_distance;
    g.tele = cfg->teleport > 0.f ? cfg->teleport : cfg->aoi_distance / 8.0f;
    g.max_slots = s->max_slots;
    // H = 2D + teleport + 1 (the +1 covers float32 rounding of the window
    // bounds for |x| < 2^24)
    const double H = 2.0 * (double)g.D + (double)g.tele + 1.0;
    g.H = (float)H;
    for (uint32_t q = 0; q < g.S; ++q) {
        if (q + 1 < g.S) g.edge[q] = cfg->edges[q];
        const double lo_q = q == 0 ? -INFINITY : (double)cfg->edges[q - 1] - H;
        const double hi_q = q + 1 == g.S ? INFINITY : (double)cfg->edges[q] + H;
        float fl = (float)lo_q, fh = (float)hi_q;  // round outward
        if ((double)fl > lo_q) fl = std::nextafter(fl, -INFINITY);
        if ((double)fh < hi_q) fh = std::nextafter(fh, INFINITY);
        g.rlo[q] = fl;
        g.rhi[q] = fh;
    }
    const size_t N = s->max_slots;
    auto fail = [&](int rc) {
        gwaoi_strips_destroy(s);
        return rc;
    };
    if (hipMalloc((void **)&s->cur, N * sizeof(Rec16)) != hipSuccess ||
        hipMalloc((void **)&s->prv, N * sizeof(Rec16)) != hipSuccess ||
        hipMalloc((void **)&s->ptick, N * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&s->ttick, N * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&s->err, sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&s->terr, sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&s->small_d, SM_WORDS * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&s->kstat, (GWAOI_MAX_STRIPS + 1) * KS * sizeof(int)) != hipSuccess ||
        hipMalloc((void **)&s->tcnt, 2 * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc((void **)&s->small_h, SM_WORDS * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess)
        return fail(GWAOI_ENOMEM);
    std::memset(s->small_h, 0, SM_WORDS * sizeof(uint32_t));
    if (hipMemsetAsync(s->cur, 0xFF, N * sizeof(Rec16), s->st) != hipSuccess ||  // x = NaN: absent
        hipMemsetAsync(s->prv, 0xFF, N * sizeof(Rec16), s->st) != hipSuccess ||
        hipMemsetAsync(s->ptick, 0, N * sizeof(uint32_t), s->st) != hipSuccess ||
        hipMemsetAsync(s->ttick, 0, N * sizeof(uint32_t), s->st) != hipSuccess ||
        hipMemsetAsync(s->err, 0, sizeof(uint32_t), s->st) != hipSuccess ||
        hipMemsetAsync(s->terr, 0, sizeof(uint32_t), s->st) != hipSuccess ||
        hipStreamSynchronize(s->st) != hipSuccess)
        return fail(GWAOI_EDEVICE);
    *out = s;
    return GWAOI_OK;
    });
}

int gwaoi_strips_halo(const gwaoi_strips *s, float *halo) {
    return gw::api_guard([&]() -> int {
    if (!s || !halo) return GWAOI_EINVAL;
    *halo = s->geo.H;
    return GWAOI_OK;
    });
}

}  // extern "C"

namespace {
// Route phase 0 and its totals, queued (no wait).  Behind the previous tick, if one is pending:
// its filter and totals land before this route's totals, so the route's one wait completes both.
int route_launch(gwaoi_strips *s, const gwaoi_halo_rec *d_ops, size_t n) {
    const uint32_t K = s->geo.S + 1;
    const uint32_t nb = std::max(1u, cdivu(n, BT));
    s->kinds_valid = false;
    s->routed = false;
    if (int rc = ensure_split(s, K, nb)) return rc;
    hipStream_t st = s->st;
    S_TRY(hipMemsetAsync(s->err, 0, sizeof(uint32_t), st));
    k_kstat_init<<<1, 64, 0, st>>>(s->kstat, s->geo.S);
    k_route<<<nb, BT, 0, st>>>(0, d_ops, (uint32_t)n, s->cur, s->geo, s->counts, nullptr, nb, s->err, nullptr,
                               nullptr, s->kstat);
    gw::scan_exclusive(s->counts, s->counts, (size_t)K * nb + 1, s->scan_tmp, st);
    k_totals<<<1, 128, 0, st>>>(s->counts, K, nb, s->err, s->small_d + SM_ROUTE);
    S_TRY(hipGetLastError());
    s->r_ops = d_ops;
    s->r_n = (uint32_t)n;
    s->r_nb = nb;
    return GWAOI_OK;
}

// The route's totals and kind statistics to the host (queued after whatever else the caller
// queued), then the tick's one host wait; it also completes the previous tick.
int route_finish(gwaoi_strips *s, uint64_t *counts) {
    const uint32_t K = s->geo.S + 1;
    hipStream_t st = s->st;
    S_TRY(hipMemcpyAsync(s->small_h + SM_ROUTE, s->small_d + SM_ROUTE, (K + 2) * sizeof(uint32_t),
                         hipMemcpyDeviceToHost, st));
    S_TRY(hipMemcpyAsync(s->small_h + SM_KIND, s->kstat, (size_t)s->geo.S * KS * sizeof(int), hipMemcpyDeviceToHost,
                         st));
    if (int rc = wait(s)) return rc;  // the one host wait of a strip tick
    if (int rc = complete_or_break(s, true)) return rc;
    if (int rc = strip_err(s, s->small_h[SM_ROUTE + K + 1], "route")) return rc;
    for (uint32_t q = 0; q < K; ++q) counts[q] = s->small_h[SM_ROUTE + q + 1] - s->small_h[SM_ROUTE + q];
    s->routed = true;
    s->kinds_valid = true;
    return GWAOI_OK;
}
}  // namespace

extern "C" {

int gwaoi_strips_route(gwaoi_strips *s, const gwaoi_halo_rec *d_ops, size_t n, uint64_t *counts) {
    return gw::api_guard([&]() -> int {
    if (!s || !counts || (n && !d_ops) || n > 0x7FFFFFFFu || s->row_pending) return GWAOI_EINVAL;
    if (int rc = route_launch(s, d_ops, n)) return rc;
    return route_finish(s, counts);
    });
}

int gwaoi_strips_route_row_words(const gwaoi_strips *s, uint32_t *words) {
    return gw::api_guard([&]() -> int {
    if (!s || !words) return GWAOI_EINVAL;
    *words = row_words(s->geo.S);
    return GWAOI_OK;
    });
}

int gwaoi_strips_route_begin(gwaoi_strips *s, const gwaoi_halo_rec *d_ops, size_t n, uint32_t *d_row) {
    return gw::api_guard([&]() -> int {
    if (!s || !d_row || (n && !d_ops) || n > 0x7FFFFFFFu || s->row_pending) return GWAOI_EINVAL;
    if (s->broken) {
        s->last_error = s->broken_msg;
        return GWAOI_ESTATE;
    }
    if (int rc = route_launch(s, d_ops, n)) return rc;
    k_route_row<<<1, 256, 0, s->st>>>(s->small_d + SM_ROUTE, s->kstat, s->geo.S, d_row);
    S_TRY(hipGetLastError());
    s->row_pending = true;
    return GWAOI_OK;
    });
}

int gwaoi_strips_route_end(gwaoi_strips *s, const uint32_t *d_matrix, const uint32_t **h_matrix, uint64_t *counts) {
    return gw::api_guard([&]() -> int {
    if (!s || !d_matrix || !h_matrix || !counts || !s->row_pending) return GWAOI_EINVAL;
    s->row_pending = false;
    const size_t words = (size_t)s->geo.S * row_words(s->geo.S);
    if (!s->row_h) {
        S_TRY(hipHostMalloc((void **)&s->row_h, words * sizeof(uint32_t), hipHostMallocDefault));
    }
    S_TRY(hipMemcpyAsync(s->row_h, d_matrix, words * sizeof(uint32_t), hipMemcpyDeviceToHost, s->st));
    if (int rc = route_finish(s, counts)) return rc;
    // every strip's route error (its own was checked by route_finish)
    const uint32_t W = row_words(s->geo.S);
    for (uint32_t q = 0; q < s->geo.S; ++q)
        if (uint32_t e = s->row_h[(size_t)q * W + W - 1]) {
            s->routed = false;
            return strip_err(s, e, "route of another strip");
        }
    *h_matrix = s->row_h;
    return GWAOI_OK;
    });
}

int gwaoi_strips_route_kinds(const gwaoi_strips *s, uint64_t *enters, uint64_t *leaves, float *enter_boxes) {
    return gw::api_guard([&]() -> int {
    if (!s || !s->kinds_valid) return GWAOI_EINVAL;
    for (uint32_t q = 0; q < s->geo.S; ++q) {
        const int *k = reinterpret_cast<const int *>(s->small_h + SM_KIND) + (size_t)q * KS;
        if (enters) enters[q] = (uint32_t)k[0];
        if (leaves) leaves[q] = (uint32_t)k[1];
        if (enter_boxes) {
            float *b = enter_boxes + 4 * q;
            if (k[0]) {
                b[0] = o2f(k[2]); b[1] = o2f(k[3]); b[2] = o2f(k[4]); b[3] = o2f(k[5]);
            } else {
                b[0] = b[1] = INFINITY;
                b[2] = b[3] = -INFINITY;
            }
        }
    }
    return GWAOI_OK;
    });
}

int gwaoi_strips_route_scatter(gwaoi_strips *s, gwaoi_halo_rec *d_send, gwaoi_tele_rec *d_tele) {
    return gw::api_guard([&]() -> int {
    if (!s || !s->routed) return GWAOI_EINVAL;
    s->routed = false;
    k_route<<<s->r_nb, BT, 0, s->st>>>(1, s->r_ops, s->r_n, s->cur, s->geo, s->counts, s->counts, s->r_nb, s->err,
                                       d_send, d_tele, nullptr);
    S_TRY(hipGetLastError());  // complete in stream order on the world's stream (gwaoi_stream): no host wait
    return GWAOI_OK;
    });
}

int gwaoi_strips_tick_async(gwaoi_strips *s, const gwaoi_halo_rec *d_local, size_t n_local,
                            const gwaoi_halo_rec *d_recv, size_t n_recv, const gwaoi_tele_rec *d_tele, size_t n_tele,
                            uint64_t n_enter_recs, uint64_t n_leave_recs, const float *enter_box) {
    return gw::api_guard([&]() -> int {
    if (!s || (n_local && !d_local) || (n_recv && !d_recv) || (n_tele && !d_tele) || n_tele > 0x7FFFFFFFu ||
        n_local + n_recv > 0x7FFFFFFFu || n_enter_recs + n_leave_recs > n_local + n_recv)
        return GWAOI_EINVAL;
    if (int rc = complete_or_break(s, false)) return rc;
    const size_t n_all = n_local + n_recv;
    const uint32_t n_ent = (uint32_t)n_enter_recs, n_lev = (uint32_t)n_leave_recs;
    const uint32_t n_move = (uint32_t)n_all - n_ent - n_lev;
    s->n_enter = s->n_leave = 0;
    const uint32_t tick = ++s->tick;
    hipStream_t st = s->st;
    // ---- own + received records -> world ops [moves | enters | leaves] + per-slot state
    const uint32_t nb = std::max(1u, cdivu(n_all, BT));
    if (int rc = ensure_split(s, 3, nb)) return rc;
    if (int rc = ensure_moves(s, std::max<size_t>(n_all, 1))) return rc;
    S_TRY(hipMemsetAsync(s->terr, 0, sizeof(uint32_t), st));
    k_recv<<<nb, BT, 0, st>>>(0, d_local, (uint32_t)n_local, d_recv, (uint32_t)n_all, s->cur, s->prv, s->ptick, tick,
                              s->max_slots, s->counts, nullptr, nb, s->terr, nullptr, nullptr, nullptr, nullptr, nullptr);
    gw::scan_exclusive(s->counts, s->counts, (size_t)3 * nb + 1, s->scan_tmp, st);
    k_recv<<<nb, BT, 0, st>>>(1, d_local, (uint32_t)n_local, d_recv, (uint32_t)n_all, s->cur, s->prv, s->ptick, tick,
                              s->max_slots, s->counts, s->counts, nb, s->terr, s->m_slot, s->m_x, s->m_z, s->m_seq,
                              nullptr);
    k_recv_check<<<1, 64, 0, st>>>(s->counts, nb, n_move, n_ent, n_lev, s->terr);
    if (n_tele) k_tele_mark<<<cdivu(n_tele, 256), 256, 0, st>>>(d_tele, (uint32_t)n_tele, s->ttick, tick, s->max_slots);
    S_TRY(hipGetLastError());
    // ---- the world's ops, all device batches: Leaves, Enters, Moves (one record per slot)
    auto wfail = [&](int rc, const char *what) {
        s->last_error = std::string(what) + ": " + gwaoi_last_error(s->w);
        return rc;
    };
    const uint64_t *seqs = reinterpret_cast<const uint64_t *>(s->m_seq);
    if (n_lev)
        if (int rc = gwaoi_leave_batch_device(s->w, s->space, s->m_slot + n_move + n_ent, n_lev))
            return wfail(rc, "world leaves");
    if (n_ent)
        if (int rc = gwaoi_enter_batch_device(s->w, s->space, s->m_slot + n_move, s->m_x + n_move, s->m_z + n_move,
                                              seqs + n_move, n_ent, enter_box))
            return wfail(rc, "world enters");
    if (n_move)
        if (int rc = gwaoi_moved_batch_device_seq(s->w, s->m_slot, s->m_x, s->m_z, seqs, n_move))
            return wfail(rc, "world moves");
    gwaoi_debug dbg{};
    (void)gwaoi_debug_counters(s->w, &dbg);
    s->pend_regrows = dbg.event_regrows;
    if (int rc = gwaoi_tick_begin(s->w)) return wfail(rc, "world tick");
    // ---- teleporter pairs: one pass into buffers that hold every possible pair (n (n-1) per kind)
    S_TRY(hipMemsetAsync(s->tcnt, 0, 2 * sizeof(unsigned long long), st));
    uint64_t tcap = n_tele > 1 ? (uint64_t)n_tele * (n_tele - 1) : 0;
    if (tcap > TELE_PAIRS_MAX) {  // a teleport storm: count first (one more host wait), then size exactly
        k_tele_pairs<<<cdivu(n_tele, 256), 256, 0, st>>>(0, d_tele, (uint32_t)n_tele, s->geo, s->tcnt, nullptr,
                                                         nullptr, 0);
        unsigned long long hc[2];
        S_TRY(hipMemcpyAsync(hc, s->tcnt, sizeof(hc), hipMemcpyDeviceToHost, st));
        if (int rc = wait(s)) return rc;
        tcap = std::max<uint64_t>(std::max(hc[0], hc[1]), 1);
        S_TRY(hipMemsetAsync(s->tcnt, 0, 2 * sizeof(unsigned long long), st));
    }
    // the pair buffers hold at least 2^16 pairs per kind: a tick-to-tick change of the teleporter
    // count does not reallocate them (a reallocation waits for the stream)
    tcap = std::max<uint64_t>(tcap, 1u << 16);
    if (int rc = grow(s, &s->tpairs, s->tpairs_cap, 2 * tcap + 1)) return rc;
    if (n_tele > 1)
        k_tele_pairs<<<cdivu(n_tele, 256), 256, 0, st>>>(1, d_tele, (uint32_t)n_tele, s->geo, s->tcnt, s->tpairs,
                                                         s->tpairs + tcap, tcap);
    // ---- filter the world's events to this strip's: [filter enters | tele enters | filter leaves | tele leaves]
    if (int rc = launch_filter(s, tcap)) return rc;
    s->pend_tcap = tcap;
    s->pending = true;
    return GWAOI_OK;
    });
}

int gwaoi_strips_wait(gwaoi_strips *s, uint64_t *n_enter, uint64_t *n_leave) {
    return gw::api_guard([&]() -> int {
    if (!s) return GWAOI_EINVAL;
    const int rc = complete_or_break(s, false);
    if (n_enter) *n_enter = s->n_enter;
    if (n_leave) *n_leave = s->n_leave;
    return rc;
    });
}

int gwaoi_strips_tick(gwaoi_strips *s, const gwaoi_halo_rec *d_local, size_t n_local, const gwaoi_halo_rec *d_recv,
                      size_t n_recv, const gwaoi_tele_rec *d_tele, size_t n_tele, uint64_t *n_enter,
                      uint64_t *n_leave) {
    return gw::api_guard([&]() -> int {
    if (n_enter) *n_enter = 0;
    if (n_leave) *n_leave = 0;
    if (!s || (n_local && !d_local) || (n_recv && !d_recv) || n_local + n_recv > 0x7FFFFFFFu) return GWAOI_EINVAL;
    if (int rc = complete_or_break(s, false)) return rc;
    // no announced counts: the records' kinds and the box of their Enters are read here first
    const size_t n_all = n_local + n_recv;
    const uint32_t nb = std::max(1u, cdivu(n_all, BT));
    if (int rc = ensure_split(s, 3, nb)) return rc;
    hipStream_t st = s->st;
    int *ks = s->kstat + (size_t)GWAOI_MAX_STRIPS * KS;
    S_TRY(hipMemsetAsync(s->err, 0, sizeof(uint32_t), st));
    k_kstat_init<<<1, 64, 0, st>>>(ks, 1);
    k_recv<<<nb, BT, 0, st>>>(0, d_local, (uint32_t)n_local, d_recv, (uint32_t)n_all, s->cur, s->prv, s->ptick,
                              s->tick + 1, s->max_slots, s->counts, nullptr, nb, s->err, nullptr, nullptr, nullptr,
                              nullptr, ks);
    S_TRY(hipGetLastError());
    S_TRY(hipMemcpyAsync(s->small_h + SM_RECV, s->err, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    S_TRY(hipMemcpyAsync(s->small_h + SM_RECV + 2, ks, KS * sizeof(int), hipMemcpyDeviceToHost, st));
    if (int rc = wait(s)) return rc;
    if (int rc = strip_err(s, s->small_h[SM_RECV], "recv")) return rc;
    const int *k = reinterpret_cast<const int *>(s->small_h + SM_RECV + 2);
    const float box[4] = {o2f(k[2]), o2f(k[3]), o2f(k[4]), o2f(k[5])};
    if (int rc = gwaoi_strips_tick_async(s, d_local, n_local, d_recv, n_recv, d_tele, n_tele, (uint32_t)k[0],
                                         (uint32_t)k[1], k[0] ? box : nullptr))
        return rc;
    return gwaoi_strips_wait(s, n_enter, n_leave);
    });
}

int gwaoi_strips_host_waits(const gwaoi_strips *s, uint64_t *waits) {
    return gw::api_guard([&]() -> int {
    if (!s || !waits) return GWAOI_EINVAL;
    *waits = s->waits;
    return GWAOI_OK;
    });
}

int gwaoi_strips_events_device(gwaoi_strips *s, const uint32_t **d_enter, const uint32_t **d_leave) {
    return gw::api_guard([&]() -> int {
    if (!s) return GWAOI_EINVAL;
    if (int rc = complete_or_break(s, false)) return rc;
    if (d_enter) *d_enter = reinterpret_cast<const uint32_t *>(s->out);
    if (d_leave) *d_leave = reinterpret_cast<const uint32_t *>(s->out + s->n_enter);
    return GWAOI_OK;
    });
}

int gwaoi_strips_events(gwaoi_strips *s, gwaoi_events *out) {
    return gw::api_guard([&]() -> int {
    if (!s || !out) return GWAOI_EINVAL;
    if (int rc = complete_or_break(s, false)) return rc;
    const uint64_t tot = s->n_enter + s->n_leave;
    if (tot > s->h_cap || !s->h_events) {
        if (s->h_events) (void)hipHostFree(s->h_events);
        s->h_events = nullptr;
        s->h_cap = 0;
        const size_t c = std::max<size_t>(tot + tot / 4, 1024);
        S_TRY(hipHostMalloc((void **)&s->h_events, 2 * c * sizeof(uint32_t), hipHostMallocDefault));
        s->h_cap = c;
    }
    if (tot) {
        S_TRY(hipMemcpyAsync(s->h_events, s->out, tot * sizeof(uint2), hipMemcpyDeviceToHost, s->st));
        if (int rc = wait(s)) return rc;
    }
    out->n_enter = s->n_enter;
    out->n_leave = s->n_leave;
    out->enter = s->h_events;
    out->leave = s->h_events + 2 * s->n_enter;
    return GWAOI_OK;
    });
}

const char *gwaoi_strips_last_error(gwaoi_strips *s) { return s ? s->last_error.c_str() : "null strips"; }

}  // extern "C"
