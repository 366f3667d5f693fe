// gwaoi_kernels.hip -- HIP kernels of the AOI tick for gfx950 (MI355X).
//
// One flush (gwaoi_tick) runs, on one stream:
//   ops_claim/ops_apply  last-writer-wins application of the queued
//                        Enter/Leave/Moved calls (seq = call order) onto the
//                        working copy S' of the previous frame
//   keygen               cell key per entity (space-major uniform grid)
//   radix sort           stable LSD sort of (key, index), wave64 multisplit
//   gather               new frame (sorted SoA) + old state in the new order
//   cell_count + scan    cell_start table
//   pairs (x4)           count/fill of enter events over the new grid and of
//                        leave events over the previous grid; both evaluate
//                        go-aoi's float32 window predicate with last-mover
//                        ownership at both times
//
// The path is sort/scan/gather/compaction: integer and float32-compare work
// bounded by HBM and on-chip bandwidth, no dense contraction, so no MFMA.
// Compile with -ffp-contract=off: the window bounds must be plain float32
// sums exactly as in go-aoi (`coord - sl.aoidist`).

#include "gwaoi_internal.h"

#include <algorithm>

namespace gw {
namespace {

constexpr int WAVE = 64;

__device__ __forceinline__ uint32_t lane() { return __lane_id(); }
__device__ __forceinline__ unsigned long long lanemask_lt() { return (1ull << lane()) - 1ull; }

inline uint32_t cdiv(size_t a, size_t b) { return (uint32_t)((a + b - 1) / b); }

// Monotone non-decreasing in v (IEEE sub/mul round monotonically; clamp is
// monotone).  keygen and every query use this one function.
__device__ __forceinline__ int cell_of(float v, float o, float inv, uint32_t g) {
    float t = (v - o) * inv;
    t = fmaxf(t, 0.0f);
    t = fminf(t, (float)(g - 1));
    return (int)t;
}

// L inside W's window [fl32(w-D), fl32(w+D)]^2 (bounds precomputed by the caller)
__device__ __forceinline__ bool in_win(float lx, float lz, float lox, float hix, float loz, float hiz) {
    return lx >= lox && lx <= hix && lz >= loz && lz <= hiz;
}

// go-aoi relation of a pair under last-mover ownership
__device__ __forceinline__ bool related(float xa, float za, uint64_t sa, float lox, float hix, float loz, float hiz,
                                        float xb, float zb, uint64_t sb, float D) {
    return sa > sb ? in_win(xb, zb, lox, hix, loz, hiz) : in_win(xa, za, xb - D, xb + D, zb - D, zb + D);
}

// ------------------------------------------------------------ op apply ------

__global__ void k_init_appended(const uint32_t *__restrict__ new_slots, uint32_t n_app, uint32_t n_prev,
                                uint32_t *s_slot, uint32_t *s_sp, uint64_t *s_seq, uint32_t *rank) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_app) return;
    uint32_t s = new_slots[i];
    uint32_t idx = n_prev + i;
    s_slot[idx] = s;
    s_sp[idx] = SP_DEAD;
    s_seq[idx] = 0;
    rank[s] = idx;
}

__global__ void k_ops_claim(const uint32_t *__restrict__ op_slot, uint32_t n, uint32_t max_slots,
                            unsigned long long *lastop, uint32_t tick, uint32_t *err) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint32_t s = op_slot[j];
    if (s >= max_slots) {
        atomicOr(err, ERR_BAD_SLOT);
        return;
    }
    atomicMax(&lastop[s], ((unsigned long long)tick << 32) | j);
}

// The last op of a slot in this flush determines its state (closed form:
// only the final position and the final seq matter).
__global__ void k_ops_apply(const uint32_t *__restrict__ op_slot, const float *__restrict__ op_x,
                            const float *__restrict__ op_z, const uint32_t *__restrict__ op_sp, uint32_t n,
                            uint32_t max_slots, const unsigned long long *__restrict__ lastop, uint32_t tick,
                            const uint32_t *__restrict__ rank, uint32_t n_total, uint64_t seq_base, float *s_x,
                            float *s_z, uint64_t *s_seq, uint32_t *s_sp, const uint32_t *__restrict__ s_slot,
                            uint32_t *err) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint32_t s = op_slot[j];
    if (s >= max_slots) return;
    if (lastop[s] != (((unsigned long long)tick << 32) | j)) return;
    uint32_t idx = rank[s];
    if (idx >= n_total || s_slot[idx] != s) {
        atomicOr(err, ERR_MOVE_DEAD);
        return;
    }
    uint32_t sp = op_sp[j];
    if (sp == SP_DEAD) {  // Leave
        s_sp[idx] = SP_DEAD;
        s_seq[idx] = seq_base + j;
        return;
    }
    if (sp == SP_KEEP) {  // device-side Moved
        sp = s_sp[idx];
        if (sp == SP_DEAD) {
            atomicOr(err, ERR_MOVE_DEAD);
            return;
        }
    }
    float x = op_x[j], z = op_z[j];
    if (!isfinite(x) || !isfinite(z)) {
        atomicOr(err, ERR_NONFINITE);
        return;
    }
    s_x[idx] = x;
    s_z[idx] = z;
    s_seq[idx] = seq_base + j;
    s_sp[idx] = sp;
}

// --------------------------------------------------------------- keygen ------

__global__ void k_keygen(const float *__restrict__ x, const float *__restrict__ z, const uint32_t *__restrict__ sp,
                         uint32_t n, const SpaceGrid *__restrict__ grid, uint32_t sentinel, uint32_t *keys,
                         uint32_t *vals) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t s = sp[i];
    uint32_t key = sentinel;
    if (s != SP_DEAD) {
        const SpaceGrid g = grid[s];
        int cx = cell_of(x[i], g.ox, g.inv, g.gx);
        int cz = cell_of(z[i], g.oz, g.inv, g.gz);
        key = g.base + (uint32_t)cz * g.gx + (uint32_t)cx;
    }
    keys[i] = key;
    vals[i] = i;
}

// ----------------------------------------------------------------- scan ------

constexpr int SC_T = 256;
constexpr int SC_I = 16;
constexpr int SC_TILE = SC_T * SC_I;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        uint32_t y = __shfl_up(x, o);
        if ((int)lane() >= o) x += y;
    }
    return x;
}

// exclusive scan of one value per thread over a 256-thread block
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *ws, uint32_t &total) {
    uint32_t x = wave_incl_scan(v);
    const int w = threadIdx.x / WAVE;
    if (lane() == WAVE - 1) ws[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < SC_T / WAVE; ++i) {
        uint32_t t = ws[i];
        pre += (i < w) ? t : 0u;
        tot += t;
    }
    total = tot;
    return pre + x - v;
}

__device__ __forceinline__ void load16(const uint32_t *in, size_t base, size_t n, uint32_t (&v)[SC_I]) {
    if (base + SC_I <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(in + base);
#pragma unroll
        for (int q = 0; q < SC_I / 4; ++q) {
            uint4 t = p[q];
            v[4 * q] = t.x;
            v[4 * q + 1] = t.y;
            v[4 * q + 2] = t.z;
            v[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < SC_I; ++q) v[q] = (base + q < n) ? in[base + q] : 0u;
    }
}

__global__ __launch_bounds__(SC_T) void k_scan_reduce(const uint32_t *__restrict__ in, size_t n, uint32_t *sums) {
    __shared__ uint32_t ws[SC_T / WAVE];
    uint32_t v[SC_I];
    load16(in, (size_t)blockIdx.x * SC_TILE + (size_t)threadIdx.x * SC_I, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < SC_I; ++q) s += v[q];
    uint32_t tot;
    block_excl_scan(s, ws, tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SC_T) void k_scan_down(const uint32_t *in, uint32_t *out, size_t n,
                                                    const uint32_t *__restrict__ block_off) {
    __shared__ uint32_t ws[SC_T / WAVE];
    const size_t base = (size_t)blockIdx.x * SC_TILE + (size_t)threadIdx.x * SC_I;
    uint32_t v[SC_I];
    load16(in, base, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < SC_I; ++q) s += v[q];
    uint32_t tot;
    uint32_t run = block_excl_scan(s, ws, tot) + (block_off ? block_off[blockIdx.x] : 0u);
    if (base + SC_I <= n) {
        uint4 *p = reinterpret_cast<uint4 *>(out + base);
#pragma unroll
        for (int q = 0; q < SC_I / 4; ++q) {
            uint4 t;
            t.x = run; run += v[4 * q];
            t.y = run; run += v[4 * q + 1];
            t.z = run; run += v[4 * q + 2];
            t.w = run; run += v[4 * q + 3];
            p[q] = t;
        }
    } else {
#pragma unroll
        for (int q = 0; q < SC_I; ++q)
            if (base + q < n) {
                out[base + q] = run;
                run += v[q];
            }
    }
}

// ----------------------------------------------------------- radix sort ------
// Tile = 4 waves x 8 items x 64 lanes.  Element (wave w, item j, lane l) is
// index tile*2048 + w*512 + j*64 + l, so processing items in order per wave
// and waves in order keeps the sort stable.

constexpr int RS_T = 256;
constexpr int RS_I = 8;
constexpr int RS_TILE = RS_T * RS_I;
constexpr int RS_WAVES = RS_T / WAVE;
constexpr int RS_WSEG = WAVE * RS_I;

__global__ __launch_bounds__(RS_T) void k_rs_upsweep(const uint32_t *__restrict__ keys, uint32_t n, int shift,
                                                     int nbits, uint32_t *hist, uint32_t ntiles) {
    __shared__ uint32_t h[256];
    const int bins = 1 << nbits;
    const uint32_t mask = (uint32_t)bins - 1u;
    for (int i = threadIdx.x; i < bins; i += RS_T) h[i] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * RS_TILE;
#pragma unroll
    for (int i = 0; i < RS_I; ++i) {
        size_t idx = base + (size_t)i * RS_T + threadIdx.x;
        if (idx < n) atomicAdd(&h[(keys[idx] >> shift) & mask], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < bins; d += RS_T) hist[(size_t)d * ntiles + blockIdx.x] = h[d];
}

__global__ __launch_bounds__(RS_T) void k_rs_downsweep(const uint32_t *__restrict__ keys_in,
                                                       const uint32_t *__restrict__ vals_in, uint32_t *keys_out,
                                                       uint32_t *vals_out, uint32_t n, int shift, int nbits,
                                                       const uint32_t *__restrict__ hist_scanned, uint32_t ntiles) {
    __shared__ uint32_t wcnt[RS_WAVES][256];
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
    for (int d = threadIdx.x; d < bins; d += RS_T) {
        uint32_t run = hist_scanned[(size_t)d * ntiles + blockIdx.x];
#pragma unroll
        for (int ww = 0; ww < RS_WAVES; ++ww) {
            uint32_t c = wcnt[ww][d];
            wcnt[ww][d] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        const size_t idx = wbase + (size_t)j * WAVE + l;
        if (idx < n) {
            const uint32_t d = (k[j] >> shift) & mask;
            const uint32_t pos = wcnt[w][d] + rk[j];
            keys_out[pos] = k[j];
            vals_out[pos] = v[j];
        }
    }
}

// --------------------------------------------------------------- gather ------

__global__ void k_gather(const uint32_t *__restrict__ perm, uint32_t n_new, uint32_t n_prev,
                         const float *__restrict__ s_x, const float *__restrict__ s_z,
                         const uint64_t *__restrict__ s_seq, const uint32_t *__restrict__ s_sp,
                         const uint32_t *__restrict__ s_slot, const float *__restrict__ p_x,
                         const float *__restrict__ p_z, const uint64_t *__restrict__ p_seq,
                         const uint32_t *__restrict__ p_sp, float *f_x, float *f_z, uint64_t *f_seq, uint32_t *f_sp,
                         uint32_t *f_slot, float *o_x, float *o_z, uint64_t *o_seq, uint32_t *o_sp, uint32_t *rank,
                         const uint32_t *__restrict__ sorted_keys, uint32_t sentinel, uint32_t n_total,
                         uint32_t *err) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0 && n_new < n_total && sorted_keys[n_new] != sentinel) atomicOr(err, ERR_COUNT_MISMATCH);
    if (k >= n_new) return;
    if (sorted_keys[k] == sentinel) atomicOr(err, ERR_COUNT_MISMATCH);
    const uint32_t i = perm[k];
    const uint32_t slot = s_slot[i];
    f_x[k] = s_x[i];
    f_z[k] = s_z[i];
    f_seq[k] = s_seq[i];
    f_sp[k] = s_sp[i];
    f_slot[k] = slot;
    rank[slot] = k;
    if (i < n_prev) {
        o_x[k] = p_x[i];
        o_z[k] = p_z[i];
        o_seq[k] = p_seq[i];
        o_sp[k] = p_sp[i];
    } else {
        o_x[k] = 0.0f;
        o_z[k] = 0.0f;
        o_seq[k] = 0;
        o_sp[k] = SP_DEAD;
    }
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
// MODE 0 (enter): F = new frame, O = previous state of the same entities in
//   F's order; emit (A,B) when related now and not related before.
// MODE 1 (leave): F = previous frame, O = new state in F's order; emit (A,B)
//   when related before and not related now.
// "Related at the other time" requires both entities live in the same space
// as now at that time (each space is its own go-aoi manager).  Pairs where
// neither entity was touched this flush cannot change and are skipped.

template <int MODE, bool FILL>
__global__ __launch_bounds__(256) void k_pairs(FrameView F, StateView O, uint64_t seq_base, uint32_t *counts,
                                               const uint32_t *__restrict__ offsets, uint2 *out, uint64_t out_cap,
                                               unsigned long long *total64) {
    const uint32_t a = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t cnt = 0;
    if (a < F.n) {
        const float xa = F.x[a], za = F.z[a];
        const uint64_t sa = F.seq[a];
        const uint32_t spa = F.sp[a];
        const SpaceGrid g = F.grid[spa];
        const float D = g.D;
        const uint32_t osp_a = O.sp[a];
        const uint64_t osa = O.seq[a];
        const float oxa = O.x[a], oza = O.z[a];
        const bool a_other = (osp_a == spa);
        const bool chg_a = (MODE == 0 ? sa : osa) >= seq_base;
        const float lox = xa - D, hix = xa + D, loz = za - D, hiz = za + D;
        const float olox = oxa - D, ohix = oxa + D, oloz = oza - D, ohiz = oza + D;
        // conservative query box: covers P_A(B) and P_B(A) under float32
        // rounding of the bounds (|dx| <= D + (|x|+2D)*2^-24)
        const float mx = (fabsf(xa) + 2.0f * D) * 0x1p-21f;
        const float mz = (fabsf(za) + 2.0f * D) * 0x1p-21f;
        const float qlox = lox - mx, qhix = hix + mx, qloz = loz - mz, qhiz = hiz + mz;
        const int cx0 = cell_of(qlox, g.ox, g.inv, g.gx), cx1 = cell_of(qhix, g.ox, g.inv, g.gx);
        const int cz0 = cell_of(qloz, g.oz, g.inv, g.gz), cz1 = cell_of(qhiz, g.oz, g.inv, g.gz);
        const uint32_t wbase = FILL ? offsets[a] : 0u;
        const uint32_t slot_a = FILL ? F.slot[a] : 0u;
        for (int cz = cz0; cz <= cz1; ++cz) {
            const uint32_t row = g.base + (uint32_t)cz * g.gx;
            const uint32_t jb = F.cell_start[row + (uint32_t)cx0];
            const uint32_t je = F.cell_start[row + (uint32_t)cx1 + 1u];
            for (uint32_t b = jb; b < je; ++b) {
                if (b == a) continue;
                const float xb = F.x[b], zb = F.z[b];
                if (xb < qlox || xb > qhix || zb < qloz || zb > qhiz) continue;
                const uint64_t sb = F.seq[b];
                uint64_t osb = 0;
                bool chg_b;
                if (MODE == 0) {
                    chg_b = sb >= seq_base;
                } else {
                    osb = O.seq[b];
                    chg_b = osb >= seq_base;
                }
                if (!chg_a && !chg_b) continue;
                if (!related(xa, za, sa, lox, hix, loz, hiz, xb, zb, sb, D)) continue;
                bool other = false;
                if (a_other && O.sp[b] == spa) {
                    if (MODE == 0) osb = O.seq[b];
                    other = related(oxa, oza, osa, olox, ohix, oloz, ohiz, O.x[b], O.z[b], osb, D);
                }
                if (other) continue;
                if (FILL) {
                    const uint64_t pos = (uint64_t)wbase + cnt;
                    if (pos < out_cap) out[pos] = make_uint2(slot_a, F.slot[b]);
                }
                ++cnt;
            }
        }
        if (!FILL) counts[a] = cnt;
    }
    if (!FILL) {
        unsigned long long c = cnt;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        if (lane() == 0 && c) atomicAdd(total64, c);
    }
}

__global__ void k_finish(const uint32_t *__restrict__ offsets, uint32_t n_new, uint32_t n_prev,
                         const uint32_t *__restrict__ err, const unsigned long long *__restrict__ total64,
                         TickResult *res) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    res->n_enter = offsets[n_new];
    res->n_total = offsets[(size_t)n_new + n_prev];
    res->err = *err;
    res->total64 = *total64;
}

// ----------------------------------------------------------------- bbox ------

__device__ __forceinline__ int f2o(float f) {
    int i = __float_as_int(f);
    return i ^ ((i >> 31) & 0x7FFFFFFF);
}

__global__ void k_bbox(FrameView F, int *bbox, uint32_t max_spaces) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = k < F.n;
    const uint32_t sp = valid ? F.sp[k] : SP_DEAD;
    int mnx = valid ? f2o(F.x[k]) : INT_MAX, mnz = valid ? f2o(F.z[k]) : INT_MAX;
    int mxx = valid ? mnx : INT_MIN, mxz = valid ? mnz : INT_MIN;
    const uint32_t sp0 = __shfl(sp, 0);
    if (__all(!valid || sp == sp0)) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            mnx = min(mnx, __shfl_xor(mnx, o));
            mnz = min(mnz, __shfl_xor(mnz, o));
            mxx = max(mxx, __shfl_xor(mxx, o));
            mxz = max(mxz, __shfl_xor(mxz, o));
        }
        if (lane() == 0 && sp0 != SP_DEAD && sp0 < max_spaces) {
            atomicMin(&bbox[sp0], mnx);
            atomicMin(&bbox[max_spaces + sp0], mnz);
            atomicMax(&bbox[2 * max_spaces + sp0], mxx);
            atomicMax(&bbox[3 * max_spaces + sp0], mxz);
        }
    } else if (valid && sp < max_spaces) {
        atomicMin(&bbox[sp], mnx);
        atomicMin(&bbox[max_spaces + sp], mnz);
        atomicMax(&bbox[2 * max_spaces + sp], mxx);
        atomicMax(&bbox[3 * max_spaces + sp], mxz);
    }
}

// ------------------------------------------------------------ neighbors ------

__global__ __launch_bounds__(256) void k_neighbors(FrameView F, const uint32_t *__restrict__ rank, uint32_t slot,
                                                   uint32_t *out, uint32_t cap, uint32_t *count) {
    const uint32_t a = rank[slot];
    if (a >= F.n || F.slot[a] != slot) return;
    const float xa = F.x[a], za = F.z[a];
    const uint64_t sa = F.seq[a];
    const SpaceGrid g = F.grid[F.sp[a]];
    const float D = g.D;
    const float lox = xa - D, hix = xa + D, loz = za - D, hiz = za + D;
    const float mx = (fabsf(xa) + 2.0f * D) * 0x1p-21f, mz = (fabsf(za) + 2.0f * D) * 0x1p-21f;
    const int cx0 = cell_of(lox - mx, g.ox, g.inv, g.gx), cx1 = cell_of(hix + mx, g.ox, g.inv, g.gx);
    const int cz0 = cell_of(loz - mz, g.oz, g.inv, g.gz), cz1 = cell_of(hiz + mz, g.oz, g.inv, g.gz);
    for (int cz = cz0; cz <= cz1; ++cz) {
        const uint32_t row = g.base + (uint32_t)cz * g.gx;
        const uint32_t jb = F.cell_start[row + (uint32_t)cx0], je = F.cell_start[row + (uint32_t)cx1 + 1u];
        for (uint32_t b = jb + threadIdx.x; b < je; b += blockDim.x) {
            if (b == a) continue;
            if (related(xa, za, sa, lox, hix, loz, hiz, F.x[b], F.z[b], F.seq[b], D)) {
                uint32_t p = atomicAdd(count, 1u);
                if (p < cap) out[p] = F.slot[b];
            }
        }
    }
}

}  // namespace

// ============================================================ launchers ======

void launch_init_appended(const uint32_t *new_slots, uint32_t n_app, uint32_t n_prev, uint32_t *s_slot,
                          uint32_t *s_sp, uint64_t *s_seq, uint32_t *rank, hipStream_t st) {
    if (!n_app) return;
    k_init_appended<<<cdiv(n_app, 256), 256, 0, st>>>(new_slots, n_app, n_prev, s_slot, s_sp, s_seq, rank);
}

void launch_ops_claim(const uint32_t *op_slot, uint32_t n_ops, uint32_t max_slots, unsigned long long *lastop,
                      uint32_t tick_id, uint32_t *err, hipStream_t st) {
    if (!n_ops) return;
    k_ops_claim<<<cdiv(n_ops, 256), 256, 0, st>>>(op_slot, n_ops, max_slots, lastop, tick_id, err);
}

void launch_ops_apply(const uint32_t *op_slot, const float *op_x, const float *op_z, const uint32_t *op_sp,
                      uint32_t n_ops, uint32_t max_slots, const unsigned long long *lastop, uint32_t tick_id,
                      const uint32_t *rank, uint32_t n_total, uint64_t seq_base, float *s_x, float *s_z,
                      uint64_t *s_seq, uint32_t *s_sp, const uint32_t *s_slot, uint32_t *err, hipStream_t st) {
    if (!n_ops) return;
    k_ops_apply<<<cdiv(n_ops, 256), 256, 0, st>>>(op_slot, op_x, op_z, op_sp, n_ops, max_slots, lastop, tick_id,
                                                  rank, n_total, seq_base, s_x, s_z, s_seq, s_sp, s_slot, err);
}

void launch_keygen(const float *s_x, const float *s_z, const uint32_t *s_sp, uint32_t n_total,
                   const SpaceGrid *grid, uint32_t sentinel, uint32_t *keys, uint32_t *vals, hipStream_t st) {
    if (!n_total) return;
    k_keygen<<<cdiv(n_total, 256), 256, 0, st>>>(s_x, s_z, s_sp, n_total, grid, sentinel, keys, vals);
}

size_t scan_tmp_elems(size_t n) {
    size_t nb = cdiv(n, SC_TILE);
    if (nb <= 1) return 0;
    return ((nb + 3) & ~(size_t)3) + scan_tmp_elems(nb);
}

void scan_exclusive(const uint32_t *in, uint32_t *out, size_t n, uint32_t *tmp, hipStream_t st) {
    if (!n) return;
    const size_t nb = cdiv(n, SC_TILE);
    if (nb == 1) {
        k_scan_down<<<1, SC_T, 0, st>>>(in, out, n, nullptr);
        return;
    }
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

void launch_gather(const uint32_t *perm, uint32_t n_new, uint32_t n_prev, const float *s_x, const float *s_z,
                   const uint64_t *s_seq, const uint32_t *s_sp, const uint32_t *s_slot, const float *p_x,
                   const float *p_z, const uint64_t *p_seq, const uint32_t *p_sp, float *f_x, float *f_z,
                   uint64_t *f_seq, uint32_t *f_sp, uint32_t *f_slot, float *o_x, float *o_z, uint64_t *o_seq,
                   uint32_t *o_sp, uint32_t *rank, const uint32_t *sorted_keys, uint32_t sentinel,
                   uint32_t n_total, uint32_t *err, hipStream_t st) {
    const uint32_t nt = std::max<uint32_t>(n_new, 1u);
    k_gather<<<cdiv(nt, 256), 256, 0, st>>>(perm, n_new, n_prev, s_x, s_z, s_seq, s_sp, s_slot, p_x, p_z, p_seq,
                                            p_sp, f_x, f_z, f_seq, f_sp, f_slot, o_x, o_z, o_seq, o_sp, rank,
                                            sorted_keys, sentinel, n_total, err);
}

void launch_cell_count(const uint32_t *sorted_keys, uint32_t n, uint32_t *cnt, hipStream_t st) {
    if (!n) return;
    k_cell_count<<<cdiv(n, 256), 256, 0, st>>>(sorted_keys, n, cnt);
}

void launch_pairs(int mode, bool fill, FrameView F, StateView O, uint64_t seq_base, uint32_t *counts,
                  const uint32_t *offsets, uint32_t *out_pairs, uint64_t out_cap, unsigned long long *total64,
                  hipStream_t st) {
    if (!F.n) return;
    const uint32_t nb = cdiv(F.n, 256);
    uint2 *out = reinterpret_cast<uint2 *>(out_pairs);
    if (mode == 0) {
        if (fill)
            k_pairs<0, true><<<nb, 256, 0, st>>>(F, O, seq_base, counts, offsets, out, out_cap, total64);
        else
            k_pairs<0, false><<<nb, 256, 0, st>>>(F, O, seq_base, counts, offsets, out, out_cap, total64);
    } else {
        if (fill)
            k_pairs<1, true><<<nb, 256, 0, st>>>(F, O, seq_base, counts, offsets, out, out_cap, total64);
        else
            k_pairs<1, false><<<nb, 256, 0, st>>>(F, O, seq_base, counts, offsets, out, out_cap, total64);
    }
}

void launch_finish(const uint32_t *offsets, uint32_t n_new, uint32_t n_prev, const uint32_t *err,
                   const unsigned long long *total64, TickResult *res, hipStream_t st) {
    k_finish<<<1, 64, 0, st>>>(offsets, n_new, n_prev, err, total64, res);
}

void launch_bbox(FrameView F, int *bbox, uint32_t max_spaces, hipStream_t st) {
    if (!F.n) return;
    k_bbox<<<cdiv(F.n, 256), 256, 0, st>>>(F, bbox, max_spaces);
}

void launch_neighbors(FrameView F, const uint32_t *rank, uint32_t slot, uint32_t *out, uint32_t cap,
                      uint32_t *count, hipStream_t st) {
    k_neighbors<<<1, 256, 0, st>>>(F, rank, slot, out, cap, count);
}

}  // namespace gw
