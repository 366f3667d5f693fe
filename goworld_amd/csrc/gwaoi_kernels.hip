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
//   build_tiles          rows split into tiles of <= 256 entities
//   pairs (x2)           one workgroup per tile stages the tile's candidate
//                        rows in LDS and emits enter events (new grid) or
//                        leave events (previous grid); both evaluate go-aoi's
//                        float32 window predicate with last-mover ownership
//                         at both times
//   reorder              events into deterministic tile order
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

__global__ void k_copy_state(uint32_t n, const float *__restrict__ p_x, const float *__restrict__ p_z,
                             const uint64_t *__restrict__ p_seq, const uint32_t *__restrict__ p_sp,
                             const uint32_t *__restrict__ p_slot, float *s_x, float *s_z, uint64_t *s_seq,
                             uint32_t *s_sp, uint32_t *s_slot) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    s_x[i] = p_x[i];
    s_z[i] = p_z[i];
    s_seq[i] = p_seq[i];
    s_sp[i] = p_sp[i];
    s_slot[i] = p_slot[i];
}

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

__global__ void k_ops_claim(const uint32_t *__restrict__ slots, uint32_t n, uint32_t j0, uint32_t max_slots,
                            unsigned long long *lastop, uint32_t tick, uint32_t *err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slots[i];
    if (s >= max_slots) {
        atomicOr(err, ERR_BAD_SLOT);
        return;
    }
    atomicMax(&lastop[s], ((unsigned long long)tick << 32) | (j0 + i));
}

// The last op of a slot in this flush determines its state (closed form:
// only the final position and the final seq matter).
__global__ void k_ops_apply(const uint32_t *__restrict__ slots, const float *__restrict__ xs,
                            const float *__restrict__ zs, const uint32_t *__restrict__ sps, uint32_t n, uint32_t j0,
                            uint32_t max_slots, const unsigned long long *__restrict__ lastop, uint32_t tick,
                            const uint32_t *__restrict__ rank, uint32_t n_total, uint64_t seq_base, float *s_x,
                            float *s_z, uint64_t *s_seq, uint32_t *s_sp, const uint32_t *__restrict__ s_slot,
                            uint32_t *err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = j0 + i;
    const uint32_t s = slots[i];
    if (s >= max_slots) return;
    if (lastop[s] != (((unsigned long long)tick << 32) | j)) return;
    const uint32_t idx = rank[s];
    if (idx >= n_total || s_slot[idx] != s) {
        atomicOr(err, ERR_MOVE_DEAD);
        return;
    }
    uint32_t sp = sps ? sps[i] : SP_KEEP;
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
    const float x = xs[i], z = zs[i];
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

// Also folds d_rel = max over "near" entities (live at t-1 and t in the same
// space, moved at most FAR_FRAC*D per axis) of displacement / D.
__global__ void k_keygen(const float *__restrict__ x, const float *__restrict__ z, const uint32_t *__restrict__ sp,
                         uint32_t n, const SpaceGrid *__restrict__ grid, uint32_t sentinel, uint32_t *keys,
                         uint32_t *vals, const float *__restrict__ p_x, const float *__restrict__ p_z,
                         const uint32_t *__restrict__ p_sp, const SpaceGrid *__restrict__ p_grid, uint32_t n_prev,
                         int *d_rel) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    float dr = 0.0f;
    if (i < n) {
        const uint32_t s = sp[i];
        uint32_t key = sentinel;
        const float xi = x[i], zi = z[i];
        if (s != SP_DEAD) {
            const SpaceGrid g = grid[s];
            const int cx = cell_of(xi, g.ox, g.inv, g.gx);
            const int cz = cell_of(zi, g.oz, g.inv, g.gz);
            key = g.base + (uint32_t)cz * g.gx + (uint32_t)cx;
            if (i < n_prev && p_sp[i] == s) {
                const float D = p_grid[s].D;
                const float dx = fabsf(xi - p_x[i]), dz = fabsf(zi - p_z[i]);
                const float thr = 0.25f * D;
                if (dx <= thr && dz <= thr) dr = fmaxf(dx, dz) / D;
            }
        }
        keys[i] = key;
        vals[i] = i;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dr = fmaxf(dr, __shfl_xor(dr, o));
    if (lane() == 0 && dr > 0.0f) atomicMax(d_rel, __float_as_int(dr));
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

// ---------------------------------------------------------------- tiles ------

__global__ void k_row_space(const SpaceGrid *__restrict__ grid, uint32_t n_spaces, uint32_t *row_space) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_spaces) return;
    const SpaceGrid g = grid[s];
    for (uint32_t cz = 0; cz < g.gz; ++cz) row_space[g.row_base + cz] = s;
}

__global__ void k_row_tiles(FrameView F, const uint32_t *__restrict__ row_space, uint32_t n_rows, uint32_t *cnt) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const SpaceGrid g = F.grid[row_space[r]];
    const uint32_t c0 = g.base + (r - g.row_base) * g.gx;
    const uint32_t n_row = F.cell_start[c0 + g.gx] - F.cell_start[c0];
    cnt[r] = (n_row + TILE_A - 1) / TILE_A;
}

__global__ void k_fill_tiles(FrameView F, const uint32_t *__restrict__ row_space, uint32_t n_rows,
                             const uint32_t *__restrict__ off, Tile *tiles) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const SpaceGrid g = F.grid[row_space[r]];
    const uint32_t c0 = g.base + (r - g.row_base) * g.gx;
    const uint32_t b = F.cell_start[c0], e = F.cell_start[c0 + g.gx];
    uint32_t t = off[r];
    for (uint32_t k = b; k < e; k += TILE_A, ++t) {
        Tile T;
        T.e0 = k;
        T.e1 = min(k + TILE_A, e);
        T.row = r;
        T.pad = 0;
        tiles[t] = T;
    }
}

// ---------------------------------------------------------------- pairs ------
// A flush's events are the diff of the go-aoi relation N between the
// previous state (t-1) and the new state (t) of every pair:
//   enter(A,B) = N_t(A,B) && !N_t-1(A,B),   leave(A,B) = N_t-1(A,B) && !N_t(A,B)
// N is symmetric in the pair, so each unordered pair is evaluated once and
// emitted in both directions.
//
// MODE 2 (combined): over the NEW grid.  The entity with the lower frame index
//   enumerates its partners (own cell row from a+1, then the rows above)
//   inside the symmetric box |dx|,|dz| <= H + margin, H = D(1 + 2 d_rel),
//   d_rel = the largest displacement / D of any "near" entity this flush.
//   Every pair with N_t is inside the box; so is every pair with N_t-1 whose
//   members both moved at most d_rel*D ("near").
// MODE 1 (special): over the PREVIOUS grid, only for entities that left,
//   changed space, or moved more than D/4 ("special").  Emits the leaves of
//   pairs the combined pass could not see (box test false at t).  A pair of
//   two specials is emitted by the one with the lower previous-frame index.
// Invalid other-time state (not live in this space then) is staged as NaN
// coordinates, which makes every window test false.

constexpr int PT = (int)TILE_A;  // threads per workgroup = entities per tile
constexpr int PCAP = 1024;       // candidates staged in LDS per chunk
constexpr int PS = 8;            // events buffered in LDS per thread
constexpr int PMAXR = 32;        // candidate rows a tile may span (else global path)
constexpr float FAR_FRAC = 0.25f;  // displacement > FAR_FRAC * D => special
constexpr uint32_t KIND_LEAVE = 0x80000000u;

// go-aoi relation: the owner (larger seq) W's window [fl32(w-D), fl32(w+D)]^2 contains the other
__device__ __forceinline__ bool rel(float xa, float za, uint64_t sa, float xb, float zb, uint64_t sb, float D) {
    const bool own = sa > sb;
    const float wx = own ? xa : xb, wz = own ? za : zb;
    const float px = own ? xb : xa, pz = own ? zb : za;
    return (int)(px >= wx - D) & (int)(px <= wx + D) & (int)(pz >= wz - D) & (int)(pz <= wz + D);
}

// symmetric candidate box: |b-a| <= H + (max|coord| + K) * 2^-20 per axis
__device__ __forceinline__ bool near_sym(float xa, float za, float xb, float zb, float H, float K) {
    const float mx = (fmaxf(fabsf(xa), fabsf(xb)) + K) * 0x1p-20f;
    const float mz = (fmaxf(fabsf(za), fabsf(zb)) + K) * 0x1p-20f;
    return (int)(fabsf(xb - xa) <= H + mx) & (int)(fabsf(zb - za) <= H + mz);
}

// "special" = left / changed space (NaN new position) or moved more than thr
__device__ __forceinline__ bool is_special(float xn, float zn, float xo, float zo, float thr) {
    return !((int)(fabsf(xn - xo) <= thr) & (int)(fabsf(zn - zo) <= thr));
}

__device__ __forceinline__ float load_drel(const float *p) { return p ? *p : 0.0f; }

struct Rec {  // 16 B staged record
    float x, z;
    uint64_t s;
};

template <int MODE>
struct PairIn {  // the entity that enumerates (A)
    Rec now, oth;  // MODE 2: now = t, oth = t-1; MODE 1: now = t-1, oth = t
    uint32_t a;    // frame index
    float D, H, K, thr;
    uint64_t seq_base;
    bool chg;
};

// frame entry j as (this-frame record, other-time record with NaN if invalid)
__device__ __forceinline__ void load_rec(const FrameView &F, const StateView &O, uint32_t j, Rec &now, Rec &oth) {
    now.x = F.x[j];
    now.z = F.z[j];
    now.s = F.seq[j];
    const bool ok = O.sp[j] == F.sp[j];
    oth.x = ok ? O.x[j] : __int_as_float(0x7FC00000);
    oth.z = ok ? O.z[j] : __int_as_float(0x7FC00000);
    oth.s = O.seq[j];
}

// Event kind of pair (A, B): 0 none, 1 enter, 2 leave.
template <int MODE>
__device__ __forceinline__ int pair_kind(const PairIn<MODE> &A, const Rec &bn, const Rec &bo, uint32_t b) {
    if (MODE == 2) {
        if (!near_sym(A.now.x, A.now.z, bn.x, bn.z, A.H, A.K)) return 0;
        if (!A.chg && bn.s < A.seq_base) return 0;  // neither touched: unchanged
        const bool nt = rel(A.now.x, A.now.z, A.now.s, bn.x, bn.z, bn.s, A.D);
        const bool no = rel(A.oth.x, A.oth.z, A.oth.s, bo.x, bo.z, bo.s, A.D);
        return nt == no ? 0 : (nt ? 1 : 2);
    } else {
        // previous grid; A is special.  now = t-1 state, oth = t state
        if (!near_sym(A.now.x, A.now.z, bn.x, bn.z, A.D, 2.0f * A.D)) return 0;
        if (!rel(A.now.x, A.now.z, A.now.s, bn.x, bn.z, bn.s, A.D)) return 0;       // not related at t-1
        if (rel(A.oth.x, A.oth.z, A.oth.s, bo.x, bo.z, bo.s, A.D)) return 0;         // still related at t
        if (near_sym(A.oth.x, A.oth.z, bo.x, bo.z, A.H, A.K)) return 0;              // combined pass saw it
        if (is_special(bo.x, bo.z, bn.x, bn.z, A.thr) && b < A.a) return 0;          // the other special emits
        return 2;
    }
}

// Row-major enumeration of A's partners straight from HBM/L2 (fallback and
// overflow path; same order and predicate as the LDS path).  Counts events
// per kind; when WRITE, writes (A,B),(B,A) for events number >= skip.
template <int MODE, bool WRITE>
__device__ void enum_global(const FrameView &F, const StateView &O, const SpaceGrid &g, const PairIn<MODE> &A,
                            int cx0, int cx1, int cz0, int cz1, uint32_t skip, uint2 *out, unsigned long long pe,
                            unsigned long long pl, uint64_t cap, uint32_t &ne, uint32_t &nl) {
    const uint32_t slot_a = WRITE ? F.slot[A.a] : 0u;
    uint32_t k = 0;
    for (int cz = cz0; cz <= cz1; ++cz) {
        const uint32_t row = g.base + (uint32_t)cz * g.gx;
        uint32_t jb = F.cell_start[row + (uint32_t)cx0];
        const uint32_t je = F.cell_start[row + (uint32_t)cx1 + 1u];
        if (MODE == 2 && cz == cz0) jb = A.a + 1;
        for (uint32_t b = jb; b < je; ++b) {
            if (MODE == 1 && b == A.a) continue;
            Rec bn, bo;
            load_rec(F, O, b, bn, bo);
            const int kind = pair_kind<MODE>(A, bn, bo, b);
            if (!kind) continue;
            if (WRITE && k >= skip) {
                const uint32_t slot_b = F.slot[b];
                const unsigned long long p = kind == 1 ? pe + 2ull * ne : pl + 2ull * nl;
                if (p + 1 < cap) {
                    out[p] = make_uint2(slot_a, slot_b);
                    out[p + 1] = make_uint2(slot_b, slot_a);
                }
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
__global__ __launch_bounds__(PT) void k_pairs(FrameView F, StateView O, TileSet TS, uint64_t seq_base,
                                              const float *__restrict__ d_rel, unsigned long long *counter,
                                              uint2 *tmp, uint64_t cap, uint32_t *tile_total,
                                              unsigned long long *tile_base, uint32_t tile_off, uint32_t leave_off) {
    __shared__ float4 s_now[PCAP];
    __shared__ float4 s_oth[PCAP];
    __shared__ uint32_t s_slot[PCAP];
    __shared__ uint32_t s_ev[PS * PT];
    __shared__ int s_box[4];
    __shared__ uint32_t s_seg[PMAXR];
    __shared__ uint32_t s_pre[PMAXR + 1];
    __shared__ uint32_t s_ws[PT / WAVE];
    __shared__ unsigned long long s_base;

    const uint32_t t = blockIdx.x;
    if (t >= *TS.n_tiles) return;  // uniform per workgroup
    const Tile T = TS.tiles[t];
    const uint32_t tid = threadIdx.x;
    const SpaceGrid g = F.grid[TS.row_space[T.row]];
    const float drel = load_drel(d_rel);
    PairIn<MODE> A;
    A.D = g.D;
    A.H = g.D * (1.0f + 2.0f * drel);
    A.K = 3.0f * g.D;
    A.thr = FAR_FRAC * g.D;
    A.seq_base = seq_base;
    A.a = T.e0 + tid;
    bool active = A.a < T.e1;
    int cx0 = 0, cx1 = -1, cz0 = 0, cz1 = -1;
    if (active) {
        load_rec(F, O, A.a, A.now, A.oth);
        if (MODE == 2) {
            A.chg = A.now.s >= seq_base;
            const float mr = (fabsf(A.now.x) + 2.0f * A.H + A.K) * 0x1p-19f;
            const float mz = (fabsf(A.now.z) + 2.0f * A.H + A.K) * 0x1p-19f;
            cx0 = cell_of(A.now.x - A.H - mr, g.ox, g.inv, g.gx);
            cx1 = cell_of(A.now.x + A.H + mr, g.ox, g.inv, g.gx);
            cz0 = cell_of(A.now.z, g.oz, g.inv, g.gz);  // own row (= the tile's row)
            cz1 = cell_of(A.now.z + A.H + mz, g.oz, g.inv, g.gz);
        } else {
            A.chg = true;
            active = is_special(A.oth.x, A.oth.z, A.now.x, A.now.z, A.thr);
            const float mr = (fabsf(A.now.x) + 3.0f * A.D) * 0x1p-19f;
            const float mz = (fabsf(A.now.z) + 3.0f * A.D) * 0x1p-19f;
            cx0 = cell_of(A.now.x - A.D - mr, g.ox, g.inv, g.gx);
            cx1 = cell_of(A.now.x + A.D + mr, g.ox, g.inv, g.gx);
            cz0 = cell_of(A.now.z - A.D - mz, g.oz, g.inv, g.gz);
            cz1 = cell_of(A.now.z + A.D + mz, g.oz, g.inv, g.gz);
        }
    }
    if (MODE == 1 && !__syncthreads_or(active)) {  // no special entity in this tile
        if (tid == 0) {
            tile_total[tile_off + t] = 0;
            tile_total[leave_off + tile_off + t] = 0;
        }
        return;
    }
    // tile box = union of the active entities' query cells (wave reductions, then LDS)
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
    const bool staged = nrows <= PMAXR;
    uint32_t ne = 0, nl = 0, nk = 0;  // enters, leaves, buffered
    if (staged) {
        if ((int)tid < nrows) {
            const uint32_t row = g.base + (uint32_t)(CZ0 + (int)tid) * g.gx;
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
                Rec bn, bo;
                load_rec(F, O, j, bn, bo);
                s_now[i] = make_float4(bn.x, bn.z, __uint_as_float((uint32_t)bn.s), __uint_as_float((uint32_t)(bn.s >> 32)));
                s_oth[i] = make_float4(bo.x, bo.z, __uint_as_float((uint32_t)bo.s), __uint_as_float((uint32_t)(bo.s >> 32)));
                s_slot[i] = F.slot[j];
            }
            __syncthreads();
            if (active) {
                for (int cz = cz0; cz <= cz1; ++cz) {
                    const int rr = cz - CZ0;
                    const uint32_t row = g.base + (uint32_t)cz * g.gx;
                    uint32_t jb = F.cell_start[row + (uint32_t)cx0];
                    const uint32_t je = F.cell_start[row + (uint32_t)cx1 + 1u];
                    if (MODE == 2 && cz == cz0) jb = A.a + 1;
                    const uint32_t vb = s_pre[rr] + (jb - s_seg[rr]);
                    const uint32_t ve = vb + (je - jb);
                    const uint32_t lo = max(vb, base), hi = min(ve, base + lim);
                    for (uint32_t v = lo; v < hi; ++v) {
                        const uint32_t i = v - base;
                        const uint32_t b = jb + (v - vb);
                        if (MODE == 1 && b == A.a) continue;
                        const float4 qn = s_now[i], qo = s_oth[i];
                        Rec bn, bo;
                        bn.x = qn.x; bn.z = qn.y;
                        bn.s = ((uint64_t)__float_as_uint(qn.w) << 32) | __float_as_uint(qn.z);
                        bo.x = qo.x; bo.z = qo.y;
                        bo.s = ((uint64_t)__float_as_uint(qo.w) << 32) | __float_as_uint(qo.z);
                        const int kind = pair_kind<MODE>(A, bn, bo, b);
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
        enum_global<MODE, false>(F, O, g, A, cx0, cx1, cz0, cz1, 0, nullptr, 0, 0, 0, ne, nl);
    }
    // offsets: directed pairs = 2 per event, enters then leaves of the tile
    uint32_t te, tl;
    const uint32_t oe = block_excl_scan(2 * ne, s_ws, te);
    __syncthreads();
    const uint32_t ol = block_excl_scan(2 * nl, s_ws, tl);
    if (tid == 0) {
        const uint32_t tot = te + tl;
        const unsigned long long b = tot ? atomicAdd(counter, (unsigned long long)tot) : 0ull;
        s_base = b;
        tile_total[tile_off + t] = te;
        tile_base[tile_off + t] = b;
        tile_total[leave_off + tile_off + t] = tl;
        tile_base[leave_off + tile_off + t] = b + te;
    }
    __syncthreads();
    if (active && (ne | nl)) {
        const unsigned long long pe = s_base + oe, pl = s_base + te + ol;
        if (staged) {
            const uint32_t slot_a = F.slot[A.a];
            const uint32_t k = min(nk, (uint32_t)PS);
            uint32_t ie = 0, il = 0;
            for (uint32_t q = 0; q < k; ++q) {
                const uint32_t e = s_ev[q * PT + tid];
                const uint32_t slot_b = e & ~KIND_LEAVE;
                const bool lv = (e & KIND_LEAVE) != 0u;
                const unsigned long long p = lv ? pl + 2ull * il : pe + 2ull * ie;
                il += (uint32_t)lv;
                ie += (uint32_t)!lv;
                if (p + 1 < cap) {
                    tmp[p] = make_uint2(slot_a, slot_b);
                    tmp[p + 1] = make_uint2(slot_b, slot_a);
                }
            }
            if (nk > PS) {
                uint32_t we = 0, wl = 0;  // continue after the buffered events, in order
                enum_global<MODE, true>(F, O, g, A, cx0, cx1, cz0, cz1, PS, tmp, pe + 2ull * ie, pl + 2ull * il,
                                        cap, we, wl);
            }
        } else {
            uint32_t we = 0, wl = 0;
            enum_global<MODE, true>(F, O, g, A, cx0, cx1, cz0, cz1, 0, tmp, pe, pl, cap, we, wl);
        }
    }
}

__global__ void k_reorder(const uint32_t *__restrict__ dest, const uint32_t *__restrict__ tile_total,
                          const unsigned long long *__restrict__ tile_base, uint32_t n_entries,
                          const uint2 *__restrict__ tmp, uint2 *out, uint64_t cap) {
    const uint32_t e = blockIdx.x;
    if (e >= n_entries) return;
    const uint32_t cnt = tile_total[e];
    if (!cnt) return;
    const unsigned long long src = tile_base[e];
    const uint64_t dst = dest[e];
    for (uint32_t k = threadIdx.x; k < cnt; k += blockDim.x)
        if (src + k < cap && dst + k < cap) out[dst + k] = tmp[src + k];
}

__global__ void k_finish(const uint32_t *__restrict__ dest, uint32_t n_enter_entries, uint32_t n_entries,
                         const uint32_t *__restrict__ err, const unsigned long long *__restrict__ counter,
                         TickResult *res) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    res->n_enter = dest[n_enter_entries];
    res->n_total = dest[n_entries];
    res->err = *err;
    res->total64 = *counter;
}

// ----------------------------------------------------------------- bbox ------

__device__ __forceinline__ int f2o(float f) {
    int i = __float_as_int(f);
    return i ^ ((i >> 31) & 0x7FFFFFFF);
}

__device__ __forceinline__ void bbox_flush(int *bbox, uint32_t ms, uint32_t sp, int mnx, int mnz, int mxx, int mxz) {
    atomicMin(&bbox[sp], mnx);
    atomicMin(&bbox[ms + sp], mnz);
    atomicMax(&bbox[2 * ms + sp], mxx);
    atomicMax(&bbox[3 * ms + sp], mxz);
}

constexpr uint32_t BB_PER_THREAD = 16;

// Per-space bounding box of the frame (for the next flush's grid).  Each lane
// folds 16 consecutive entries; runs of one space are merged per wave.
__global__ void k_bbox(FrameView F, int *bbox, uint32_t ms) {
    const uint32_t k0 = (blockIdx.x * blockDim.x + threadIdx.x) * BB_PER_THREAD;
    const uint32_t k1 = min(k0 + BB_PER_THREAD, F.n);
    uint32_t cur = SP_DEAD;
    int mnx = INT_MAX, mnz = INT_MAX, mxx = INT_MIN, mxz = INT_MIN;
    for (uint32_t k = k0; k < k1; ++k) {
        const uint32_t sp = F.sp[k];
        if (sp != cur) {
            if (cur != SP_DEAD && cur < ms) bbox_flush(bbox, ms, cur, mnx, mnz, mxx, mxz);
            cur = sp;
            mnx = mnz = INT_MAX;
            mxx = mxz = INT_MIN;
        }
        const int ix = f2o(F.x[k]), iz = f2o(F.z[k]);
        mnx = min(mnx, ix);
        mnz = min(mnz, iz);
        mxx = max(mxx, ix);
        mxz = max(mxz, iz);
    }
    const uint32_t first = __shfl(cur, 0);
    if (__all(cur == first || cur == SP_DEAD)) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            mnx = min(mnx, __shfl_xor(mnx, o));
            mnz = min(mnz, __shfl_xor(mnz, o));
            mxx = max(mxx, __shfl_xor(mxx, o));
            mxz = max(mxz, __shfl_xor(mxz, o));
        }
        if (lane() == 0 && first != SP_DEAD && first < ms) bbox_flush(bbox, ms, first, mnx, mnz, mxx, mxz);
    } else if (cur != SP_DEAD && cur < ms) {
        bbox_flush(bbox, ms, cur, mnx, mnz, mxx, mxz);
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

void launch_copy_state(uint32_t n, const float *p_x, const float *p_z, const uint64_t *p_seq, const uint32_t *p_sp,
                       const uint32_t *p_slot, float *s_x, float *s_z, uint64_t *s_seq, uint32_t *s_sp,
                       uint32_t *s_slot, hipStream_t st) {
    if (!n) return;
    k_copy_state<<<cdiv(n, 256), 256, 0, st>>>(n, p_x, p_z, p_seq, p_sp, p_slot, s_x, s_z, s_seq, s_sp, s_slot);
}

void launch_init_appended(const uint32_t *new_slots, uint32_t n_app, uint32_t n_prev, uint32_t *s_slot,
                          uint32_t *s_sp, uint64_t *s_seq, uint32_t *rank, hipStream_t st) {
    if (!n_app) return;
    k_init_appended<<<cdiv(n_app, 256), 256, 0, st>>>(new_slots, n_app, n_prev, s_slot, s_sp, s_seq, rank);
}

void launch_ops_claim(const uint32_t *slots, uint32_t n, uint32_t j0, uint32_t max_slots, unsigned long long *lastop,
                      uint32_t tick_id, uint32_t *err, hipStream_t st) {
    if (!n) return;
    k_ops_claim<<<cdiv(n, 256), 256, 0, st>>>(slots, n, j0, max_slots, lastop, tick_id, err);
}

void launch_ops_apply(const uint32_t *slots, const float *x, const float *z, const uint32_t *sp, uint32_t n,
                      uint32_t j0, uint32_t max_slots, const unsigned long long *lastop, uint32_t tick_id,
                      const uint32_t *rank, uint32_t n_total, uint64_t seq_base, float *s_x, float *s_z,
                      uint64_t *s_seq, uint32_t *s_sp, const uint32_t *s_slot, uint32_t *err, hipStream_t st) {
    if (!n) return;
    k_ops_apply<<<cdiv(n, 256), 256, 0, st>>>(slots, x, z, sp, n, j0, max_slots, lastop, tick_id, rank, n_total,
                                              seq_base, s_x, s_z, s_seq, s_sp, s_slot, err);
}

void launch_keygen(const float *s_x, const float *s_z, const uint32_t *s_sp, uint32_t n_total,
                   const SpaceGrid *grid, uint32_t sentinel, uint32_t *keys, uint32_t *vals, const float *p_x,
                   const float *p_z, const uint32_t *p_sp, const SpaceGrid *p_grid, uint32_t n_prev, int *d_rel,
                   hipStream_t st) {
    if (!n_total) return;
    k_keygen<<<cdiv(n_total, 256), 256, 0, st>>>(s_x, s_z, s_sp, n_total, grid, sentinel, keys, vals, p_x, p_z,
                                                 p_sp, p_grid, n_prev, d_rel);
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

void build_tiles(FrameView F, uint32_t n_space_ids, uint32_t n_rows, uint32_t *row_space, uint32_t *row_ntiles,
                 Tile *tiles, uint32_t *scan_tmp, hipStream_t st) {
    if (n_space_ids) k_row_space<<<cdiv(n_space_ids, 256), 256, 0, st>>>(F.grid, n_space_ids, row_space);
    (void)hipMemsetAsync(row_ntiles + n_rows, 0, sizeof(uint32_t), st);
    if (n_rows) k_row_tiles<<<cdiv(n_rows, 256), 256, 0, st>>>(F, row_space, n_rows, row_ntiles);
    scan_exclusive(row_ntiles, row_ntiles, (size_t)n_rows + 1, scan_tmp, st);
    if (n_rows) k_fill_tiles<<<cdiv(n_rows, 256), 256, 0, st>>>(F, row_space, n_rows, row_ntiles, tiles);
}

void launch_pairs(int mode, FrameView F, StateView O, TileSet T, uint64_t seq_base, const float *d_rel,
                  unsigned long long *counter, uint32_t *tmp_pairs, uint64_t cap, uint32_t *tile_total,
                  unsigned long long *tile_base, uint32_t tile_off, uint32_t leave_off, hipStream_t st) {
    if (!F.n || !T.bound) return;
    uint2 *tmp = reinterpret_cast<uint2 *>(tmp_pairs);
    if (mode == 2)
        k_pairs<2><<<T.bound, PT, 0, st>>>(F, O, T, seq_base, d_rel, counter, tmp, cap, tile_total, tile_base,
                                           tile_off, leave_off);
    else
        k_pairs<1><<<T.bound, PT, 0, st>>>(F, O, T, seq_base, d_rel, counter, tmp, cap, tile_total, tile_base,
                                           tile_off, leave_off);
}

void launch_reorder(const uint32_t *dest, const uint32_t *tile_total, const unsigned long long *tile_base,
                    uint32_t n_entries, const uint32_t *tmp_pairs, uint32_t *out_pairs, uint64_t cap,
                    hipStream_t st) {
    if (!n_entries) return;
    k_reorder<<<n_entries, 128, 0, st>>>(dest, tile_total, tile_base, n_entries,
                                         reinterpret_cast<const uint2 *>(tmp_pairs),
                                         reinterpret_cast<uint2 *>(out_pairs), cap);
}

void launch_finish(const uint32_t *dest, uint32_t n_enter_entries, uint32_t n_entries, const uint32_t *err,
                   const unsigned long long *counter, TickResult *res, hipStream_t st) {
    k_finish<<<1, 64, 0, st>>>(dest, n_enter_entries, n_entries, err, counter, res);
}

void launch_bbox(FrameView F, int *bbox, uint32_t max_spaces, hipStream_t st) {
    if (!F.n) return;
    const uint32_t threads = cdiv(F.n, BB_PER_THREAD);
    k_bbox<<<cdiv(threads, 256), 256, 0, st>>>(F, bbox, max_spaces);
}

void launch_neighbors(FrameView F, const uint32_t *rank, uint32_t slot, uint32_t *out, uint32_t cap,
                      uint32_t *count, hipStream_t st) {
    k_neighbors<<<1, 256, 0, st>>>(F, rank, slot, out, cap, count);
}

}  // namespace gw
