// Sparse flush: a flush of a few Moved calls (the game loop's read-after-write case: a timer
// callback moves an entity, the next one reads interest sets) priced by its calls, not by the
// world.  The full flush rebuilds the frame (keys, sort, gather, the band sweep of every entity:
// ~0.2 ms at 1M entities whatever the call count).  Here, with the frame of the last flush in place:
//
//   1. k_ops_claim (gwaoi_kernels.hip): the last op of each slot wins, as in every flush;
//   2. k_sp_events<0>: one workgroup per winning op A scans the grid cells around A's old and new
//      positions; a partner B that is no mover keeps its frame state, so the pair's relation before
//      is rel(A_old, B) and after rel(A_new, B) (go-aoi's window test with A's new, largest seq).
//      Mover pairs are taken from the op list (the lower slot of the two), both states from the
//      frame and the ops.  Counts enters / leaves per op;
//   3. k_sp_scan: the per-op offsets, the flush summary, the capacity check;
//   4. k_sp_events<1>: the same scan, writing the directed pairs [enters | leaves] in op order;
//   5. k_sp_apply (one workgroup): the frame patched in place -- each winner's record, and a winner
//      whose cell changed shifted into its new cell (the entries between move by one, cell starts
//      by one, SlotInfo.rank follows).  The frame stays exactly the stable sort a full flush makes
//      of it, up to the order inside a cell (which nothing depends on).
//
// Steps 3 and 5 decline (TickOut.pad != 0, nothing mutated) when the events outgrow the flush
// set's buffer or the shifts are long; the host then runs the full flush over the same queue.
// The pair relation between flushes is the closed form over the frame, so
// the events are exactly those of the full flush of the same queue.
#include "gwaoi_device.h"

namespace gw {
namespace {

constexpr int WAVE = 64;
constexpr uint32_t SP_T = 256;         // threads per op workgroup
constexpr uint32_t SA_T = 1024;        // threads of the apply workgroup
constexpr uint32_t SP_MAX_CHANGERS = 64;     // winners changing cell one sparse flush shifts
constexpr uint32_t SP_MAX_SHIFT = 1u << 17;  // frame entries those shifts may move in total

struct SparseArgs {
    Rec16 *rec;
    SlotSp *ss;
    uint32_t *key;
    uint32_t *cell_start;
    const SpaceGrid *grid;
    SlotTab info;
    const uint32_t *op_slot;
    const float *op_x, *op_z;
    const unsigned long long *op_seq;  // nullptr: op j's seq is seq0 + j
    unsigned long long seq0;
    uint32_t k;
    uint32_t tick;
    uint32_t *cnt;  // [0, k): enters per op, [k, 2k): leaves, their exclusive scans [2k, 4k), totals [4k, 4k+2), declined [4k+2]
    uint2 *out;
    uint64_t cap;
    TickOut *res;
};

__device__ __forceinline__ unsigned long long op_seq(const SparseArgs &A, uint32_t j) {
    return A.op_seq ? A.op_seq[j] : A.seq0 + j;
}

__device__ __forceinline__ bool winner(const SparseArgs &A, uint32_t j, uint32_t slot) {
    return A.info.lastop[slot] == (((unsigned long long)A.tick << 32) | j);
}

// Block-wide exclusive scan of two flags, in thread order, and their block totals.
__device__ __forceinline__ void scan2(bool e, bool l, uint32_t *ws, uint32_t &pe, uint32_t &pl, uint32_t &te,
                                      uint32_t &tl) {
    const unsigned long long me = __ballot(e), ml = __ballot(l);
    const uint32_t w = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    const unsigned long long lt = (1ull << __lane_id()) - 1ull;
    __syncthreads();
    if (__lane_id() == 0) {
        ws[w] = (uint32_t)__popcll(me);
        ws[nw + w] = (uint32_t)__popcll(ml);
    }
    __syncthreads();
    uint32_t be = 0, bl = 0;
    te = tl = 0;
    for (uint32_t q = 0; q < nw; ++q) {
        if (q < w) {
            be += ws[q];
            bl += ws[nw + q];
        }
        te += ws[q];
        tl += ws[nw + q];
    }
    pe = be + (uint32_t)__popcll(me & lt);
    pl = bl + (uint32_t)__popcll(ml & lt);
}

template <int PHASE>
__global__ __launch_bounds__(SP_T) void k_sp_events(SparseArgs A) {
    __shared__ uint32_t ws[2 * SP_T / WAVE];
    const uint32_t j = blockIdx.x, tid = threadIdx.x;
    const uint32_t slot = A.op_slot[j];
    if (!winner(A, j, slot)) {
        if (PHASE == 0 && tid == 0) A.cnt[j] = A.cnt[A.k + j] = 0;
        return;
    }
    const uint32_t ra = A.info.rank[slot];
    const Rec16 ao = ld_rec(A.rec, ra);
    const uint32_t sp = ld_ss(A.ss, ra).sp;
    const SpaceGrid g = A.grid[sp];
    const float D = g.D;
    const float nx = A.op_x[j], nz = A.op_z[j];
    const unsigned long long ns = op_seq(A, j);
    // every B related to A before or after lies within D (+ the float32 rounding of fl32(w +- D))
    // of A's old or new position
    const float mx = (fmaxf(fabsf(ao.x), fabsf(nx)) + 3.0f * D) * 0x1p-20f;
    const float mz = (fmaxf(fabsf(ao.z), fabsf(nz)) + 3.0f * D) * 0x1p-20f;
    const int cx0 = cell_of(fminf(ao.x, nx) - D - mx, g.ox, g.inv, g.gx);
    const int cx1 = cell_of(fmaxf(ao.x, nx) + D + mx, g.ox, g.inv, g.gx);
    const int cz0 = cell_of(fminf(ao.z, nz) - D - mz, g.oz, g.inv, g.gz);
    const int cz1 = cell_of(fmaxf(ao.z, nz) + D + mz, g.oz, g.inv, g.gz);
    uint32_t ne = 0, nl = 0;
    unsigned long long pe = 0, pl = 0;  // PHASE 1: this op's next enter / leave position (directed pairs)
    if (PHASE == 1) {
        pe = 2ull * A.cnt[2 * A.k + j];
        pl = 2ull * ((unsigned long long)A.cnt[4 * A.k] + A.cnt[3 * A.k + j]);
    }
    auto emit = [&](bool valid, int kind, uint32_t b_slot) {
        uint32_t oe, ol, te, tl;
        scan2(valid && kind == 1, valid && kind == 2, ws, oe, ol, te, tl);
        if (PHASE == 1 && valid && kind) {
            const unsigned long long p = kind == 1 ? pe + 2ull * oe : pl + 2ull * ol;
            if (p + 1 < A.cap) {
                A.out[p] = make_uint2(slot, b_slot);
                A.out[p + 1] = make_uint2(b_slot, slot);
            }
        }
        ne += te;
        nl += tl;
        pe += 2ull * te;
        pl += 2ull * tl;
    };
    // partners in the frame that are not movers of this flush (their state is the frame's)
    for (int cz = cz0; cz <= cz1; ++cz) {
        const uint32_t row = g.base + (uint32_t)cz * g.gx;
        const uint32_t jb = A.cell_start[row + (uint32_t)cx0], je = A.cell_start[row + (uint32_t)cx1 + 1u];
        for (uint32_t b0 = jb; b0 < je; b0 += SP_T) {
            const uint32_t b = b0 + tid;
            int kind = 0;
            uint32_t b_slot = 0;
            if (b < je && b != ra) {
                b_slot = ld_ss(A.ss, b).slot;
                if ((uint32_t)(A.info.lastop[b_slot] >> 32) != A.tick) {
                    const Rec16 br = ld_rec(A.rec, b);
                    const bool was = rel(ao.x, ao.z, ao.s, br.x, br.z, br.s, D);
                    const bool is = rel(nx, nz, ns, br.x, br.z, br.s, D);
                    kind = was == is ? 0 : is ? 1 : 2;
                }
            }
            emit(b < je, kind, b_slot);
        }
    }
    // pairs of two movers, from the lower slot: both states from the frame and the ops
    for (uint32_t q0 = 0; q0 < A.k; q0 += SP_T) {
        const uint32_t q = q0 + tid;
        int kind = 0;
        uint32_t b_slot = 0;
        if (q < A.k) {
            b_slot = A.op_slot[q];
            if (b_slot > slot && winner(A, q, b_slot)) {
                const uint32_t rb = A.info.rank[b_slot];
                if (ld_ss(A.ss, rb).sp == sp) {
                    const Rec16 bo = ld_rec(A.rec, rb);
                    const bool was = rel(ao.x, ao.z, ao.s, bo.x, bo.z, bo.s, D);
                    const bool is = rel(nx, nz, ns, A.op_x[q], A.op_z[q], op_seq(A, q), D);
                    kind = was == is ? 0 : is ? 1 : 2;
                }
            }
        }
        emit(q < A.k, kind, b_slot);
    }
    if (PHASE == 0 && tid == 0) {
        A.cnt[j] = ne;
        A.cnt[A.k + j] = nl;
    }
}

// Per-op offsets (exclusive scans of the enter and leave counts), the summary, the capacity check.
__global__ __launch_bounds__(SA_T) void k_sp_scan(SparseArgs A) {
    __shared__ uint32_t ws[2 * SA_T / WAVE];
    __shared__ uint32_t carry[2];
    if (threadIdx.x == 0) carry[0] = carry[1] = 0;
    for (uint32_t j0 = 0; j0 < A.k; j0 += SA_T) {
        const uint32_t j = j0 + threadIdx.x;
        const uint32_t e = j < A.k ? A.cnt[j] : 0u, l = j < A.k ? A.cnt[A.k + j] : 0u;
        // exclusive scan of counts (not flags): wave scan, then the waves' totals
        uint32_t ie = e, il = l;
        for (int o = 1; o < WAVE; o <<= 1) {
            const uint32_t te = (uint32_t)__shfl_up((int)ie, o), tl = (uint32_t)__shfl_up((int)il, o);
            if ((int)__lane_id() >= o) {
                ie += te;
                il += tl;
            }
        }
        const uint32_t w = threadIdx.x / WAVE, nw = SA_T / WAVE;
        __syncthreads();
        if (__lane_id() == WAVE - 1) {
            ws[w] = ie;
            ws[nw + w] = il;
        }
        __syncthreads();
        uint32_t be = carry[0], bl = carry[1], te = 0, tl = 0;
        for (uint32_t q = 0; q < nw; ++q) {
            if (q < w) {
                be += ws[q];
                bl += ws[nw + q];
            }
            te += ws[q];
            tl += ws[nw + q];
        }
        if (j < A.k) {
            A.cnt[2 * A.k + j] = be + ie - e;
            A.cnt[3 * A.k + j] = bl + il - l;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            carry[0] += te;
            carry[1] += tl;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const uint32_t E = carry[0], L = carry[1];
        A.cnt[4 * A.k] = E;
        A.cnt[4 * A.k + 1] = L;
        const unsigned long long tot = 2ull * ((unsigned long long)E + L);
        A.res->n_enter = 2 * E;
        A.res->n_total = (uint32_t)tot;
        A.res->err = 0;
        const uint32_t declined = tot > A.cap ? 1u : 0u;  // the flush set's buffer is too small (the full flush grows it)
        A.cnt[4 * A.k + 2] = declined;
        A.res->pad = declined;
        A.res->total64 = tot;
        A.res->seq_max = 0;
        for (int q = 0; q < (int)DBG_N; ++q) A.res->dbg[q] = 0;
    }
}

// Shift one mover (now at frame index p, key k1, new key k2 != k1) into its new cell: the entries
// between move by one (in place, in chunks ordered so that no entry is overwritten before it is
// read), the cell starts between by one, and SlotInfo.rank of every moved entry follows.
__device__ void sp_shift(const SparseArgs &A, uint32_t p, uint32_t k1, uint32_t k2) {
    __shared__ uint4 s_rec[SA_T];
    __shared__ uint2 s_ss[SA_T];
    __shared__ uint32_t s_key[SA_T];
    __shared__ uint4 m_rec;
    __shared__ uint2 m_ss;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) {
        m_rec = reinterpret_cast<const uint4 *>(A.rec)[p];
        m_ss = reinterpret_cast<const uint2 *>(A.ss)[p];
    }
    uint32_t dst;
    if (k2 > k1) {  // entries p+1 .. e down by one, the mover to e
        const uint32_t e = A.cell_start[k2 + 1] - 1u;
        __syncthreads();
        for (uint32_t c0 = p + 1; c0 <= e; c0 += SA_T) {
            const uint32_t i = c0 + tid;
            const bool v = i <= e;
            if (v) {
                s_rec[tid] = reinterpret_cast<const uint4 *>(A.rec)[i];
                s_ss[tid] = reinterpret_cast<const uint2 *>(A.ss)[i];
                s_key[tid] = A.key[i];
            }
            __syncthreads();
            if (v) {
                reinterpret_cast<uint4 *>(A.rec)[i - 1] = s_rec[tid];
                reinterpret_cast<uint2 *>(A.ss)[i - 1] = s_ss[tid];
                A.key[i - 1] = s_key[tid];
                A.info.rank[s_ss[tid].x] = i - 1;
            }
            __syncthreads();
        }
        for (uint32_t c = k1 + 1 + tid; c <= k2; c += SA_T) A.cell_start[c] -= 1u;
        dst = e;
    } else {  // entries s .. p-1 up by one, the mover to s
        const uint32_t s = A.cell_start[k2 + 1];
        __syncthreads();
        for (uint32_t hi = p; hi > s;) {  // chunks from the top down
            const uint32_t lo = hi - s > SA_T ? hi - SA_T : s;
            const uint32_t i = lo + tid;
            const bool v = i < hi;
            if (v) {
                s_rec[tid] = reinterpret_cast<const uint4 *>(A.rec)[i];
                s_ss[tid] = reinterpret_cast<const uint2 *>(A.ss)[i];
                s_key[tid] = A.key[i];
            }
            __syncthreads();
            if (v) {
                reinterpret_cast<uint4 *>(A.rec)[i + 1] = s_rec[tid];
                reinterpret_cast<uint2 *>(A.ss)[i + 1] = s_ss[tid];
                A.key[i + 1] = s_key[tid];
                A.info.rank[s_ss[tid].x] = i + 1;
            }
            __syncthreads();
            hi = lo;
        }
        for (uint32_t c = k2 + 1 + tid; c <= k1; c += SA_T) A.cell_start[c] += 1u;
        dst = s;
    }
    __syncthreads();
    if (tid == 0) {
        reinterpret_cast<uint4 *>(A.rec)[dst] = m_rec;
        reinterpret_cast<uint2 *>(A.ss)[dst] = m_ss;
        A.key[dst] = k2;
        A.info.rank[m_ss.x] = dst;
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t key_of(const SpaceGrid &g, float x, float z) {
    return g.base + (uint32_t)cell_of(z, g.oz, g.inv, g.gz) * g.gx + (uint32_t)cell_of(x, g.ox, g.inv, g.gx);
}

// The frame patched in place (one workgroup): first decide (no write before the decision), then
// the winners' records, then the cell changers one after another in op order.  win(j, slot): op j
// is the last op of its slot in this flush.
template <class Win>
__device__ void sp_apply_body(const SparseArgs &A, Win win) {
    __shared__ uint32_t n_chg, shift_sum;
    __shared__ uint32_t chg[SP_MAX_CHANGERS];
    const uint32_t tid = threadIdx.x;
    if (tid == 0) n_chg = shift_sum = 0;
    __syncthreads();
    for (uint32_t j = tid; j < A.k; j += SA_T) {
        const uint32_t slot = A.op_slot[j];
        if (!win(j, slot)) continue;
        const uint32_t r = A.info.rank[slot];
        const uint32_t k1 = A.key[r], k2 = key_of(A.grid[ld_ss(A.ss, r).sp], A.op_x[j], A.op_z[j]);
        if (k1 == k2) continue;
        const uint32_t c = atomicAdd(&n_chg, 1u);
        if (c < SP_MAX_CHANGERS) chg[c] = j;
        // entries this shift moves (against the starts before any shift: an estimate of the total)
        const uint32_t d = k2 > k1 ? A.cell_start[k2 + 1] - 1u - r : r - A.cell_start[k2 + 1];
        atomicAdd(&shift_sum, min(d, SP_MAX_SHIFT + 1u));
    }
    __syncthreads();
    if (n_chg > SP_MAX_CHANGERS || shift_sum > SP_MAX_SHIFT) {
        if (tid == 0) A.res->pad = 2u;  // declined: too much of the frame would move
        return;
    }
    // the winners' records (a changer's record moves with it below)
    for (uint32_t j = tid; j < A.k; j += SA_T) {
        const uint32_t slot = A.op_slot[j];
        if (!win(j, slot)) continue;
        Rec16 r;
        r.x = A.op_x[j];
        r.z = A.op_z[j];
        r.s = op_seq(A, j);
        st_rec(A.rec, A.info.rank[slot], r);
    }
    // changers in op order (deterministic frame): rank-sort the short list
    __shared__ uint32_t ord[SP_MAX_CHANGERS];
    const uint32_t nc = n_chg;
    if (tid < nc) {
        uint32_t pos = 0;
        for (uint32_t q = 0; q < nc; ++q) pos += chg[q] < chg[tid];
        ord[pos] = chg[tid];
    }
    __syncthreads();
    for (uint32_t c = 0; c < nc; ++c) {
        const uint32_t j = ord[c], slot = A.op_slot[j];
        const uint32_t p = A.info.rank[slot];
        const uint32_t k1 = A.key[p], k2 = key_of(A.grid[ld_ss(A.ss, p).sp], A.op_x[j], A.op_z[j]);
        sp_shift(A, p, k1, k2);
    }
}

__global__ __launch_bounds__(SA_T) void k_sp_apply(SparseArgs A) {
    if (A.cnt[4 * A.k + 2]) return;  // declined by the scan
    sp_apply_body(A, [&](uint32_t j, uint32_t slot) { return winner(A, j, slot); });
}

// ---- the fused form: one launch for a flush of up to SP_FUSED_MAX ops --------------------------
// One workgroup per op finds its events and keeps them in a scratch row of its own; the workgroup
// that finishes last (told by the value its arrival add returns) lays them out [enters | leaves] in
// op order and patches the frame.  Claims are not stored: every workgroup holds the ops' slots in
// an LDS hash set (the last op of a slot is its winner; a frame partner in the set is a mover of
// this flush, whose pairs come from the op list).  The candidates of an op are the two windows
// around its old and new positions (the new one less the cells of the old), laid end to end as
// row ranges and dealt to the lanes flat, so a candidate costs one round trip whatever the row.
// An op with more events than the scratch row holds, or more row ranges than SF_MAXSEG, makes the
// flush decline (pad 3) before any write: the host then runs the kernels above.
constexpr uint32_t SP_FUSED_MAX = 256;
constexpr uint32_t SF_HASH = 1024;  // LDS hash set of the op slots (load factor <= 1/4)
constexpr uint32_t SF_MAXSEG = 128;
constexpr uint32_t SF_EMPTY = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t sf_hash(uint32_t s) { return (s * 2654435761u) >> 22; }  // 10 bits

__device__ __forceinline__ bool sf_find(const uint32_t *hs, uint32_t s) {
    for (uint32_t h = sf_hash(s);; h = (h + 1u) & (SF_HASH - 1u)) {
        const uint32_t v = hs[h];
        if (v == s) return true;
        if (v == SF_EMPTY) return false;
    }
}

__global__ __launch_bounds__(SA_T) void k_sp_fused(SparseArgs A, uint32_t *scr, uint32_t scr_cap, uint32_t *done) {
    __shared__ uint32_t hs[SF_HASH], hl[SF_HASH];  // slot set, the last op index of each slot
    __shared__ uint32_t s_slot[SP_FUSED_MAX], s_pos[SP_FUSED_MAX];
    __shared__ uint32_t seg_b[SF_MAXSEG], seg_c[SF_MAXSEG + 1];
    __shared__ uint32_t ws[2 * SA_T / WAVE];
    __shared__ uint32_t s_off[2][SP_FUSED_MAX + 1];
    __shared__ uint32_t s_flag;
    const uint32_t tid = threadIdx.x, j = blockIdx.x, k = A.k;
    for (uint32_t i = tid; i < SF_HASH; i += SA_T) {
        hs[i] = SF_EMPTY;
        hl[i] = 0;
    }
    if (tid < k) s_slot[tid] = A.op_slot[tid];
    __syncthreads();
    if (tid < k) {
        const uint32_t sl = s_slot[tid];
        uint32_t h = sf_hash(sl);
        for (;; h = (h + 1u) & (SF_HASH - 1u)) {
            const uint32_t old = atomicCAS(&hs[h], SF_EMPTY, sl);
            if (old == SF_EMPTY || old == sl) break;
        }
        atomicMax(&hl[h], tid);
        s_pos[tid] = h;
    }
    __syncthreads();
    auto win = [&](uint32_t q) { return hl[s_pos[q]] == q; };
    const uint32_t slot = s_slot[j];
    uint32_t *se = scr + (size_t)j * 2u * scr_cap, *sl_ = se + scr_cap;  // this op's enters, leaves (B slots)
    uint32_t ne = 0, nl = 0;
    bool ovf = false;
    if (win(j)) {
        const uint32_t ra = A.info.rank[slot];
        const Rec16 ao = ld_rec(A.rec, ra);
        const uint32_t sp = ld_ss(A.ss, ra).sp;
        const SpaceGrid g = A.grid[sp];
        const float D = g.D;
        const float nx = A.op_x[j], nz = A.op_z[j];
        const unsigned long long ns = op_seq(A, j);
        // every B related to A before or after lies within D (+ the float32 rounding of fl32(w +- D))
        // of A's old or new position
        const float mx = (fmaxf(fabsf(ao.x), fabsf(nx)) + 3.0f * D) * 0x1p-20f;
        const float mz = (fmaxf(fabsf(ao.z), fabsf(nz)) + 3.0f * D) * 0x1p-20f;
        const int ox0 = cell_of(ao.x - D - mx, g.ox, g.inv, g.gx), ox1 = cell_of(ao.x + D + mx, g.ox, g.inv, g.gx);
        const int oz0 = cell_of(ao.z - D - mz, g.oz, g.inv, g.gz), oz1 = cell_of(ao.z + D + mz, g.oz, g.inv, g.gz);
        const int nx0 = cell_of(nx - D - mx, g.ox, g.inv, g.gx), nx1 = cell_of(nx + D + mx, g.ox, g.inv, g.gx);
        const int nz0 = cell_of(nz - D - mz, g.oz, g.inv, g.gz), nz1 = cell_of(nz + D + mz, g.oz, g.inv, g.gz);
        const uint32_t nO = (uint32_t)(oz1 - oz0 + 1), nN = (uint32_t)(nz1 - nz0 + 1);
        const uint32_t nseg = nO + 2u * nN;
        if (nseg <= SF_MAXSEG) {
            // row ranges: the old window's rows, then each new-window row less the old window's cells
            if (tid < nO + nN) {
                int r, c0[2], c1[2];
                if (tid < nO) {
                    r = oz0 + (int)tid;
                    c0[0] = ox0;
                    c1[0] = ox1;
                    c0[1] = 1;
                    c1[1] = 0;
                } else {
                    r = nz0 + (int)(tid - nO);
                    if (r >= oz0 && r <= oz1) {
                        c0[0] = nx0;
                        c1[0] = min(nx1, ox0 - 1);
                        c0[1] = max(nx0, ox1 + 1);
                        c1[1] = nx1;
                    } else {
                        c0[0] = nx0;
                        c1[0] = nx1;
                        c0[1] = 1;
                        c1[1] = 0;
                    }
                }
                const uint32_t row = g.base + (uint32_t)r * g.gx;
                const uint32_t nq = tid < nO ? 1u : 2u, s0 = tid < nO ? tid : nO + 2u * (tid - nO);
                for (uint32_t q = 0; q < nq; ++q) {
                    uint32_t b = 0, e = 0;
                    if (c0[q] <= c1[q]) {
                        b = A.cell_start[row + (uint32_t)c0[q]];
                        e = A.cell_start[row + (uint32_t)c1[q] + 1u];
                    }
                    seg_b[s0 + q] = b;
                    seg_c[s0 + q + 1] = e - b;
                }
            }
            __syncthreads();
            if (tid == 0) {  // lengths -> cumulative (nseg <= 128)
                uint32_t c = 0;
                seg_c[0] = 0;
                for (uint32_t q = 1; q <= nseg; ++q) {
                    c += seg_c[q];
                    seg_c[q] = c;
                }
            }
            __syncthreads();
            const uint32_t T = seg_c[nseg];
            auto emit = [&](bool valid, int kind, uint32_t b_slot) {
                uint32_t oe, ol, te, tl;
                scan2(valid && kind == 1, valid && kind == 2, ws, oe, ol, te, tl);
                if (valid && kind == 1 && ne + oe < scr_cap) se[ne + oe] = b_slot;
                if (valid && kind == 2 && nl + ol < scr_cap) sl_[nl + ol] = b_slot;
                ne += te;
                nl += tl;
            };
            // partners in the frame that are not movers of this flush (their state is the frame's)
            for (uint32_t p0 = 0; p0 < T; p0 += SA_T) {
                const uint32_t p = p0 + tid;
                int kind = 0;
                uint32_t b_slot = 0;
                if (p < T) {
                    uint32_t lo = 0, hi = nseg;  // the segment holding p: seg_c[lo] <= p < seg_c[lo + 1]
                    while (hi - lo > 1u) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (seg_c[mid] <= p) lo = mid;
                        else hi = mid;
                    }
                    const uint32_t b = seg_b[lo] + (p - seg_c[lo]);
                    if (b != ra) {
                        const SlotSp bs = ld_ss(A.ss, b);
                        const Rec16 br = ld_rec(A.rec, b);
                        b_slot = bs.slot;
                        if (!sf_find(hs, b_slot)) {
                            const bool was = rel(ao.x, ao.z, ao.s, br.x, br.z, br.s, D);
                            const bool is = rel(nx, nz, ns, br.x, br.z, br.s, D);
                            kind = was == is ? 0 : is ? 1 : 2;
                        }
                    }
                }
                emit(p < T, kind, b_slot);
            }
            // pairs of two movers, from the lower slot: both states from the frame and the ops
            for (uint32_t q0 = 0; q0 < k; q0 += SA_T) {
                const uint32_t q = q0 + tid;
                int kind = 0;
                uint32_t b_slot = 0;
                if (q < k) {
                    b_slot = s_slot[q];
                    if (b_slot > slot && win(q)) {
                        const uint32_t rb = A.info.rank[b_slot];
                        if (ld_ss(A.ss, rb).sp == sp) {
                            const Rec16 bo = ld_rec(A.rec, rb);
                            const bool was = rel(ao.x, ao.z, ao.s, bo.x, bo.z, bo.s, D);
                            const bool is = rel(nx, nz, ns, A.op_x[q], A.op_z[q], op_seq(A, q), D);
                            kind = was == is ? 0 : is ? 1 : 2;
                        }
                    }
                }
                emit(q < k, kind, b_slot);
            }
            ovf = ne > scr_cap || nl > scr_cap;
        } else {
            ovf = true;
        }
    }
    // arrive: this workgroup's counts (~0u: it cannot be taken here) and scratch rows are published
    // by one agent-scope add; the workgroup whose add comes last goes on
    __syncthreads();
    if (tid == 0) {
        A.cnt[j] = ovf ? ~0u : ne;
        A.cnt[k + j] = ovf ? ~0u : nl;
        __threadfence();
        s_flag = atomicAdd(done, 1u) == k - 1u ? 1u : 0u;
    }
    __syncthreads();
    if (!s_flag) return;
    __threadfence();
    // ---- the last workgroup: offsets, summary, layout, then the frame patch
    if (tid == 0) *done = 0u;  // re-armed for the next flush (every other workgroup has arrived)
    bool bad = false;
    if (tid < k) {
        s_off[0][tid + 1] = A.cnt[tid];
        s_off[1][tid + 1] = A.cnt[k + tid];
        bad = s_off[0][tid + 1] == ~0u;
    }
    const bool any_bad = __syncthreads_or(bad);
    if (any_bad) {
        if (tid == 0) {
            A.res->pad = 3u;
            A.res->n_enter = A.res->n_total = 0;
            A.res->total64 = 0;
        }
        return;
    }
    if (tid < 2) {  // exclusive scans of the per-op counts (k <= 256)
        uint32_t c = 0;
        s_off[tid][0] = 0;
        for (uint32_t q = 1; q <= k; ++q) {
            c += s_off[tid][q];
            s_off[tid][q] = c;
        }
    }
    __syncthreads();
    const uint32_t E = s_off[0][k], L = s_off[1][k];
    const unsigned long long tot = 2ull * ((unsigned long long)E + L);
    const bool declined = tot > A.cap;  // the flush set's buffer is too small (the full flush grows it)
    if (tid == 0) {
        A.res->n_enter = 2 * E;
        A.res->n_total = (uint32_t)tot;
        A.res->err = 0;
        A.res->pad = declined ? 1u : 0u;
        A.res->total64 = tot;
        A.res->seq_max = 0;
        for (int q = 0; q < (int)DBG_N; ++q) A.res->dbg[q] = 0;
    }
    if (declined) return;
    for (uint32_t p = tid; p < E + L; p += SA_T) {  // directed pairs [enters | leaves], op order
        const uint32_t kd = p < E ? 0u : 1u, v = p < E ? p : p - E;
        uint32_t lo = 0, hi = k;  // s_off[kd][lo] <= v < s_off[kd][lo + 1]
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_off[kd][mid] <= v) lo = mid;
            else hi = mid;
        }
        const uint32_t b = scr[((size_t)lo * 2u + kd) * scr_cap + (v - s_off[kd][lo])], a = s_slot[lo];
        const size_t o = 2u * (size_t)p;
        A.out[o] = make_uint2(a, b);
        A.out[o + 1] = make_uint2(b, a);
    }
    sp_apply_body(A, [&](uint32_t q, uint32_t) { return win(q); });
}

}  // namespace

size_t sparse_cnt_elems(uint32_t k) { return 4 * (size_t)k + 3; }

void launch_sparse(Rec16 *rec, SlotSp *ss, uint32_t *key, uint32_t *cell_start, const SpaceGrid *grid,
                   SlotTab info, const uint32_t *op_slot, const float *op_x, const float *op_z,
                   const unsigned long long *op_seq, uint64_t seq0, uint32_t k, uint32_t tick, uint32_t *cnt,
                   uint32_t *out, uint64_t cap, TickOut *res, hipStream_t st) {
    SparseArgs A{rec, ss, key, cell_start, grid, info, op_slot, op_x, op_z, op_seq, seq0, k, tick, cnt,
                 reinterpret_cast<uint2 *>(out), cap, res};
    k_sp_events<0><<<k, SP_T, 0, st>>>(A);
    k_sp_scan<<<1, SA_T, 0, st>>>(A);
    k_sp_events<1><<<k, SP_T, 0, st>>>(A);
    k_sp_apply<<<1, SA_T, 0, st>>>(A);
}

uint32_t sparse_fused_max() { return SP_FUSED_MAX; }

void launch_sparse_fused(Rec16 *rec, SlotSp *ss, uint32_t *key, uint32_t *cell_start, const SpaceGrid *grid,
                         SlotTab info, const uint32_t *op_slot, const float *op_x, const float *op_z,
                         const unsigned long long *op_seq, uint64_t seq0, uint32_t k, uint32_t *cnt, uint32_t *scr,
                         uint32_t scr_cap, uint32_t *done, uint32_t *out, uint64_t cap, TickOut *res, hipStream_t st) {
    SparseArgs A{rec, ss, key, cell_start, grid, info, op_slot, op_x, op_z, op_seq, seq0, k, 0u, cnt,
                 reinterpret_cast<uint2 *>(out), cap, res};
    k_sp_fused<<<k, SA_T, 0, st>>>(A, scr, scr_cap, done);
}

}  // namespace gw
