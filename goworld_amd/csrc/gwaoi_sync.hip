// gwaoi_sync.hip -- entity position sync around the AOI path (include/gwaoi_sync.h).
//
// Three device passes, all on the world's stream:
//   decode    HandleSyncPositionYawFromClient (GameService.go:392-404): one
//             lane per 32-B record, entity-id hash lookup, the record becomes
//             op i of a device Moved batch (SLOT_NONE = skipped), Y/yaw by
//             last-writer claim, sifSyncNeighborClients.
//   fan-out   CollectEntitySyncInfos (Entity.go:1221-1267), receiver side:
//             one lane per frame entity B with a client; its records are its
//             own (sifSyncOwnClient) and one per flagged A with rel(A,B) (the
//             go-aoi relation of the last flush: B in A.InterestedBy).
//   route     Entity.interest/uninterest -> sendCreateEntity/sendDestroyEntity
//             (Entity.go:236-246, GameClient.go:37-59): the flush's events
//             whose first entity has a client, grouped by gate.
// Grouping by gate is a multisplit: a first pass counts records per
// (gate, block) in LDS, an exclusive scan gives every (gate, block) its
// base, a second pass writes each block's runs (the fan-out's first pass
// also lists every record's sender, so the AOI window is walked once).
// The output is HBM write bound (48 B per record).

#include "gwaoi_device.h"
#include "gwaoi_internal.h"
#include "../../include/gwaoi_sync.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace gw {
namespace {

constexpr uint32_t NO_GATE = 0xFFFFFFFFu;
constexpr uint32_t H_EMPTY = 0xFFFFFFFFu;  // hash bucket never used
constexpr uint32_t H_TOMB = 0xFFFFFFFEu;   // hash bucket freed
constexpr int ST = 256;                    // threads per workgroup of the sync kernels
constexpr uint32_t SCR_FULL = 0xFFFFFFFFu; // fan-out: the block's hits did not fit the scratch

inline uint32_t cdivu(size_t a, size_t b) { return (uint32_t)((a + b - 1) / b); }

// Hash of a 16-byte id (host and device agree).
__host__ __device__ inline uint32_t id_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    unsigned long long h = (((unsigned long long)b << 32) | a) * 0x9E3779B97F4A7C15ull;
    h ^= (((unsigned long long)d << 32) | c) + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    return (uint32_t)h;
}

// The fan-out's 16-B output and scratch stores.  Plain stores: the non-temporal form was
// slower.
// 16-B record stores that nothing in the kernel reads back: nontemporal (A/B,
// profiles/r06_ab_fan_write.txt: k_fan_write 661 -> 630 us against plain stores)
__device__ __forceinline__ void st_stream(uint4 *p, const uint4 &v) {
#ifdef GWAOI_EXP_FW_PLAIN
    *p = v;
#else
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4u *>(p));
#endif
}

__device__ __forceinline__ bool eq4(uint4 a, uint4 b) {
    return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
}

// ------------------------------------------------------------ scatter ------
// Host-side state changes reach the device as (array, index, value) writes.
constexpr int MAX_ARR = 8;
struct ArrTable {
    void *p[MAX_ARR];
    uint32_t stride[MAX_ARR];  // elements between consecutive indices (fields of packed per-slot records)
};
struct W32 {
    uint32_t arr, idx, val, pad;
};
struct W128 {
    uint32_t arr, idx, pad0, pad1;
    uint4 val;
};

__global__ void k_scatter32(const W32 *__restrict__ w, uint32_t n, ArrTable T) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const W32 e = w[i];
    static_cast<uint32_t *>(T.p[e.arr])[(size_t)e.idx * T.stride[e.arr]] = e.val;
}

__global__ void k_scatter128(const W128 *__restrict__ w, uint32_t n, ArrTable T) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const W128 e = w[i];
    static_cast<uint4 *>(T.p[e.arr])[(size_t)e.idx * T.stride[e.arr]] = e.val;
}

// Per-slot sync state is packed so that one pass touches one line per slot:
//   one 64-B record per slot (SLOT_U4 uint4): sst {gate index, space in call
//           order, syncing, sync flags}, pos {x, y, z, yaw}, eid, cid -- the
//           fan-out's sender pass reads the first three from one line, the
//           decode writes pos and the flags into it
//   cl[s]   ulonglong2 {Position claim, yaw claim}
//   htab    64-B buckets {3 entity ids; their 3 slots}: a probe reads keys and
//           values from one line (see lookup).
enum SstField { SST_GATE = 0, SST_SPACE = 1, SST_SYNCING = 2, SST_FLAGS = 3 };
constexpr uint32_t SLOT_U4 = 4;             // uint4 per slot record: sst, pos, eid, cid
constexpr uint32_t SLOT_W = 4 * SLOT_U4;    // its 32-bit words

// Host position/yaw writes (set_position_yaw, entity_set_position_yaw,
// entity_enter_plain) and flag-only ops (Space.enter): claim, then the winner
// writes.  Position (x, y, z) and yaw have claims of their own: outside an AOI
// space setPositionYaw changes yaw but not Position (Space.go:253-257), so the
// last write of each may come from different calls.
constexpr uint32_t SIDE_POS = 0x100u;  // op writes Position (x, y, z)
constexpr uint32_t SIDE_YAW = 0x200u;  // op writes yaw
constexpr uint32_t SIDE_SIF = GWAOI_SIF_OWN_CLIENT | GWAOI_SIF_NEIGHBOR_CLIENTS;
struct SideOp {
    uint32_t slot, bits;  // bits: SIDE_POS | SIDE_YAW | sync flags
    unsigned long long claim;
    float4 pos;  // x, y, z, yaw
};

__global__ void k_side_claim(const SideOp *__restrict__ ops, uint32_t n, unsigned long long *cl, uint32_t *sst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SideOp o = ops[i];
    if (o.bits & SIDE_POS) atomicMax(&cl[2 * (size_t)o.slot], o.claim);
    if (o.bits & SIDE_YAW) atomicMax(&cl[2 * (size_t)o.slot + 1], o.claim);
    if (o.bits & SIDE_SIF) atomicOr(&sst[SLOT_W * (size_t)o.slot + SST_FLAGS], o.bits & SIDE_SIF);
}

__global__ void k_side_write(const SideOp *__restrict__ ops, uint32_t n, const unsigned long long *cl, float4 *pos) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SideOp o = ops[i];
    float *p = reinterpret_cast<float *>(pos + SLOT_U4 * (size_t)o.slot);
    if ((o.bits & SIDE_POS) && cl[2 * (size_t)o.slot] == o.claim) {
        p[0] = o.pos.x;
        p[1] = o.pos.y;
        p[2] = o.pos.z;
    }
    if ((o.bits & SIDE_YAW) && cl[2 * (size_t)o.slot + 1] == o.claim) p[3] = o.pos.w;
}

// ------------------------------------------------------------- decode ------
struct DecodeArgs {
    const uint4 *pay;  // 2 uint4 per record: id, (x, y, z, yaw) bits
    uint32_t n;
    const uint4 *htab;
    uint32_t hmask;  // buckets - 1 (power of two)
    uint32_t *sst;
    uint32_t *o_slot, *o_sp;  // the device Moved batch (SLOT_NONE: no move)
    float *o_x, *o_z;
    uint32_t *o_ys;  // slot of an applied record (SLOT_NONE: skipped), for k_decode_yaw
    unsigned long long claim0;
    unsigned long long *cl;
    float4 *pos;
    uint32_t *oflag, *oflag_n;  // slots flagged outside every AOI space (own-client records)
    uint32_t *h_ndec;           // pinned host word: *oflag_n once the batch is decoded
    uint32_t oflag_cap;         // entries oflag holds (max_slots: one per slot, see k_decode)
    uint32_t *dups, *ndup;      // slots with a record whose claim store did not survive (1)
};

// The id table: 64-B buckets (one line), three entries each: keys in words 0..11,
// the three slots in words 12..14 (H_EMPTY never used, H_TOMB freed).  Linear
// probing over entries e = 3 b + way, so a probe reads one line per step and
// almost always stops in the first (half the bytes of the 32-B bucket layout).
// One bucket's three entries against id: true when the probe ends here (found, or an
// empty entry: not in the table), with the slot (or SLOT_NONE) in *out.
__device__ __forceinline__ bool probe_bucket(const uint4 (&k)[3], const uint4 &m, const uint4 &id, uint32_t *out) {
    const uint32_t v[3] = {m.x, m.y, m.z};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        if (v[q] == H_EMPTY) {
            *out = SLOT_NONE;
            return true;
        }
        if (v[q] != H_TOMB && eq4(k[q], id)) {
            *out = v[q];
            return true;
        }
    }
    return false;
}

__device__ __forceinline__ uint32_t lookup(const uint4 *__restrict__ htab, uint32_t bmask, uint4 id,
                                           uint32_t probe0 = 0) {
    uint32_t b = (id_hash(id.x, id.y, id.z, id.w) + probe0) & bmask;
    for (uint32_t probe = probe0; probe <= bmask; ++probe, b = (b + 1) & bmask) {
        uint4 k[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) k[q] = htab[4 * (size_t)b + (uint32_t)q];
        const uint4 m = htab[4 * (size_t)b + 3];
        const uint32_t v[3] = {m.x, m.y, m.z};
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            if (v[q] == H_EMPTY) return SLOT_NONE;
            if (v[q] != H_TOMB && eq4(k[q], id)) return v[q];
        }
    }
    return SLOT_NONE;
}

// The record's effects once its slot is known (s: the looked-up slot or SLOT_NONE; st: its
// slot record when s != SLOT_NONE).
__device__ __forceinline__ void decode_rest(const DecodeArgs &A, uint32_t i, const uint4 &pv, uint32_t s,
                                            const uint4 &st) {
    uint32_t sp = SP_DEAD, old = 0;
    if (s != SLOT_NONE) {
        sp = st.y;  // SST_SPACE
        old = st.w;  // SST_FLAGS
        if (!st.z) s = SLOT_NONE;  // SST_SYNCING
    }
    const bool move = s != SLOT_NONE && sp != SP_DEAD;
    A.o_slot[i] = move ? s : SLOT_NONE;
    A.o_x[i] = __uint_as_float(pv.x);
    A.o_z[i] = __uint_as_float(pv.z);
    A.o_sp[i] = sp;
    A.o_ys[i] = s;
    if (s != SLOT_NONE) {
        // Plain stores, no atomics (a device-scope atomic is performed memory-side
        // on gfx950, ~17x slower than a store for 64 lanes on 64 lines): the
        // claims of this batch are larger than every claim already applied, so a
        // store replaces them; among records of one slot in this batch a random
        // store survives, and k_decode_fix folds the others in.
        const unsigned long long c = A.claim0 + i;
        if (move) reinterpret_cast<ulonglong2 *>(A.cl)[s] = make_ulonglong2(c, c);
        else A.cl[2 * (size_t)s + 1] = c;
        // (the flags word came with the slot's record; records of one slot all set the same bit)
        uint32_t *fl = A.sst + SLOT_W * (size_t)s + SST_FLAGS;
        if (!move && old == 0u) {
            // first flag of a slot outside the frame since the last collect: the flag is
            // claimed atomically, so a slot with several records in the batch is listed
            // once and the list never holds more than one entry per slot (rare path: only
            // entities outside every AOI space get here)
            if (atomicOr(fl, GWAOI_SIF_NEIGHBOR_CLIENTS) == 0u) {
                const uint32_t k = atomicAdd(A.oflag_n, 1u);
                if (k < A.oflag_cap) A.oflag[k] = s;
            }
        } else if (!(old & GWAOI_SIF_NEIGHBOR_CLIENTS)) {
            *fl = old | GWAOI_SIF_NEIGHBOR_CLIENTS;
        }
    }
}


// OnSyncPositionYawFromClient: unknown id -> skip (EntityManager.go:486-490);
// syncPositionYawFromClient: only if syncing (Entity.go:432).  setPositionYaw
// (Entity.go:1189-1205) then runs for every entity: e.Space is nilSpace, not
// nil, outside every space.  In an AOI space it is a Moved (op i of the
// batch) plus Position; elsewhere Space.move returns before Position
// (Space.go:253-257) and only yaw changes.  Both raise sifSyncNeighborClients.
// PER records per thread, strided by the block: every slot record is loaded before any is used.
#ifndef GWAOI_DEC_PER
#define GWAOI_DEC_PER 2  // records per k_decode thread (2: 102 vs 113 us at 1M records, profiles/archive/r04_variants_sync.log)
#endif
template <int PER>
__global__ __launch_bounds__(ST) void k_decode(DecodeArgs A) {
    const uint32_t i0 = blockIdx.x * (ST * PER) + threadIdx.x;
    if (i0 == 0) *A.ndup = 0u;  // read by k_decode_apply, the next launch on the stream
    uint4 id[PER], pv[PER];
    uint32_t s[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const uint32_t i = i0 + (uint32_t)u * ST;
        const size_t ic = i < A.n ? i : 0u;  // (clamped: the loads issue together)
        id[u] = A.pay[2 * ic];
        pv[u] = A.pay[2 * ic + 1];
    }
    // the first bucket of every record's probe in flight together (a probe almost always ends
    // there); the rare longer probe continues from the next bucket
    uint4 hk[PER][3], hm[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const size_t b = id_hash(id[u].x, id[u].y, id[u].z, id[u].w) & A.hmask;
#pragma unroll
        for (int q = 0; q < 3; ++q) hk[u][q] = A.htab[4 * b + (uint32_t)q];
        hm[u] = A.htab[4 * b + 3];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        s[u] = SLOT_NONE;
        if (i0 + (uint32_t)u * ST < A.n && !probe_bucket(hk[u], hm[u], id[u], &s[u]))
            s[u] = lookup(A.htab, A.hmask, id[u], 1u);
    }
    uint4 st[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {  // every slot record in flight together (clamped slot: no branch)
        st[u] = reinterpret_cast<const uint4 *>(A.sst)[SLOT_U4 * (size_t)(s[u] != SLOT_NONE ? s[u] : 0u)];
        if (s[u] == SLOT_NONE) st[u] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const uint32_t i = i0 + (uint32_t)u * ST;
        if (i < A.n) decode_rest(A, i, pv[u], s[u], st[u]);
    }
}


// The claim fold and the apply in one pass.  A record whose claim store survived
// (cs == c) applies its position / yaw; one whose store was overwritten by another
// record of the same slot folds its claim in with atomicMax and lists the slot.
// Whatever the interleaving, every slot with two or more records in the batch is
// listed by one of them, and k_decode_dups then applies the record that holds the
// final (largest) claim.  A batch without repeated slots pays no atomic and
// lists nothing: the separate read-only fold pass (k_decode_fix) is gone.
__global__ __launch_bounds__(ST) void k_decode_apply(DecodeArgs A) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n) return;
    const uint32_t s = A.o_ys[i];
    if (s == SLOT_NONE) return;
    const unsigned long long c = A.claim0 + i;
    const uint4 pv = A.pay[2 * (size_t)i + 1];
    float *p = reinterpret_cast<float *>(A.pos + SLOT_U4 * (size_t)s);
    const ulonglong2 cs = reinterpret_cast<const ulonglong2 *>(A.cl)[s];
    const bool moves = A.o_sp[i] != SP_DEAD;
    if (moves && cs.x == c && cs.y == c) {  // the common case: one 16-B store of position and yaw
        A.pos[SLOT_U4 * (size_t)s] = make_float4(__uint_as_float(pv.x), __uint_as_float(pv.y), __uint_as_float(pv.z),
                               __uint_as_float(pv.w));
        return;
    }
    bool lost = false;
    if (moves) {
        if (cs.x == c) {
            p[0] = __uint_as_float(pv.x);
            p[1] = __uint_as_float(pv.y);
            p[2] = __uint_as_float(pv.z);
        } else {
            atomicMax(&A.cl[2 * (size_t)s], c);
            lost = true;
        }
    }
    if (cs.y == c) {
        p[3] = __uint_as_float(pv.w);
    } else {
        atomicMax(&A.cl[2 * (size_t)s + 1], c);
        lost = true;
    }
    if (lost) A.dups[atomicAdd(A.ndup, 1u)] = s;
}

// Listed slots (rare; may repeat): apply the records holding the final claims.
__global__ __launch_bounds__(ST) void k_decode_dups(DecodeArgs A) {
    const uint32_t nd = *A.ndup;
    if (blockIdx.x == 0 && threadIdx.x == 0) *A.h_ndec = *A.oflag_n;  // (for the collect, no copy)
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nd; k += gridDim.x * blockDim.x) {
        const uint32_t s = A.dups[k];
        const ulonglong2 cs = reinterpret_cast<const ulonglong2 *>(A.cl)[s];
        float *p = reinterpret_cast<float *>(A.pos + SLOT_U4 * (size_t)s);
        const unsigned long long ix = cs.x - A.claim0, iy = cs.y - A.claim0;  // claims of older batches wrap
        if (ix < A.n && A.o_ys[ix] == s && A.o_sp[ix] != SP_DEAD) {
            const uint4 pv = A.pay[2 * (size_t)ix + 1];
            p[0] = __uint_as_float(pv.x);
            p[1] = __uint_as_float(pv.y);
            p[2] = __uint_as_float(pv.z);
        }
        if (iy < A.n && A.o_ys[iy] == s) p[3] = __uint_as_float(A.pay[2 * (size_t)iy + 1].w);
    }
}

// ------------------------------------------------------------ fan-out ------
// Receiver side: CollectEntitySyncInfos sends entity A's record to the client
// of every B in A.InterestedBy, i.e. every B with rel(A,B).  One lane per
// frame entity B with a client (gate g): its records are its own one (if B's
// sifSyncOwnClient is set) plus one per A in B's window with rel(A,B) and
// sifSyncNeighborClients set on A.  All of a lane's records go to one gate,
// so a lane reserves its whole run with one LDS atomic and writes it
// contiguously.  k_fan_prep first lays the senders out in frame order
// (flags, id, position/yaw) so that the window walk reads them next to the
// frame records, and clears the flags.
struct FanArgs {
    FrameView F;
    SlotTab info;  // slot -> frame index (rank) of the world
    const uint32_t *left;  // flagged slots outside the frame (own-client records only), may repeat
    uint32_t n_left;
    const uint4 *eid, *cid;
    uint32_t *sst;
    const float4 *pos;
    // frame-ordered (n + n_left entries), written by k_fan_prep
    uint32_t *snd;    // sender flags
    uint32_t *rg;     // receiver gate (NO_GATE: no client)
    uint4 *srec;      // 2 per entry: sender id, then x, y, z, yaw (one 32-B load per record)
    uint4 *frec;      // frame records (x, z, seq) with sifSyncNeighborClients in bit 63
    uint4 *fcid;      // receiver's ClientID (entries with a client; from the slot record's line)
    uint32_t *fcnt, *fsb;  // records of each entry, its run in the scratch
    uint32_t *scr;         // hits: sender entry of each record, receiver-contiguous runs
    unsigned long long *scr_cursor;
    unsigned long long scr_cap;  // < SCR_FULL
    uint32_t G, nb;
    uint32_t *blk_cnt;  // [G][nb] (pass 1 writes, the scan turns it into bases)
    uint4 *out;         // 3 uint4 per record (pass 2)
    unsigned long long out_recs;  // records out holds (pass 2 writes nothing past a larger total)
};

__global__ __launch_bounds__(ST) void k_fan_prep(FanArgs A) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nf = A.F.n;
    if (i == 0) {  // the hits pass's scratch cursor and the scan's extra count (first attempt)
        *A.scr_cursor = 0ull;
        A.blk_cnt[(size_t)A.G * A.nb] = 0u;
    }
    if (i >= nf + A.n_left) return;
    const bool in_frame = i < nf;
    const uint32_t s = in_frame ? ld_ss(A.F.ss, i).slot : A.left[i - nf];
    // the slot's whole 64-B record and the frame record, all loaded before any is used (a load
    // under a per-lane branch is waited for before the next one issues)
    const uint4 *rec = reinterpret_cast<const uint4 *>(A.sst) + SLOT_U4 * (size_t)s;
    const uint4 st = rec[0];  // gate, space, syncing, flags
    const uint4 pw = rec[1];  // Position, yaw
    const uint4 id = rec[2];  // EntityID
    const uint4 ci = rec[3];  // ClientID
    const uint4 q = reinterpret_cast<const uint4 *>(A.F.rec)[in_frame ? i : 0u];
    uint32_t fl;
    if (in_frame) {
        fl = st.w;
        if (fl) A.sst[SLOT_W * (size_t)s + SST_FLAGS] = 0u;
    } else {
        // a listed slot back in the frame is its frame entry's; a slot listed twice is sent once
        const uint32_t r = A.info.rank[s];
        fl = (r < nf && ld_ss(A.F.ss, r).slot == s) ? 0u : atomicExch(&A.sst[SLOT_W * (size_t)s + SST_FLAGS], 0u);
    }
    A.snd[i] = fl;
    A.rg[i] = st.x;
    A.fcid[i] = ci;  // (the receiver's, read in frame order by the write pass)
    if (in_frame) {  // the walk's candidate record: x, z, seq with the sender flag in bit 63
        uint4 f = q;
        if (fl & GWAOI_SIF_NEIGHBOR_CLIENTS) f.w |= 0x80000000u;
        A.frec[i] = f;
    }
    if (fl) {
        // the frame holds the AOI position; outside the frame, the last Position written
        const uint32_t x = in_frame ? q.x : pw.x, z = in_frame ? q.y : pw.z;
        A.srec[2 * (size_t)i] = id;
        A.srec[2 * (size_t)i + 1] = make_uint4(x, pw.y, z, pw.w);
    }
}

__device__ __forceinline__ uint32_t s_lane() { return __lane_id(); }

// Exclusive scan of n (<= ST * k) LDS words in place by one workgroup.
__device__ void lds_excl_scan(uint32_t *a, uint32_t n, uint32_t *ws) {
    const uint32_t k = (n + ST - 1) / ST, b = threadIdx.x * k;
    uint32_t sum = 0;
    for (uint32_t q = 0; q < k && b + q < n; ++q) sum += a[b + q];
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if ((int)s_lane() >= o) x += y;
    }
    const uint32_t w = threadIdx.x / 64;
    if (s_lane() == 63) ws[w] = x;
    __syncthreads();
    uint32_t pre = x - sum;
    for (uint32_t q = 0; q < w; ++q) pre += ws[q];
    for (uint32_t q = 0; q < k && b + q < n; ++q) {
        const uint32_t v = a[b + q];
        a[b + q] = pre;
        pre += v;
    }
    __syncthreads();
}

// Block-wide exclusive scan of one value per thread (ST threads).
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t *ws, uint32_t &total) {
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if ((int)s_lane() >= o) x += y;
    }
    const uint32_t w = threadIdx.x / 64;
    if (s_lane() == 63) ws[w] = x;
    __syncthreads();
    uint32_t pre = x - v;
    total = 0;
    for (uint32_t q = 0; q < ST / 64; ++q) {
        if (q < w) pre += ws[q];
        total += ws[q];
    }
    __syncthreads();
    return pre;
}

// The go-aoi window of receiver entry i (cells), widened by the float32
// rounding margin of the window bounds.
struct FanWin {
    Rec16 R;
    float D;
    uint32_t row0, gx;  // cell index of (cx0, cz0), grid row length
    int cx0, cx1, cz0, cz1;
};
__device__ __forceinline__ FanWin fan_window(const FrameView &F, uint32_t i) {
    FanWin W;
    W.R = ld_rec(F.rec, i);
    const SpaceGrid gr = F.grid[ld_ss(F.ss, i).sp];
    W.D = gr.D;
    const float mx = (fabsf(W.R.x) + 3.0f * W.D) * 0x1p-20f, mz = (fabsf(W.R.z) + 3.0f * W.D) * 0x1p-20f;
    W.cx0 = cell_of(W.R.x - W.D - mx, gr.ox, gr.inv, gr.gx);
    W.cx1 = cell_of(W.R.x + W.D + mx, gr.ox, gr.inv, gr.gx);
    W.cz0 = cell_of(W.R.z - W.D - mz, gr.oz, gr.inv, gr.gz);
    W.cz1 = cell_of(W.R.z + W.D + mz, gr.oz, gr.inv, gr.gz);
    W.gx = gr.gx;
    W.row0 = gr.base + (uint32_t)W.cz0 * gr.gx + (uint32_t)W.cx0;
    return W;
}

// Fan-out pass 1 (hits).  Entry i (frame order, then the listed slots outside
// the frame) with a client is a receiver: it lists the senders of its records
// in the scratch, itself first if sifSyncOwnClient, then every A in its go-aoi
// window with sifSyncNeighborClients and rel(A,B), rows in order and frame
// order inside a row.  Its scratch run is sized by the window's candidate
// count (one lane per entry, cell_start loads only) and placed by one atomic
// per block, so the window is walked once; a block past the scratch capacity
// writes no hits (the host regrows the scratch and reruns this pass; it has no
// other side effect).  The walk takes a wave per receiver (FAN_NR of a wave's
// receivers at a time): the window rows are laid end to end (lane j loads row
// j's bounds; a DPP scan gives each row's first position) and the wave deals
// out 64 consecutive positions per step.  A lane's candidate is found from the
// rows starting in the step (an LDS mark per position, a ballot) and the row's
// offset (LDS), so one load instruction reads 64 consecutive candidates instead
// of one candidate from each of 64 windows (the round-5 lane-per-receiver walk:
// 353 against 249 us, profiles/r06_ab_fan_hits.txt), and the hits are
// compacted by a ballot into consecutive 4-B stores.
#ifndef GWAOI_FAN_WU
#define GWAOI_FAN_WU 2  // steps of 64 positions per receiver with their loads in flight together
#endif
constexpr int FAN_WU = GWAOI_FAN_WU;
#ifndef GWAOI_FAN_NR
#define GWAOI_FAN_NR 2  // receivers of a wave dealt together (A/B, profiles/r06_ab_fan_hits.txt: k_fan_hits
                        // 252 us at NR 2 / WU 2, 259 at 3 / 2, 279 at 4 / 2, 283 at 2 / 4, 267 at 1 / 4)
#endif
constexpr int FAN_NR = GWAOI_FAN_NR;
#ifndef GWAOI_FAN_UBU
#define GWAOI_FAN_UBU 4  // window rows whose bounds the run sizing loads together
#endif
constexpr int FAN_UBU = GWAOI_FAN_UBU;

__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t k) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)k);
}

__global__ __launch_bounds__(ST) void k_fan_hits_wave(FanArgs A) {
    extern __shared__ uint32_t gcnt[];  // [G] records per gate of the block
    __shared__ uint32_t s_ws[ST / 64];
    __shared__ uint32_t s_base;
    __shared__ uint32_t s_adj[ST / 64][FAN_NR][64];            // candidate index - position, per non-empty row
    __shared__ uint32_t s_mark[ST / 64][FAN_NR][FAN_WU * 64];  // a non-empty row starts at this position
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x);
    const uint32_t nf = A.F.n, ne = nf + A.n_left;
    const uint32_t w = threadIdx.x / 64, ln = s_lane();
    for (uint32_t q = threadIdx.x; q < A.G; q += blockDim.x) gcnt[q] = 0u;
    const uint32_t i = blk * ST + threadIdx.x;
    const uint32_t g = i < ne ? A.rg[i] : NO_GATE;
    const bool on = g != NO_GATE;
    const bool own = on && (A.snd[i] & GWAOI_SIF_OWN_CLIENT);
    const bool walk = on && i < nf;
    const uint32_t *cs = A.F.cell_start;
    FanWin W{};
    uint32_t ub = own ? 1u : 0u;
    if (walk) {
        W = fan_window(A.F, i);
        const uint32_t span = (uint32_t)(W.cx1 - W.cx0) + 1u;
        for (int cz = W.cz0; cz <= W.cz1; cz += FAN_UBU) {  // FAN_UBU rows' bounds in flight together
            uint32_t lo[FAN_UBU], hi[FAN_UBU];
#pragma unroll
            for (int u = 0; u < FAN_UBU; ++u) {
                const uint32_t rb = W.row0 + (uint32_t)(min(cz + u, W.cz1) - W.cz0) * W.gx;
                lo[u] = cs[rb];
                hi[u] = cs[rb + span];
            }
#pragma unroll
            for (int u = 0; u < FAN_UBU; ++u)
                if (cz + u <= W.cz1) ub += hi[u] - lo[u];
        }
    }
    ub = (ub + 3u) & ~3u;  // (runs start 16-B aligned)
    uint32_t tot;
    const uint32_t off = block_excl(ub, s_ws, tot);
    if (threadIdx.x == 0) {
        const unsigned long long b = tot ? atomicAdd(A.scr_cursor, (unsigned long long)tot) : 0ull;
        s_base = b + tot <= A.scr_cap ? (uint32_t)b : SCR_FULL;
    }
    __syncthreads();
    const bool fits = s_base != SCR_FULL;
    const uint32_t sb = s_base + off;
    if (own && fits) A.scr[sb] = i;
    uint32_t c = own ? 1u : 0u;
    const unsigned long long lt = (1ull << ln) - 1ull;
    const unsigned long long le = ln == 63 ? ~0ull : (2ull << ln) - 1ull;
    unsigned long long todo = __ballot(walk);
#ifdef GWAOI_EXP_FAN_NOWALK  // timing only: the run sizing and placement without the walks (no neighbour records)
    todo = 0;
#endif
    while (todo) {
        // FAN_NR receivers at a time, their steps interleaved (a receiver's chain of row-bound
        // loads, then candidate loads, is latency-bound alone); a missing one has no rows
        uint32_t k[FAN_NR], ri[FAN_NR], row0[FAN_NR], gx[FAN_NR], span[FAN_NR], nrows[FAN_NR], rsb[FAN_NR],
            rc[FAN_NR];
        float rx[FAN_NR], rz[FAN_NR], D[FAN_NR];
        unsigned long long rs[FAN_NR];
        uint32_t maxrows = 0;
#pragma unroll
        for (int r = 0; r < FAN_NR; ++r) {
            k[r] = todo ? (uint32_t)__builtin_ctzll(todo) : 64u;
            todo &= todo - 1ull;
            const uint32_t kk = min(k[r], 63u);
            ri[r] = blk * ST + w * 64u + kk;
            rx[r] = __uint_as_float(rdl(__float_as_uint(W.R.x), kk));
            rz[r] = __uint_as_float(rdl(__float_as_uint(W.R.z), kk));
            D[r] = __uint_as_float(rdl(__float_as_uint(W.D), kk));
            rs[r] = ((unsigned long long)rdl((uint32_t)(W.R.s >> 32), kk) << 32) | rdl((uint32_t)W.R.s, kk);
            row0[r] = rdl(W.row0, kk);
            gx[r] = rdl(W.gx, kk);
            span[r] = rdl((uint32_t)(W.cx1 - W.cx0), kk) + 1u;
            nrows[r] = k[r] < 64u ? rdl((uint32_t)(W.cz1 - W.cz0), kk) + 1u : 0u;
            rsb[r] = rdl(sb, kk);
            rc[r] = rdl(c, kk);
            maxrows = max(maxrows, nrows[r]);
        }
        for (uint32_t j0 = 0; j0 < maxrows; j0 += 64u) {
            // lane t: row j0 + t of each window, its candidates [jb, jb + len)
            const uint32_t t = j0 + ln;
            uint32_t jb[FAN_NR], je[FAN_NR], len[FAN_NR], ex[FAN_NR], T[FAN_NR];
#pragma unroll
            for (int r = 0; r < FAN_NR; ++r) {
                const uint32_t rb = row0[r] + min(t, max(nrows[r], 1u) - 1u) * gx[r];
                jb[r] = cs[rb];
                je[r] = cs[rb + span[r]];
            }
            uint32_t Tm = 0;
#pragma unroll
            for (int r = 0; r < FAN_NR; ++r) {
                len[r] = t < nrows[r] ? je[r] - jb[r] : 0u;
                const uint32_t incl = wave_scan_add(len[r]);
                ex[r] = incl - len[r];
                T[r] = rdl(incl, 63);
                Tm = max(Tm, T[r]);
                const unsigned long long nem = __ballot(len[r] != 0u);
                if (len[r]) s_adj[w][r][__popcll(nem & lt)] = jb[r] - ex[r];
            }
            for (uint32_t p0 = 0; p0 < Tm; p0 += FAN_WU * 64u) {
#pragma unroll
                for (int r = 0; r < FAN_NR; ++r)
#pragma unroll
                    for (int u = 0; u < FAN_WU; ++u) s_mark[w][r][u * 64 + ln] = 0u;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                uint32_t nr[FAN_NR];  // non-empty rows started before this step
#pragma unroll
                for (int r = 0; r < FAN_NR; ++r) {
                    if (len[r] && ex[r] >= p0 && ex[r] - p0 < FAN_WU * 64u) s_mark[w][r][ex[r] - p0] = 1u;
                    nr[r] = (uint32_t)__popcll(__ballot(len[r] != 0u && ex[r] < p0));
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                uint32_t b[FAN_NR][FAN_WU];
                uint4 q[FAN_NR][FAN_WU];
#pragma unroll
                for (int r = 0; r < FAN_NR; ++r)
#pragma unroll
                    for (int u = 0; u < FAN_WU; ++u) {
                        const unsigned long long m = __ballot(s_mark[w][r][u * 64 + ln] != 0u);
                        const uint32_t p = p0 + (uint32_t)u * 64u + ln;
                        const uint32_t row = nr[r] + (uint32_t)__popcll(m & le);  // rows started at or before p
                        nr[r] += (uint32_t)__popcll(m);
                        b[r][u] = p < T[r] ? p + s_adj[w][r][row - 1u] : ri[r];  // (row >= 1 whenever p < T)
                        q[r][u] = A.frec[b[r][u]];
                    }
#pragma unroll
                for (int r = 0; r < FAN_NR; ++r)
#pragma unroll
                    for (int u = 0; u < FAN_WU; ++u) {
                        const uint32_t p = p0 + (uint32_t)u * 64u + ln;
                        const uint4 &Q = q[r][u];
                        const unsigned long long bs = ((unsigned long long)(Q.w & 0x7FFFFFFFu) << 32) | Q.z;
                        const bool hit = p < T[r] && b[r][u] != ri[r] && (Q.w >> 31) &&
                                         rel(rx[r], rz[r], rs[r], __uint_as_float(Q.x), __uint_as_float(Q.y), bs, D[r]);
                        const unsigned long long hm = __ballot(hit);
                        if (hit && fits) A.scr[rsb[r] + rc[r] + (uint32_t)__popcll(hm & lt)] = b[r][u];
                        rc[r] += (uint32_t)__popcll(hm);
                    }
            }
            __builtin_amdgcn_wave_barrier();  // s_adj is rewritten by the next row group
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
#pragma unroll
        for (int r = 0; r < FAN_NR; ++r)
            if (ln == k[r]) c = rc[r];
    }
    if (i < ne) {
        A.fcnt[i] = c;
        A.fsb[i] = sb;
    }
    if (c) atomicAdd(&gcnt[g], c);
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < A.G; q += blockDim.x) A.blk_cnt[(size_t)q * A.nb + blk] = gcnt[q];
}

// Fan-out pass 2 (write): block blk expands the hits of its receivers into
// 48-B records (receiver's ClientID, sender's EntityID, x, y, z, yaw).  The
// receivers are regrouped by gate (stable), so the block's records of gate g
// form one run starting at the scanned base of (g, blk).  Thread t writes
// records t, t + ST, ... of the block: consecutive threads write consecutive
// records of a run (coalesced stores), each finding its receiver by a binary
// search of the inclusive record prefix in LDS.  (GoWorld's own per-gate
// order is Go map order, EntityManager.go's entity loop: the order of
// records inside a gate is not part of the contract.)
#ifndef GWAOI_FW_G
#define GWAOI_FW_G 12  // A/B (profiles/r06_ab_fan_write.txt): collect 1.355 (4), 1.285 (6), 1.242 (8), 1.203 (12), 1.210 (16) ms once the hit loads stopped serialising
#endif
constexpr int FW_G = GWAOI_FW_G;  // record groups of 64 per wave with their loads in flight together

__global__ __launch_bounds__(ST) void k_fan_write(FanArgs A) {
    extern __shared__ uint32_t lds[];  // bin[G + 1] | gbase[G] | seg[G]
    __shared__ uint32_t s_pre[ST], s_sb[ST], s_gate[ST];
    __shared__ uint4 s_cli[ST];
    __shared__ uint4 s_rec[ST / 64][3 * 64];  // a wave's 64 records, staged for contiguous stores
    __shared__ uint32_t s_pos[ST / 64][64];
    __shared__ uint32_t s_ws[ST / 64];
    // launched behind the hits pass without a host round trip: nothing to do when the hits
    // overflowed the scratch or the total (the scan's last entry) outgrew the output; the host
    // sees both after its one sync and reruns
    if (*A.scr_cursor > A.scr_cap || A.blk_cnt[(size_t)A.G * A.nb] > A.out_recs) return;
    uint32_t *bin = lds, *gbase = lds + A.G + 1, *seg = gbase + A.G;
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x);
    const uint32_t ne = A.F.n + A.n_left;
    const uint32_t w = threadIdx.x / 64, ln = s_lane();
    for (uint32_t q = threadIdx.x; q <= A.G; q += blockDim.x) bin[q] = 0u;
    for (uint32_t q = threadIdx.x; q < A.G; q += blockDim.x) gbase[q] = A.blk_cnt[(size_t)q * A.nb + blk];
    __syncthreads();
    const uint32_t i = blk * ST + threadIdx.x;
    // the receiver's gate, record count, run and ClientID in one round trip (clamped index, no
    // load under a branch)
    const uint32_t ic = i < ne ? i : 0u;
    const uint32_t g0 = A.rg[ic], cnt0 = A.fcnt[ic], sb0 = A.fsb[ic];
    const uint4 cli = A.fcid[ic];
    const uint32_t g = i < ne ? g0 : NO_GATE;
    const uint32_t key = g == NO_GATE ? A.G : g;
    const uint32_t r0 = atomicAdd(&bin[key], 1u);
    __syncthreads();
    lds_excl_scan(bin, A.G + 1, s_ws);
    const uint32_t p = bin[key] + r0;  // (the order inside a gate's run is not part of the contract)
    const uint32_t c = g != NO_GATE ? cnt0 : 0u;
    s_pre[p] = c;
    s_sb[p] = c ? sb0 : 0u;
    s_gate[p] = key;
    if (c) s_cli[p] = cli;
    __syncthreads();
    uint32_t R;
    const uint32_t mine = s_pre[threadIdx.x];
    const uint32_t ex = block_excl(mine, s_ws, R);
    s_pre[threadIdx.x] = ex + mine;  // inclusive
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < A.G; q += blockDim.x) seg[q] = bin[q] ? s_pre[bin[q] - 1] : 0u;
    __syncthreads();
    const uint4 *srec = A.srec;
    // record r of receiver q -> (its scratch entry, output position)
    auto place = [&](uint32_t r, uint32_t q, uint32_t &sidx, uint32_t &pos) {
        const uint32_t gq = s_gate[q];
        sidx = s_sb[q] + r - (q ? s_pre[q - 1] : 0u);
        pos = gbase[gq] + (r - seg[gq]);
    };
    auto search = [&](uint32_t r) {  // first receiver q with s_pre[q] > r
        uint32_t lo = 0, hi = ST - 1;
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (s_pre[m] > r) hi = m;
            else lo = m + 1;
        }
        return lo;
    };
    // stage a wave's 64 records in LDS, then store them as 3 x 64 consecutive 16-B words
    auto emit = [&](uint32_t nrec, bool ok, uint32_t q, uint32_t pos, const uint4 &id, const uint4 &pv) {
        if (ok) {
            s_pos[w][ln] = pos;
            s_rec[w][3 * ln] = s_cli[q];
            s_rec[w][3 * ln + 1] = id;
            s_rec[w][3 * ln + 2] = pv;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (uint32_t j = 0; j < 3; ++j) {
            const uint32_t e = ln + 64u * j, rr = e / 3u;
            if (rr < nrec)
                st_stream(A.out + 3 * (size_t)s_pos[w][rr] + (e - 3u * rr), s_rec[w][e]);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    };
    // wave w: one contiguous chunk [c0, c1) of the block's records, FW_G consecutive groups of 64
    // per step with all groups' loads in flight.  A lane's records are then exactly 64 apart
    // (under one receiver on average), so its receiver is found by a forward scan from the last
    // one instead of a binary search over the block per record.
    const uint32_t per = (R + ST - 1u) / ST * 64u;  // ST / 64 waves
    const uint32_t c0 = min(R, w * per), c1 = min(R, c0 + per);
    uint32_t qc = c0 + ln < c1 ? search(c0 + ln) : 0u;
    for (uint32_t rw = c0; rw < c1; rw += FW_G * 64) {
        uint32_t q[FW_G], pos[FW_G], h[FW_G];
        bool ok[FW_G];
#pragma unroll
        for (int k = 0; k < FW_G; ++k) {
            const uint32_t r = rw + (uint32_t)k * 64u + ln;
            ok[k] = r < c1;
            uint32_t sidx = 0;
            q[k] = pos[k] = 0;
            if (ok[k]) {
                while (s_pre[qc] <= r) ++qc;  // ends: s_pre[ST - 1] = R > r
                q[k] = qc;
                place(r, qc, sidx, pos[k]);
            }
            h[k] = A.scr[sidx];  // (sidx 0 when !ok: a load under a per-lane branch is waited for
        }                        // before the next one issues, which serialised the groups)
        uint4 id[FW_G], pv[FW_G];
#pragma unroll
        for (int k = 0; k < FW_G; ++k) {
            id[k] = pv[k] = make_uint4(0, 0, 0, 0);
            if (ok[k]) {
                id[k] = srec[2 * (size_t)h[k]];
                pv[k] = srec[2 * (size_t)h[k] + 1];
            }
        }
#pragma unroll
        for (int k = 0; k < FW_G; ++k) {
            const uint32_t rk = rw + (uint32_t)k * 64u;
            if (rk < c1) emit(min(64u, c1 - rk), ok[k], q[k], pos[k], id[k], pv[k]);
        }
    }
}

// -------------------------------------------------------------- route ------
struct RouteArgs {
    const uint32_t *ev;  // (a,b) pairs: [enters | leaves]
    uint32_t n_enter, n_total;
    FrameView F;
    SlotTab info;
    const uint4 *eid, *cid;
    const uint32_t *sst;
    const float4 *pos;
    uint32_t G, nb;
    uint32_t *blk_cnt;  // [2][G][nb]: creates then destroys
    uint4 *out_c;       // 3 uint4 per create record
    uint4 *out_d;       // 2 uint4 per destroy record
    uint32_t split;     // destroy bases start at split (one scan over both parts)
};

template <int PASS>
__global__ __launch_bounds__(ST) void k_route(RouteArgs A) {
    extern __shared__ uint32_t lds[];  // [2][G]
    const uint32_t blk = blockIdx.x;
    for (uint32_t g = threadIdx.x; g < 2 * A.G; g += blockDim.x)
        lds[g] = PASS == 0 ? 0u : A.blk_cnt[(size_t)g * A.nb + blk];
    __syncthreads();
    const uint32_t e = blk * ST + threadIdx.x;
    if (e < A.n_total) {
        const uint2 ab = reinterpret_cast<const uint2 *>(A.ev)[e];
        const uint32_t g = A.sst[SLOT_W * (size_t)ab.x + SST_GATE];
        if (g != NO_GATE) {
            const bool create = e < A.n_enter;
            const uint32_t p = atomicAdd(&lds[(create ? 0u : A.G) + g], 1u);
            if (PASS == 1) {
                if (create) {
                    const uint32_t r = A.info.rank[ab.y];  // b is live after the flush
                    const Rec16 B = ld_rec(A.F.rec, r);
                    const float4 P = A.pos[SLOT_U4 * (size_t)ab.y];
                    uint4 *o = A.out_c + 3 * (size_t)p;
                    o[0] = A.cid[SLOT_U4 * (size_t)ab.x];
                    o[1] = A.eid[SLOT_U4 * (size_t)ab.y];
                    o[2] = make_uint4(__float_as_uint(B.x), __float_as_uint(P.y), __float_as_uint(B.z),
                                      __float_as_uint(P.w));
                } else {
                    uint4 *o = A.out_d + 2 * (size_t)(p - A.split);
                    o[0] = A.cid[SLOT_U4 * (size_t)ab.x];
                    o[1] = A.eid[SLOT_U4 * (size_t)ab.y];
                }
            }
        }
    }
    __syncthreads();
    if (PASS == 0)
        for (uint32_t g = threadIdx.x; g < 2 * A.G; g += blockDim.x) A.blk_cnt[(size_t)g * A.nb + blk] = lds[g];
}

// offsets[k] = scanned[k * nb] for k in [0, parts]; scanned has parts*nb + 1 entries
__global__ void k_part_offsets(const uint32_t *__restrict__ scanned, uint32_t parts, uint32_t nb,
                               unsigned long long *off, const unsigned long long *extra) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k <= parts) off[k] = scanned[(size_t)k * nb];
    if (k == parts) off[parts + 1] = extra ? *extra : 0ull;  // (one copy brings both to the host)
}

}  // namespace

// ======================================================== host state ======

struct SyncState {
    gwaoi_world *w = nullptr;
    hipStream_t st = nullptr;
    uint32_t max_slots = 0;
    // device, per slot
    uint4 *slots = nullptr;   // SLOT_U4 per slot (the allocation); the fields below point into it
    uint4 *eid = nullptr, *cid = nullptr;
    uint32_t *sst = nullptr;  // gate, space, syncing, flags
    float4 *pos = nullptr;
    unsigned long long *cl = nullptr;  // 2 per slot: Position / yaw last-writer claims
    uint32_t *oflag = nullptr, *oflag_n = nullptr;  // decode: slots flagged outside every AOI space
    uint32_t oflag_cap = 0;                           // entries of oflag (max_slots)
    bool decoded = false;                           // a decode ran since the last collect
    uint32_t *h_ndec = nullptr;                     // pinned: oflag_n after the last decode
    hipEvent_t ndec_ev = nullptr;                   // that copy
    // id -> slot hash table (device, host mirror)
    uint4 *htab = nullptr;  // 4 per bucket: 3 keys, (slot, slot, slot, -)
    uint32_t hcap = 0, hused = 0;  // entries (3 per 64-B bucket), live + tombstones
    uint32_t hbuckets = 0;         // power of two
    std::vector<uint4> h_hkey;
    std::vector<uint32_t> h_hval;
    std::vector<uint4> h_tab;  // rehash upload staging
    // host mirrors
    std::vector<uint4> h_eid;
    std::vector<uint8_t> h_bound, h_client;
    std::vector<uint8_t> h_plain;  // in a space without AOI (gwaoi_entity_enter_plain)
    std::vector<uint32_t> h_bucket;  // slot -> its hash bucket (if bound)
    std::unordered_map<uint32_t, uint32_t> gate_idx;  // gate id -> dense index
    std::vector<uint16_t> gate_ids;
    // pending device writes
    std::vector<W32> w32;
    std::vector<W128> w128;
    std::vector<SideOp> side;
    std::vector<uint32_t> left;  // slots flagged outside the frame since the last collect (host ops)
    unsigned long long claim_next = 1;
    // staging (pinned host + device), reused once the previous upload has landed
    void *h_stage = nullptr, *d_stage = nullptr;
    size_t stage_cap = 0;
    hipEvent_t stage_ev = nullptr;
    bool stage_pending = false;
    // decode arenas: alive until the flush that consumes them
    struct Chunk {
        char *p;
        size_t cap, used;
    };
    std::vector<Chunk> arena;
    uint64_t arena_tick = ~0ull;
    // collect scratch / outputs
    uint32_t *blk_cnt = nullptr, *scan_tmp = nullptr;
    size_t blk_cap = 0, scan_cap = 0;
    unsigned long long *d_off = nullptr;
    size_t off_cap = 0;
    uint8_t *h_offp = nullptr;  // pinned: d_off (and the extra word) on the host
    size_t h_offp_cap = 0;
    uint32_t *d_left = nullptr;
    size_t left_cap = 0;
    // fan-out scratch, frame order (fan_cap entries each)
    uint32_t *f_snd = nullptr, *f_rg = nullptr, *f_cnt = nullptr, *f_sb = nullptr;
    uint32_t *scr = nullptr;  // fan-out hits (sender entries), receiver runs
    size_t scr_cap = 0;
    unsigned long long *scr_cursor = nullptr;
    uint4 *f_rec = nullptr;  // 2 per entry
    uint4 *f_frec = nullptr, *f_cid = nullptr;
    size_t fan_cap = 0;
    uint4 *out = nullptr, *out_d = nullptr;
    size_t out_cap = 0, outd_cap = 0;  // in uint4
    std::vector<unsigned long long> h_off_raw;
    std::vector<uint64_t> h_off, h_off_c, h_off_d;
    uint8_t *h_rec = nullptr, *h_rec_d = nullptr;
    size_t h_rec_cap = 0, h_recd_cap = 0;
};

namespace {

template <class T>
int salloc(SyncState *S, T **p, size_t n) {
    *p = nullptr;
    if (hipMalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
        *p = nullptr;
        world_set_error(S->w, "sync: hipMalloc failed");
        return GWAOI_ENOMEM;
    }
    return GWAOI_OK;
}
template <class T>
void sfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

#define SY_TRY(expr)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            world_set_error(S->w, (std::string(#expr) + ": " + hipGetErrorString(e_)).c_str()); \
            return GWAOI_EDEVICE;                                                        \
        }                                                                                \
    } while (0)

enum Arr { A_CGATE, A_QSPACE, A_SYNCING, A_SFLAGS, A_HVAL, A_N32 };
enum Arr128 { B_EID, B_CID, B_HKEY, B_N128 };

ArrTable table32(SyncState *S) {
    ArrTable T{};
    T.p[A_CGATE] = S->sst + SST_GATE;
    T.p[A_QSPACE] = S->sst + SST_SPACE;
    T.p[A_SYNCING] = S->sst + SST_SYNCING;
    T.p[A_SFLAGS] = S->sst + SST_FLAGS;
    for (int a = A_CGATE; a <= A_SFLAGS; ++a) T.stride[a] = SLOT_W;
    T.p[A_HVAL] = reinterpret_cast<uint32_t *>(S->htab);  // index: the slot word of an entry (hval_word)
    T.stride[A_HVAL] = 1;
    return T;
}
ArrTable table128(SyncState *S) {
    ArrTable T{};
    T.p[B_EID] = S->eid;
    T.stride[B_EID] = SLOT_U4;
    T.p[B_CID] = S->cid;
    T.stride[B_CID] = SLOT_U4;
    T.p[B_HKEY] = S->htab;  // index: the key of an entry (hkey_vec)
    T.stride[B_HKEY] = 1;
    return T;
}

void put32(SyncState *S, Arr a, uint32_t idx, uint32_t v) { S->w32.push_back(W32{(uint32_t)a, idx, v, 0}); }
void put128(SyncState *S, Arr128 a, uint32_t idx, uint4 v) { S->w128.push_back(W128{(uint32_t)a, idx, 0, 0, v}); }

int ensure_stage(SyncState *S, size_t bytes) {
    if (S->stage_pending) {
        SY_TRY(hipEventSynchronize(S->stage_ev));
        S->stage_pending = false;
    }
    if (bytes <= S->stage_cap) return GWAOI_OK;
    if (S->h_stage) (void)hipHostFree(S->h_stage);
    sfree(S->d_stage);
    S->h_stage = nullptr;
    S->stage_cap = 0;
    const size_t cap = std::max<size_t>(bytes + bytes / 2, 1 << 16);
    SY_TRY(hipHostMalloc(&S->h_stage, cap, hipHostMallocDefault));
    if (int rc = salloc(S, (char **)&S->d_stage, cap)) return rc;
    S->stage_cap = cap;
    return GWAOI_OK;
}

// Keep the last write per (array, index): one scatter launch has no order.
template <class T>
void last_wins(std::vector<T> &v) {
    if (v.size() < 2) return;
    std::vector<uint32_t> ord(v.size());
    for (uint32_t i = 0; i < ord.size(); ++i) ord[i] = i;
    auto key = [&](uint32_t i) { return ((unsigned long long)v[i].arr << 32) | v[i].idx; };
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
    std::vector<T> out;
    out.reserve(v.size());
    for (size_t k = 0; k < ord.size(); ++k)
        if (k + 1 == ord.size() || key(ord[k + 1]) != key(ord[k])) out.push_back(v[ord[k]]);
    v.swap(out);
}

// Upload the pending host-side writes and Y/yaw ops (stream order).
int push(SyncState *S) {
    last_wins(S->w32);
    last_wins(S->w128);
    const size_t b32 = S->w32.size() * sizeof(W32), b128 = S->w128.size() * sizeof(W128);
    const size_t bside = S->side.size() * sizeof(SideOp);
    const size_t total = b128 + b32 + bside;
    if (!total) return GWAOI_OK;
    if (int rc = ensure_stage(S, total)) return rc;
    char *h = static_cast<char *>(S->h_stage);
    char *d = static_cast<char *>(S->d_stage);
    std::memcpy(h, S->w128.data(), b128);
    std::memcpy(h + b128, S->w32.data(), b32);
    std::memcpy(h + b128 + b32, S->side.data(), bside);
    SY_TRY(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, S->st));
    SY_TRY(hipEventRecord(S->stage_ev, S->st));
    S->stage_pending = true;
    // 128-bit writes first (hash keys before the values that publish them)
    if (!S->w128.empty())
        k_scatter128<<<cdivu(S->w128.size(), ST), ST, 0, S->st>>>(reinterpret_cast<const W128 *>(d),
                                                                   (uint32_t)S->w128.size(), table128(S));
    if (!S->w32.empty())
        k_scatter32<<<cdivu(S->w32.size(), ST), ST, 0, S->st>>>(reinterpret_cast<const W32 *>(d + b128),
                                                                 (uint32_t)S->w32.size(), table32(S));
    if (!S->side.empty()) {
        const SideOp *o = reinterpret_cast<const SideOp *>(d + b128 + b32);
        const uint32_t n = (uint32_t)S->side.size();
        k_side_claim<<<cdivu(n, ST), ST, 0, S->st>>>(o, n, S->cl, S->sst);
        k_side_write<<<cdivu(n, ST), ST, 0, S->st>>>(o, n, S->cl, S->pos);
    }
    SY_TRY(hipGetLastError());
    S->w32.clear();
    S->w128.clear();
    S->side.clear();
    return GWAOI_OK;
}

int create(gwaoi_world *w, SyncState **out) {
    SyncState *S = new (std::nothrow) SyncState();
    if (!S) return GWAOI_ENOMEM;
    const WorldView v = world_view(w);
    S->w = w;
    S->st = v.st;
    S->max_slots = v.max_slots;
    uint32_t nbk = 512;  // buckets of three: at least 2 entries per slot
    while (3ull * nbk < 2ull * v.max_slots) nbk <<= 1;
    const uint32_t cap = 3 * nbk;
    S->hbuckets = nbk;
    S->hcap = cap;
    const size_t N = v.max_slots;
    S->oflag_cap = (uint32_t)N;
    int rc;
    if ((rc = salloc(S, &S->slots, SLOT_U4 * N)) || (rc = salloc(S, &S->cl, 2 * N)) || (rc = salloc(S, &S->oflag, N)) ||
        (rc = salloc(S, &S->oflag_n, 1)) || (rc = salloc(S, &S->htab, 4 * (size_t)nbk))) {
        sync_destroy(S);
        return rc;
    }
    S->sst = reinterpret_cast<uint32_t *>(S->slots);
    S->pos = reinterpret_cast<float4 *>(S->slots + 1);
    S->eid = S->slots + 2;
    S->cid = S->slots + 3;
    bool ok = hipMemsetAsync(S->slots, 0, N * 16 * SLOT_U4, S->st) == hipSuccess &&
              hipMemsetAsync(S->cl, 0, N * 16, S->st) == hipSuccess &&
              hipMemsetAsync(S->oflag_n, 0, 4, S->st) == hipSuccess &&
              hipMemsetAsync(S->htab, 0xFF, (size_t)nbk * 64, S->st) == hipSuccess &&  // every entry H_EMPTY
              hipEventCreateWithFlags(&S->stage_ev, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&S->ndec_ev, hipEventDisableTiming) == hipSuccess &&
              hipHostMalloc((void **)&S->h_ndec, 4, hipHostMallocDefault) == hipSuccess;
    if (!ok) {
        sync_destroy(S);
        return GWAOI_EDEVICE;
    }
    // space of every slot in call order (the world may hold entities already)
    std::vector<uint4> qs(N);
    for (uint32_t s = 0; s < N; ++s) qs[s] = make_uint4(NO_GATE, world_slot_space(w, s), 0u, 0u);
    if (hipMemcpy2DAsync(S->sst, 16 * SLOT_U4, qs.data(), 16, 16, N, hipMemcpyHostToDevice, S->st) != hipSuccess ||
        hipStreamSynchronize(S->st) != hipSuccess) {
        sync_destroy(S);
        return GWAOI_EDEVICE;
    }
    S->h_hkey.assign(cap, make_uint4(0, 0, 0, 0));
    S->h_hval.assign(cap, H_EMPTY);
    S->h_eid.assign(N, make_uint4(0, 0, 0, 0));
    S->h_bound.assign(N, 0);
    S->h_client.assign(N, 0);
    S->h_plain.assign(N, 0);
    S->h_bucket.assign(N, H_EMPTY);
    *out = S;
    return GWAOI_OK;
}

int state(gwaoi_world *w, SyncState **out) {
    if (!w) return GWAOI_EINVAL;
    SyncState *&S = world_sync(w);
    if (!S) {
        if (int rc = create(w, &S)) return rc;
    }
    *out = S;
    return GWAOI_OK;
}

uint4 load_id(const uint8_t *p) {
    uint4 v;
    std::memcpy(&v, p, 16);
    return v;
}

bool same(const uint4 &a, const uint4 &b) { return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w; }

// Entry e of the id table: bucket e / 3, way e % 3 (see lookup).
uint32_t hkey_vec(uint32_t e) { return 4 * (e / 3) + e % 3; }        // uint4 index of its key
uint32_t hval_word(uint32_t e) { return 16 * (e / 3) + 12 + e % 3; }  // uint32 index of its slot
uint32_t h_first(const SyncState *S, const uint4 &id) {  // the probe's first entry
    return 3 * (id_hash(id.x, id.y, id.z, id.w) & (S->hbuckets - 1));
}
uint32_t h_next(const SyncState *S, uint32_t e) { return e + 1 == S->hcap ? 0 : e + 1; }

// entry of id, or H_EMPTY
uint32_t h_find(const SyncState *S, const uint4 &id) {
    uint32_t h = h_first(S, id);
    for (uint32_t p = 0; p < S->hcap; ++p, h = h_next(S, h)) {
        const uint32_t v = S->h_hval[h];
        if (v == H_EMPTY) return H_EMPTY;
        if (v != H_TOMB && same(S->h_hkey[h], id)) return h;
    }
    return H_EMPTY;
}

// Rebuild the table without tombstones and upload it whole.
int h_rehash(SyncState *S) {
    std::fill(S->h_hval.begin(), S->h_hval.end(), H_EMPTY);
    S->hused = 0;
    for (uint32_t s = 0; s < S->max_slots; ++s) {
        if (!S->h_bound[s]) continue;
        const uint4 id = S->h_eid[s];
        uint32_t h = h_first(S, id);
        while (S->h_hval[h] != H_EMPTY) h = h_next(S, h);
        S->h_hkey[h] = id;
        S->h_hval[h] = s;
        S->h_bucket[s] = h;
        S->hused++;
    }
    // drop pending table writes: the whole table goes up now (after the other pending writes)
    std::vector<W32> k32;
    for (const W32 &e : S->w32)
        if (e.arr != A_HVAL) k32.push_back(e);
    S->w32.swap(k32);
    std::vector<W128> k128;
    for (const W128 &e : S->w128)
        if (e.arr != B_HKEY) k128.push_back(e);
    S->w128.swap(k128);
    if (int rc = push(S)) return rc;
    S->h_tab.assign(4 * (size_t)S->hbuckets, make_uint4(H_EMPTY, H_EMPTY, H_EMPTY, H_EMPTY));
    for (uint32_t h = 0; h < S->hcap; ++h) {
        S->h_tab[hkey_vec(h)] = S->h_hkey[h];
        reinterpret_cast<uint32_t *>(S->h_tab.data())[hval_word(h)] = S->h_hval[h];
    }
    SY_TRY(hipMemcpyAsync(S->htab, S->h_tab.data(), S->h_tab.size() * 16, hipMemcpyHostToDevice, S->st));
    SY_TRY(hipStreamSynchronize(S->st));  // h_tab is pageable staging
    return GWAOI_OK;
}

int bind_one(SyncState *S, uint32_t slot, const uint4 &id) {
    if (slot >= S->max_slots) return GWAOI_EBADSLOT;
    const uint32_t hb = h_find(S, id);
    if (S->h_bound[slot]) return (hb != H_EMPTY && S->h_hval[hb] == slot) ? GWAOI_OK : GWAOI_ESTATE;
    if (hb != H_EMPTY) return GWAOI_ESTATE;  // id bound to another slot
    if (S->hused + 1 > S->hcap / 4 * 3) {
        // too many tombstones (live entries are <= max_slots <= hcap/2)
        if (int rc = h_rehash(S)) return rc;
    }
    uint32_t h = h_first(S, id);
    while (S->h_hval[h] != H_EMPTY && S->h_hval[h] != H_TOMB) h = h_next(S, h);
    if (S->h_hval[h] == H_EMPTY) S->hused++;
    S->h_hkey[h] = id;
    S->h_hval[h] = slot;
    S->h_bucket[slot] = h;
    S->h_bound[slot] = 1;
    S->h_eid[slot] = id;
    put128(S, B_HKEY, hkey_vec(h), id);
    put32(S, A_HVAL, hval_word(h), slot);
    put128(S, B_EID, slot, id);
    return GWAOI_OK;
}

int ensure_u32(SyncState *S, uint32_t **p, size_t *cap, size_t n) {
    if (n <= *cap) return GWAOI_OK;
    sfree(*p);
    *cap = 0;
    const size_t c = std::max<size_t>(n + n / 4, 1024);
    if (int rc = salloc(S, p, c)) return rc;
    *cap = c;
    return GWAOI_OK;
}

// (device) records, grown to n uint4
int ensure_out(SyncState *S, uint4 **p, size_t *cap, size_t n) {
    if (n <= *cap) return GWAOI_OK;
    sfree(*p);
    *cap = 0;
    const size_t c = std::max<size_t>(n + n / 8, 3 * 1024);
    if (int rc = salloc(S, p, c)) return rc;
    *cap = c;
    return GWAOI_OK;
}

int ensure_host(SyncState *S, uint8_t **p, size_t *cap, size_t bytes) {
    if (bytes <= *cap) return GWAOI_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t c = std::max<size_t>(bytes + bytes / 8, 1 << 16);
    SY_TRY(hipHostMalloc((void **)p, c, hipHostMallocDefault));
    *cap = c;
    return GWAOI_OK;
}

// Multisplit bases: blk_cnt [parts][nb] -> exclusive scan (parts*nb + 1
// entries, the last is the total) -> h_off_raw[0..parts].
int fetch_bases(SyncState *S, uint32_t parts, bool sync);

unsigned long long unpack_bases(SyncState *S, uint32_t parts) {  // -> the extra word
    const unsigned long long *h = reinterpret_cast<const unsigned long long *>(S->h_offp);
    S->h_off_raw.assign(h, h + parts + 1);
    return h[parts + 1];
}

// per-part bases of the [parts][nb] counts in blk_cnt (scanned in place) into d_off[0, parts],
// with *extra (a device word, e.g. a cursor) in d_off[parts + 1]
int part_bases(SyncState *S, uint32_t parts, uint32_t nb, bool sync = true, bool copy = true,
               const unsigned long long *extra = nullptr) {
    const size_t n = (size_t)parts * nb + 1;
    if (int rc = ensure_u32(S, &S->scan_tmp, &S->scan_cap, scan_tmp_elems(n) + 4)) return rc;
    if (parts + 2 > S->off_cap) {
        sfree(S->d_off);
        if (int rc = salloc(S, &S->d_off, parts + 2)) return rc;
        S->off_cap = parts + 2;
    }
    scan_exclusive(S->blk_cnt, S->blk_cnt, n, S->scan_tmp, S->st);
    k_part_offsets<<<cdivu(parts + 1, ST), ST, 0, S->st>>>(S->blk_cnt, parts, nb, S->d_off, extra);
    SY_TRY(hipGetLastError());
    return copy ? fetch_bases(S, parts, sync) : GWAOI_OK;
}

// the bases part_bases left in d_off (and the extra word), to pinned host memory; unpack_bases
// turns them into h_off_raw once the stream has reached the copy
int fetch_bases(SyncState *S, uint32_t parts, bool sync) {
    if (int rc = ensure_host(S, &S->h_offp, &S->h_offp_cap, (parts + 2) * 8)) return rc;
    SY_TRY(hipMemcpyAsync(S->h_offp, S->d_off, (parts + 2) * 8, hipMemcpyDeviceToHost, S->st));
    if (sync) {
        SY_TRY(hipStreamSynchronize(S->st));
        unpack_bases(S, parts);
    }
    return GWAOI_OK;
}

void fill_out(SyncState *S, gwaoi_gate_records *o, const std::vector<uint64_t> &off, const uint8_t *rec) {
    o->n_gates = (uint32_t)S->gate_ids.size();
    o->gate_ids = S->gate_ids.data();
    o->offsets = off.data();
    o->records = rec;
}

int collect_sync(gwaoi_world *w, gwaoi_gate_records *out, bool to_host) {
    if (!w || !out) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = state(w, &S)) return rc;
    const WorldView v = world_view(w);
    if (v.pending_ops) return GWAOI_ESTATE;
    if (int rc = push(S)) return rc;
    // flagged slots outside the frame get their own-client record only (InterestedBy is empty
    // outside an AOI space): the host ops' list, then the slots k_decode listed
    std::vector<uint32_t> left;
    std::sort(S->left.begin(), S->left.end());
    S->left.erase(std::unique(S->left.begin(), S->left.end()), S->left.end());
    for (uint32_t s : S->left)
        if (world_slot_space(w, s) == SP_DEAD) left.push_back(s);
    S->left.clear();
    uint32_t n_dec = 0;
    if (S->decoded) {  // copied behind the last decode: done by now unless that flush is still running
        SY_TRY(hipEventSynchronize(S->ndec_ev));
        n_dec = *S->h_ndec;
        S->decoded = false;
        n_dec = std::min(n_dec, S->oflag_cap);  // k_decode lists a slot at most once (atomicOr claim)
    }
    const size_t n_left = left.size() + n_dec;
    if (n_left) {
        if (int rc = ensure_u32(S, &S->d_left, &S->left_cap, n_left)) return rc;
        if (!left.empty())
            SY_TRY(hipMemcpyAsync(S->d_left, left.data(), left.size() * 4, hipMemcpyHostToDevice, S->st));
        if (n_dec) {
            SY_TRY(hipMemcpyAsync(S->d_left + left.size(), S->oflag, (size_t)n_dec * 4, hipMemcpyDeviceToDevice,
                                  S->st));
            SY_TRY(hipMemsetAsync(S->oflag_n, 0, 4, S->st));
        }
    }
    const uint32_t G = (uint32_t)S->gate_ids.size();
    const uint32_t n_ent = v.F.n + (uint32_t)n_left;
    const uint32_t nb = std::max(1u, cdivu(n_ent, ST));
    FanArgs A{};
    A.F = v.F;
    A.info = v.info;
    A.left = S->d_left;
    A.n_left = (uint32_t)n_left;
    A.eid = S->eid;
    A.cid = S->cid;
    A.sst = S->sst;
    A.pos = S->pos;
    A.G = G;
    A.nb = nb;
    if (int rc = ensure_u32(S, &S->blk_cnt, &S->blk_cap, (size_t)G * nb + 1)) return rc;
    A.blk_cnt = S->blk_cnt;
    if (n_ent > S->fan_cap) {
        sfree(S->f_snd); sfree(S->f_rg); sfree(S->f_rec); sfree(S->f_frec); sfree(S->f_cid);
        sfree(S->f_cnt); sfree(S->f_sb);
        S->fan_cap = 0;
        const size_t c = std::max<size_t>(n_ent + n_ent / 8, 1024);
        int rc;
        if ((rc = salloc(S, &S->f_snd, c)) || (rc = salloc(S, &S->f_rg, c)) ||
            (rc = salloc(S, &S->f_rec, 2 * c)) || (rc = salloc(S, &S->f_frec, c)) || (rc = salloc(S, &S->f_cid, c)) || (rc = salloc(S, &S->f_cnt, c)) ||
            (rc = salloc(S, &S->f_sb, c)))
            return rc;
        S->fan_cap = c;
    }
    int rc_scr = GWAOI_OK;
    if (!S->scr_cursor && (rc_scr = salloc(S, &S->scr_cursor, 1))) return rc_scr;
    A.fcnt = S->f_cnt;
    A.fsb = S->f_sb;
    A.snd = S->f_snd;
    A.rg = S->f_rg;
    A.srec = S->f_rec;
    A.frec = S->f_frec;
    A.fcid = S->f_cid;
    A.scr_cursor = S->scr_cursor;
    if (n_ent) k_fan_prep<<<cdivu(n_ent, ST), ST, 0, S->st>>>(A);  // also clears the flags
    uint64_t total = 0;
    S->h_off_raw.assign((size_t)G + 1, 0);  // G gates, all empty unless the passes below run
    if (G && n_ent) {
        // pass 1: hits into the scratch; a run past the capacity is redone after a regrow
        for (int attempt = 0;; ++attempt) {
            if (S->scr_cap == 0 && (rc_scr = ensure_u32(S, &S->scr, &S->scr_cap, 32 * (size_t)n_ent))) return rc_scr;
            A.scr = S->scr;
            A.scr_cap = std::min<unsigned long long>(S->scr_cap, SCR_FULL - 1ull);
            if (attempt) {  // (k_fan_prep zeroed them for the first)
                SY_TRY(hipMemsetAsync(S->scr_cursor, 0, 8, S->st));
                SY_TRY(hipMemsetAsync(S->blk_cnt + (size_t)G * nb, 0, 4, S->st));
            }
            k_fan_hits_wave<<<nb, ST, (size_t)G * 4, S->st>>>(A);
            SY_TRY(hipGetLastError());
            // the per-gate bases are scanned before the capacity check: one host round trip
            // for both (a rerun rewrites every count the scan read).  The write pass follows on
            // the device with the output as it is (the last collect's size), queued before the
            // (pageable, host-blocking) copies of the bases and the cursor; it writes nothing
            // when either capacity fell short, which the host sees below
            if (int rc = part_bases(S, G, nb, false, false, S->scr_cursor)) return rc;
            A.out = S->out;
            A.out_recs = S->out_cap / 3;
#ifdef GWAOI_EXP_FW_ROUNDTRIP  // A/B: the write pass launched after the host's sync (before round 6)
            A.out_recs = 0;
#endif
            if (A.out_recs) {
                k_fan_write<<<nb, ST, (3 * (size_t)G + 1) * 4, S->st>>>(A);
                SY_TRY(hipGetLastError());
            }
            if (int rc = fetch_bases(S, G, false)) return rc;
            SY_TRY(hipStreamSynchronize(S->st));
            const unsigned long long used = unpack_bases(S, G);
            if (used <= A.scr_cap) break;
            if (attempt || used >= SCR_FULL) {
                world_set_error(w, "sync: fan-out scratch exceeds 2^32 entries");
                return GWAOI_ENOMEM;
            }
            if ((rc_scr = ensure_u32(S, &S->scr, &S->scr_cap, (size_t)used))) return rc_scr;
        }
        total = S->h_off_raw[G];
    }
    if (total > A.out_recs) {  // (first collect, or more records than the output holds)
        if (int rc = ensure_out(S, &S->out, &S->out_cap, 3 * total)) return rc;
        A.out = S->out;
        A.out_recs = S->out_cap / 3;
        k_fan_write<<<nb, ST, (3 * (size_t)G + 1) * 4, S->st>>>(A);
        SY_TRY(hipGetLastError());
    }
    if (int rc = ensure_out(S, &S->out, &S->out_cap, 3)) return rc;  // (an empty collect's pointer)
    S->h_off.assign(S->h_off_raw.begin(), S->h_off_raw.end());
    if (to_host) {
        if (int rc = ensure_host(S, &S->h_rec, &S->h_rec_cap, std::max<uint64_t>(total, 1) * 48)) return rc;
        if (total) SY_TRY(hipMemcpyAsync(S->h_rec, S->out, total * 48, hipMemcpyDeviceToHost, S->st));
        SY_TRY(hipStreamSynchronize(S->st));
        fill_out(S, out, S->h_off, S->h_rec);
    } else {
        fill_out(S, out, S->h_off, reinterpret_cast<const uint8_t *>(S->out));
    }
    return GWAOI_OK;
}

int decode(gwaoi_world *w, const uint8_t *payload, size_t n, bool on_device) {
    if (!w || (n && !payload)) return GWAOI_EINVAL;
    if (on_device && (reinterpret_cast<uintptr_t>(payload) & 15u)) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = state(w, &S)) return rc;
    if (world_view(w).in_flight) return GWAOI_ESTATE;  // a flush in flight reads the sync state's stream
    if (!n) return GWAOI_OK;
    if (n > 0x7FFFFFFFull) return GWAOI_EINVAL;
    // arena of the current flush (older chunks were consumed by earlier flushes)
    uint64_t ticks_now;
    {
        gwaoi_info inf;
        gwaoi_world_info(w, &inf);
        ticks_now = inf.ticks;
    }
    if (S->arena_tick != ticks_now) {
        if (S->arena.size() > 1) {  // keep the largest chunk only
            SY_TRY(hipStreamSynchronize(S->st));
            std::sort(S->arena.begin(), S->arena.end(),
                      [](const SyncState::Chunk &a, const SyncState::Chunk &b) { return a.cap > b.cap; });
            for (size_t k = 1; k < S->arena.size(); ++k) (void)hipFree(S->arena[k].p);
            S->arena.resize(1);
        }
        for (auto &c : S->arena) c.used = 0;
        S->arena_tick = ticks_now;
    }
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t need = 6 * al(n * 4) + al(4) + (on_device ? 0 : al(n * 32));
    SyncState::Chunk *ch = nullptr;
    for (auto &c : S->arena)
        if (c.cap - c.used >= need) {
            ch = &c;
            break;
        }
    if (!ch) {
        SyncState::Chunk c{nullptr, std::max<size_t>(need, 1 << 20), 0};
        SY_TRY(hipMalloc((void **)&c.p, c.cap));
        S->arena.push_back(c);
        ch = &S->arena.back();
    }
    char *base = ch->p + ch->used;
    ch->used += need;
    uint32_t *o_slot = reinterpret_cast<uint32_t *>(base);
    float *o_x = reinterpret_cast<float *>(base + al(n * 4));
    float *o_z = reinterpret_cast<float *>(base + 2 * al(n * 4));
    uint32_t *o_sp = reinterpret_cast<uint32_t *>(base + 3 * al(n * 4));
    uint32_t *o_ys = reinterpret_cast<uint32_t *>(base + 4 * al(n * 4));
    const uint4 *pay;
    if (on_device) {
        pay = reinterpret_cast<const uint4 *>(payload);
    } else {
        char *dp = base + 6 * al(n * 4) + al(4);
        SY_TRY(hipMemcpyAsync(dp, payload, n * 32, hipMemcpyHostToDevice, S->st));
        pay = reinterpret_cast<const uint4 *>(dp);
    }
    if (int rc = push(S)) return rc;
    DecodeArgs A{};
    A.pay = pay;
    A.n = (uint32_t)n;
    A.htab = S->htab;
    A.hmask = S->hbuckets - 1;
    A.sst = S->sst;
    A.o_slot = o_slot;
    A.o_sp = o_sp;
    A.o_x = o_x;
    A.o_z = o_z;
    A.o_ys = o_ys;
    A.claim0 = S->claim_next;
    A.cl = S->cl;
    A.pos = S->pos;
    A.oflag = S->oflag;
    A.oflag_n = S->oflag_n;
    A.h_ndec = S->h_ndec;
    A.oflag_cap = S->oflag_cap;
    A.dups = reinterpret_cast<uint32_t *>(base + 5 * al(n * 4));
    A.ndup = reinterpret_cast<uint32_t *>(base + 6 * al(n * 4));
    S->claim_next += n;
    S->decoded = true;
    k_decode<GWAOI_DEC_PER><<<cdivu(n, ST * GWAOI_DEC_PER), ST, 0, S->st>>>(A);
    k_decode_apply<<<cdivu(n, ST), ST, 0, S->st>>>(A);
    k_decode_dups<<<std::min<uint32_t>(cdivu(n, ST), 64u), ST, 0, S->st>>>(A);
    SY_TRY(hipGetLastError());
    SY_TRY(hipEventRecord(S->ndec_ev, S->st));
    return world_queue_decoded(w, o_slot, o_x, o_z, o_sp, n);
}

}  // namespace

void sync_note_slot(SyncState *S, uint32_t slot, uint32_t space_or_dead) {
    put32(S, A_QSPACE, slot, space_or_dead);
    if (space_or_dead == SP_DEAD)
        S->left.push_back(slot);
    else  // Space.enter: syncInfoFlag |= sifSyncOwnClient | sifSyncNeighborClients (Space.go:205)
        S->side.push_back(SideOp{slot, SIDE_SIF, 0ull, make_float4(0.f, 0.f, 0.f, 0.f)});
}

bool sync_slot_plain(const SyncState *S, uint32_t slot) { return slot < S->max_slots && S->h_plain[slot]; }

void sync_destroy(SyncState *S) {
    if (!S) return;
    if (S->st) (void)hipStreamSynchronize(S->st);
    sfree(S->slots);
    sfree(S->cl); sfree(S->oflag); sfree(S->oflag_n);
    sfree(S->htab);
    sfree(S->f_snd); sfree(S->f_rg); sfree(S->f_rec); sfree(S->f_frec); sfree(S->f_cid);
    sfree(S->blk_cnt); sfree(S->scan_tmp); sfree(S->scr); sfree(S->scr_cursor); sfree(S->f_cnt); sfree(S->f_sb); sfree(S->d_off); sfree(S->d_left); sfree(S->out); sfree(S->out_d);
    sfree(S->d_stage);
    for (auto &c : S->arena) (void)hipFree(c.p);
    if (S->h_stage) (void)hipHostFree(S->h_stage);
    if (S->h_rec) (void)hipHostFree(S->h_rec);
    if (S->h_rec_d) (void)hipHostFree(S->h_rec_d);
    if (S->stage_ev) (void)hipEventDestroy(S->stage_ev);
    if (S->ndec_ev) (void)hipEventDestroy(S->ndec_ev);
    if (S->h_ndec) (void)hipHostFree(S->h_ndec);
    if (S->h_offp) (void)hipHostFree(S->h_offp);
    delete S;
}

}  // namespace gw

// =============================================================== C ABI =======

using gw::SyncState;

extern "C" {

int gwaoi_entity_bind(gwaoi_world *w, uint32_t slot, const uint8_t eid[GWAOI_ID_LEN]) {
    return gw::api_guard([&]() -> int {
    if (!w || !eid) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = gw::state(w, &S)) return rc;
    return gw::bind_one(S, slot, gw::load_id(eid));
    });
}

int gwaoi_entity_bind_batch(gwaoi_world *w, const uint32_t *slots, const uint8_t *eids, size_t n) {
    return gw::api_guard([&]() -> int {
    if (!w || (n && (!slots || !eids))) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = gw::state(w, &S)) return rc;
    for (size_t i = 0; i < n; ++i)
        if (int rc = gw::bind_one(S, slots[i], gw::load_id(eids + 16 * i))) return rc;
    return GWAOI_OK;
    });
}

int gwaoi_entity_unbind(gwaoi_world *w, uint32_t slot) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = gw::state(w, &S)) return rc;
    if (slot >= S->max_slots) return GWAOI_EBADSLOT;
    if (!S->h_bound[slot]) return GWAOI_ESTATE;
    const uint32_t h = S->h_bucket[slot];
    S->h_hval[h] = gw::H_TOMB;
    gw::put32(S, gw::A_HVAL, gw::hval_word(h), gw::H_TOMB);
    S->h_bound[slot] = 0;
    S->h_bucket[slot] = gw::H_EMPTY;
    if (S->h_client[slot]) {
        S->h_client[slot] = 0;
        gw::put32(S, gw::A_CGATE, slot, gw::NO_GATE);
    }
    gw::put32(S, gw::A_SYNCING, slot, 0);
    return GWAOI_OK;
    });
}

int gwaoi_entity_set_client(gwaoi_world *w, uint32_t slot, uint16_t gate_id, const uint8_t *clientid) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = gw::state(w, &S)) return rc;
    if (slot >= S->max_slots) return GWAOI_EBADSLOT;
    if (!clientid) {
        S->h_client[slot] = 0;
        gw::put32(S, gw::A_CGATE, slot, gw::NO_GATE);
        return GWAOI_OK;
    }
    auto it = S->gate_idx.find(gate_id);
    uint32_t g;
    if (it == S->gate_idx.end()) {
        if (S->gate_ids.size() >= GWAOI_MAX_GATES) return GWAOI_ECAPACITY;
        g = (uint32_t)S->gate_ids.size();
        S->gate_idx.emplace(gate_id, g);
        S->gate_ids.push_back(gate_id);
    } else {
        g = it->second;
    }
    S->h_client[slot] = 1;
    gw::put128(S, gw::B_CID, slot, gw::load_id(clientid));
    gw::put32(S, gw::A_CGATE, slot, g);
    return GWAOI_OK;
    });
}

int gwaoi_entity_set_syncing(gwaoi_world *w, uint32_t slot, int syncing) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = gw::state(w, &S)) return rc;
    if (slot >= S->max_slots) return GWAOI_EBADSLOT;
    gw::put32(S, gw::A_SYNCING, slot, syncing ? 1u : 0u);
    return GWAOI_OK;
    });
}

int gwaoi_entity_set_position_yaw(gwaoi_world *w, uint32_t slot, float x, float y, float z, float yaw) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = gw::state(w, &S)) return rc;
    if (slot >= S->max_slots) return GWAOI_EBADSLOT;
    S->side.push_back(gw::SideOp{slot, gw::SIDE_POS | gw::SIDE_YAW, S->claim_next++, make_float4(x, y, z, yaw)});
    return GWAOI_OK;
    });
}

int gwaoi_set_position_yaw(gwaoi_world *w, uint32_t slot, float x, float y, float z, float yaw) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = gw::state(w, &S)) return rc;
    if (slot >= S->max_slots) return GWAOI_EBADSLOT;
    if (gw::world_slot_space(w, slot) != gw::SP_DEAD) {  // Space.move of an AOI space: Position + Moved
        if (int rc = gwaoi_moved(w, slot, x, z)) return rc;
        S->side.push_back(gw::SideOp{slot, gw::SIDE_POS | gw::SIDE_YAW | gw::SIDE_SIF, S->claim_next++,
                                     make_float4(x, y, z, yaw)});
        return GWAOI_OK;
    }
    // nilSpace or a space without AOI: Space.move returns before Position (Space.go:253-257); yaw
    // and both flags are still set (Entity.go:1196-1204)
    S->side.push_back(gw::SideOp{slot, gw::SIDE_YAW | gw::SIDE_SIF, S->claim_next++, make_float4(x, y, z, yaw)});
    S->left.push_back(slot);
    return GWAOI_OK;
    });
}

int gwaoi_entity_enter_plain(gwaoi_world *w, uint32_t slot, float x, float y, float z) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = gw::state(w, &S)) return rc;
    if (slot >= S->max_slots) return GWAOI_EBADSLOT;
    // Space.enter panics unless the entity is in nilSpace (Space.go:193-195)
    if (S->h_plain[slot] || gw::world_slot_space(w, slot) != gw::SP_DEAD) return GWAOI_ESTATE;
    S->h_plain[slot] = 1;
    S->side.push_back(gw::SideOp{slot, gw::SIDE_POS | gw::SIDE_SIF, S->claim_next++, make_float4(x, y, z, 0.f)});
    S->left.push_back(slot);
    return GWAOI_OK;
    });
}

int gwaoi_entity_leave_plain(gwaoi_world *w, uint32_t slot) {
    return gw::api_guard([&]() -> int {
    if (!w) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = gw::state(w, &S)) return rc;
    if (slot >= S->max_slots) return GWAOI_EBADSLOT;
    if (!S->h_plain[slot]) return GWAOI_ESTATE;  // Space.leave panics for another space (Space.go:229-231)
    S->h_plain[slot] = 0;
    return GWAOI_OK;
    });
}

int gwaoi_sync_from_clients(gwaoi_world *w, const uint8_t *payload, size_t n_rec) {
    return gw::api_guard([&]() -> int {
    return gw::decode(w, payload, n_rec, false);
    });
}

int gwaoi_sync_from_clients_device(gwaoi_world *w, const uint8_t *d_payload, size_t n_rec) {
    return gw::api_guard([&]() -> int {
    return gw::decode(w, d_payload, n_rec, true);
    });
}

int gwaoi_collect_sync_infos(gwaoi_world *w, gwaoi_gate_records *out) { return gw::api_guard([&]() -> int { return gw::collect_sync(w, out, true); }); }

int gwaoi_collect_sync_infos_device(gwaoi_world *w, gwaoi_gate_records *out) {
    return gw::api_guard([&]() -> int {
    return gw::collect_sync(w, out, false);
    });
}

int gwaoi_collect_client_events(gwaoi_world *w, gwaoi_gate_records *creates, gwaoi_gate_records *destroys) {
    return gw::api_guard([&]() -> int {
    using namespace gw;
    if (!w || !creates || !destroys) return GWAOI_EINVAL;
    SyncState *S;
    if (int rc = state(w, &S)) return rc;
    const WorldView v = world_view(w);
    if (v.pending_ops) return GWAOI_ESTATE;
    if (int rc = push(S)) return rc;
    const uint32_t G = (uint32_t)S->gate_ids.size();
    const uint64_t n_total = v.n_enter + v.n_leave;
    S->h_off_c.assign(G + 1, 0);
    S->h_off_d.assign(G + 1, 0);
    uint64_t nc = 0, nd = 0;
    if (G && n_total) {
        const uint32_t nb = cdivu(n_total, ST);
        if (int rc = ensure_u32(S, &S->blk_cnt, &S->blk_cap, 2 * (size_t)G * nb + 1)) return rc;
        RouteArgs A{};
        A.ev = v.events;
        A.n_enter = (uint32_t)v.n_enter;
        A.n_total = (uint32_t)n_total;
        A.F = v.F;
        A.info = v.info;
        A.eid = S->eid;
        A.cid = S->cid;
        A.sst = S->sst;
        A.pos = S->pos;
        A.G = G;
        A.nb = nb;
        A.blk_cnt = S->blk_cnt;
        const size_t lds = 2 * (size_t)G * 4;
        SY_TRY(hipMemsetAsync(S->blk_cnt + 2 * (size_t)G * nb, 0, 4, S->st));
        k_route<0><<<nb, ST, lds, S->st>>>(A);
        SY_TRY(hipGetLastError());
        if (int rc = part_bases(S, 2 * G, nb)) return rc;
        const uint64_t split = S->h_off_raw[G];  // creates occupy [0, split) of one index space
        nc = split;
        nd = S->h_off_raw[2 * G] - split;
        if (int rc = ensure_out(S, &S->out, &S->out_cap, 3 * std::max<uint64_t>(nc, 1))) return rc;
        if (int rc = ensure_out(S, &S->out_d, &S->outd_cap, 2 * std::max<uint64_t>(nd, 1))) return rc;
        A.out_c = S->out;
        A.out_d = S->out_d;
        A.split = (uint32_t)split;
        k_route<1><<<nb, ST, lds, S->st>>>(A);
        SY_TRY(hipGetLastError());
        for (uint32_t g = 0; g <= G; ++g) {
            S->h_off_c[g] = S->h_off_raw[g];
            S->h_off_d[g] = S->h_off_raw[G + g] - split;
        }
    }
    if (int rc = ensure_host(S, &S->h_rec, &S->h_rec_cap, std::max<uint64_t>(nc, 1) * 48)) return rc;
    if (int rc = ensure_host(S, &S->h_rec_d, &S->h_recd_cap, std::max<uint64_t>(nd, 1) * 32)) return rc;
    if (nc) SY_TRY(hipMemcpyAsync(S->h_rec, S->out, nc * 48, hipMemcpyDeviceToHost, S->st));
    if (nd) SY_TRY(hipMemcpyAsync(S->h_rec_d, S->out_d, nd * 32, hipMemcpyDeviceToHost, S->st));
    SY_TRY(hipStreamSynchronize(S->st));
    fill_out(S, creates, S->h_off_c, S->h_rec);
    fill_out(S, destroys, S->h_off_d, S->h_rec_d);
    return GWAOI_OK;
    });
}

}  // extern "C"
