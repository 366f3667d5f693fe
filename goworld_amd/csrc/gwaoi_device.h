// Device helpers shared by the HIP translation units of libgwaoi
// (gwaoi_kernels.hip, gwaoi_sync.hip): record loads/stores, the grid's cell
// function and go-aoi's window relation.  Not part of the public ABI.
#pragma once

#include "gwaoi_internal.h"

namespace gw {

// Monotone non-decreasing in v (IEEE sub/mul round monotonically; clamp is
// monotone).  keygen and every query use this one function.
__device__ __forceinline__ int cell_of(float v, float o, float inv, uint32_t g) {
    float t = (v - o) * inv;
    t = fmaxf(t, 0.0f);
    t = fminf(t, (float)(g - 1));
    return (int)t;
}

__device__ __forceinline__ Rec16 ld_rec(const Rec16 *p, uint32_t i) {
    const uint4 q = reinterpret_cast<const uint4 *>(p)[i];
    Rec16 r;
    r.x = __uint_as_float(q.x);
    r.z = __uint_as_float(q.y);
    r.s = ((unsigned long long)q.w << 32) | q.z;
    return r;
}

__device__ __forceinline__ void st_rec(Rec16 *p, uint32_t i, const Rec16 &r) {
    reinterpret_cast<uint4 *>(p)[i] =
        make_uint4(__float_as_uint(r.x), __float_as_uint(r.z), (uint32_t)r.s, (uint32_t)(r.s >> 32));
}

__device__ __forceinline__ SlotSp ld_ss(const SlotSp *p, uint32_t i) {
    const uint2 q = reinterpret_cast<const uint2 *>(p)[i];
    SlotSp r;
    r.slot = q.x;
    r.sp = q.y;
    return r;
}

__device__ __forceinline__ void st_ss(SlotSp *p, uint32_t i, uint32_t slot, uint32_t sp) {
    reinterpret_cast<uint2 *>(p)[i] = make_uint2(slot, sp);
}

__device__ __forceinline__ float qnan() { return __int_as_float(0x7FC00000); }

// go-aoi relation: the owner (larger seq) W's window [fl32(w-D), fl32(w+D)]^2 contains the other
__device__ __forceinline__ bool rel(float xa, float za, unsigned long long sa, float xb, float zb,
                                    unsigned long long sb, float D) {
    const bool own = sa > sb;
    const float wx = own ? xa : xb, wz = own ? za : zb;
    const float px = own ? xb : xa, pz = own ? zb : za;
    return (int)(px >= wx - D) & (int)(px <= wx + D) & (int)(pz >= wz - D) & (int)(pz <= wz + D);
}

// Workgroups are dispatched round-robin over the 8 XCDs, each with its own
// L2.  Neighbouring blocks read the same candidate rows, so give every XCD a
// contiguous run of blocks: XCD x (bid % 8 == x) takes blocks
// [x*q + min(x, r), ...) in order, q = nb / 8, r = nb % 8.
constexpr uint32_t N_XCD = 8;
__device__ __forceinline__ uint32_t xcd_block(uint32_t bid, uint32_t nb) {
    const uint32_t x = bid % N_XCD, k = bid / N_XCD, q = nb / N_XCD, r = nb % N_XCD;
    return x * q + min(x, r) + k;
}

// The XCD this wave runs on (s_getreg HW_REG_XCC_ID: id 20, offset 0, 4 bits), 0..7.  Placement
// information, for speed only: nothing's correctness depends on it.
__device__ __forceinline__ uint32_t xcc_id() {
    return (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & (N_XCD - 1u);
}

// n directed pairs from event stream q (one returning atomic on the shard's own line); the
// encoded stream position of the first (ev_phys gives the scratch index).
__device__ __forceinline__ unsigned long long ev_alloc(TickScalars *sc, uint32_t q, uint32_t n) {
    return ev_enc(q, atomicAdd(reinterpret_cast<unsigned long long *>(&sc->shard[q][2]), (unsigned long long)n));
}

// The directed pair (a,b), (b,a) at stream position p (even: both in one chunk), if it fits.
__device__ __forceinline__ void ev_put2(uint2 *out, uint64_t cap, unsigned long long p, uint32_t a, uint32_t b) {
    const unsigned long long i = ev_phys(p);
    if (i + 1 < cap) {
        out[i] = make_uint2(a, b);
        out[i + 1] = make_uint2(b, a);
    }
}

// Inclusive wave-wide scans by DPP (rows of 16 lanes, then the row broadcasts).
__device__ __forceinline__ uint32_t dpp_shr(uint32_t v, int n) {
    switch (n) {
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    case 4: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    default: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    }
}
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v) {
    v += dpp_shr(v, 1);
    v += dpp_shr(v, 2);
    v += dpp_shr(v, 4);
    v += dpp_shr(v, 8);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
__device__ __forceinline__ uint32_t wave_scan_max(uint32_t v) {
    v = max(v, dpp_shr(v, 1));
    v = max(v, dpp_shr(v, 2));
    v = max(v, dpp_shr(v, 4));
    v = max(v, dpp_shr(v, 8));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}

}  // namespace gw
