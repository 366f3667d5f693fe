// calib_fetch.hip -- calibrates rocprofv3's FETCH_SIZE on gfx950 for the read
// patterns of k_combined (MI355X_MICROARCH.md: FETCH_SIZE is exact only after
// doubling for wide streaming reads; "calibrate on a known byte count in your
// own access pattern").  A 2 GiB table (past the 256 MiB Infinity Cache) is
// read in four patterns whose distinct 64-B and 128-B line counts are known:
//   stream    16 B per lane, coalesced: 2 GiB
//   gather1   one 16-B record per 128-B line, lines in random order: R lines
//   gather2   both 64-B halves of R lines, the second half read by a later
//             launch-half (no merging in flight): a 128-B fetch serves both,
//             a 64-B one does not
//   runs4     4 consecutive records (one 64-B half-line) per lane at random
//             64-B-aligned positions: the k_combined candidate-run shape
// Each is one launch; rocprofv3 --pmc FETCH_SIZE gives the counted bytes,
// printed beside the known distinct 64-B / 128-B bytes by tools/calib_fetch.py.
// Build: hipcc --offload-arch=gfx950 -O3 -o goworld_amd/lib/calib_fetch tools/calib_fetch.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ void k_stream(const uint4 *__restrict__ t, size_t n, unsigned *out) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = t[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// idx[i] = record index to read (one per lane)
__global__ void k_gather(const uint4 *__restrict__ t, const unsigned *__restrict__ idx, size_t n, unsigned *out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 v = t[idx[i]];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = 1;
}

// 4 consecutive records per lane from record idx[i]
__global__ void k_runs4(const uint4 *__restrict__ t, const unsigned *__restrict__ idx, size_t n, unsigned *out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned b = idx[i];
    unsigned acc = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = t[b + q];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = 1;
}

int main() {
    const size_t recs = (size_t)1 << 27;  // 2 GiB of 16-B records
    const size_t lines = recs / 8;        // 128-B lines
    const size_t R = (size_t)1 << 22;     // lines touched by the gathers
    uint4 *t;
    unsigned *idx, *out;
    CK(hipMalloc(&t, recs * sizeof(uint4)));
    CK(hipMemset(t, 1, recs * sizeof(uint4)));
    CK(hipMalloc(&idx, 2 * R * sizeof(unsigned)));
    CK(hipMalloc(&out, 4));
    std::mt19937_64 g(7);
    std::vector<unsigned> L(lines);
    for (size_t i = 0; i < lines; ++i) L[i] = (unsigned)i;
    std::shuffle(L.begin(), L.end(), g);
    std::vector<unsigned> h(2 * R);
    // gather1: record 0 of R random lines
    for (size_t i = 0; i < R; ++i) h[i] = L[i] * 8u;
    CK(hipMemcpy(idx, h.data(), R * 4, hipMemcpyHostToDevice));
    k_stream<<<4096, 256>>>(t, recs, out);
    CK(hipDeviceSynchronize());
    k_gather<<<(R + 255) / 256, 256>>>(t, idx, R, out);
    CK(hipDeviceSynchronize());
    // gather2: R other lines, first halves then (second half of the launch) second halves
    for (size_t i = 0; i < R; ++i) {
        h[i] = L[R + i] * 8u;
        h[R + i] = L[R + i] * 8u + 4u;
    }
    CK(hipMemcpy(idx, h.data(), 2 * R * 4, hipMemcpyHostToDevice));
    k_gather<<<(2 * R + 255) / 256, 256>>>(t, idx, 2 * R, out);
    CK(hipDeviceSynchronize());
    // runs4: 64-B half-lines of R further lines
    for (size_t i = 0; i < R; ++i) h[i] = L[2 * R + i] * 8u + (unsigned)(g() & 1u) * 4u;
    CK(hipMemcpy(idx, h.data(), R * 4, hipMemcpyHostToDevice));
    k_runs4<<<(R + 255) / 256, 256>>>(t, idx, R, out);
    CK(hipDeviceSynchronize());
    std::printf("{\"stream_bytes\": %zu, \"gather1_lines\": %zu, \"gather2_lines\": %zu, \"runs4_halflines\": %zu}\n",
                recs * sizeof(uint4), R, R, R);
    return 0;
}
