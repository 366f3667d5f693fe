// gwaoi_wire.hip -- the position-sync wire path between gate, dispatcher and
// game, regrouped on the GPU (include/gwaoi_wire.h).
//
// Each regroup is a stable partition of fixed-size records by a 32-bit
// destination key:
//   k_wire_keys    one lane per record: key = dispatcher id (two id bytes,
//                  hash.go:7-12), or a 16-B id looked up in a hash table
//                  (entity -> game, client -> proxy index); unknown -> the
//                  drop key, which sorts after every destination
//   radix sort     the world's stable LSD sort of (key, record index)
//   k_wire_heads   group starts of the sorted keys; a scan numbers them
//   k_wire_groups  (key, first record) of every group
//   k_wire_gather  the records in group order (two 16-B words per lane)
// The work is byte movement (HBM bound): 32 or 48 B in, 32 B out per record.
// The id tables live on the host (open addressing, 16-B keys) and reach the
// device as changed 32-B buckets {key; value} before the next regroup.

#include "gwaoi_internal.h"
#include "../../include/gwaoi_wire.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

namespace {

constexpr int WT = 256;
constexpr uint32_t H_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t H_TOMB = 0xFFFFFFFEu;
constexpr uint32_t ID_BYTES = 16, SYNC_BYTES = 16;
constexpr uint32_t REC32 = ID_BYTES + SYNC_BYTES;             // EntityID | x, y, z, yaw
constexpr uint32_t REC48 = ID_BYTES + ID_BYTES + SYNC_BYTES;  // ClientID | EntityID | x, y, z, yaw

inline uint32_t cdivu(size_t a, size_t b) { return (uint32_t)((a + b - 1) / b); }

__host__ __device__ inline uint32_t wid_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    unsigned long long h = (((unsigned long long)b << 32) | a) * 0x9E3779B97F4A7C15ull;
    h ^= (((unsigned long long)d << 32) | c) + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    return (uint32_t)h;
}

__device__ __forceinline__ uint32_t wlookup(const uint4 *__restrict__ tab, uint32_t mask, uint4 id, uint32_t miss) {
    uint32_t h = wid_hash(id.x, id.y, id.z, id.w) & mask;
    for (uint32_t p = 0; p <= mask; ++p, h = (h + 1) & mask) {
        const uint4 k = tab[2 * (size_t)h];  // one 32-B bucket: key, then value
        const uint32_t v = tab[2 * (size_t)h + 1].x;
        if (v == H_EMPTY) return miss;
        if (v != H_TOMB && k.x == id.x && k.y == id.y && k.z == id.z && k.w == id.w) return v;
    }
    return miss;
}

__global__ void k_wire_put(const uint4 *__restrict__ src, const uint32_t *__restrict__ idx, uint32_t n, uint4 *tab) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    tab[2 * (size_t)idx[i]] = src[2 * (size_t)i];
    tab[2 * (size_t)idx[i] + 1] = src[2 * (size_t)i + 1];
}

enum KeyMode { KM_DISPATCHER = 0, KM_TABLE = 1 };

// key of record i: its id at byte id_off of the record (16-B aligned)
__global__ __launch_bounds__(WT) void k_wire_keys(const uint4 *__restrict__ rec, uint32_t n, uint32_t words,
                                                  uint32_t id_word, int mode, uint32_t n_disp,
                                                  const uint4 *__restrict__ tab, uint32_t mask, uint32_t drop,
                                                  uint32_t *keys, uint32_t *vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 id = rec[(size_t)i * words + id_word];
    uint32_t key;
    if (mode == KM_DISPATCHER) {
        // id[14] * 256 + id[15]: the last two bytes of the id (little-endian word w)
        const uint32_t h = ((id.w >> 16) & 0xFFu) * 256u + (id.w >> 24);
        key = h % n_disp + 1u;
    } else {
        key = wlookup(tab, mask, id, drop);
    }
    keys[i] = key;
    vals[i] = i;
}

// head[j] = 1 where a kept group starts; *n_keep = index of the first dropped record
__global__ __launch_bounds__(WT) void k_wire_heads(const uint32_t *__restrict__ sk, uint32_t n, uint32_t drop,
                                                   uint32_t *head, uint32_t *n_keep) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > n) return;
    if (j == n) {
        head[n] = 0u;
        if (n == 0 || sk[n - 1] != drop) *n_keep = n;
        return;
    }
    const uint32_t k = sk[j];
    const bool first = j == 0 || sk[j - 1] != k;
    head[j] = (first && k != drop) ? 1u : 0u;
    if (first && k == drop) *n_keep = j;
}

__global__ __launch_bounds__(WT) void k_wire_groups(const uint32_t *__restrict__ sk, const uint32_t *__restrict__ pos,
                                                    uint32_t n, uint32_t *gkey, uint32_t *gstart) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n || pos[j + 1] == pos[j]) return;
    gkey[pos[j]] = sk[j];
    gstart[pos[j]] = j;
}

// out record j (2 words) = words [src_word, src_word + 2) of input record perm[j]
__global__ __launch_bounds__(WT) void k_wire_gather(const uint4 *__restrict__ rec, uint32_t words, uint32_t src_word,
                                                    const uint32_t *__restrict__ perm, uint32_t n_keep, uint4 *out) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;  // one 16-B word of the output per lane
    if (e >= 2 * n_keep) return;
    const uint32_t j = e >> 1;
    out[e] = rec[(size_t)perm[j] * words + src_word + (e & 1u)];
}

int bitlen(uint32_t v) {
    int b = 0;
    while (v) {
        ++b;
        v >>= 1;
    }
    return b;
}

// Host side of one id table: 16-B id -> u32, linear probing, tombstones; the
// device copy is updated bucket by bucket.
struct IdTable {
    uint32_t cap = 0, used = 0, live = 0;
    std::vector<uint4> key;
    std::vector<uint32_t> val;
    std::vector<uint32_t> dirty;
    uint4 *d = nullptr;
    uint32_t max_val = 0;  // largest value ever set (the key range of the regroup)

    uint32_t find(const uint4 &id) const {
        const uint32_t mask = cap - 1;
        uint32_t h = wid_hash(id.x, id.y, id.z, id.w) & mask;
        for (uint32_t p = 0; p < cap; ++p, h = (h + 1) & mask) {
            if (val[h] == H_EMPTY) return H_EMPTY;
            if (val[h] != H_TOMB && !std::memcmp(&key[h], &id, 16)) return h;
        }
        return H_EMPTY;
    }
};

}  // namespace

struct gwaoi_wire {
    int device = 0;
    hipStream_t st = nullptr;
    std::string err;
    IdTable games, clients;
    // scratch
    uint32_t *keys[2] = {nullptr, nullptr}, *vals[2] = {nullptr, nullptr};
    uint32_t *hist = nullptr, *scan_tmp = nullptr, *head = nullptr, *gkey = nullptr, *gstart = nullptr;
    uint32_t *small = nullptr;  // [0] n_keep
    size_t n_cap = 0, hist_cap = 0, scan_cap = 0;
    uint4 *d_in = nullptr, *d_out = nullptr;
    size_t in_cap = 0, out_cap = 0;  // bytes
    uint8_t *h_in = nullptr, *h_out = nullptr;
    size_t h_in_cap = 0, h_out_cap = 0;
    uint4 *d_put = nullptr;
    uint32_t *d_put_idx = nullptr;
    size_t put_cap = 0;
    std::vector<uint4> h_put;
    std::vector<uint32_t> h_put_idx;
    // last output
    std::vector<uint32_t> o_keys, o_start;
    std::vector<uint64_t> o_off;
};

namespace {

#define W_TRY(expr)                                                                      \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            w->err = std::string(#expr) + ": " + hipGetErrorString(e_);                  \
            return GWAOI_EDEVICE;                                                        \
        }                                                                                \
    } while (0)

template <class T>
int walloc(gwaoi_wire *w, T **p, size_t n) {
    *p = nullptr;
    if (hipMalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
        *p = nullptr;
        w->err = "hipMalloc failed";
        return GWAOI_ENOMEM;
    }
    return GWAOI_OK;
}
template <class T>
void wfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}
void hfree(uint8_t *&p) {
    if (p) (void)hipHostFree(p);
    p = nullptr;
}

int table_init(gwaoi_wire *w, IdTable &t, uint32_t cap) {
    wfree(t.d);
    t.cap = cap;
    t.used = t.live = 0;
    t.key.assign(cap, make_uint4(0, 0, 0, 0));
    t.val.assign(cap, H_EMPTY);
    t.dirty.clear();
    if (int rc = walloc(w, &t.d, 2 * (size_t)cap)) return rc;
    W_TRY(hipMemsetAsync(t.d, 0xFF, (size_t)cap * 32, w->st));  // every value H_EMPTY
    return GWAOI_OK;
}

// Rebuild at twice the size when live + tombstones pass 3/4 (the whole table goes up).
int table_grow(gwaoi_wire *w, IdTable &t) {
    std::vector<uint4> k;
    std::vector<uint32_t> v;
    for (uint32_t h = 0; h < t.cap; ++h)
        if (t.val[h] != H_EMPTY && t.val[h] != H_TOMB) {
            k.push_back(t.key[h]);
            v.push_back(t.val[h]);
        }
    uint32_t cap = t.cap;
    while ((size_t)k.size() * 2 >= cap) cap *= 2;
    if (cap == t.cap && t.used - t.live < t.cap / 4) cap *= 2;
    const uint32_t mv = t.max_val;
    if (int rc = table_init(w, t, cap)) return rc;
    t.max_val = mv;
    const uint32_t mask = cap - 1;
    for (size_t i = 0; i < k.size(); ++i) {
        uint32_t h = wid_hash(k[i].x, k[i].y, k[i].z, k[i].w) & mask;
        while (t.val[h] != H_EMPTY) h = (h + 1) & mask;
        t.key[h] = k[i];
        t.val[h] = v[i];
        t.used++;
        t.live++;
    }
    std::vector<uint4> buf(2 * (size_t)cap);
    for (uint32_t h = 0; h < cap; ++h) {
        buf[2 * (size_t)h] = t.key[h];
        buf[2 * (size_t)h + 1] = make_uint4(t.val[h], 0, 0, 0);
    }
    W_TRY(hipMemcpyAsync(t.d, buf.data(), buf.size() * 16, hipMemcpyHostToDevice, w->st));
    W_TRY(hipStreamSynchronize(w->st));  // buf is pageable
    t.dirty.clear();
    return GWAOI_OK;
}

int table_set(gwaoi_wire *w, IdTable &t, const uint8_t *ids, const uint32_t *vals, size_t n, bool remove) {
    if (n && !ids) return GWAOI_EINVAL;
    if (!remove && n && !vals) return GWAOI_EINVAL;
    if (!remove)  // validate the whole batch before touching the table: a rejected call changes nothing
        for (size_t i = 0; i < n; ++i)
            if (vals[i] >= H_TOMB) return GWAOI_EINVAL;
    for (size_t i = 0; i < n; ++i) {
        uint4 id;
        std::memcpy(&id, ids + 16 * i, 16);
        const uint32_t at = t.find(id);
        if (remove) {
            if (at == H_EMPTY) continue;
            t.val[at] = H_TOMB;
            t.live--;
            t.dirty.push_back(at);
            continue;
        }
        if (at != H_EMPTY) {
            t.val[at] = vals[i];
            t.dirty.push_back(at);
        } else {
            if ((size_t)t.used + 1 > (size_t)t.cap / 4 * 3)
                if (int rc = table_grow(w, t)) return rc;
            const uint32_t mask = t.cap - 1;
            uint32_t h = wid_hash(id.x, id.y, id.z, id.w) & mask;
            while (t.val[h] != H_EMPTY && t.val[h] != H_TOMB) h = (h + 1) & mask;
            if (t.val[h] == H_EMPTY) t.used++;
            t.live++;
            t.key[h] = id;
            t.val[h] = vals[i];
            t.dirty.push_back(h);
        }
        t.max_val = std::max(t.max_val, vals[i]);
    }
    return GWAOI_OK;
}

// Upload the changed buckets (last state of each) before a regroup reads the table.
int table_push(gwaoi_wire *w, IdTable &t) {
    if (t.dirty.empty()) return GWAOI_OK;
    std::sort(t.dirty.begin(), t.dirty.end());
    t.dirty.erase(std::unique(t.dirty.begin(), t.dirty.end()), t.dirty.end());
    const size_t n = t.dirty.size();
    if (n > w->put_cap) {
        wfree(w->d_put);
        wfree(w->d_put_idx);
        w->put_cap = 0;
        const size_t c = std::max<size_t>(n + n / 2, 1024);
        if (int rc = walloc(w, &w->d_put, 2 * c)) return rc;
        if (int rc = walloc(w, &w->d_put_idx, c)) return rc;
        w->put_cap = c;
    }
    w->h_put.resize(2 * n);
    w->h_put_idx.assign(t.dirty.begin(), t.dirty.end());
    for (size_t i = 0; i < n; ++i) {
        w->h_put[2 * i] = t.key[t.dirty[i]];
        w->h_put[2 * i + 1] = make_uint4(t.val[t.dirty[i]], 0, 0, 0);
    }
    W_TRY(hipMemcpyAsync(w->d_put, w->h_put.data(), 2 * n * 16, hipMemcpyHostToDevice, w->st));
    W_TRY(hipMemcpyAsync(w->d_put_idx, w->h_put_idx.data(), n * 4, hipMemcpyHostToDevice, w->st));
    k_wire_put<<<cdivu(n, WT), WT, 0, w->st>>>(w->d_put, w->d_put_idx, (uint32_t)n, t.d);
    W_TRY(hipGetLastError());
    W_TRY(hipStreamSynchronize(w->st));  // the pageable staging vectors are reused
    t.dirty.clear();
    return GWAOI_OK;
}

int ensure_n(gwaoi_wire *w, size_t n) {
    const size_t hist = gw::radix_hist_elems((uint32_t)std::max<size_t>(n, 1));
    const size_t scan = std::max(gw::scan_tmp_elems(n + 1), gw::scan_tmp_elems(hist)) + 4;
    if (n + 1 > w->n_cap) {
        for (int b = 0; b < 2; ++b) {
            wfree(w->keys[b]);
            wfree(w->vals[b]);
        }
        wfree(w->head);
        wfree(w->gkey);
        wfree(w->gstart);
        w->n_cap = 0;
        const size_t c = std::max<size_t>(n + 1 + n / 4, 4096);
        for (int b = 0; b < 2; ++b) {
            if (int rc = walloc(w, &w->keys[b], c)) return rc;
            if (int rc = walloc(w, &w->vals[b], c)) return rc;
        }
        if (int rc = walloc(w, &w->head, c)) return rc;
        if (int rc = walloc(w, &w->gkey, c)) return rc;
        if (int rc = walloc(w, &w->gstart, c)) return rc;
        w->n_cap = c;
    }
    if (hist > w->hist_cap) {
        wfree(w->hist);
        w->hist_cap = 0;
        if (int rc = walloc(w, &w->hist, hist)) return rc;
        w->hist_cap = hist;
    }
    if (scan > w->scan_cap) {
        wfree(w->scan_tmp);
        w->scan_cap = 0;
        if (int rc = walloc(w, &w->scan_tmp, scan)) return rc;
        w->scan_cap = scan;
    }
    return GWAOI_OK;
}

int ensure_dev(gwaoi_wire *w, uint4 **p, size_t *cap, size_t bytes) {
    if (bytes <= *cap) return GWAOI_OK;
    wfree(*p);
    *cap = 0;
    const size_t c = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    if (int rc = walloc(w, (uint8_t **)p, c)) return rc;
    *cap = c;
    return GWAOI_OK;
}

int ensure_pinned(gwaoi_wire *w, uint8_t **p, size_t *cap, size_t bytes) {
    if (bytes <= *cap) return GWAOI_OK;
    hfree(*p);
    *cap = 0;
    const size_t c = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    W_TRY(hipHostMalloc((void **)p, c, hipHostMallocDefault));
    *cap = c;
    return GWAOI_OK;
}

// One regroup: records of rec_bytes (32 or 48) keyed at id_word, 32-B output
// words [src_word, src_word + 2).
int regroup(gwaoi_wire *w, const uint8_t *records, size_t n, bool on_device, uint32_t rec_bytes, uint32_t id_word,
            uint32_t src_word, int mode, uint32_t n_disp, IdTable *tab, gwaoi_wire_groups *out) {
    if (!w || !out || (n && !records)) return GWAOI_EINVAL;
    if (n > 0x7FFFFFF0ull) return GWAOI_EINVAL;
    if (on_device && (reinterpret_cast<uintptr_t>(records) & 15u)) return GWAOI_EINVAL;
    W_TRY(hipSetDevice(w->device));
    *out = gwaoi_wire_groups{};
    out->rec_bytes = REC32;
    uint32_t max_key;
    if (mode == KM_DISPATCHER) {
        if (n_disp == 0 || n_disp > 0xFFFFu) return GWAOI_EINVAL;
        max_key = n_disp;
    } else {
        if (int rc = table_push(w, *tab)) return rc;
        max_key = tab->max_val;
    }
    const int bits = std::max(1, bitlen(max_key + 1u));
    const uint32_t drop = bits >= 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;  // > every key
    if (int rc = ensure_n(w, n)) return rc;
    if (int rc = ensure_dev(w, &w->d_out, &w->out_cap, std::max<size_t>(n, 1) * REC32)) return rc;
    const uint4 *d_rec = reinterpret_cast<const uint4 *>(records);
    if (!on_device && n) {
        if (int rc = ensure_pinned(w, &w->h_in, &w->h_in_cap, n * rec_bytes)) return rc;
        if (int rc = ensure_dev(w, &w->d_in, &w->in_cap, n * rec_bytes)) return rc;
        std::memcpy(w->h_in, records, n * rec_bytes);
        W_TRY(hipMemcpyAsync(w->d_in, w->h_in, n * rec_bytes, hipMemcpyHostToDevice, w->st));
        d_rec = w->d_in;
    }
    const uint32_t words = rec_bytes / 16;
    uint32_t n_keep = 0, n_groups = 0;
    const uint32_t *sk = w->keys[0], *perm = w->vals[0];
    if (n) {
        k_wire_keys<<<cdivu(n, WT), WT, 0, w->st>>>(d_rec, (uint32_t)n, words, id_word, mode, n_disp,
                                                     tab ? tab->d : nullptr, tab ? tab->cap - 1 : 0u, drop,
                                                     w->keys[0], w->vals[0]);
        gw::SortBuffers sb;
        sb.keys[0] = w->keys[0];
        sb.keys[1] = w->keys[1];
        sb.vals[0] = w->vals[0];
        sb.vals[1] = w->vals[1];
        sb.hist = w->hist;
        sb.scan_tmp = w->scan_tmp;
        const int which = gw::radix_sort(sb, (uint32_t)n, bits, w->st);
        sk = w->keys[which];
        perm = w->vals[which];
        k_wire_heads<<<cdivu(n + 1, WT), WT, 0, w->st>>>(sk, (uint32_t)n, drop, w->head, w->small);
        gw::scan_exclusive(w->head, w->head, n + 1, w->scan_tmp, w->st);
        k_wire_groups<<<cdivu(n, WT), WT, 0, w->st>>>(sk, w->head, (uint32_t)n, w->gkey, w->gstart);
        W_TRY(hipGetLastError());
        uint32_t sm[2];
        W_TRY(hipMemcpyAsync(&sm[0], w->small, 4, hipMemcpyDeviceToHost, w->st));
        W_TRY(hipMemcpyAsync(&sm[1], w->head + n, 4, hipMemcpyDeviceToHost, w->st));
        W_TRY(hipStreamSynchronize(w->st));
        n_keep = sm[0];
        n_groups = sm[1];
        if (n_keep)
            k_wire_gather<<<cdivu(2 * (size_t)n_keep, WT), WT, 0, w->st>>>(d_rec, words, src_word, perm, n_keep,
                                                                         w->d_out);
        W_TRY(hipGetLastError());
    }
    w->o_keys.resize(n_groups);
    w->o_start.resize(n_groups);
    if (n_groups) {
        W_TRY(hipMemcpyAsync(w->o_keys.data(), w->gkey, n_groups * 4, hipMemcpyDeviceToHost, w->st));
        W_TRY(hipMemcpyAsync(w->o_start.data(), w->gstart, n_groups * 4, hipMemcpyDeviceToHost, w->st));
    }
    const uint8_t *recs_out = reinterpret_cast<const uint8_t *>(w->d_out);
    if (!on_device) {
        if (int rc = ensure_pinned(w, &w->h_out, &w->h_out_cap, std::max<size_t>(n_keep, 1) * REC32)) return rc;
        if (n_keep)
            W_TRY(hipMemcpyAsync(w->h_out, w->d_out, (size_t)n_keep * REC32, hipMemcpyDeviceToHost, w->st));
        recs_out = w->h_out;
    }
    W_TRY(hipStreamSynchronize(w->st));
    w->o_off.resize((size_t)n_groups + 1);
    for (uint32_t g = 0; g < n_groups; ++g) w->o_off[g] = w->o_start[g];
    w->o_off[n_groups] = n_keep;
    out->n_groups = n_groups;
    out->keys = w->o_keys.data();
    out->offsets = w->o_off.data();
    out->records = recs_out;
    out->n_dropped = n - n_keep;
    return GWAOI_OK;
}

}  // namespace

extern "C" {

int gwaoi_wire_create(int device, gwaoi_wire **out) {
    return gw::api_guard([&]() -> int {
        if (!out) return GWAOI_EINVAL;
        *out = nullptr;
        if (hipSetDevice(device) != hipSuccess) return GWAOI_EDEVICE;
        gwaoi_wire *w = new gwaoi_wire();
        w->device = device;
        if (hipStreamCreateWithFlags(&w->st, hipStreamNonBlocking) != hipSuccess) {
            delete w;
            return GWAOI_EDEVICE;
        }
        int rc;
        if ((rc = walloc(w, &w->small, 4)) || (rc = table_init(w, w->games, 1024)) ||
            (rc = table_init(w, w->clients, 1024))) {
            gwaoi_wire_destroy(w);
            return rc;
        }
        *out = w;
        return GWAOI_OK;
    });
}

void gwaoi_wire_destroy(gwaoi_wire *w) {
    if (!w) return;
    (void)hipSetDevice(w->device);
    if (w->st) (void)hipStreamSynchronize(w->st);
    for (int b = 0; b < 2; ++b) {
        wfree(w->keys[b]);
        wfree(w->vals[b]);
    }
    wfree(w->hist); wfree(w->scan_tmp); wfree(w->head); wfree(w->gkey); wfree(w->gstart); wfree(w->small);
    wfree(w->d_in); wfree(w->d_out); wfree(w->d_put); wfree(w->d_put_idx);
    wfree(w->games.d); wfree(w->clients.d);
    hfree(w->h_in);
    hfree(w->h_out);
    if (w->st) (void)hipStreamDestroy(w->st);
    delete w;
}

const char *gwaoi_wire_last_error(gwaoi_wire *w) { return w ? w->err.c_str() : "null wire handle"; }

int gwaoi_wire_set_entity_games(gwaoi_wire *w, const uint8_t *entity_ids, const uint16_t *game_ids, size_t n) {
    return gw::api_guard([&]() -> int {
        if (!w || (n && !game_ids)) return GWAOI_EINVAL;
        W_TRY(hipSetDevice(w->device));
        std::vector<uint32_t> v(game_ids, game_ids + n);
        return table_set(w, w->games, entity_ids, v.data(), n, false);
    });
}

int gwaoi_wire_remove_entities(gwaoi_wire *w, const uint8_t *entity_ids, size_t n) {
    return gw::api_guard([&]() -> int {
        if (!w) return GWAOI_EINVAL;
        W_TRY(hipSetDevice(w->device));
        return table_set(w, w->games, entity_ids, nullptr, n, true);
    });
}

int gwaoi_wire_set_clients(gwaoi_wire *w, const uint8_t *client_ids, const uint32_t *client_index, size_t n) {
    return gw::api_guard([&]() -> int {
        if (!w) return GWAOI_EINVAL;
        W_TRY(hipSetDevice(w->device));
        return table_set(w, w->clients, client_ids, client_index, n, false);
    });
}

int gwaoi_wire_remove_clients(gwaoi_wire *w, const uint8_t *client_ids, size_t n) {
    return gw::api_guard([&]() -> int {
        if (!w) return GWAOI_EINVAL;
        W_TRY(hipSetDevice(w->device));
        return table_set(w, w->clients, client_ids, nullptr, n, true);
    });
}

int gwaoi_wire_gate_from_clients(gwaoi_wire *w, const uint8_t *records, size_t n, uint32_t n_dispatchers,
                                 gwaoi_wire_groups *out) {
    return gw::api_guard([&]() -> int {
        return regroup(w, records, n, false, REC32, 0, 0, KM_DISPATCHER, n_dispatchers, nullptr, out);
    });
}

int gwaoi_wire_gate_from_clients_device(gwaoi_wire *w, const uint8_t *d_records, size_t n, uint32_t n_dispatchers,
                                        gwaoi_wire_groups *out) {
    return gw::api_guard([&]() -> int {
        return regroup(w, d_records, n, true, REC32, 0, 0, KM_DISPATCHER, n_dispatchers, nullptr, out);
    });
}

int gwaoi_wire_dispatcher_to_games(gwaoi_wire *w, const uint8_t *records, size_t n, gwaoi_wire_groups *out) {
    return gw::api_guard([&]() -> int {
        if (!w) return GWAOI_EINVAL;
        return regroup(w, records, n, false, REC32, 0, 0, KM_TABLE, 0, &w->games, out);
    });
}

int gwaoi_wire_dispatcher_to_games_device(gwaoi_wire *w, const uint8_t *d_records, size_t n,
                                          gwaoi_wire_groups *out) {
    return gw::api_guard([&]() -> int {
        if (!w) return GWAOI_EINVAL;
        return regroup(w, d_records, n, true, REC32, 0, 0, KM_TABLE, 0, &w->games, out);
    });
}

int gwaoi_wire_gate_to_clients(gwaoi_wire *w, const uint8_t *records, size_t n, gwaoi_wire_groups *out) {
    return gw::api_guard([&]() -> int {
        if (!w) return GWAOI_EINVAL;
        return regroup(w, records, n, false, REC48, 0, 1, KM_TABLE, 0, &w->clients, out);
    });
}

int gwaoi_wire_gate_to_clients_device(gwaoi_wire *w, const uint8_t *d_records, size_t n, gwaoi_wire_groups *out) {
    return gw::api_guard([&]() -> int {
        if (!w) return GWAOI_EINVAL;
        return regroup(w, d_records, n, true, REC48, 0, 1, KM_TABLE, 0, &w->clients, out);
    });
}

}  // extern "C"
