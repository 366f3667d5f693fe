/*
 * oracle/closed_form.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * Batch restatement of the XZ-list neighbour relation:
 * after any sequence of Enter/Moved/Leave calls on go-aoi's XZListAOIManager
 * (go.mod:29, external, absent here), live entities A and B of one space are
 * neighbours iff P_W(L) holds at their current positions, where W is the one
 * whose most recent Enter/Moved call came last (larger seq) and
 *   P_W(L) := L.x >= fl32(W.x-D) && L.x <= fl32(W.x+D)
 *          && L.z >= fl32(W.z-D) && L.z <= fl32(W.z+D).
 * This file evaluates that relation by brute-force bucketing on the CPU so
 * that tests can check (1) the sequential restatement (xzlist.c) against the
 * closed form and (2) the HIP path against both.
 *
 * PARITY UNPINNED (see xzlist.c header): no reference fixture exists.
 *
 * Inputs are per-entity arrays; sp[i] = space id, or 0xFFFFFFFF when entity i
 * is not live.  D is indexed by space id.  Output: every directed neighbour
 * pair as a uint64 key (a << 32 | b), sorted ascending.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define DEAD 0xFFFFFFFFu

static inline int pred(float wx, float wz, float lx, float lz, float D) {
    const float lox = wx - D, hix = wx + D, loz = wz - D, hiz = wz + D;
    return lx >= lox && lx <= hix && lz >= loz && lz <= hiz;
}

typedef struct {
    uint32_t sp;
    int64_t cx, cz;
    int32_t i;
} cell_ent;

static int cmp_cell(const void *pa, const void *pb) {
    const cell_ent *a = (const cell_ent *)pa, *b = (const cell_ent *)pb;
    if (a->sp != b->sp) return a->sp < b->sp ? -1 : 1;
    if (a->cx != b->cx) return a->cx < b->cx ? -1 : 1;
    if (a->cz != b->cz) return a->cz < b->cz ? -1 : 1;
    return a->i < b->i ? -1 : (a->i > b->i);
}

static int cmp_u64(const void *pa, const void *pb) {
    uint64_t a = *(const uint64_t *)pa, b = *(const uint64_t *)pb;
    return a < b ? -1 : (a > b);
}

/* first index in [0,n) whose (sp,cx,cz) >= key */
static int64_t lower(const cell_ent *e, int64_t n, uint32_t sp, int64_t cx, int64_t cz) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        const cell_ent *m = &e[mid];
        int less = m->sp != sp ? m->sp < sp : (m->cx != cx ? m->cx < cx : m->cz < cz);
        if (less) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* neighbour relation; returns number of pairs written to *out (malloc'd,
 * caller frees via cf_free); sorted ascending when `sort` is set */
int64_t cf_pairs_ex(int64_t n, const float *x, const float *z, const uint64_t *seq, const uint32_t *sp,
                    const float *D, uint64_t **out, int sort) {
    cell_ent *e = (cell_ent *)malloc(sizeof(cell_ent) * (n ? n : 1));
    int64_t m = 0;
    for (int64_t i = 0; i < n; i++) {
        if (sp[i] == DEAD) continue;
        double C = 2.0 * (double)D[sp[i]];
        e[m].sp = sp[i];
        e[m].cx = (int64_t)floor((double)x[i] / C);
        e[m].cz = (int64_t)floor((double)z[i] / C);
        e[m].i = (int32_t)i;
        m++;
    }
    qsort(e, m, sizeof(cell_ent), cmp_cell);
    size_t cap = 1024, len = 0;
    uint64_t *pairs = (uint64_t *)malloc(cap * sizeof(uint64_t));
    for (int64_t k = 0; k < m; k++) {
        int32_t a = e[k].i;
        float Dsp = D[e[k].sp];
        for (int dx = -1; dx <= 1; dx++)
            for (int dz = -1; dz <= 1; dz++) {
                int64_t j = lower(e, m, e[k].sp, e[k].cx + dx, e[k].cz + dz);
                for (; j < m && e[j].sp == e[k].sp && e[j].cx == e[k].cx + dx && e[j].cz == e[k].cz + dz; j++) {
                    int32_t b = e[j].i;
                    if (b == a) continue;
                    int nb = seq[a] > seq[b] ? pred(x[a], z[a], x[b], z[b], Dsp)
                                             : pred(x[b], z[b], x[a], z[a], Dsp);
                    if (!nb) continue;
                    if (len == cap) {
                        cap *= 2;
                        pairs = (uint64_t *)realloc(pairs, cap * sizeof(uint64_t));
                    }
                    pairs[len++] = ((uint64_t)(uint32_t)a << 32) | (uint32_t)b;
                }
            }
    }
    free(e);
    if (sort) qsort(pairs, len, sizeof(uint64_t), cmp_u64);
    *out = pairs;
    return (int64_t)len;
}

int64_t cf_pairs(int64_t n, const float *x, const float *z, const uint64_t *seq, const uint32_t *sp,
                 const float *D, uint64_t **out) {
    return cf_pairs_ex(n, x, z, seq, sp, D, out, 1);
}

void cf_free(void *p) { free(p); }

/* ---- tick diff of the relation (multithreaded) ------------------------------
 * cf_diff evaluates the relation at two states (t-1: x0,z0,s0,sp0 and t:
 * x1,z1,s1,sp1; sp = DEAD when not live) and returns the flush's net events
 * as the GPU path reports them (per-tick recipe): enter
 * = pairs related at t and not at t-1, leave = the converse, both directions,
 * as uint64 keys a << 32 | b sorted ascending.  Every space is its own
 * manager: an entity whose space changed leaves all its old pairs and enters
 * all its new ones, even with the same partner.  Entities are bucketed in
 * cells of C = D (1 + 2^-10) per space: a window [fl32(w-D), fl32(w+D)] is
 * narrower than 2C even after rounding, so it needs only the 3x3 cells around
 * its own. */

typedef struct {
    uint64_t key; /* space << 42 | (cx + 2^20) << 21 | (cz + 2^20) */
    int32_t i;
} gent;

typedef struct {
    gent *e;
    int64_t m;
} grid_t;

static inline uint64_t gkey(uint32_t sp, int64_t cx, int64_t cz) {
    return ((uint64_t)sp << 42) | ((uint64_t)((cx + (1 << 20)) & 0x1FFFFF) << 21) |
           (uint64_t)((cz + (1 << 20)) & 0x1FFFFF);
}

static inline int64_t cell_of2(float v, float D) {
    return (int64_t)floor((double)v / ((double)D * (1.0 + 0x1p-10)));
}

static int cmp_gent(const void *pa, const void *pb) {
    const gent *a = (const gent *)pa, *b = (const gent *)pb;
    if (a->key != b->key) return a->key < b->key ? -1 : 1;
    return a->i < b->i ? -1 : (a->i > b->i);
}

static grid_t grid_build(int64_t n, const float *x, const float *z, const uint32_t *sp, const float *D) {
    grid_t g;
    g.e = (gent *)malloc(sizeof(gent) * (n ? n : 1));
    g.m = 0;
    for (int64_t i = 0; i < n; i++) {
        if (sp[i] == DEAD) continue;
        const float d = D[sp[i]];
        g.e[g.m].key = gkey(sp[i], cell_of2(x[i], d), cell_of2(z[i], d));
        g.e[g.m].i = (int32_t)i;
        g.m++;
    }
    qsort(g.e, g.m, sizeof(gent), cmp_gent);
    return g;
}

static int64_t glower(const grid_t *g, uint64_t key) {
    int64_t lo = 0, hi = g->m;
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (g->e[mid].key < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

typedef struct {
    uint32_t *v;
    int64_t n, cap;
} vec32;

static void v32_push(vec32 *v, uint32_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 256;
        v->v = (uint32_t *)realloc(v->v, (size_t)v->cap * sizeof(uint32_t));
    }
    v->v[v->n++] = x;
}

typedef struct {
    uint64_t *v;
    int64_t n, cap;
} vec64;

static void v64_push(vec64 *v, uint64_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 1024;
        v->v = (uint64_t *)realloc(v->v, (size_t)v->cap * sizeof(uint64_t));
    }
    v->v[v->n++] = x;
}

static int cmp_u32(const void *pa, const void *pb) {
    uint32_t a = *(const uint32_t *)pa, b = *(const uint32_t *)pb;
    return a < b ? -1 : (a > b);
}

/* sorted neighbours of a at one state into out (cleared first) */
static void row_of(const grid_t *g, int32_t a, const float *x, const float *z, const uint64_t *seq,
                   const uint32_t *sp, const float *D, vec32 *out) {
    out->n = 0;
    if (sp[a] == DEAD) return;
    const float d = D[sp[a]];
    const int64_t cx = cell_of2(x[a], d), cz = cell_of2(z[a], d);
    for (int dx = -1; dx <= 1; dx++) {  /* cells (cx+dx, cz-1..cz+1) are consecutive keys */
        const uint64_t k0 = gkey(sp[a], cx + dx, cz - 1), k1 = gkey(sp[a], cx + dx, cz + 1);
        for (int64_t j = glower(g, k0); j < g->m && g->e[j].key <= k1; j++) {
                const int32_t b = g->e[j].i;
                if (b == a) continue;
                const int nb = seq[a] > seq[b] ? pred(x[a], z[a], x[b], z[b], d) : pred(x[b], z[b], x[a], z[a], d);
                if (nb) v32_push(out, (uint32_t)b);
            }
        }
    if (out->n > 1) qsort(out->v, out->n, sizeof(uint32_t), cmp_u32);
}

int cf_diff(int64_t n, const float *x0, const float *z0, const uint64_t *s0, const uint32_t *sp0, const float *x1,
            const float *z1, const uint64_t *s1, const uint32_t *sp1, const float *D, uint64_t **enter,
            int64_t *n_enter, uint64_t **leave, int64_t *n_leave, int threads) {
    grid_t g0 = grid_build(n, x0, z0, sp0, D), g1 = grid_build(n, x1, z1, sp1, D);
    if (threads < 1) threads = 1;
    const int64_t chunks = (int64_t)threads * 16;
    vec64 *ce = (vec64 *)calloc((size_t)chunks, sizeof(vec64)), *cl = (vec64 *)calloc((size_t)chunks, sizeof(vec64));
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
    for (int64_t c = 0; c < chunks; c++) {
        vec32 r0 = {0, 0, 0}, r1 = {0, 0, 0};
        const int64_t a0 = n * c / chunks, a1 = n * (c + 1) / chunks;
        for (int64_t a = a0; a < a1; a++) {
            row_of(&g0, (int32_t)a, x0, z0, s0, sp0, D, &r0);
            row_of(&g1, (int32_t)a, x1, z1, s1, sp1, D, &r1);
            const uint64_t hi = (uint64_t)a << 32;
            if (sp0[a] != sp1[a]) {  /* another manager: every old pair leaves, every new one enters */
                for (int64_t k = 0; k < r1.n; k++) v64_push(&ce[c], hi | r1.v[k]);
                for (int64_t k = 0; k < r0.n; k++) v64_push(&cl[c], hi | r0.v[k]);
                continue;
            }
            int64_t i = 0, j = 0;
            while (i < r0.n || j < r1.n) {
                if (j == r1.n || (i < r0.n && r0.v[i] < r1.v[j])) v64_push(&cl[c], hi | r0.v[i++]);
                else if (i == r0.n || r1.v[j] < r0.v[i]) v64_push(&ce[c], hi | r1.v[j++]);
                else { i++; j++; }
            }
        }
        free(r0.v);
        free(r1.v);
    }
    int64_t ne = 0, nl = 0;
    for (int64_t c = 0; c < chunks; c++) {
        ne += ce[c].n;
        nl += cl[c].n;
    }
    uint64_t *E = (uint64_t *)malloc(sizeof(uint64_t) * (ne ? ne : 1));
    uint64_t *L = (uint64_t *)malloc(sizeof(uint64_t) * (nl ? nl : 1));
    ne = nl = 0;
    for (int64_t c = 0; c < chunks; c++) {
        if (ce[c].n) memcpy(E + ne, ce[c].v, (size_t)ce[c].n * sizeof(uint64_t));
        if (cl[c].n) memcpy(L + nl, cl[c].v, (size_t)cl[c].n * sizeof(uint64_t));
        ne += ce[c].n;
        nl += cl[c].n;
        free(ce[c].v);
        free(cl[c].v);
    }
    free(ce);
    free(cl);
    free(g0.e);
    free(g1.e);
    *enter = E;
    *leave = L;
    *n_enter = ne;
    *n_leave = nl;
    return 0;
}

/* Sorted neighbour rows of the entities q[0..nq) at one state: row k is
 * out[off[k] .. off[k+1]); off has nq + 1 entries. */
int64_t cf_rows(int64_t n, const float *x, const float *z, const uint64_t *seq, const uint32_t *sp, const float *D,
                int64_t nq, const int32_t *q, int64_t *off, uint32_t **out) {
    grid_t g = grid_build(n, x, z, sp, D);
    vec32 r = {0, 0, 0}, all = {0, 0, 0};
    off[0] = 0;
    for (int64_t k = 0; k < nq; k++) {
        row_of(&g, q[k], x, z, seq, sp, D, &r);
        for (int64_t j = 0; j < r.n; j++) v32_push(&all, r.v[j]);
        off[k + 1] = all.n;
    }
    free(r.v);
    free(g.e);
    *out = all.v;
    return all.n;
}

/* the single-pair predicate, exported for known-answer tests */
int cf_pred(float wx, float wz, float lx, float lz, float D) { return pred(wx, wz, lx, lz, D); }
