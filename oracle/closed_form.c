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

/* the single-pair predicate, exported for known-answer tests */
int cf_pred(float wx, float wz, float lx, float lz, float D) { return pred(wx, wz, lx, lz, D); }
