/*
 * oracle/cpu_grid.c -- CPU BASELINE ONLY (bench.py's cpu_baseline leg; also
 * checked by tests/test_oracle.py).  Never a product path.
 *
 * "CPU-grid" of BASELINE.md: a multithreaded CPU implementation of the same
 * tick the GPU path computes, as a stronger comparator than the sequential
 * XZ-list restatement.  One space.  Per tick:
 *   1. apply the Moved batch in call order (position + seq = call index);
 *   2. counting-sort the entities into cells of C = D (1 + 2^-10): every
 *      window [fl32(w-D), fl32(w+D)] lies in the 3x3 cells around its own;
 *   3. per entity A (OpenMP, dynamic chunks): its neighbour row -- every B in
 *      the 3x3 cells with go-aoi's relation P_W(L), W the later mover (SURVEY.md
 *      Appendix B) -- diffed against A's row of the previous tick with a
 *      per-thread mark array: enters = new \ old, leaves = old \ new
 *      (directed; both directions come from the two rows);
 *   4. the new rows replace the old ones (chunk-local storage).
 * The same relation the GPU reports, evaluated from scratch every tick on all
 * host cores; the counts are checked against the closed form in the tests.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline int pred(float wx, float wz, float lx, float lz, float D) {
    const float lox = wx - D, hix = wx + D, loz = wz - D, hiz = wz + D;
    return lx >= lox && lx <= hix && lz >= loz && lz <= hiz;
}

typedef struct {
    uint32_t *v;
    int64_t n, cap;
} buf32;

static void b_push(buf32 *b, uint32_t x) {
    if (b->n == b->cap) {
        b->cap = b->cap ? 2 * b->cap : 4096;
        b->v = (uint32_t *)realloc(b->v, (size_t)b->cap * sizeof(uint32_t));
    }
    b->v[b->n++] = x;
}

typedef struct {
    int64_t n;
    float D;
    int threads;
    int64_t nchunk;
    float *x, *z;
    uint64_t *seq;
    uint64_t next_seq;
    /* rows of the previous tick: row a = rows[chk[a]].v + off[a], len[a] */
    buf32 *rows, *rows_new;
    int64_t *off, *off_new;
    uint32_t *len, *len_new, *chk, *chk_new;
    float *xs, *zs;   /* positions and seqs in cell order (the candidate scans read these) */
    uint64_t *ss;
    /* grid */
    uint32_t *cell_start, *cell_idx, *ent_cell;
    uint8_t *marks; /* per thread, n bytes, all zero between entities */
    int64_t cells_cap;
    buf32 *ev_e, *ev_l; /* per chunk: events of the last tick (a << 32 | b as two words) */
} cgrid;

void *cg_new(int64_t n, float D, int threads) {
    cgrid *g = (cgrid *)calloc(1, sizeof(cgrid));
    g->n = n;
    g->D = D;
    g->threads = threads > 0 ? threads : 1;
    g->nchunk = (int64_t)g->threads * 32;
    g->x = (float *)malloc(sizeof(float) * n);
    g->z = (float *)malloc(sizeof(float) * n);
    g->seq = (uint64_t *)malloc(sizeof(uint64_t) * n);
    g->rows = (buf32 *)calloc((size_t)g->nchunk, sizeof(buf32));
    g->rows_new = (buf32 *)calloc((size_t)g->nchunk, sizeof(buf32));
    g->ev_e = (buf32 *)calloc((size_t)g->nchunk, sizeof(buf32));
    g->ev_l = (buf32 *)calloc((size_t)g->nchunk, sizeof(buf32));
    g->off = (int64_t *)calloc((size_t)n, sizeof(int64_t));
    g->off_new = (int64_t *)calloc((size_t)n, sizeof(int64_t));
    g->len = (uint32_t *)calloc((size_t)n, sizeof(uint32_t));
    g->len_new = (uint32_t *)calloc((size_t)n, sizeof(uint32_t));
    g->chk = (uint32_t *)calloc((size_t)n, sizeof(uint32_t));
    g->chk_new = (uint32_t *)calloc((size_t)n, sizeof(uint32_t));
    g->xs = (float *)malloc(sizeof(float) * n);
    g->zs = (float *)malloc(sizeof(float) * n);
    g->ss = (uint64_t *)malloc(sizeof(uint64_t) * n);
    g->cell_idx = (uint32_t *)malloc(sizeof(uint32_t) * n);
    g->ent_cell = (uint32_t *)malloc(sizeof(uint32_t) * n);
    g->marks = (uint8_t *)calloc((size_t)g->threads * (size_t)n, 1);
    g->next_seq = 1;
    return g;
}

void cg_free(void *p) {
    cgrid *g = (cgrid *)p;
    if (!g) return;
    for (int64_t c = 0; c < g->nchunk; c++) {
        free(g->rows[c].v);
        free(g->rows_new[c].v);
        free(g->ev_e[c].v);
        free(g->ev_l[c].v);
    }
    free(g->rows);
    free(g->rows_new);
    free(g->ev_e);
    free(g->ev_l);
    free(g->off);
    free(g->off_new);
    free(g->len);
    free(g->len_new);
    free(g->chk);
    free(g->chk_new);
    free(g->xs);
    free(g->zs);
    free(g->ss);
    free(g->x);
    free(g->z);
    free(g->seq);
    free(g->cell_start);
    free(g->cell_idx);
    free(g->ent_cell);
    free(g->marks);
    free(g);
}

/* grid of the current positions; returns gx (cells per row); cell (cx, cz) = cz * gx + cx */
static int64_t build_grid(cgrid *g, double *ox, double *oz, int64_t *gz_out, double *C_out) {
    const int64_t n = g->n;
    float x0 = g->x[0], x1 = g->x[0], z0 = g->z[0], z1 = g->z[0];
    for (int64_t i = 1; i < n; i++) {
        if (g->x[i] < x0) x0 = g->x[i];
        if (g->x[i] > x1) x1 = g->x[i];
        if (g->z[i] < z0) z0 = g->z[i];
        if (g->z[i] > z1) z1 = g->z[i];
    }
    const double C = (double)g->D * (1.0 + 0x1p-10);
    *ox = (double)x0 - C;
    *oz = (double)z0 - C;
    const int64_t gx = (int64_t)((x1 - x0) / C) + 3, gz = (int64_t)((z1 - z0) / C) + 3;
    const int64_t cells = gx * gz;
    if (cells + 1 > g->cells_cap) {
        free(g->cell_start);
        g->cells_cap = cells + 1;
        g->cell_start = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)g->cells_cap);
    }
    memset(g->cell_start, 0, sizeof(uint32_t) * (size_t)(cells + 1));
    for (int64_t i = 0; i < n; i++) {
        const int64_t cx = (int64_t)floor(((double)g->x[i] - *ox) / C), cz = (int64_t)floor(((double)g->z[i] - *oz) / C);
        g->ent_cell[i] = (uint32_t)(cz * gx + cx);
        g->cell_start[g->ent_cell[i] + 1]++;
    }
    for (int64_t c = 0; c < cells; c++) g->cell_start[c + 1] += g->cell_start[c];
    /* scatter (stable in entity order) using cell_idx as cursor space */
    uint32_t *cur = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)cells);
    memcpy(cur, g->cell_start, sizeof(uint32_t) * (size_t)cells);
    for (int64_t i = 0; i < n; i++) g->cell_idx[cur[g->ent_cell[i]]++] = (uint32_t)i;
    free(cur);
    for (int64_t j = 0; j < n; j++) {
        const uint32_t i = g->cell_idx[j];
        g->xs[j] = g->x[i];
        g->zs[j] = g->z[i];
        g->ss[j] = g->seq[i];
    }
    *gz_out = gz;
    *C_out = C;
    return gx;
}

/* relation rows of every entity, diffed against the previous rows when `diff` */
static void rows_and_diff(cgrid *g, int diff, int64_t *n_enter, int64_t *n_leave) {
    double ox, oz, C;
    int64_t gz;
    const int64_t gx = build_grid(g, &ox, &oz, &gz, &C);
    const int64_t n = g->n, nch = g->nchunk;
    const float D = g->D;
    int64_t ne = 0, nl = 0;
#pragma omp parallel for num_threads(g->threads) schedule(dynamic, 1) reduction(+ : ne, nl)
    for (int64_t c = 0; c < nch; c++) {
        uint8_t *mark = g->marks + (size_t)omp_get_thread_num() * (size_t)n;
        buf32 *out = &g->rows_new[c];
        out->n = 0;
        g->ev_e[c].n = g->ev_l[c].n = 0;
        /* entities in cell order: neighbouring A scan the same cells */
        const int64_t j0 = n * c / nch, j1 = n * (c + 1) / nch;
        for (int64_t ja = j0; ja < j1; ja++) {
            const int64_t a = g->cell_idx[ja];
            const int64_t start = out->n;
            const int64_t cell = g->ent_cell[a], cx = cell % gx, cz = cell / gx;
            const float ax = g->xs[ja], az = g->zs[ja];
            const uint64_t as = g->ss[ja];
            for (int64_t dz = -1; dz <= 1; dz++) {
                const int64_t r = cz + dz;
                if (r < 0 || r >= gz) continue;
                const int64_t c0 = cx > 0 ? cx - 1 : 0, c1 = cx + 1 < gx ? cx + 1 : gx - 1;
                const uint32_t jb = g->cell_start[r * gx + c0], je = g->cell_start[r * gx + c1 + 1];
                for (uint32_t j = jb; j < je; j++) {
                    if ((int64_t)j == ja) continue;
                    const float bx = g->xs[j], bz = g->zs[j];
                    const int nb = as > g->ss[j] ? pred(ax, az, bx, bz, D) : pred(bx, bz, ax, az, D);
                    if (nb) b_push(out, g->cell_idx[j]);
                }
            }
            g->off_new[a] = start;
            g->len_new[a] = (uint32_t)(out->n - start);
            g->chk_new[a] = (uint32_t)c;
            if (!diff) continue;
            /* diff against the previous row of a with the thread's marks: 1 = old only, 2 = in both */
            const uint32_t *o = g->rows[g->chk[a]].v + g->off[a], *q = out->v + start;
            const int64_t no = g->len[a], nq = out->n - start;
            for (int64_t i = 0; i < no; i++) mark[o[i]] = 1;
            for (int64_t k = 0; k < nq; k++) {
                if (mark[q[k]]) {
                    mark[q[k]] = 2;
                } else {
                    b_push(&g->ev_e[c], (uint32_t)a);
                    b_push(&g->ev_e[c], q[k]);
                    ne++;
                }
            }
            for (int64_t i = 0; i < no; i++) {
                if (mark[o[i]] == 1) {
                    b_push(&g->ev_l[c], (uint32_t)a);
                    b_push(&g->ev_l[c], o[i]);
                    nl++;
                }
                mark[o[i]] = 0;
            }
        }
    }
    /* the new rows become the previous ones */
    buf32 *t = g->rows;
    g->rows = g->rows_new;
    g->rows_new = t;
    int64_t *to = g->off;
    g->off = g->off_new;
    g->off_new = to;
    uint32_t *tl = g->len;
    g->len = g->len_new;
    g->len_new = tl;
    uint32_t *tc = g->chk;
    g->chk = g->chk_new;
    g->chk_new = tc;
    if (n_enter) *n_enter = ne;
    if (n_leave) *n_leave = nl;
}

/* Enter entities 0..n-1 in index order; returns the directed relation size. */
int64_t cg_init(void *p, const float *x, const float *z) {
    cgrid *g = (cgrid *)p;
    memcpy(g->x, x, sizeof(float) * (size_t)g->n);
    memcpy(g->z, z, sizeof(float) * (size_t)g->n);
    for (int64_t i = 0; i < g->n; i++) g->seq[i] = g->next_seq++;
    rows_and_diff(g, 0, NULL, NULL);
    int64_t tot = 0;
    for (int64_t i = 0; i < g->n; i++) tot += g->len[i];
    return tot;
}

/* One tick: m Moved calls in call order, then the relation diff.  Directed
 * event counts out; the events themselves stay in per-chunk buffers. */
void cg_tick(void *p, int64_t m, const int32_t *slots, const float *x, const float *z, int64_t *n_enter,
             int64_t *n_leave) {
    cgrid *g = (cgrid *)p;
    for (int64_t k = 0; k < m; k++) {
        const int32_t s = slots[k];
        g->x[s] = x[k];
        g->z[s] = z[k];
        g->seq[s] = g->next_seq++;
    }
    rows_and_diff(g, 1, n_enter, n_leave);
}
