/*
 * oracle/xzlist.c -- TEST INFRASTRUCTURE ONLY (parity oracle; never linked into
 * or called by the product path in goworld_amd/).
 *
 * Clean-room sequential restatement of go-aoi v0.2.0 `XZListAOIManager`
 * (third-party module github.com/xiaonanln/go-aoi v0.2.0, pinned at
 * /root/reference/go.mod:29; NOT present in this container, so this follows
 * the behavioural spec in SURVEY.md Appendix A).
 *
 * PARITY UNPINNED: the reference holds no AOI test, fixture or golden vector
 *  and go-aoi cannot be built or fetched here (no Go
 * toolchain, no network).  The restatement is pinned only by the reference's
 * call sites and by the known-answer tests of SURVEY.md Appendix C.
 *
 * Reference call sites this mirrors:
 *   NewXZListAOIManager(dist)      engine/entity/Space.go:105
 *   Enter(aoi, x, z)               engine/entity/Space.go:211,221
 *   Leave(aoi)                     engine/entity/Space.go:243
 *   Moved(aoi, x, z)               engine/entity/Space.go:259
 *   OnEnterAOI / OnLeaveAOI        engine/entity/Entity.go:227-233
 *
 * Data structure (Appendix A): two coordinate-sorted doubly linked sweep lists
 * (x and z), a per-node mark counter, and a per-node neighbour hash set.
 * `adjust(a)` marks every node inside [fl32(a.c-D), fl32(a.c+D)] on each
 * axis, diffs the previous neighbour set against markVal==2, emits the
 * leaves, then re-walks the x window to emit the enters, then clears the z
 * window.  All coordinate arithmetic is IEEE float32 (compile without
 * -ffast-math and with -ffp-contract=off).
 *
 * Node ids are manager-local dense integers in [0, cap).
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NIL (-1)
#define H_EMPTY (-1)
#define H_TOMB (-2)

typedef struct {
    int32_t *slot;
    uint32_t cap;   /* power of two, 0 when unallocated */
    uint32_t len;   /* live keys */
    uint32_t used;  /* live + tombstones */
} nset;

enum { EV_ENTER = 1, EV_LEAVE = 2 };

typedef struct {
    float D;
    int32_t cap;
    float *x, *z;
    int32_t *xprev, *xnext, *zprev, *znext;
    int32_t *mark;
    uint8_t *live;
    nset *nb;
    int32_t xhead, xtail, zhead, ztail;
    /* event sink */
    int record;
    int64_t n_enter, n_leave;
    uint8_t *ev_t;
    int32_t *ev_a, *ev_b;
    size_t ev_len, ev_cap;
} xzmgr;

/* ---------------------------------------------------------------- nset -- */

static inline uint32_t h32(int32_t k) { return (uint32_t)k * 0x9E3779B1u; }

static void nset_rehash(nset *s, uint32_t ncap) {
    int32_t *old = s->slot;
    uint32_t ocap = s->cap;
    s->slot = (int32_t *)malloc(sizeof(int32_t) * ncap);
    for (uint32_t i = 0; i < ncap; i++) s->slot[i] = H_EMPTY;
    s->cap = ncap;
    s->len = 0;
    s->used = 0;
    for (uint32_t i = 0; i < ocap; i++) {
        int32_t k = old[i];
        if (k >= 0) {
            uint32_t m = ncap - 1, p = h32(k) & m;
            while (s->slot[p] != H_EMPTY) p = (p + 1) & m;
            s->slot[p] = k;
            s->len++;
            s->used++;
        }
    }
    free(old);
}

static void nset_add(nset *s, int32_t k) {
    if (s->cap == 0) nset_rehash(s, 8);
    if ((s->used + 1) * 2 > s->cap) {
        uint32_t ncap = s->cap;
        while ((s->len + 1) * 4 > ncap) ncap *= 2; /* grow, or same size to drop tombstones */
        nset_rehash(s, ncap);
    }
    uint32_t m = s->cap - 1, p = h32(k) & m;
    int32_t tomb = -1;
    while (s->slot[p] != H_EMPTY) {
        if (s->slot[p] == k) return;
        if (s->slot[p] == H_TOMB && tomb < 0) tomb = (int32_t)p;
        p = (p + 1) & m;
    }
    if (tomb >= 0) {
        s->slot[tomb] = k;
    } else {
        s->slot[p] = k;
        s->used++;
    }
    s->len++;
}

static void nset_del(nset *s, int32_t k) {
    if (s->cap == 0) return;
    uint32_t m = s->cap - 1, p = h32(k) & m;
    while (s->slot[p] != H_EMPTY) {
        if (s->slot[p] == k) {
            s->slot[p] = H_TOMB;
            s->len--;
            return;
        }
        p = (p + 1) & m;
    }
}

/* ---------------------------------------------------------- event sink -- */

static void emit(xzmgr *m, int type, int32_t a, int32_t b) {
    if (type == EV_ENTER) m->n_enter++; else m->n_leave++;
    if (!m->record) return;
    if (m->ev_len == m->ev_cap) {
        size_t nc = m->ev_cap ? m->ev_cap * 2 : 1024;
        m->ev_t = (uint8_t *)realloc(m->ev_t, nc);
        m->ev_a = (int32_t *)realloc(m->ev_a, nc * sizeof(int32_t));
        m->ev_b = (int32_t *)realloc(m->ev_b, nc * sizeof(int32_t));
        m->ev_cap = nc;
    }
    m->ev_t[m->ev_len] = (uint8_t)type;
    m->ev_a[m->ev_len] = a;
    m->ev_b[m->ev_len] = b;
    m->ev_len++;
}

/* ------------------------------------------------------ sweep-list ops -- */
/* The two axes share one implementation through pointer selection. */

typedef struct {
    float *c;
    int32_t *prev, *next;
    int32_t *head, *tail;
} axis;

static inline axis ax_x(xzmgr *m) { axis a = {m->x, m->xprev, m->xnext, &m->xhead, &m->xtail}; return a; }
static inline axis ax_z(xzmgr *m) { axis a = {m->z, m->zprev, m->znext, &m->zhead, &m->ztail}; return a; }

/* insert before the first node whose coord >= the new coord, scanning from the head */
static void list_insert(axis A, int32_t n) {
    float c = A.c[n];
    if (*A.head == NIL) {
        *A.head = *A.tail = n;
        A.prev[n] = A.next[n] = NIL;
        return;
    }
    int32_t p = *A.head;
    while (p != NIL && A.c[p] < c) p = A.next[p];
    if (p == NIL) {
        int32_t t = *A.tail;
        A.next[t] = n;
        A.prev[n] = t;
        A.next[n] = NIL;
        *A.tail = n;
    } else {
        int32_t pr = A.prev[p];
        A.next[n] = p;
        A.prev[p] = n;
        A.prev[n] = pr;
        if (pr != NIL) A.next[pr] = n; else *A.head = n;
    }
}

static void list_remove(axis A, int32_t n) {
    int32_t pr = A.prev[n], nx = A.next[n];
    if (pr != NIL) A.next[pr] = nx; else *A.head = nx;
    if (nx != NIL) A.prev[nx] = pr; else *A.tail = pr;
    A.prev[n] = A.next[n] = NIL;
}

/* relink after the coordinate changed from oldc to A.c[n] (called only when they differ) */
static void list_move(axis A, int32_t n, float oldc) {
    float c = A.c[n];
    if (c > oldc) {
        int32_t nx = A.next[n];
        if (nx == NIL || A.c[nx] >= c) return;
        int32_t pr = A.prev[n];
        if (pr != NIL) A.next[pr] = nx; else *A.head = nx;
        A.prev[nx] = pr;
        pr = nx;
        nx = A.next[nx];
        while (nx != NIL && A.c[nx] < c) { pr = nx; nx = A.next[nx]; }
        A.next[pr] = n;
        A.prev[n] = pr;
        if (nx != NIL) A.prev[nx] = n; else *A.tail = n;
        A.next[n] = nx;
    } else {
        int32_t pr = A.prev[n];
        if (pr == NIL || A.c[pr] <= c) return;
        int32_t nx = A.next[n];
        if (nx != NIL) A.prev[nx] = pr; else *A.tail = pr;
        A.next[pr] = nx;
        nx = pr;
        pr = A.prev[pr];
        while (pr != NIL && A.c[pr] > c) { nx = pr; pr = A.prev[pr]; }
        A.prev[nx] = n;
        A.next[n] = nx;
        if (pr != NIL) A.next[pr] = n; else *A.head = n;
        A.prev[n] = pr;
    }
}

/* markVal += 1 for every node (other than n) with coord in [fl32(c-D), fl32(c+D)] */
static void list_mark(axis A, int32_t *mark, int32_t n, float D) {
    float c = A.c[n];
    const float lo = c - D, hi = c + D; /* fl32 bounds, exactly as go-aoi */
    for (int32_t p = A.prev[n]; p != NIL && A.c[p] >= lo; p = A.prev[p]) mark[p]++;
    for (int32_t p = A.next[n]; p != NIL && A.c[p] <= hi; p = A.next[p]) mark[p]++;
}

static void list_clear(axis A, int32_t *mark, int32_t n, float D) {
    float c = A.c[n];
    const float lo = c - D, hi = c + D;
    for (int32_t p = A.prev[n]; p != NIL && A.c[p] >= lo; p = A.prev[p]) mark[p] = 0;
    for (int32_t p = A.next[n]; p != NIL && A.c[p] <= hi; p = A.next[p]) mark[p] = 0;
}

static void enter_pair(xzmgr *m, int32_t a, int32_t o) {
    nset_add(&m->nb[a], o);
    emit(m, EV_ENTER, a, o); /* a.callback.OnEnterAOI(o) */
    nset_add(&m->nb[o], a);
    emit(m, EV_ENTER, o, a); /* o.callback.OnEnterAOI(a) */
}

/* the x-window re-walk: every node with markVal==2 becomes a neighbour; all reset to 0 */
static void list_get_clear_marked(xzmgr *m, axis A, int32_t n) {
    float c = A.c[n];
    const float lo = c - m->D, hi = c + m->D;
    for (int32_t p = A.prev[n]; p != NIL && A.c[p] >= lo; p = A.prev[p]) {
        if (m->mark[p] == 2) enter_pair(m, n, p);
        m->mark[p] = 0;
    }
    for (int32_t p = A.next[n]; p != NIL && A.c[p] <= hi; p = A.next[p]) {
        if (m->mark[p] == 2) enter_pair(m, n, p);
        m->mark[p] = 0;
    }
}

static void adjust(xzmgr *m, int32_t a) {
    list_mark(ax_x(m), m->mark, a, m->D);
    list_mark(ax_z(m), m->mark, a, m->D);
    nset *s = &m->nb[a];
    for (uint32_t i = 0; i < s->cap; i++) {
        int32_t o = s->slot[i];
        if (o < 0) continue;
        if (m->mark[o] == 2) {
            m->mark[o] = -2; /* kept */
        } else {
            nset_del(s, o);
            emit(m, EV_LEAVE, a, o);
            nset_del(&m->nb[o], a);
            emit(m, EV_LEAVE, o, a);
        }
    }
    list_get_clear_marked(m, ax_x(m), a);
    list_clear(ax_z(m), m->mark, a, m->D);
}

/* ------------------------------------------------------------- public -- */

xzmgr *xz_new(float D, int32_t cap) {
    xzmgr *m = (xzmgr *)calloc(1, sizeof(xzmgr));
    m->D = D;
    m->cap = cap;
    m->x = (float *)calloc(cap, sizeof(float));
    m->z = (float *)calloc(cap, sizeof(float));
    m->xprev = (int32_t *)malloc(cap * sizeof(int32_t));
    m->xnext = (int32_t *)malloc(cap * sizeof(int32_t));
    m->zprev = (int32_t *)malloc(cap * sizeof(int32_t));
    m->znext = (int32_t *)malloc(cap * sizeof(int32_t));
    m->mark = (int32_t *)calloc(cap, sizeof(int32_t));
    m->live = (uint8_t *)calloc(cap, 1);
    m->nb = (nset *)calloc(cap, sizeof(nset));
    for (int32_t i = 0; i < cap; i++) m->xprev[i] = m->xnext[i] = m->zprev[i] = m->znext[i] = NIL;
    m->xhead = m->xtail = m->zhead = m->ztail = NIL;
    return m;
}

void xz_free(xzmgr *m) {
    if (!m) return;
    for (int32_t i = 0; i < m->cap; i++) free(m->nb[i].slot);
    free(m->x); free(m->z); free(m->xprev); free(m->xnext); free(m->zprev); free(m->znext);
    free(m->mark); free(m->live); free(m->nb);
    free(m->ev_t); free(m->ev_a); free(m->ev_b);
    free(m);
}

void xz_set_record(xzmgr *m, int record) { m->record = record; }

/* Enter(aoi, x, z): errors mirror a Go panic (non-zero return) */
int xz_enter(xzmgr *m, int32_t id, float x, float z) {
    if (id < 0 || id >= m->cap || m->live[id]) return -1;
    m->live[id] = 1;
    m->x[id] = x;
    m->z[id] = z;
    m->mark[id] = 0;
    list_insert(ax_x(m), id);
    list_insert(ax_z(m), id);
    adjust(m, id);
    return 0;
}

int xz_leave(xzmgr *m, int32_t id) {
    if (id < 0 || id >= m->cap || !m->live[id]) return -1;
    list_remove(ax_x(m), id);
    list_remove(ax_z(m), id);
    adjust(m, id); /* unlinked node marks nobody: every neighbour gets a leave */
    m->live[id] = 0;
    return 0;
}

int xz_moved(xzmgr *m, int32_t id, float x, float z) {
    if (id < 0 || id >= m->cap || !m->live[id]) return -1;
    float ox = m->x[id], oz = m->z[id];
    m->x[id] = x;
    m->z[id] = z;
    if (ox != x) list_move(ax_x(m), id, ox);
    if (oz != z) list_move(ax_z(m), id, oz);
    adjust(m, id); /* always, even when the position is unchanged */
    return 0;
}

/* Apply a batch of ops in array order.  op: 0 = Moved, 1 = Enter, 2 = Leave.
 * Returns the index of the first failing op, or -1 when all succeeded. */
int64_t xz_apply(xzmgr *m, int64_t n, const uint8_t *op, const int32_t *id, const float *x, const float *z) {
    for (int64_t i = 0; i < n; i++) {
        int r;
        switch (op[i]) {
        case 0: r = xz_moved(m, id[i], x[i], z[i]); break;
        case 1: r = xz_enter(m, id[i], x[i], z[i]); break;
        case 2: r = xz_leave(m, id[i]); break;
        default: r = -1;
        }
        if (r) return i;
    }
    return -1;
}

/* Bulk equivalent of Enter(id[0..n)) in array order on an empty manager: the
 * same sorted lists and the same neighbour sets (closed form with seq = array
 * position) in O(n + E) instead of go-aoi's O(n^2)
 * head-scan inserts.  No events are emitted.  Used only to populate the
 * bench's cpu_baseline (1M entities at config 3, 2^24 at config 5); tests check
 * it against real Enters.  The lists come from a stable LSD radix sort of the
 * coordinates (equal coordinates keep array order); the neighbour sets from a
 * grid of 2D cells, one thread per entity's own set (OpenMP). */
static inline uint32_t fkey(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

/* positions 0..n-1 ordered stably by key[] (4 passes of 8 bits) */
static void radix_order(int64_t n, const uint32_t *key, int32_t *ord) {
    int32_t *tmp = (int32_t *)malloc(sizeof(int32_t) * (n ? n : 1));
    for (int64_t i = 0; i < n; i++) ord[i] = (int32_t)i;
    for (int sh = 0; sh < 32; sh += 8) {
        int64_t cnt[257] = {0};
        for (int64_t i = 0; i < n; i++) cnt[((key[ord[i]] >> sh) & 255u) + 1]++;
        for (int b = 0; b < 256; b++) cnt[b + 1] += cnt[b];
        for (int64_t i = 0; i < n; i++) tmp[cnt[(key[ord[i]] >> sh) & 255u]++] = ord[i];
        int32_t *t = ord;
        memcpy(t, tmp, sizeof(int32_t) * n);
    }
    free(tmp);
}

static inline int bulk_pred(float wx, float wz, float lx, float lz, float D) {
    const float lox = wx - D, hix = wx + D, loz = wz - D, hiz = wz + D;
    return lx >= lox && lx <= hix && lz >= loz && lz <= hiz;
}

int xz_bulk_enter(xzmgr *m, int64_t n, const int32_t *id, const float *x, const float *z) {
    if (m->xhead != NIL || m->zhead != NIL) return -1;
    for (int64_t i = 0; i < n; i++)
        if (id[i] < 0 || id[i] >= m->cap || m->live[id[i]]) return -1;
    for (int64_t i = 0; i < n; i++) {
        m->live[id[i]] = 1;
        m->x[id[i]] = x[i];
        m->z[id[i]] = z[i];
        m->mark[id[i]] = 0;
    }
    int32_t *ord = (int32_t *)malloc(sizeof(int32_t) * (n ? n : 1));
    uint32_t *key = (uint32_t *)malloc(sizeof(uint32_t) * (n ? n : 1));
    for (int a = 0; a < 2; a++) {
        axis A = a == 0 ? ax_x(m) : ax_z(m);
        const float *c = a == 0 ? x : z;
        for (int64_t i = 0; i < n; i++) key[i] = fkey(c[i]);
        radix_order(n, key, ord);
        for (int64_t k = 0; k < n; k++) {
            const int32_t e = id[ord[k]];
            A.prev[e] = k ? id[ord[k - 1]] : NIL;
            A.next[e] = k + 1 < n ? id[ord[k + 1]] : NIL;
        }
        *A.head = n ? id[ord[0]] : NIL;
        *A.tail = n ? id[ord[n - 1]] : NIL;
    }
    free(key);
    free(ord);
    if (n < 2) return 0;
    /* cells of side C = 2D: a window [fl32(w-D), fl32(w+D)] spans at most the 3x3 cells around w */
    /* (wider cells for a sparse world: any side >= 2D keeps the 3x3 neighbourhood complete) */
    const float D = m->D;
    double x0 = INFINITY, z0 = INFINITY, x1 = -INFINITY, z1 = -INFINITY;
    for (int64_t i = 0; i < n; i++) {
        x0 = fmin(x0, x[i]); x1 = fmax(x1, x[i]);
        z0 = fmin(z0, z[i]); z1 = fmax(z1, z[i]);
    }
    double C = 2.0 * (double)D;
    while (((x1 - x0) / C + 2.0) * ((z1 - z0) / C + 2.0) > 4.0 * (double)n + 1024.0) C *= 2.0;
    int64_t cx0 = INT64_MAX, cz0 = INT64_MAX, cx1 = INT64_MIN, cz1 = INT64_MIN;
    int64_t *cxz = (int64_t *)malloc(sizeof(int64_t) * 2 * n);
    for (int64_t i = 0; i < n; i++) {
        const int64_t cx = (int64_t)floor((double)x[i] / C), cz = (int64_t)floor((double)z[i] / C);
        cxz[2 * i] = cx;
        cxz[2 * i + 1] = cz;
        if (cx < cx0) cx0 = cx;
        if (cx > cx1) cx1 = cx;
        if (cz < cz0) cz0 = cz;
        if (cz > cz1) cz1 = cz;
    }
    const int64_t gx = cx1 - cx0 + 1, gz = cz1 - cz0 + 1;
    int64_t *start = (int64_t *)calloc((size_t)(gx * gz + 1), sizeof(int64_t));
    int32_t *cell = (int32_t *)malloc(sizeof(int32_t) * n);
    for (int64_t i = 0; i < n; i++) start[(cxz[2 * i] - cx0) * gz + (cxz[2 * i + 1] - cz0) + 1]++;
    for (int64_t c = 0; c < gx * gz; c++) start[c + 1] += start[c];
    {
        int64_t *fill = (int64_t *)malloc(sizeof(int64_t) * (size_t)(gx * gz));
        memcpy(fill, start, sizeof(int64_t) * (size_t)(gx * gz));
        for (int64_t i = 0; i < n; i++) cell[fill[(cxz[2 * i] - cx0) * gz + (cxz[2 * i + 1] - cz0)]++] = (int32_t)i;
        free(fill);
    }
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t i = 0; i < n; i++) {
        const int64_t cx = cxz[2 * i] - cx0, cz = cxz[2 * i + 1] - cz0;
        nset *s = &m->nb[id[i]];
        for (int64_t ux = cx - 1; ux <= cx + 1; ux++) {
            if (ux < 0 || ux >= gx) continue;
            for (int64_t uz = cz - 1; uz <= cz + 1; uz++) {
                if (uz < 0 || uz >= gz) continue;
                const int64_t c = ux * gz + uz;
                for (int64_t k = start[c]; k < start[c + 1]; k++) {
                    const int64_t j = cell[k];
                    if (j == i) continue;
                    /* the later of the two (larger array position = larger seq) owns the window */
                    const int nb = j < i ? bulk_pred(x[i], z[i], x[j], z[j], D) : bulk_pred(x[j], z[j], x[i], z[i], D);
                    if (nb) nset_add(s, id[j]);
                }
            }
        }
    }
    free(start);
    free(cell);
    free(cxz);
    return 0;
}

/* Moved() over a prefix of a batch; used by the bench's cpu_baseline leg */
int64_t xz_moved_batch(xzmgr *m, int64_t n, const int32_t *id, const float *x, const float *z) {
    for (int64_t i = 0; i < n; i++)
        if (xz_moved(m, id[i], x[i], z[i])) return i;
    return -1;
}

void xz_counts(const xzmgr *m, int64_t *n_enter, int64_t *n_leave) {
    *n_enter = m->n_enter;
    *n_leave = m->n_leave;
}

size_t xz_num_events(const xzmgr *m) { return m->ev_len; }

size_t xz_take_events(xzmgr *m, uint8_t *t, int32_t *a, int32_t *b, size_t cap) {
    size_t n = m->ev_len < cap ? m->ev_len : cap;
    memcpy(t, m->ev_t, n);
    memcpy(a, m->ev_a, n * sizeof(int32_t));
    memcpy(b, m->ev_b, n * sizeof(int32_t));
    m->ev_len = 0;
    return n;
}

int32_t xz_neighbor_count(const xzmgr *m, int32_t id) {
    if (id < 0 || id >= m->cap) return -1;
    return (int32_t)m->nb[id].len;
}

/* unsorted neighbour ids of `id` */
int32_t xz_neighbors(const xzmgr *m, int32_t id, int32_t *out, int32_t cap) {
    if (id < 0 || id >= m->cap) return -1;
    const nset *s = &m->nb[id];
    int32_t n = 0;
    for (uint32_t i = 0; i < s->cap; i++)
        if (s->slot[i] >= 0) {
            if (n < cap) out[n] = s->slot[i];
            n++;
        }
    return n;
}

/* total directed neighbour pairs */
int64_t xz_total_pairs(const xzmgr *m) {
    int64_t t = 0;
    for (int32_t i = 0; i < m->cap; i++) t += m->nb[i].len;
    return t;
}

/* check both sweep lists are sorted and consistent; returns 0 when sound */
int xz_check(const xzmgr *m) {
    const float *cs[2] = {m->x, m->z};
    const int32_t *nexts[2] = {m->xnext, m->znext};
    const int32_t *prevs[2] = {m->xprev, m->zprev};
    const int32_t heads[2] = {m->xhead, m->zhead};
    for (int a = 0; a < 2; a++) {
        int32_t p = heads[a], prev = NIL;
        while (p != NIL) {
            if (prevs[a][p] != prev) return 1 + a;
            if (prev != NIL && cs[a][prev] > cs[a][p]) return 3 + a;
            prev = p;
            p = nexts[a][p];
        }
    }
    return 0;
}
