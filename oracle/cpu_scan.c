/*
 * cpu_scan.c -- TEST / BASELINE INFRASTRUCTURE ONLY (never the product).
 *
 * The second CPU baseline line of bench.py: an optimised C kNN over one window with the
 * build contract of orc_knn_contract (candidates = cell in C u G and
 * d <= r, one entry per objID -- its minimum-(d, idx) occurrence --, sorted by (d, objID),
 * first k).  What a competent host implementation would do instead of the reference's object
 * pipeline: OpenMP over contiguous point ranges, integer Chebyshev cell test (no strings, no
 * hash sets), a squared-distance prefilter against the thread's running k-th distance, a
 * bounded top-k-distinct max-heap per thread (objID -> heap slot hash), one final merge.
 */
#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#include "geoflink_oracle.h"

typedef struct { double d; int64_t obj, idx; } ent;

static int ent_lt(const ent* a, const ent* b) {
  if (a->d != b->d) return a->d < b->d;
  if (a->obj != b->obj) return a->obj < b->obj;
  return a->idx < b->idx;
}

/* bounded max-heap of distinct objIDs + open-addressing objID -> slot map */
typedef struct {
  ent* h;
  int32_t n, k;
  int64_t* hk;   /* keys */
  int32_t* hv;   /* slot, -1 empty */
  uint64_t mask;
} topk;

static uint64_t mix(int64_t v) {
  uint64_t x = (uint64_t)v * 0x9E3779B97F4A7C15ull;
  return x ^ (x >> 29);
}
static int64_t map_find(const topk* t, int64_t obj) {
  for (uint64_t i = mix(obj) & t->mask;; i = (i + 1) & t->mask) {
    if (t->hv[i] < 0) return -1;
    if (t->hk[i] == obj) return (int64_t)i;
  }
}
static void map_put(topk* t, int64_t obj, int32_t slot) {
  uint64_t i = mix(obj) & t->mask;
  while (t->hv[i] >= 0 && t->hk[i] != obj) i = (i + 1) & t->mask;
  t->hk[i] = obj;
  t->hv[i] = slot;
}
static void map_del(topk* t, int64_t obj) {  /* linear probing, backward-shift deletion */
  int64_t f = map_find(t, obj);
  if (f < 0) return;
  uint64_t i = (uint64_t)f, j = i;
  for (;;) {
    j = (j + 1) & t->mask;
    if (t->hv[j] < 0) break;
    const uint64_t home = mix(t->hk[j]) & t->mask;
    const int stays = i <= j ? (home > i && home <= j) : (home > i || home <= j);  /* home in (i, j] */
    if (stays) continue;
    t->hk[i] = t->hk[j];
    t->hv[i] = t->hv[j];
    i = j;
  }
  t->hv[i] = -1;
}
static void put_slot(topk* t, int32_t s, ent e) {
  t->h[s] = e;
  int64_t m = map_find(t, e.obj);
  if (m >= 0) t->hv[m] = s; else map_put(t, e.obj, s);
}
static void sift_up(topk* t, int32_t s) {
  ent e = t->h[s];
  while (s > 0) {
    int32_t p = (s - 1) / 2;
    if (!ent_lt(&t->h[p], &e)) break;
    put_slot(t, s, t->h[p]);
    s = p;
  }
  put_slot(t, s, e);
}
static void sift_down(topk* t, int32_t s) {
  ent e = t->h[s];
  for (;;) {
    int32_t c = 2 * s + 1;
    if (c >= t->n) break;
    if (c + 1 < t->n && ent_lt(&t->h[c], &t->h[c + 1])) ++c;
    if (!ent_lt(&e, &t->h[c])) break;
    put_slot(t, s, t->h[c]);
    s = c;
  }
  put_slot(t, s, e);
}
static void topk_offer(topk* t, ent e) {
  int64_t m = map_find(t, e.obj);
  if (m >= 0) {  /* objID present: keep its smaller occurrence (a smaller key sinks in a max-heap) */
    int32_t s = t->hv[m];
    if (ent_lt(&e, &t->h[s])) { t->h[s] = e; sift_down(t, s); }
    return;
  }
  if (t->n < t->k) {
    t->h[t->n] = e;
    map_put(t, e.obj, t->n);
    t->n++;
    sift_up(t, t->n - 1);
  } else if (ent_lt(&e, &t->h[0])) {
    map_del(t, t->h[0].obj);
    t->h[0] = e;
    map_put(t, e.obj, 0);
    sift_down(t, 0);
  }
}

static int cmp_ent(const void* a, const void* b) {
  const ent* p = (const ent*)a; const ent* q = (const ent*)b;
  return ent_lt(p, q) ? -1 : (ent_lt(q, p) ? 1 : 0);
}

int32_t orc_knn_scan_omp(const orc_grid* g, int64_t n, const double* x, const double* y,
                         const int64_t* objID, double qx, double qy, double r, int32_t k,
                         int metric, int nthreads, int64_t* out_objID, double* out_d, int64_t* out_idx) {
  if (k <= 0) return ORC_ERR_ARG;
  const int T = nthreads < 1 ? 1 : nthreads;
  int32_t qcx, qcy;
  orc_cell_of(g, qx, qy, &qcx, &qcy);
  const int64_t gl = orc_guaranteed_layers(g, r), cl = orc_candidate_layers(g, r), N = g->n;
  ent* all = (ent*)malloc(sizeof(ent) * (size_t)T * (size_t)k);
  int32_t* cnt = (int32_t*)calloc((size_t)T, sizeof(int32_t));
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    topk K;
    uint64_t cap = 16;
    while (cap < 4 * (uint64_t)k) cap <<= 1;
    K.h = all + (size_t)t * k; K.n = 0; K.k = k; K.mask = cap - 1;
    K.hk = (int64_t*)malloc(sizeof(int64_t) * cap);
    K.hv = (int32_t*)malloc(sizeof(int32_t) * cap);
    for (uint64_t i = 0; i < cap; i++) K.hv[i] = -1;
    double thr_s = INFINITY;  /* prefilter: s above it cannot beat the heap's maximum */
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; i++) {
      const double dx = qx - x[i], dy = qy - y[i];
      const double s = dx * dx + dy * dy;
      if (s > thr_s) continue;
      int32_t cx, cy;
      orc_cell_of(g, x[i], y[i], &cx, &cy);
      const int64_t ax = (int64_t)cx - qcx, ay = (int64_t)cy - qcy;
      const int valid = cx >= 0 && cy >= 0 && cx < N && cy < N;
      const int inC = cl > 0 && valid && ax <= cl && ax >= -cl && ay <= cl && ay >= -cl;
      const int inG = gl == 0 && ax == 0 && ay == 0;
      if (!(inC || inG)) continue;
      const double d = orc_distance(qx, qy, x[i], y[i], metric);
      if (!(d <= r)) continue;
      ent e = {d, objID[i], i};
      topk_offer(&K, e);
      if (K.n == K.k) thr_s = K.h[0].d * K.h[0].d * (1.0 + 1e-12);
    }
    cnt[t] = K.n;
    free(K.hk);
    free(K.hv);
  }
  /* merge: every thread's top-k-distinct list, sorted, first occurrence of each objID */
  int64_t m = 0;
  for (int t = 0; t < T; t++) {
    memmove(all + m, all + (size_t)t * k, sizeof(ent) * (size_t)cnt[t]);
    m += cnt[t];
  }
  qsort(all, (size_t)m, sizeof(ent), cmp_ent);
  int32_t nout = 0;
  for (int64_t i = 0; i < m && nout < k; i++) {
    int dup = 0;
    for (int32_t j = 0; j < nout && !dup; j++) dup = out_objID[j] == all[i].obj;
    if (dup) continue;
    out_objID[nout] = all[i].obj; out_d[nout] = all[i].d; out_idx[nout] = all[i].idx;
    nout++;
  }
  free(all);
  free(cnt);
  return nout;
}

/* ------------------------------------------------------------------------------------ */
/* Optimised OpenMP range / join lines (bench cpu_baseline "optimized_scan" of C1, C3, C4): */
/* integer cells instead of String keys, a class byte per grid cell (the union of the       */
/* queries' guaranteed / candidate sets, UniformGrid.java:165-229,368-411), per-thread      */
/* outputs.  Same results as orc_range_pp / orc_range_ppoly / orc_join_pp.                  */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint8_t* cls; int64_t n; int32_t* xg; int64_t nxg, cxg; } cellcls;

static void cls_init(cellcls* c, int64_t n) {
  c->n = n; c->cls = (uint8_t*)calloc((size_t)(n * n), 1); c->xg = NULL; c->nxg = c->cxg = 0;
}
static void cls_free(cellcls* c) { free(c->cls); free(c->xg); }
/* guaranteed (2) / candidate (1) cells of query cell (qcx, qcy); g == 0: the cell itself without
 * validKey (kept in xg when outside the grid) */
static void cls_mark(cellcls* c, int64_t qcx, int64_t qcy, int32_t gl, int32_t cl) {
  const int64_t n = c->n;
  if (gl == 0) {
    if (qcx >= 0 && qcy >= 0 && qcx < n && qcy < n) c->cls[qcy * n + qcx] = 2;
    else {
      if (c->nxg == c->cxg) { c->cxg = c->cxg ? 2 * c->cxg : 16; c->xg = (int32_t*)realloc(c->xg, 8 * (size_t)c->cxg); }
      c->xg[2 * c->nxg] = (int32_t)qcx; c->xg[2 * c->nxg + 1] = (int32_t)qcy; c->nxg++;
    }
  }
  for (int pass = 0; pass < 2; pass++) {
    const int64_t L = pass == 0 ? gl : cl;
    if (L <= 0) continue;
    for (int64_t j = qcy - L < 0 ? 0 : qcy - L; j <= (qcy + L < n - 1 ? qcy + L : n - 1); j++)
      for (int64_t i = qcx - L < 0 ? 0 : qcx - L; i <= (qcx + L < n - 1 ? qcx + L : n - 1); i++) {
        uint8_t* v = &c->cls[j * n + i];
        if (pass == 0) *v = 2;
        else if (*v == 0) *v = 1;
      }
  }
}
static int cls_of(const cellcls* c, int32_t cx, int32_t cy) {
  if (cx >= 0 && cy >= 0 && cx < c->n && cy < c->n) return c->cls[(int64_t)cy * c->n + cx];
  for (int64_t k = 0; k < c->nxg; k++)
    if (c->xg[2 * k] == cx && c->xg[2 * k + 1] == cy) return 2;
  return 0;
}

typedef struct { int64_t* v; int64_t n, cap; } ovec;
static void ovec_push(ovec* a, int64_t x) {
  if (a->n == a->cap) { a->cap = a->cap ? 2 * a->cap : 1024; a->v = (int64_t*)realloc(a->v, 8 * (size_t)a->cap); }
  a->v[a->n++] = x;
}
/* per-thread results of contiguous point ranges, concatenated in thread order (ascending) */
static int64_t ovec_concat(ovec* res, int T, int64_t* out, int64_t cap) {
  int64_t w = 0;
  for (int t = 0; t < T; t++) {
    for (int64_t i = 0; i < res[t].n; i++, w++)
      if (w < cap) out[w] = res[t].v[i];
    free(res[t].v);
  }
  return w;
}

int64_t orc_range_pp_omp(const orc_grid* g, int64_t n, const double* x, const double* y, int32_t nq,
                         const double* qx, const double* qy, double r, int approximate, int metric, int nthreads,
                         int64_t* out_idx, int64_t cap) {
  const int T = nthreads < 1 ? 1 : nthreads;
  const int32_t gl = orc_guaranteed_layers(g, r), cl = orc_candidate_layers(g, r);
  cellcls c;
  cls_init(&c, g->n);
  for (int32_t q = 0; q < nq; q++) {
    int32_t a, b;
    orc_cell_of(g, qx[q], qy[q], &a, &b);
    cls_mark(&c, a, b, gl, cl);
  }
  ovec* res = (ovec*)calloc((size_t)T, sizeof(ovec));
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    for (int64_t i = n * t / T; i < n * (t + 1) / T; i++) {
      int32_t a, b;
      orc_cell_of(g, x[i], y[i], &a, &b);
      const int k = cls_of(&c, a, b);
      if (k == 2) { ovec_push(&res[t], i); continue; }
      if (k != 1) continue;
      if (approximate) { for (int32_t q = 0; q < nq; q++) ovec_push(&res[t], i); continue; }
      for (int32_t q = 0; q < nq; q++)
        if (orc_distance(qx[q], qy[q], x[i], y[i], metric) <= r) { ovec_push(&res[t], i); break; }
    }
  }
  int64_t cnt = ovec_concat(res, T, out_idx, cap);
  free(res);
  cls_free(&c);
  return cnt;
}

int64_t orc_range_ppoly_omp(const orc_grid* g, int64_t n, const double* x, const double* y, const orc_polygons* P,
                            double r, int approximate, int metric, int nthreads, int64_t* out_idx, int64_t cap) {
  const int T = nthreads < 1 ? 1 : nthreads;
  const int32_t gl = orc_guaranteed_layers(g, r), cl = orc_candidate_layers(g, r);
  const int64_t N = g->n;
  cellcls c;
  cls_init(&c, N);
  double* bb = (double*)malloc(sizeof(double) * 4 * (size_t)(P->npoly > 0 ? P->npoly : 1));
  /* candidate polygons per cell: those whose bbox grown by r (plus a rounding margin) reaches it */
  int64_t* cnt = (int64_t*)calloc((size_t)(N * N + 1), 8);
  int32_t(*rng)[4] = malloc(sizeof(int32_t[4]) * (size_t)(P->npoly > 0 ? P->npoly : 1));
  for (int32_t p = 0; p < P->npoly; p++) {
    const int32_t v0 = P->vert_off[P->ring_off[p]], v1 = P->vert_off[P->ring_off[p] + 1];
    double x1 = P->vx[v0], x2 = x1, y1 = P->vy[v0], y2 = y1;
    for (int32_t v = v0; v < v1; v++) {
      x1 = fmin(x1, P->vx[v]); x2 = fmax(x2, P->vx[v]); y1 = fmin(y1, P->vy[v]); y2 = fmax(y2, P->vy[v]);
    }
    bb[4 * p] = x1; bb[4 * p + 1] = y1; bb[4 * p + 2] = x2; bb[4 * p + 3] = y2;
    int32_t a1, b1, a2, b2;
    orc_cell_of(g, x1, y1, &a1, &b1);
    orc_cell_of(g, x2, y2, &a2, &b2);
    for (int64_t a = a1; a <= a2; a++)
      for (int64_t b = b1; b <= b2; b++) cls_mark(&c, a, b, gl, cl);
    const double m = r * (1.0 + 1e-9) + 1e-9;
    int32_t e1, f1, e2, f2;
    orc_cell_of(g, x1 - m, y1 - m, &e1, &f1);
    orc_cell_of(g, x2 + m, y2 + m, &e2, &f2);
    rng[p][0] = e1 < 0 ? 0 : e1; rng[p][1] = f1 < 0 ? 0 : f1;
    rng[p][2] = e2 > N - 1 ? (int32_t)N - 1 : e2; rng[p][3] = f2 > N - 1 ? (int32_t)N - 1 : f2;
    for (int64_t b = rng[p][1]; b <= rng[p][3]; b++)
      for (int64_t a = rng[p][0]; a <= rng[p][2]; a++) cnt[b * N + a + 1]++;
  }
  for (int64_t k = 0; k < N * N; k++) cnt[k + 1] += cnt[k];
  int32_t* lst = (int32_t*)malloc(4 * (size_t)(cnt[N * N] > 0 ? cnt[N * N] : 1));
  {
    int64_t* cur = (int64_t*)malloc(8 * (size_t)(N * N));
    memcpy(cur, cnt, 8 * (size_t)(N * N));
    for (int32_t p = 0; p < P->npoly; p++)  /* ascending polygon order per cell (the reference's loop order) */
      for (int64_t b = rng[p][1]; b <= rng[p][3]; b++)
        for (int64_t a = rng[p][0]; a <= rng[p][2]; a++) lst[cur[b * N + a]++] = p;
    free(cur);
  }
  ovec* res = (ovec*)calloc((size_t)T, sizeof(ovec));
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    for (int64_t i = n * t / T; i < n * (t + 1) / T; i++) {
      int32_t a, b;
      orc_cell_of(g, x[i], y[i], &a, &b);
      const int k = cls_of(&c, a, b);
      if (k == 2) { ovec_push(&res[t], i); continue; }
      if (k != 1) continue;  /* candidate cells are in-grid */
      const int64_t s = (int64_t)b * N + a;
      for (int64_t u = cnt[s]; u < cnt[s + 1]; u++) {
        const int32_t p = lst[u];
        const double* e = bb + 4 * p;
        const double d = approximate ? orc_point_bbox_distance(x[i], y[i], e[0], e[1], e[2], e[3])
                                     : orc_point_polygon_distance(x[i], y[i], P, p, metric);
        if (d <= r) { ovec_push(&res[t], i); break; }
      }
    }
  }
  int64_t m = ovec_concat(res, T, out_idx, cap);
  free(res); free(bb); free(cnt); free(rng); free(lst);
  cls_free(&c);
  return m;
}

/* point-point join on one grid: queries counting-sorted by clamped cell, each ordinary point
 * (in the grid) scans the cells within c layers; pairs sorted by (ordinary, query) */
static int cmp_pair64(const void* a, const void* b) {
  const int64_t* x = (const int64_t*)a; const int64_t* y = (const int64_t*)b;
  if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
  return x[1] < y[1] ? -1 : (x[1] > y[1]);
}
/* order-independent digest of a pair set: the sum (mod 2^64) of fmix64(p << 32 | q) over the pairs
 * (p, q < 2^32) -- the whole-window check of windows too large to materialise (clustered C4: 2e9
 * pairs); the bench computes the same sum over the device's pairs */
static uint64_t pair_mix(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
  return k;
}
static int64_t join_pp_omp_core(const orc_grid* grid, int64_t no, const double* ox, const double* oy, int64_t nq,
                                const double* qx, const double* qy, double r, int metric, int nthreads,
                                int64_t* out_pairs, int64_t cap, uint64_t* digest);
int64_t orc_join_pp_omp(const orc_grid* grid, int64_t no, const double* ox, const double* oy, int64_t nq,
                        const double* qx, const double* qy, double r, int metric, int nthreads, int64_t* out_pairs,
                        int64_t cap) {
  return join_pp_omp_core(grid, no, ox, oy, nq, qx, qy, r, metric, nthreads, out_pairs, cap, NULL);
}
/* the pair count (return value) and *digest of the same join, without storing any pair */
int64_t orc_join_pp_omp_digest(const orc_grid* grid, int64_t no, const double* ox, const double* oy, int64_t nq,
                               const double* qx, const double* qy, double r, int metric, int nthreads,
                               uint64_t* digest) {
  return join_pp_omp_core(grid, no, ox, oy, nq, qx, qy, r, metric, nthreads, NULL, 0, digest);
}
static int64_t join_pp_omp_core(const orc_grid* grid, int64_t no, const double* ox, const double* oy, int64_t nq,
                                const double* qx, const double* qy, double r, int metric, int nthreads,
                                int64_t* out_pairs, int64_t cap, uint64_t* digest) {
  const int T = nthreads < 1 ? 1 : nthreads;
  const int32_t cl = orc_candidate_layers(grid, r);
  if (!(r > 0) || cl <= 0) return -1;
  const int64_t n = grid->n, W = n + 2;
  int64_t* off = (int64_t*)calloc((size_t)(W * W + 1), 8);
  int32_t* qc = (int32_t*)malloc(8 * (size_t)(nq > 0 ? nq : 1));
  for (int64_t q = 0; q < nq; q++) {
    int32_t a, b;
    orc_cell_of(grid, qx[q], qy[q], &a, &b);
    qc[2 * q] = a; qc[2 * q + 1] = b;
    const int64_t ka = a < -1 ? 0 : (a > n ? n + 1 : a + 1), kb = b < -1 ? 0 : (b > n ? n + 1 : b + 1);
    off[kb * W + ka + 1]++;
  }
  for (int64_t k = 0; k < W * W; k++) off[k + 1] += off[k];
  int64_t* lst = (int64_t*)malloc(8 * (size_t)(nq > 0 ? nq : 1));
  {
    int64_t* cur = (int64_t*)malloc(8 * (size_t)(W * W));
    memcpy(cur, off, 8 * (size_t)(W * W));
    for (int64_t q = 0; q < nq; q++) {
      const int32_t a = qc[2 * q], b = qc[2 * q + 1];
      const int64_t ka = a < -1 ? 0 : (a > n ? n + 1 : a + 1), kb = b < -1 ? 0 : (b > n ? n + 1 : b + 1);
      lst[cur[kb * W + ka]++] = q;
    }
    free(cur);
  }
  ovec* res = (ovec*)calloc((size_t)T, sizeof(ovec));
  uint64_t* dsum = (uint64_t*)calloc((size_t)T * 8, sizeof(uint64_t));  /* per thread: sum, count (own lines) */
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    uint64_t ds = 0, dc = 0;
    for (int64_t p = no * t / T; p < no * (t + 1) / T; p++) {
      int32_t a, b;
      orc_cell_of(grid, ox[p], oy[p], &a, &b);
      if (a < 0 || b < 0 || a >= n || b >= n) continue;  /* p.gridID must be a replicated key */
      const int64_t j0 = b - cl < -1 ? -1 : b - cl, j1 = b + cl > n ? n : b + cl;
      const int64_t i0 = a - cl < -1 ? -1 : a - cl, i1 = a + cl > n ? n : a + cl;
      for (int64_t j = j0; j <= j1; j++)
        for (int64_t u = off[(j + 1) * W + i0 + 1]; u < off[(j + 1) * W + i1 + 2]; u++) {
          const int64_t q = lst[u];
          const int64_t dx = (int64_t)qc[2 * q] - a, dy = (int64_t)qc[2 * q + 1] - b;
          if (dx > cl || dx < -cl || dy > cl || dy < -cl) continue;  /* clamped buckets */
          if (orc_distance(ox[p], oy[p], qx[q], qy[q], metric) <= r) {
            if (digest) {
              ds += pair_mix(((uint64_t)p << 32) | (uint64_t)q);
              dc++;
            } else {
              ovec_push(&res[t], p);
              ovec_push(&res[t], q);
            }
          }
        }
    }
    dsum[8 * t] = ds;
    dsum[8 * t + 1] = dc;
  }
  if (digest) {
    uint64_t ds = 0, dc = 0;
    for (int t = 0; t < T; t++) { ds += dsum[8 * t]; dc += dsum[8 * t + 1]; }
    *digest = ds;
    free(dsum); free(res); free(off); free(qc); free(lst);
    return (int64_t)dc;
  }
  free(dsum);
  int64_t tot = 0;
  for (int t = 0; t < T; t++) tot += res[t].n;
  int64_t* all = (int64_t*)malloc(8 * (size_t)(tot > 0 ? tot : 1));
  int64_t w = 0;
  for (int t = 0; t < T; t++) {
    if (res[t].n) memcpy(all + w, res[t].v, 8 * (size_t)res[t].n);
    w += res[t].n;
    free(res[t].v);
  }
  qsort(all, (size_t)(tot / 2), 16, cmp_pair64);
  const int64_t keep = tot < 2 * cap ? tot : 2 * cap;
  if (keep > 0) memcpy(out_pairs, all, 8 * (size_t)keep);
  free(all); free(res); free(off); free(qc); free(lst);
  return tot / 2;
}
