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
