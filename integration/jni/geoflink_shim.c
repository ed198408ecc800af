/*
 * geoflink_shim.c -- the plain-C core of the JNI shim (see geoflink_shim.h).
 * Built with any C compiler against include/geoflink_hip.h and the HIP runtime:
 *
 *   gcc -O2 -fPIC -c -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ integration/jni/geoflink_shim.c
 *
 * and linked into libgeoflink_jni.so together with geoflink_jni.c (which needs a JDK), or built
 * alone as integration/jni/libgeoflink_shim.so (Makefile target `shim`, no JDK), which
 * tests/test_shim_native.py drives through ctypes.
 */
#include "geoflink_shim.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

/* a device buffer grown on demand (never shrunk) */
typedef struct {
  void* p;
  size_t cap;
} dbuf;
static int dbuf_need(dbuf* b, size_t bytes) {
  if (b->p && b->cap >= bytes) return GF_OK;
  if (b->p) hipFree(b->p);
  b->p = NULL;
  b->cap = bytes > 4096 ? bytes + bytes / 4 : 4096;
  if (hipMalloc(&b->p, b->cap) != hipSuccess) {
    b->cap = 0;
    return GF_ERR_NOMEM;
  }
  return GF_OK;
}
static void dbuf_free(dbuf* b) {
  if (b->p) hipFree(b->p);
  b->p = NULL;
  b->cap = 0;
}
/* pinned (mapped) host memory grown on demand: kernels write it, the host reads it after a sync */
typedef struct {
  void* p;
  size_t cap;
} pbuf;
static int pbuf_need(pbuf* b, size_t bytes) {
  if (b->p && b->cap >= bytes) return GF_OK;
  if (b->p) gf_pinned_free(b->p);
  b->p = NULL;
  b->cap = bytes > 4096 ? bytes + bytes / 4 : 4096;
  int st = gf_pinned_alloc(b->cap, &b->p);
  if (st) b->cap = 0;
  return st;
}
static void pbuf_free(pbuf* b) {
  if (b->p) gf_pinned_free(b->p);
  b->p = NULL;
  b->cap = 0;
}

/* a device window of at least n points, grown (recreated) only when a window is larger */
typedef struct {
  gf_window* w;
  int64_t cap;
} cached_window;
static int window_for(gf_ctx* ctx, cached_window* c, int64_t n) {
  if (c->w && c->cap >= n) return GF_OK;
  if (c->w) gf_window_destroy(c->w);
  c->w = NULL;
  c->cap = n > 1024 ? n + n / 4 : 1024;
  return gf_window_create(ctx, c->cap, &c->w);
}
/* upload the given columns (ts never: window evaluation does not read it) -> device points,
 * ordered after the copy on the context's streams */
/* An objID column in pinned memory (shim_pinned_alloc: the direct buffer the Java side fills) is
 * read in place by the kernels -- 16 B per point cross PCIe instead of 24 (only the candidates'
 * objIDs are read); any other column is copied. */
static int upload(gf_ctx* ctx, cached_window* c, const double* x, const double* y, const int64_t* objID, int64_t n,
                  gf_points* pts) {
  int st = window_for(ctx, c, n), pinned = 0;
  if (!st && objID && n > 0) st = gf_host_pinned(objID, &pinned);
  if (!st) st = pinned ? gf_window_upload_mapped(c->w, x, y, objID, n) : gf_window_upload(c->w, x, y, objID, NULL, n);
  if (!st) st = gf_window_points(c->w, pts);
  return st;
}
static void window_free(cached_window* c) {
  if (c->w) gf_window_destroy(c->w);
  c->w = NULL;
  c->cap = 0;
}

struct shim_ctx {
  gf_ctx* ctx;
  int device;
  char err[256];
  cached_window wo, wq;   /* join windows (ordinary / query or point side) */
  dbuf pairs;             /* device join pairs */
  pbuf hpairs;            /* their pinned host copy (shim_join_window's *pairs) */
  int64_t pair_hint;      /* capacity of the last join's pairs */
  dbuf text, cols;        /* ingest: device text, 4 device columns */
};

/* a copy ordered on the context's stream (after the work enqueued there, before what follows) */
static int copy(shim_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  return hipMemcpyAsync(dst, src, bytes, kind, (hipStream_t)gf_ctx_stream(c->ctx)) != hipSuccess;
}

static int fail(shim_ctx* c, int st, const char* what) {
  if (st && c) {
    const char* e = c->ctx ? gf_ctx_last_error(c->ctx) : "";
    snprintf(c->err, sizeof c->err, "%s: %s%s%s", what, gf_status_string(st), e && *e ? ": " : "", e ? e : "");
  }
  return st;
}

int shim_ctx_create(int device, shim_ctx** out) {
  *out = NULL;
  shim_ctx* c = (shim_ctx*)calloc(1, sizeof(shim_ctx));
  if (!c) return GF_ERR_NOMEM;
  int st = gf_ctx_create(device, &c->ctx);
  if (st) {
    free(c);
    return st;
  }
  c->device = device;
  *out = c;
  return GF_OK;
}

void shim_ctx_destroy(shim_ctx* c) {
  if (!c) return;
  gf_ctx_synchronize(c->ctx);
  window_free(&c->wo);
  window_free(&c->wq);
  dbuf_free(&c->pairs);
  pbuf_free(&c->hpairs);
  dbuf_free(&c->text);
  dbuf_free(&c->cols);
  gf_ctx_destroy(c->ctx);
  free(c);
}

const char* shim_last_error(shim_ctx* c) { return c ? c->err : "null context"; }
gf_ctx* shim_gf_ctx(shim_ctx* c) { return c ? c->ctx : NULL; }

/* ---- objID ------------------------------------------------------------------------------ */
int shim_objid_intern(shim_ctx* c, const char* bytes, const int64_t* offs, int64_t n, int64_t* keys) {
  gf_objid_dict* d = NULL;
  int st = gf_ctx_objid_dict(c->ctx, &d);
  if (!st) st = gf_objid_intern(d, bytes, offs, n, keys);
  return fail(c, st, "objidIntern");
}
int shim_objid_decode(shim_ctx* c, const int64_t* keys, int64_t n, char* buf, int64_t cap, int64_t* offs) {
  gf_objid_dict* d = NULL;
  int st = gf_ctx_objid_dict(c->ctx, &d);
  if (!st) st = gf_objid_decode(d, keys, n, buf, cap, offs);
  return st == GF_ERR_CAPACITY ? st : fail(c, st, "objidDecode");
}

/* ---- kNN -------------------------------------------------------------------------------- */
/* the batched sharded path (shim_knn_sharded_*): 2B slots, groups of B consecutive tickets */
#define SHIM_SHARD_MAX_BATCH 32
typedef struct {
  shim_comm* comm;
  int32_t B;
  int64_t cap_bytes;
  size_t rb, sb;                 /* record / string record bytes */
  cached_window win[2 * SHIM_SHARD_MAX_BATCH];
  gf_points pts[2 * SHIM_SHARD_MAX_BATCH];
  int64_t base[2 * SHIM_SHARD_MAX_BATCH], npts[2 * SHIM_SHARD_MAX_BATCH];
  int64_t ticket[2 * SHIM_SHARD_MAX_BATCH];  /* the ticket in the slot, -1 when read (free) */
  dbuf rec;                      /* 2B device records */
  pbuf merged;                   /* 2B merged string records (mapped pinned) */
  dbuf one;                      /* one exact record, for a flagged window's second exchange */
  pbuf one_merged;
  char* strbuf;                  /* decode scratch: the Strings of one merged record */
  int64_t* strofs;
  int64_t next, exchanged, synced;
} shard_state;

struct shim_knn {
  shim_ctx* c;
  gf_knn_plan* plan;
  int32_t k;
  cached_window win;
  dbuf rec;     /* sharded windows: this rank's device record */
  pbuf merged;  /* ... and the merged record of all ranks (mapped pinned) */
  shard_state* sh;
};

int shim_knn_plan(shim_ctx* c, const gf_grid* g, double qx, double qy, double r, int32_t k, shim_knn** out) {
  *out = NULL;
  shim_knn* h = (shim_knn*)calloc(1, sizeof(shim_knn));
  if (!h) return GF_ERR_NOMEM;
  int st = gf_knn_pp_plan_create(c->ctx, g, qx, qy, r, k, GF_METRIC_SQRT, &h->plan);
  if (st) {
    free(h);
    return fail(c, st, "knnPlan");
  }
  h->c = c;
  h->k = k;
  *out = h;
  return GF_OK;
}

int shim_knn_polygon_plan(shim_ctx* c, const gf_grid* g, const gf_polygons* poly, double r, int32_t k,
                          int approximate, shim_knn** out) {
  *out = NULL;
  shim_knn* h = (shim_knn*)calloc(1, sizeof(shim_knn));
  if (!h) return GF_ERR_NOMEM;
  int st = gf_knn_ppoly_plan_create(c->ctx, g, poly, r, k, approximate, GF_METRIC_SQRT, &h->plan);
  if (st) {
    free(h);
    return fail(c, st, "knnPolygonPlan");
  }
  h->c = c;
  h->k = k;
  *out = h;
  return GF_OK;
}

static void shard_free(shard_state* sh) {
  if (!sh) return;
  for (int i = 0; i < 2 * SHIM_SHARD_MAX_BATCH; ++i) window_free(&sh->win[i]);
  dbuf_free(&sh->rec);
  pbuf_free(&sh->merged);
  dbuf_free(&sh->one);
  pbuf_free(&sh->one_merged);
  free(sh->strbuf);
  free(sh->strofs);
  free(sh);
}

void shim_knn_destroy(shim_knn* h) {
  if (!h) return;
  gf_ctx_synchronize(h->c->ctx);
  window_free(&h->win);
  dbuf_free(&h->rec);
  pbuf_free(&h->merged);
  shard_free(h->sh);
  gf_knn_plan_destroy(h->plan);
  free(h);
}

int32_t shim_knn_k(const shim_knn* h) { return h ? h->k : 0; }

int shim_knn_window(shim_knn* h, const double* x, const double* y, const int64_t* objID, int64_t n, int64_t* out_objID,
                    double* out_dist, int64_t* out_idx, int32_t* m) {
  gf_points pts;
  *m = 0;
  int st = upload(h->c->ctx, &h->win, x, y, objID, n, &pts);
  if (!st) st = gf_knn_run(h->plan, &pts, out_objID, out_dist, out_idx, m);
  return fail(h->c, st, "knnWindow");
}

/* ---- multi-GPU kNN: one Flink subtask per GPU, the window sharded by cell-column bands; the
 * windowAll merge (PointPointKNNQuery.java:198-200, KNNQuery.java:213-272) is the RCCL record
 * exchange behind the C ABI (gf_knn_exchange_batch) -------------------------------------------- */
struct shim_comm {
  gf_comm* comm;
};

int shim_comm_unique_id(uint8_t* id) { return gf_comm_unique_id(id); }

int shim_comm_create(shim_ctx* c, const uint8_t* id, int32_t nranks, int32_t rank, shim_comm** out) {
  *out = NULL;
  shim_comm* h = (shim_comm*)calloc(1, sizeof(shim_comm));
  if (!h) return GF_ERR_NOMEM;
  int st = gf_comm_create(id, nranks, rank, c->device, &h->comm);
  if (st) {
    free(h);
    snprintf(c->err, sizeof c->err, "commCreate: %s: %s", gf_status_string(st), gf_comm_last_error(NULL));
    return st;
  }
  *out = h;
  return GF_OK;
}

int shim_comm_create_all(int32_t ndev, const int* devices, shim_comm** out) {
  gf_comm* cs[64];
  if (ndev < 1 || ndev > 64) return GF_ERR_ARG;
  for (int32_t i = 0; i < ndev; ++i) out[i] = NULL;
  int st = gf_comm_create_all(ndev, devices, cs);
  for (int32_t i = 0; !st && i < ndev; ++i) {
    out[i] = (shim_comm*)calloc(1, sizeof(shim_comm));
    if (!out[i]) st = GF_ERR_NOMEM;
    else out[i]->comm = cs[i];
  }
  if (st) {
    for (int32_t i = 0; i < ndev; ++i) {
      if (out[i]) free(out[i]);
      out[i] = NULL;
    }
  }
  return st;
}

void shim_comm_destroy(shim_comm* h) {
  if (!h) return;
  gf_comm_destroy(h->comm);
  free(h);
}

/* host lists -> a final record (status 0) in the rank's device record, for the second exchange */
static int put_exact_record(shim_knn* h, const int64_t* o, const double* d, const int64_t* ix, int32_t m) {
  const int32_t k = h->k;
  const size_t rb = gf_knn_result_bytes(k);
  char* rec = (char*)calloc(1, rb);
  if (!rec) return GF_ERR_NOMEM;
  gf_knn_header* hd = (gf_knn_header*)rec;
  hd->status = 0;
  hd->n = m;
  hd->k = k;
  double* rd = (double*)(hd + 1);
  int64_t* ro = (int64_t*)(rd + k);
  int64_t* ri = ro + k;
  memcpy(rd, d, sizeof(double) * (size_t)m);
  memcpy(ro, o, sizeof(int64_t) * (size_t)m);
  memcpy(ri, ix, sizeof(int64_t) * (size_t)m);
  int st = copy(h->c, h->rec.p, rec, rb, hipMemcpyHostToDevice) ? GF_ERR_HIP : GF_OK;
  if (!st) st = gf_ctx_synchronize(h->c->ctx);  /* rec (host) is freed below */
  free(rec);
  return st;
}

int shim_knn_window_sharded(shim_knn* h, shim_comm* comm, const double* x, const double* y, const int64_t* objID,
                            int64_t n, int64_t index_base, int64_t* out_objID, double* out_dist, int64_t* out_idx,
                            int32_t* m) {
  gf_ctx* ctx = h->c->ctx;
  const int32_t k = h->k;
  const size_t rb = gf_knn_result_bytes(k);
  gf_points pts;
  *m = 0;
  int st = upload(ctx, &h->win, x, y, objID, n, &pts);
  if (!st) st = dbuf_need(&h->rec, rb);
  if (!st) st = pbuf_need(&h->merged, rb);
  if (!st) st = gf_knn_plan_set_index_base(h->plan, index_base);
  if (!st) st = gf_knn_enqueue(h->plan, &pts, h->rec.p);
  if (!st) st = gf_knn_plan_flush(h->plan);
  if (!st) st = gf_knn_exchange_batch(comm->comm, ctx, k, h->rec.p, 1, h->merged.p);
  if (!st) st = gf_ctx_synchronize(ctx);
  if (!st && ((const gf_knn_header*)h->merged.p)->status == 1) {
    /* some rank's record needed the exact re-evaluation: the merged record is the same on every
     * rank, so every rank takes this branch -- each re-evaluates its shard exactly (the local
     * record, fetched into the merged buffer) and the ranks exchange again */
    if (copy(h->c, h->merged.p, h->rec.p, rb, hipMemcpyDeviceToHost)) st = GF_ERR_HIP;
    if (!st) st = gf_ctx_synchronize(ctx);
    if (!st) st = gf_knn_decode(h->plan, &pts, h->merged.p, out_objID, out_dist, out_idx, m);
    if (!st) st = put_exact_record(h, out_objID, out_dist, out_idx, *m);
    if (!st) st = gf_knn_exchange_batch(comm->comm, ctx, k, h->rec.p, 1, h->merged.p);
    if (!st) st = gf_ctx_synchronize(ctx);
    *m = 0;
  }
  if (!st && ((const gf_knn_header*)h->merged.p)->status != 0) st = GF_ERR_ARG;  /* 2: dictionary keys */
  if (!st) st = gf_knn_decode(h->plan, &pts, h->merged.p, out_objID, out_dist, out_idx, m);
  /* every exit path: the next knnWindow on this plan reports window-local indices */
  const int st0 = gf_knn_plan_set_index_base(h->plan, 0);
  return fail(h->c, st ? st : st0, "knnWindowSharded");
}

/* ---- the batched sharded path ------------------------------------------------------------ */
int shim_knn_sharded_begin(shim_knn* h, shim_comm* comm, int32_t batch, int64_t cap_bytes) {
  if (!h || !comm || batch < 1 || batch > SHIM_SHARD_MAX_BATCH || cap_bytes < 0 || cap_bytes > (1 << 24))
    return fail(h ? h->c : NULL, GF_ERR_ARG, "knnShardedBegin: bad argument");
  if (h->sh) return fail(h->c, GF_ERR_ARG, "knnShardedBegin: already begun on this plan");
  shard_state* sh = (shard_state*)calloc(1, sizeof(shard_state));
  if (!sh) return GF_ERR_NOMEM;
  sh->comm = comm;
  sh->B = batch;
  sh->cap_bytes = cap_bytes;
  sh->rb = gf_knn_result_bytes(h->k);
  sh->sb = gf_knn_string_record_bytes(h->k, cap_bytes);
  for (int i = 0; i < 2 * SHIM_SHARD_MAX_BATCH; ++i) sh->ticket[i] = -1;
  int st = dbuf_need(&sh->rec, 2 * (size_t)batch * sh->rb);
  if (!st) st = pbuf_need(&sh->merged, 2 * (size_t)batch * sh->sb);
  if (!st) st = dbuf_need(&sh->one, sh->rb);
  if (!st) st = pbuf_need(&sh->one_merged, sh->sb);
  sh->strbuf = (char*)malloc((size_t)cap_bytes + 64);
  sh->strofs = (int64_t*)malloc(sizeof(int64_t) * ((size_t)h->k + 1));
  if (!st && (!sh->strbuf || !sh->strofs)) st = GF_ERR_NOMEM;
  if (st) {
    shard_free(sh);
    return fail(h->c, st, "knnShardedBegin");
  }
  h->sh = sh;
  return GF_OK;
}

/* one exchange of the enqueued, not yet exchanged windows (a group's slots are contiguous: groups
 * start at multiples of B, and a flushed partial group skips the rest of its tickets) */
static int shard_exchange(shim_knn* h) {
  shard_state* sh = h->sh;
  const int64_t n = sh->next - sh->exchanged;
  if (n <= 0) return GF_OK;
  gf_objid_dict* dict = NULL;
  const size_t s0 = (size_t)(sh->exchanged % (2 * sh->B));
  int st = gf_knn_plan_flush(h->plan);  /* pipelined plans: the group's last records complete */
  if (!st) st = gf_ctx_objid_dict(h->c->ctx, &dict);
  if (!st)
    st = gf_knn_exchange_strings_batch(sh->comm->comm, dict, h->k, sh->cap_bytes, (char*)sh->rec.p + s0 * sh->rb,
                                       (int32_t)n, (char*)sh->merged.p + s0 * sh->sb);
  if (st) return st;
  sh->exchanged = sh->next = (sh->next + sh->B - 1) / sh->B * sh->B;
  return GF_OK;
}

int shim_knn_sharded_enqueue(shim_knn* h, const double* x, const double* y, const int64_t* objID, int64_t n,
                             int64_t index_base, int64_t* ticket) {
  shard_state* sh = h->sh;
  *ticket = -1;
  if (!sh) return fail(h->c, GF_ERR_ARG, "knnShardedEnqueue: knnShardedBegin first");
  const int64_t t = sh->next;
  const int s = (int)(t % (2 * sh->B));
  if (sh->ticket[s] >= 0) return fail(h->c, GF_ERR_ARG, "knnShardedEnqueue: the result of the window 2B back is unread");
  int st = upload(h->c->ctx, &sh->win[s], x, y, objID, n, &sh->pts[s]);
  if (!st) st = gf_knn_plan_set_index_base(h->plan, index_base);
  if (!st) st = gf_knn_enqueue(h->plan, &sh->pts[s], (char*)sh->rec.p + (size_t)s * sh->rb);
  const int st0 = gf_knn_plan_set_index_base(h->plan, 0);
  if (!st) st = st0;
  if (st) return fail(h->c, st, "knnShardedEnqueue");
  sh->ticket[s] = t;
  sh->base[s] = index_base;
  sh->npts[s] = n;
  sh->next = t + 1;
  *ticket = t;
  if (sh->next % sh->B == 0) st = shard_exchange(h);  /* the group is complete: its exchange */
  return fail(h->c, st, "knnShardedEnqueue");
}

int shim_knn_sharded_flush(shim_knn* h) {
  if (!h->sh) return fail(h->c, GF_ERR_ARG, "knnShardedFlush: knnShardedBegin first");
  return fail(h->c, shard_exchange(h), "knnShardedFlush");
}

/* a merged string record -> entries (dist, idx) and which of them this rank's band holds */
static int shard_decode(shim_knn* h, const void* rec, int s, double* dist, int64_t* idx, int32_t* owned, int32_t* m,
                        int32_t* status) {
  shard_state* sh = h->sh;
  int st = gf_knn_string_record_decode(rec, h->k, sh->cap_bytes, status, NULL, dist, idx, sh->strbuf,
                                       sh->cap_bytes + 64, sh->strofs, m);
  if (st || *status != 0) return st;
  for (int32_t i = 0; i < *m; ++i) owned[i] = idx[i] >= sh->base[s] && idx[i] < sh->base[s] + sh->npts[s];
  return GF_OK;
}

int shim_knn_sharded_result(shim_knn* h, int64_t ticket, double* out_dist, int64_t* out_idx, int32_t* owned,
                            int32_t* m) {
  shard_state* sh = h->sh;
  *m = 0;
  if (!sh) return fail(h->c, GF_ERR_ARG, "knnShardedResult: knnShardedBegin first");
  const int s = (int)(ticket % (2 * sh->B));
  if (ticket < 0 || ticket >= sh->exchanged || sh->ticket[s] != ticket)
    return fail(h->c, GF_ERR_ARG, "knnShardedResult: ticket not exchanged yet (knnShardedFlush) or already read");
  gf_ctx* ctx = h->c->ctx;
  int st = GF_OK;
  if (ticket >= sh->synced) {  /* one host wait per group */
    st = gf_ctx_synchronize(ctx);
    if (st) return fail(h->c, st, "knnShardedResult");
    sh->synced = sh->exchanged;
  }
  int32_t status = 0;
  st = shard_decode(h, (const char*)sh->merged.p + (size_t)s * sh->sb, s, out_dist, out_idx, owned, m, &status);
  if (!st && status == 1) {
    /* some rank's record needed the exact re-evaluation: every rank sees the same merged status,
     * re-evaluates its band exactly (its local record, on the host) and the ranks exchange the
     * exact records of this window once more */
    gf_objid_dict* dict = NULL;
    void* local = malloc(sh->rb);
    int64_t* lo = (int64_t*)malloc(sizeof(int64_t) * (size_t)h->k);
    double* ld = (double*)malloc(sizeof(double) * (size_t)h->k);
    int64_t* li = (int64_t*)malloc(sizeof(int64_t) * (size_t)h->k);
    int32_t lm = 0;
    if (!local || !lo || !ld || !li) st = GF_ERR_NOMEM;
    if (!st && copy(h->c, local, (char*)sh->rec.p + (size_t)s * sh->rb, sh->rb, hipMemcpyDeviceToHost)) st = GF_ERR_HIP;
    if (!st) st = gf_ctx_synchronize(ctx);
    if (!st) st = gf_knn_plan_set_index_base(h->plan, sh->base[s]);
    if (!st) st = gf_knn_decode(h->plan, &sh->pts[s], local, lo, ld, li, &lm);
    const int st0 = gf_knn_plan_set_index_base(h->plan, 0);
    if (!st) st = st0;
    if (!st) {
      gf_knn_header* hd = (gf_knn_header*)local;
      memset(local, 0, sh->rb);
      hd->status = 0;
      hd->n = lm;
      hd->k = h->k;
      double* rd = (double*)(hd + 1);
      memcpy(rd, ld, sizeof(double) * (size_t)lm);
      memcpy(rd + h->k, lo, sizeof(int64_t) * (size_t)lm);
      memcpy((int64_t*)(rd + h->k) + h->k, li, sizeof(int64_t) * (size_t)lm);
      if (copy(h->c, sh->one.p, local, sh->rb, hipMemcpyHostToDevice)) st = GF_ERR_HIP;
    }
    if (!st) st = gf_ctx_objid_dict(ctx, &dict);
    if (!st) st = gf_knn_exchange_strings_batch(sh->comm->comm, dict, h->k, sh->cap_bytes, sh->one.p, 1, sh->one_merged.p);
    if (!st) st = gf_ctx_synchronize(ctx);  /* (local is freed below) */
    free(local); free(lo); free(ld); free(li);
    if (!st) st = shard_decode(h, sh->one_merged.p, s, out_dist, out_idx, owned, m, &status);
  }
  if (!st && status != 0) st = status == GF_KNN_STATUS_FOREIGN_KEYS ? GF_ERR_CAPACITY : GF_ERR_ARG;
  if (st) *m = 0;
  else sh->ticket[s] = -1;  /* read: the slot may take window ticket + 2B */
  return fail(h->c, st, "knnShardedResult");
}

/* ---- sliding kNN -------------------------------------------------------------------------- */
#define SHIM_SLIDE_RECS 8
struct shim_sliding {
  shim_knn* plan;
  gf_knn_sliding* s;
  int64_t pane_ms;
  int32_t nwin;           /* device pane windows kept (the engine's ring borrows them) */
  cached_window* wins;
  void* rec[SHIM_SLIDE_RECS];      /* pinned window records */
  int64_t rec_end[SHIM_SLIDE_RECS];
  int32_t next;
  int64_t pending_end;    /* depth 2: the window whose record the next push / flush completes */
};

int shim_sliding_create(shim_knn* plan, int64_t size_ms, int64_t slide_ms, shim_sliding** out) {
  *out = NULL;
  shim_sliding* s = (shim_sliding*)calloc(1, sizeof(shim_sliding));
  if (!s) return GF_ERR_NOMEM;
  s->plan = plan;
  s->pending_end = -1;
  int32_t ppw = 0, pps = 0, ring = 0;
  int st = gf_knn_plan_set_pipeline(plan->plan, 2);  /* one fused launch per pane */
  if (!st) st = gf_knn_sliding_create(plan->plan, size_ms, slide_ms, &s->s);
  if (!st) st = gf_knn_sliding_geometry(s->s, &s->pane_ms, &ppw, &pps, &ring);
  if (!st) {
    s->nwin = ring + 1;
    s->wins = (cached_window*)calloc((size_t)s->nwin, sizeof(cached_window));
    if (!s->wins) st = GF_ERR_NOMEM;
  }
  for (int i = 0; i < SHIM_SLIDE_RECS; ++i) s->rec_end[i] = -1;
  for (int i = 0; !st && i < SHIM_SLIDE_RECS; ++i) st = gf_pinned_alloc(gf_knn_result_bytes(plan->k), &s->rec[i]);
  if (st) {
    shim_sliding_destroy(s);
    return fail(plan->c, st, "knnSlidingCreate");
  }
  *out = s;
  return GF_OK;
}

void shim_sliding_destroy(shim_sliding* s) {
  if (!s) return;
  gf_ctx_synchronize(s->plan->c->ctx);
  if (s->s) gf_knn_sliding_destroy(s->s);
  for (int32_t i = 0; s->wins && i < s->nwin; ++i) window_free(&s->wins[i]);
  free(s->wins);
  for (int i = 0; i < SHIM_SLIDE_RECS; ++i)
    if (s->rec[i]) gf_pinned_free(s->rec[i]);
  free(s);
}

int shim_sliding_pane_ms(const shim_sliding* s, int64_t* pane_ms) {
  *pane_ms = s->pane_ms;
  return GF_OK;
}

int shim_sliding_push(shim_sliding* s, int64_t pane_index, const double* x, const double* y, const int64_t* objID,
                      int64_t n, int32_t* closed, int64_t* window_end) {
  gf_ctx* ctx = s->plan->c->ctx;
  gf_points pts;
  memset(&pts, 0, sizeof pts);
  *closed = 0;
  int st = GF_OK;
  /* floor mod: panes before the epoch (negative timestamps) have negative indices */
  const int64_t slot = ((pane_index % s->nwin) + s->nwin) % s->nwin;
  if (n > 0) st = upload(ctx, &s->wins[slot], x, y, objID, n, &pts);
  const int32_t k = s->next % SHIM_SLIDE_RECS;
  if (!st) st = gf_knn_sliding_push(s->s, pane_index, &pts, s->rec[k], closed, window_end);
  if (st) return fail(s->plan->c, st, "knnSlidingPush");
  s->pending_end = -1;  /* this push completed the previous window's record */
  if (*closed) {
    s->rec_end[k] = *window_end;
    s->pending_end = *window_end;
    s->next++;
  }
  return GF_OK;
}

shim_knn* shim_sliding_plan(shim_sliding* s) { return s ? s->plan : NULL; }

int shim_sliding_flush(shim_sliding* s) {
  int st = gf_knn_sliding_flush(s->s);
  if (!st) s->pending_end = -1;
  return fail(s->plan->c, st, "knnSlidingFlush");
}

int shim_sliding_decode(shim_sliding* s, int64_t window_end, int64_t* out_objID, double* out_dist, int64_t* out_idx,
                        int32_t* m) {
  *m = 0;
  int k = -1;
  for (int i = 0; i < SHIM_SLIDE_RECS; ++i)
    if (s->rec_end[i] == window_end) k = i;
  if (k < 0) return fail(s->plan->c, GF_ERR_ARG, "knnSlidingDecode: no such closed window (decode within 8 windows)");
  int st = GF_OK;
  if (s->pending_end == window_end) st = shim_sliding_flush(s);  /* its record is written by the flush */
  if (!st) st = gf_ctx_synchronize(s->plan->c->ctx);
  if (!st) st = gf_knn_sliding_decode(s->s, window_end, s->rec[k], out_objID, out_dist, out_idx, m);
  return fail(s->plan->c, st, "knnSlidingDecode");
}

/* ---- range ------------------------------------------------------------------------------ */
struct shim_range {
  shim_ctx* c;
  gf_range_plan* plan;
  cached_window win;
  dbuf bitmap;
  pbuf idx;      /* pinned: the index list written by the device, then the count */
  int multi;     /* approximate point plan with |Q| > 1: candidate-cell points emitted |Q| times */
  dbuf mbitmap;
  pbuf midx;     /* pinned: the last window's multiplicity list, then its count */
  int64_t mcount;
};

static int range_new(shim_ctx* c, gf_range_plan* plan, int st, shim_range** out, const char* what) {
  *out = NULL;
  shim_range* h = st ? NULL : (shim_range*)calloc(1, sizeof(shim_range));
  if (st || !h) {
    if (plan) gf_range_plan_destroy(plan);
    return fail(c, st ? st : GF_ERR_NOMEM, what);
  }
  h->c = c;
  h->plan = plan;
  *out = h;
  return GF_OK;
}

int shim_range_plan(shim_ctx* c, const gf_grid* g, const double* qx, const double* qy, int32_t nq, double r,
                    int approximate, shim_range** out) {
  gf_range_plan* plan = NULL;
  int st = gf_range_pp_plan_create(c->ctx, g, qx, qy, nq, r, approximate, GF_METRIC_SQRT, &plan);
  st = range_new(c, plan, st, out, "rangePlan");
  if (!st) (*out)->multi = approximate && nq > 1;
  return st;
}

int shim_range_polygon_plan(shim_ctx* c, const gf_grid* g, const gf_polygons* polys, double r, int approximate,
                            shim_range** out) {
  gf_range_plan* plan = NULL;
  int st = gf_range_ppoly_plan_create(c->ctx, g, polys, r, approximate, GF_METRIC_SQRT, &plan);
  return range_new(c, plan, st, out, "rangePolygonPlan");
}

void shim_range_destroy(shim_range* h) {
  if (!h) return;
  gf_ctx_synchronize(h->c->ctx);
  window_free(&h->win);
  dbuf_free(&h->bitmap);
  pbuf_free(&h->idx);
  dbuf_free(&h->mbitmap);
  pbuf_free(&h->midx);
  gf_range_plan_destroy(h->plan);
  free(h);
}

int shim_range_window(shim_range* h, const double* x, const double* y, int64_t n, int32_t* out_idx, int64_t cap,
                      int64_t* count) {
  gf_points pts;
  *count = 0;
  h->mcount = 0;
  const size_t lcap = 4 * (size_t)(n > 0 ? n : 1) + 16;  /* an index list of n, then its count */
  int st = upload(h->c->ctx, &h->win, x, y, NULL, n, &pts);
  if (!st) st = dbuf_need(&h->bitmap, 8 * (size_t)((n + 63) / 64 + 1));
  if (!st) st = pbuf_need(&h->idx, lcap);
  if (!st && h->multi) st = dbuf_need(&h->mbitmap, 8 * (size_t)((n + 63) / 64 + 1));
  if (!st && h->multi) st = pbuf_need(&h->midx, lcap);
  if (!st) st = gf_range_run(h->plan, &pts, (uint64_t*)h->bitmap.p, h->multi ? (uint64_t*)h->mbitmap.p : NULL, NULL);
  /* the index list straight into pinned host memory, its count after it: one sync */
  int64_t* dcount = (int64_t*)((char*)h->idx.p + ((4 * (size_t)(n > 0 ? n : 1) + 7) / 8) * 8);
  int64_t* mcount = h->multi ? (int64_t*)((char*)h->midx.p + ((4 * (size_t)(n > 0 ? n : 1) + 7) / 8) * 8) : NULL;
  if (!st) st = gf_bitmap_to_indices_async(h->c->ctx, (const uint64_t*)h->bitmap.p, n, (uint32_t*)h->idx.p, n, dcount);
  if (!st && h->multi)
    st = gf_bitmap_to_indices_async(h->c->ctx, (const uint64_t*)h->mbitmap.p, n, (uint32_t*)h->midx.p, n, mcount);
  if (!st) st = gf_ctx_synchronize(h->c->ctx);
  if (st) return fail(h->c, st, "rangeWindow");
  if (mcount) h->mcount = *mcount;
  *count = *dcount;
  memcpy(out_idx, h->idx.p, 4 * (size_t)(*count < cap ? *count : cap));
  return *count > cap ? GF_ERR_CAPACITY : GF_OK;
}

int shim_range_window_multi(shim_range* h, int32_t* out_idx, int64_t cap, int64_t* count) {
  *count = h->multi ? h->mcount : 0;
  if (*count > 0) memcpy(out_idx, h->midx.p, 4 * (size_t)(*count < cap ? *count : cap));
  return *count > cap ? GF_ERR_CAPACITY : GF_OK;
}

/* ---- sliding range ---------------------------------------------------------------------- */
struct shim_range_sliding {
  shim_range* plan;
  gf_range_sliding* s;
  int64_t pane_ms;
  cached_window win[2];   /* pane uploads alternate (each is ordered after the work before it) */
  int32_t next;
  pbuf idx;               /* pinned: the closed window's index list, then its count */
};

/* pinned staging of a window: cap uint32 indices, then the int64 count (8-byte aligned) */
static int64_t slide_cap(const pbuf* b) { return (int64_t)((b->cap - 16) / 4); }
static int64_t* slide_count(const pbuf* b) {
  return (int64_t*)((char*)b->p + ((4 * (size_t)slide_cap(b) + 7) & ~(size_t)7));
}

int shim_range_sliding_create(shim_range* plan, int64_t size_ms, int64_t slide_ms, shim_range_sliding** out) {
  *out = NULL;
  shim_range_sliding* s = (shim_range_sliding*)calloc(1, sizeof(shim_range_sliding));
  if (!s) return GF_ERR_NOMEM;
  s->plan = plan;
  int st = gf_range_sliding_create(plan->plan, size_ms, slide_ms, &s->s);
  if (!st) st = gf_range_sliding_geometry(s->s, &s->pane_ms, NULL, NULL);
  if (!st) st = pbuf_need(&s->idx, 4096);
  if (st) {
    shim_range_sliding_destroy(s);
    return fail(plan->c, st, "rangeSlidingCreate");
  }
  *out = s;
  return GF_OK;
}

void shim_range_sliding_destroy(shim_range_sliding* s) {
  if (!s) return;
  gf_ctx_synchronize(s->plan->c->ctx);
  if (s->s) gf_range_sliding_destroy(s->s);
  window_free(&s->win[0]);
  window_free(&s->win[1]);
  pbuf_free(&s->idx);
  free(s);
}

int shim_range_sliding_pane_ms(const shim_range_sliding* s, int64_t* pane_ms) {
  *pane_ms = s->pane_ms;
  return GF_OK;
}

int shim_range_sliding_push(shim_range_sliding* s, int64_t pane_index, const double* x, const double* y, int64_t n,
                            int64_t* window_end, const uint32_t** idx, int64_t* count) {
  gf_ctx* ctx = s->plan->c->ctx;
  gf_points pts;
  memset(&pts, 0, sizeof pts);
  *window_end = -1;
  *idx = NULL;
  *count = 0;
  int st = GF_OK;
  if (n > 0) st = upload(ctx, &s->win[s->next++ & 1], x, y, NULL, n, &pts);
  int32_t closed = 0;
  int64_t end = -1, wn = 0;
  for (;;) {  /* the staging holds the window's index list, then its count */
    st = st ? st
            : gf_range_sliding_push(s->s, pane_index, &pts, (uint32_t*)s->idx.p, slide_cap(&s->idx),
                                    slide_count(&s->idx), &closed, &end, &wn);
    if (st != GF_ERR_CAPACITY) break;
    st = pbuf_need(&s->idx, 4 * (size_t)wn + 32);  /* nothing was enqueued: push the pane again */
  }
  if (!st && closed) st = gf_ctx_synchronize(ctx);
  if (st) return fail(s->plan->c, st, "rangeSlidingPush");
  if (closed) {
    *window_end = end;
    *idx = (const uint32_t*)s->idx.p;
    *count = *slide_count(&s->idx);
  }
  return GF_OK;
}

/* ---- joins ------------------------------------------------------------------------------ */
/* pairs of a join run into the context's device buffer, sized from the last join (grown and
 * re-run once on GF_ERR_CAPACITY), then copied to the pinned staging *pairs */
typedef int (*join_fn)(shim_ctx* c, const void* a, uint32_t* pairs, int64_t cap, int64_t* m);
static int join_common(shim_ctx* c, join_fn fn, const void* a, const uint32_t** pairs, int64_t* m, const char* what) {
  *pairs = NULL;
  *m = 0;
  int64_t cap = c->pair_hint > 1024 ? c->pair_hint + c->pair_hint / 8 : 1 << 16;
  int st = dbuf_need(&c->pairs, 8 * (size_t)cap);
  if (!st) st = fn(c, a, (uint32_t*)c->pairs.p, cap, m);
  if (st == GF_ERR_CAPACITY) {
    cap = *m + *m / 8 + 1024;
    st = dbuf_need(&c->pairs, 8 * (size_t)cap);
    if (!st) st = fn(c, a, (uint32_t*)c->pairs.p, cap, m);
  }
  if (!st) st = pbuf_need(&c->hpairs, 8 * (size_t)(*m > 0 ? *m : 1));
  if (!st && *m > 0 && copy(c, c->hpairs.p, c->pairs.p, 8 * (size_t)*m, hipMemcpyDeviceToHost)) st = GF_ERR_HIP;
  if (!st) st = gf_ctx_synchronize(c->ctx);
  if (st) return fail(c, st, what);
  c->pair_hint = *m;
  *pairs = (const uint32_t*)c->hpairs.p;
  return GF_OK;
}

typedef struct {
  const gf_grid *ug, *qg;
  gf_points po, pq;
  double r;
  int approximate;
} pp_args;
static int run_pp(shim_ctx* c, const void* a_, uint32_t* pairs, int64_t cap, int64_t* m) {
  const pp_args* a = (const pp_args*)a_;
  return gf_join_pp(c->ctx, a->ug, a->qg, &a->po, &a->pq, a->r, a->approximate, GF_METRIC_SQRT, pairs, cap, m);
}

int shim_join_window(shim_ctx* c, const gf_grid* ug, const gf_grid* qg, const double* ox, const double* oy, int64_t no,
                     const double* qx, const double* qy, int64_t nq, double r, int approximate, const uint32_t** pairs,
                     int64_t* m) {
  pp_args a;
  a.ug = ug; a.qg = qg; a.r = r; a.approximate = approximate;
  int st = upload(c->ctx, &c->wo, ox, oy, NULL, no, &a.po);
  if (!st) st = upload(c->ctx, &c->wq, qx, qy, NULL, nq, &a.pq);
  if (st) return fail(c, st, "joinWindow");
  return join_common(c, run_pp, &a, pairs, m, "joinWindow");
}

typedef struct {
  gf_range_plan* plan;
  const gf_grid* g;
  gf_points pts;
} ppoly_args;
static int run_ppoly(shim_ctx* c, const void* a_, uint32_t* pairs, int64_t cap, int64_t* m) {
  const ppoly_args* a = (const ppoly_args*)a_;
  (void)c;
  return gf_join_ppoly_run(a->plan, a->g, &a->pts, pairs, cap, m);
}

int shim_polygon_join_window(shim_ctx* c, const gf_grid* g, const double* x, const double* y, int64_t n,
                             const gf_polygons* polys, double r, int approximate, const uint32_t** pairs, int64_t* m) {
  ppoly_args a;
  a.g = g;
  a.plan = NULL;
  int st = gf_join_ppoly_plan_create(c->ctx, g, polys, r, approximate, GF_METRIC_SQRT, &a.plan);
  if (!st) st = upload(c->ctx, &c->wo, x, y, NULL, n, &a.pts);
  if (!st) st = join_common(c, run_ppoly, &a, pairs, m, "polygonJoinWindow");
  else fail(c, st, "polygonJoinWindow");
  if (a.plan) gf_range_plan_destroy(a.plan);
  return st;
}

/* ---- ingest ----------------------------------------------------------------------------- */
static int parse_common(shim_ctx* c, const char* text, int64_t len, int geojson, const void* schema, double* x,
                        double* y, int64_t* objID, int64_t* ts, int64_t cap, int64_t* n, int64_t* bad_line,
                        int32_t* bad_kind) {
  *n = 0;
  *bad_line = -1;
  *bad_kind = 0;
  const size_t col = 8 * (size_t)(cap > 0 ? cap : 1);
  int st = dbuf_need(&c->text, (size_t)len + 16);
  if (!st) st = dbuf_need(&c->cols, 4 * col);
  if (!st && len > 0 && copy(c, c->text.p, text, (size_t)len, hipMemcpyHostToDevice)) st = GF_ERR_HIP;
  double* dx = (double*)c->cols.p;
  double* dy = (double*)((char*)c->cols.p + col);
  int64_t* dob = (int64_t*)((char*)c->cols.p + 2 * col);
  int64_t* dts = (int64_t*)((char*)c->cols.p + 3 * col);
  if (!st)
    st = geojson ? gf_geojson_parse(c->ctx, NULL, (const char*)c->text.p, len, (const gf_geojson_schema*)schema, NULL,
                                    dx, dy, dob, dts, NULL, NULL, cap, n, bad_line, bad_kind)
                 : gf_csv_parse(c->ctx, (const char*)c->text.p, len, (const gf_csv_schema*)schema, NULL, dx, dy, dob,
                                dts, NULL, NULL, cap, n, bad_line, bad_kind);
  const size_t b = 8 * (size_t)(*n < cap ? *n : cap);
  if (!st && b && (copy(c, x, dx, b, hipMemcpyDeviceToHost) || copy(c, y, dy, b, hipMemcpyDeviceToHost) ||
                   copy(c, objID, dob, b, hipMemcpyDeviceToHost) || copy(c, ts, dts, b, hipMemcpyDeviceToHost)))
    st = GF_ERR_HIP;
  if (!st) st = gf_ctx_synchronize(c->ctx);
  return st == GF_ERR_CAPACITY ? st : fail(c, st, geojson ? "geoJsonParse" : "csvParse");
}

int shim_csv_parse(shim_ctx* c, const char* text, int64_t len, const gf_csv_schema* schema, double* x, double* y,
                   int64_t* objID, int64_t* ts, int64_t cap, int64_t* n, int64_t* bad_line, int32_t* bad_kind) {
  return parse_common(c, text, len, 0, schema, x, y, objID, ts, cap, n, bad_line, bad_kind);
}

int shim_geojson_parse(shim_ctx* c, const char* text, int64_t len, const gf_geojson_schema* schema, double* x,
                       double* y, int64_t* objID, int64_t* ts, int64_t cap, int64_t* n, int64_t* bad_line,
                       int32_t* bad_kind) {
  return parse_common(c, text, len, 1, schema, x, y, objID, ts, cap, n, bad_line, bad_kind);
}

/* ---- pinned host buffers (the Java side's objID direct buffers) ------------------------------ */
int shim_pinned_alloc(int64_t bytes, void** out) {
  *out = NULL;
  if (bytes <= 0) return GF_ERR_ARG;
  return gf_pinned_alloc((size_t)bytes, out);
}

void shim_pinned_free(void* p) { gf_pinned_free(p); }
