// sliding.cpp -- pane engine for sliding-window kNN (BASELINE configs[4]).
//
// The reference evaluates every sliding window from scratch: PointPointKNNQuery.windowBased
// keys the stream by cell and applies SlidingProcessingTimeWindows.of(size, slide) twice --
// per-cell heaps, then the windowAll merge (PointPointKNNQuery.java:158-200,
// KNNQuery.java:213-272) -- so every point is scanned size/slide times.  Here the stream is cut
// into panes of gcd(size, slide) ms: each pane is scanned ONCE (the fused kNN scan/select, one
// launch per pane) into a top-k record kept in a device ring, and a window's result is the
// top-k-distinct merge of its panes' records (one 256-thread merge launch).  Top-k-distinct of
// a union = top-k-distinct of the parts' top-k-distinct lists, so the window record equals
// evaluating the window whole -- bit for bit, including the (d, objID) order and idx.
//
// Flink window assignment (TimeWindow.getWindowStartWithOffset, offset 0): an element with
// timestamp t lies in pane floor(t / pane); window [s, s + size) (s a multiple of slide) closes
// when the pane ending at s + size is complete; a window with no element never fires.
#define GF_TU_NAME sliding_cpp
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include <algorithm>
#include <climits>
#include <numeric>
#include <vector>

#include "gf_internal.hpp"

using namespace gf;

struct gf_knn_sliding {
  gf_knn_plan* plan = nullptr;
  int64_t size_ms = 0, slide_ms = 0, pane_ms = 0;
  int32_t W = 0;   // panes per window
  int32_t S = 0;   // panes per slide
  int32_t R = 0;   // ring slots (panes kept: borrowed buffers must stay alive that long)
  size_t rb = 0;
  char* recs = nullptr;  // device ring of R pane records
  void* scratch = nullptr;  // k > kMaxK: the window merge's rank / dedupe scratch (W records)
  struct Pane {
    int64_t index = LLONG_MIN;
    gf_points pts{};
    int64_t base = 0;    // stream position of the pane's first point (idx of results)
  };
  std::vector<Pane> ring;
  bool started = false;
  int64_t first = 0;     // first pushed pane index (earlier panes are empty)
  int64_t last = 0;      // last pushed pane index
  int64_t pos = 0;       // stream position of the next pane's first point
  // depth 2: a closed window whose last pane's select has not run yet
  bool pend = false;
  int64_t pend_last = 0;
  void* pend_result = nullptr;
};

namespace {

int64_t floor_mod(int64_t a, int64_t m) {
  const int64_t r = a % m;
  return r < 0 ? r + m : r;
}
int64_t floor_div(int64_t a, int64_t m) { return (a - floor_mod(a, m)) / m; }

gf_knn_sliding::Pane& slot(gf_knn_sliding* s, int64_t p) { return s->ring[(size_t)floor_mod(p, s->R)]; }
char* rec_of(gf_knn_sliding* s, int64_t p) { return s->recs + (size_t)floor_mod(p, s->R) * s->rb; }

// the window ending with pane p: panes [p - W + 1, p]
bool window_has_points(gf_knn_sliding* s, int64_t p) {
  for (int64_t q = p - s->W + 1; q <= p; ++q) {
    const gf_knn_sliding::Pane& pn = slot(s, q);
    if (pn.index == q && pn.pts.n > 0) return true;
  }
  return false;
}

KnnMergeArgs window_merge(gf_knn_sliding* s, int64_t p, void* result) {
  KnnMergeArgs m{};
  m.result = result;
  for (int64_t q = p - s->W + 1; q <= p; ++q) {
    const gf_knn_sliding::Pane& pn = slot(s, q);
    if (pn.index == q && pn.pts.n > 0) m.list.rec[m.nrec++] = rec_of(s, q);
  }
  return m;
}

int merge_window(gf_knn_sliding* s, int64_t p, void* result) {
  const KnnMergeArgs m = window_merge(s, p, result);
  gf_ctx* ctx = s->plan->ctx;
  GF_HIP_CHECK(ctx, launch_knn_merge_list(ctx, s->plan->k, m.list, m.nrec, result, s->scratch));
  return GF_OK;
}

// windows start at multiples of slide, so they end at e = start + size: pane p closes one iff
// (p + 1) * pane - size is a multiple of slide, i.e. (p + 1 - W) mod S == 0
bool closes_window(const gf_knn_sliding* s, int64_t p) { return floor_mod(p + 1 - s->W, s->S) == 0; }

}  // namespace

extern "C" int gf_knn_sliding_create(gf_knn_plan* plan, int64_t size_ms, int64_t slide_ms, gf_knn_sliding** out) {
  if (!plan || !out || size_ms <= 0 || slide_ms <= 0) return GF_ERR_ARG;
  *out = nullptr;
  gf_ctx* ctx = plan->ctx;
  const int64_t pane = std::gcd(size_ms, slide_ms);
  const int64_t W = size_ms / pane, S = slide_ms / pane;
  if (W > kMaxMergeRecs)
    return set_err(ctx, GF_ERR_ARG, "gf_knn_sliding_create: size / gcd(size, slide) must be <= 64 panes");
  int st = bind(ctx);
  if (st) return st;
  gf_knn_sliding* s = new gf_knn_sliding();
  s->plan = plan;
  s->size_ms = size_ms; s->slide_ms = slide_ms; s->pane_ms = pane;
  s->W = (int32_t)W; s->S = (int32_t)S;
  s->R = (int32_t)(2 * W + S + 2);  // a window's panes + those pushed before its record is read
  s->rb = gf_knn_result_bytes(plan->k);
  s->ring.resize((size_t)s->R);
  hipError_t e = hipMalloc(&s->recs, s->rb * (size_t)s->R);
  if (e == hipSuccess && plan->k > kMaxK) e = hipMalloc(&s->scratch, merge_any_bytes((int32_t)W, plan->k));
  if (e != hipSuccess) {
    if (s->recs) hipFree(s->recs);
    delete s;
    return hip_err(ctx, e, "hipMalloc");
  }
  *out = s;
  return GF_OK;
}

extern "C" void gf_knn_sliding_destroy(gf_knn_sliding* s) {
  if (!s) return;
  hipSetDevice(s->plan->ctx->device);
  hipStreamSynchronize(s->plan->ctx->stream);
  if (s->recs) hipFree(s->recs);
  if (s->scratch) hipFree(s->scratch);
  delete s;
}

extern "C" int gf_knn_sliding_geometry(const gf_knn_sliding* s, int64_t* pane_ms, int32_t* panes_per_window,
                                       int32_t* panes_per_slide, int32_t* ring_panes) {
  if (!s) return GF_ERR_ARG;
  if (pane_ms) *pane_ms = s->pane_ms;
  if (panes_per_window) *panes_per_window = s->W;
  if (panes_per_slide) *panes_per_slide = s->S;
  if (ring_panes) *ring_panes = s->R;
  return GF_OK;
}

extern "C" int gf_knn_sliding_push(gf_knn_sliding* s, int64_t pane_index, const gf_points* pane, void* window_result,
                                   int32_t* closed, int64_t* window_end) {
  if (!s || !pane || !closed) return GF_ERR_ARG;
  gf_knn_plan* P = s->plan;
  gf_ctx* ctx = P->ctx;
  *closed = 0;
  if (s->started && pane_index != s->last + 1)
    return set_err(ctx, GF_ERR_ARG, "gf_knn_sliding_push: panes must be pushed consecutively (empty panes with n = 0)");
  if (pane->n < 0) return set_err(ctx, GF_ERR_ARG, "gf_knn_sliding_push: negative n");
  if (P->pipeline > 2) return set_err(ctx, GF_ERR_ARG, "gf_knn_sliding_push: the pane engine runs at pipeline depth <= 2");
  int st = bind(ctx);
  if (st) return st;
  gf_knn_sliding::Pane& pn = slot(s, pane_index);
  pn.index = pane_index;
  pn.pts = *pane;
  pn.base = s->pos;
  int merged = 0;
  if (pane->n > 0) {
    P->idx_base = s->pos;
    // depth 2: the fused launch also selects the previous non-empty pane into its ring slot
    // and, k <= 128, merges the window pending on that pane in the same block
    const KnnMergeArgs m = s->pend ? window_merge(s, s->pend_last, s->pend_result) : KnnMergeArgs{};
    if ((st = knn_enqueue_merge(P, pane, rec_of(s, pane_index), s->pend ? &m : nullptr, &merged))) return st;
  } else if ((st = gf_knn_plan_flush(P))) {
    return st;
  }
  s->pos += pane->n;
  if (!s->started) s->first = pane_index;
  s->started = true;
  s->last = pane_index;
  // every record of a pane before this one is complete (stream order); this pane's too unless
  // its select is still pending (depth 2)
  if (s->pend) {
    s->pend = false;
    if (!merged && (st = merge_window(s, s->pend_last, s->pend_result))) return st;
  }
  if (closes_window(s, pane_index) && window_has_points(s, pane_index)) {
    if (!window_result) return set_err(ctx, GF_ERR_ARG, "gf_knn_sliding_push: a window closes, result is null");
    *closed = 1;
    if (window_end) *window_end = (pane_index + 1) * s->pane_ms;
    if (P->pend_lane >= 0) {
      s->pend = true;
      s->pend_last = pane_index;
      s->pend_result = window_result;
    } else if ((st = merge_window(s, pane_index, window_result))) {
      return st;
    }
  }
  return GF_OK;
}

extern "C" int gf_knn_sliding_flush(gf_knn_sliding* s) {
  if (!s) return GF_ERR_ARG;
  int st = bind(s->plan->ctx);
  if (st || (st = gf_knn_plan_flush(s->plan))) return st;
  if (s->pend) {
    s->pend = false;
    return merge_window(s, s->pend_last, s->pend_result);
  }
  return GF_OK;
}

extern "C" int gf_pane_bounds(gf_ctx* ctx, const int64_t* ts, int64_t n, int64_t pane_ms, int64_t first_pane,
                              int32_t npanes, int64_t* bounds) {
  if (!ctx || pane_ms <= 0 || npanes < 0 || n < 0 || !bounds || (n > 0 && !ts))
    return set_err(ctx, GF_ERR_ARG, "gf_pane_bounds: bad argument");
  int st = bind(ctx);
  if (st) return st;
  GF_HIP_CHECK(ctx, launch_pane_bounds(ctx->stream, ts, n, pane_ms, first_pane, npanes + 1, bounds));
  return GF_OK;
}

extern "C" int gf_knn_sliding_decode(gf_knn_sliding* s, int64_t window_end, const void* result_host, int64_t* oo,
                                     double* od, int64_t* oi, int32_t* n_out) {
  if (!s || !result_host || !n_out) return GF_ERR_ARG;
  gf_knn_plan* P = s->plan;
  const gf_knn_header* h = (const gf_knn_header*)result_host;
  if (h->status == 0) return gf_knn_decode(P, nullptr, result_host, oo, od, oi, n_out);
  // a pane overflowed its candidate buffer or its threshold guess failed: each pane of the
  // window exactly (the plan's sorted exact path) into device records, merged on the device
  const int64_t p = floor_div(window_end, s->pane_ms) - 1;
  int st = gf_knn_sliding_flush(s);
  if (st) return st;
  gf_ctx* ctx = P->ctx;
  const int32_t k = P->k;
  const size_t rb = gf_knn_result_bytes(k);
  char* recs = nullptr;
  GF_HIP_CHECK(ctx, hipMalloc(&recs, rb * (size_t)(s->W + 1)));
  char* merged = recs + rb * (size_t)s->W;
  const int64_t saved_base = P->idx_base;
  int32_t nrec = 0;
  for (int64_t q = p - s->W + 1; q <= p && !st; ++q) {
    if (q < s->first) continue;  // before the stream: empty
    const gf_knn_sliding::Pane& pn = slot(s, q);
    if (pn.index != q) {
      st = set_err(ctx, GF_ERR_ARG, "gf_knn_sliding_decode: the window's panes left the ring");
      break;
    }
    if (pn.pts.n == 0) continue;
    P->idx_base = pn.base;
    st = knn_exact_record(P, &pn.pts, recs + rb * (size_t)nrec);
    ++nrec;
  }
  P->idx_base = saved_base;
  if (!st && nrec > 0) st = gf_knn_merge_dev(ctx, k, recs, nrec, merged);
  if (!st && nrec > 0) {
    if (hipMemcpyAsync(P->host_result, merged, rb, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
      st = set_err(ctx, GF_ERR_HIP, "gf_knn_sliding_decode: copy");
  }
  hipFree(recs);
  if (st) return st;
  if (nrec == 0) {
    *n_out = 0;
    return GF_OK;
  }
  return gf_knn_decode(P, nullptr, P->host_result, oo, od, oi, n_out);
}

// ---------------------------------------------------------------------------------------
// Sliding range (PointPointRangeQuery / PointPolygonRangeQuery under
// SlidingProcessingTimeWindows.of(size, slide), PointPointRangeQuery.java:149): the reference
// applies the window function to every window, so each point is tested size/slide times.  Here
// each pane is tested ONCE (gf_range_run into the pane's bitmap, compacted on the device into
// the pane's ascending index list + count), and a closed window's list is its panes' lists
// concatenated with the panes' window offsets (launch_range_window_gather): identical to
// evaluating the window whole, since the per-point test does not depend on the other points.
// ---------------------------------------------------------------------------------------
struct gf_range_sliding {
  gf_range_plan* plan = nullptr;
  int64_t size_ms = 0, slide_ms = 0, pane_ms = 0;
  int32_t W = 0, S = 0;
  struct Pane {
    int64_t index = LLONG_MIN;
    int64_t n = 0;
    uint64_t* bitmap = nullptr;
    uint32_t* list = nullptr;
    int64_t cap = 0;        // points the buffers hold
  };
  std::vector<Pane> ring;   // W slots: pane p in slot p mod W
  int64_t* counts = nullptr;  // device int64[W]: the slots' list lengths
  bool started = false;
  int64_t last = 0;
};

namespace {
gf_range_sliding::Pane& rslot(gf_range_sliding* s, int64_t p) { return s->ring[(size_t)floor_mod(p, s->W)]; }
bool rcloses(const gf_range_sliding* s, int64_t p) { return floor_mod(p + 1 - s->W, s->S) == 0; }
}  // namespace

extern "C" int gf_range_sliding_create(gf_range_plan* plan, int64_t size_ms, int64_t slide_ms, gf_range_sliding** out) {
  if (!plan || !out || size_ms <= 0 || slide_ms <= 0) return GF_ERR_ARG;
  *out = nullptr;
  gf_ctx* ctx = plan->ctx;
  if (plan->join) return set_err(ctx, GF_ERR_ARG, "gf_range_sliding_create: a join plan");
  const int64_t pane = std::gcd(size_ms, slide_ms);
  const int64_t W = size_ms / pane, S = slide_ms / pane;
  if (W > kMaxMergeRecs)
    return set_err(ctx, GF_ERR_ARG, "gf_range_sliding_create: size / gcd(size, slide) must be <= 64 panes");
  int st = bind(ctx);
  if (st) return st;
  gf_range_sliding* s = new gf_range_sliding();
  s->plan = plan;
  s->size_ms = size_ms; s->slide_ms = slide_ms; s->pane_ms = pane;
  s->W = (int32_t)W; s->S = (int32_t)S;
  s->ring.resize((size_t)W);
  hipError_t e = hipMalloc(&s->counts, sizeof(int64_t) * (size_t)W);
  if (e != hipSuccess) {
    delete s;
    return hip_err(ctx, e, "hipMalloc");
  }
  *out = s;
  return GF_OK;
}

extern "C" void gf_range_sliding_destroy(gf_range_sliding* s) {
  if (!s) return;
  hipSetDevice(s->plan->ctx->device);
  hipStreamSynchronize(s->plan->ctx->stream);
  for (auto& p : s->ring) {
    if (p.bitmap) hipFree(p.bitmap);
    if (p.list) hipFree(p.list);
  }
  if (s->counts) hipFree(s->counts);
  delete s;
}

extern "C" int gf_range_sliding_geometry(const gf_range_sliding* s, int64_t* pane_ms, int32_t* panes_per_window,
                                         int32_t* panes_per_slide) {
  if (!s) return GF_ERR_ARG;
  if (pane_ms) *pane_ms = s->pane_ms;
  if (panes_per_window) *panes_per_window = s->W;
  if (panes_per_slide) *panes_per_slide = s->S;
  return GF_OK;
}

extern "C" int gf_range_sliding_push(gf_range_sliding* s, int64_t pane_index, const gf_points* pane, uint32_t* idx,
                                     int64_t cap, int64_t* count, int32_t* closed, int64_t* window_end,
                                     int64_t* window_n) {
  if (!s || !pane || !closed || cap < 0) return GF_ERR_ARG;
  gf_ctx* ctx = s->plan->ctx;
  *closed = 0;
  if (s->started && pane_index != s->last + 1)
    return set_err(ctx, GF_ERR_ARG, "gf_range_sliding_push: panes must be pushed consecutively (empty panes with n = 0)");
  if (pane->n < 0 || pane->n > (int64_t)UINT32_MAX) return set_err(ctx, GF_ERR_ARG, "gf_range_sliding_push: bad n");
  int st = bind(ctx);
  if (st) return st;
  // the window this pane closes (if any) and its points, before anything changes: a too-small
  // idx is refused with nothing enqueued, so the caller can push the same pane again
  const bool closes = rcloses(s, pane_index);
  int64_t wn = 0;
  if (closes)
    for (int64_t q = pane_index - s->W + 1; q <= pane_index; ++q) {
      if (q == pane_index) wn += pane->n;
      else if (rslot(s, q).index == q) wn += rslot(s, q).n;
    }
  if (window_n) *window_n = closes ? wn : 0;
  if (closes && wn > 0) {
    if (wn > (int64_t)UINT32_MAX) return set_err(ctx, GF_ERR_ARG, "gf_range_sliding_push: window too large");
    if (cap < wn) return GF_ERR_CAPACITY;
    if (!idx || !count) return set_err(ctx, GF_ERR_ARG, "gf_range_sliding_push: a window closes, idx / count null");
  }
  gf_range_sliding::Pane& pn = rslot(s, pane_index);
  pn.index = pane_index;
  pn.n = pane->n;
  if (pane->n > 0) {
    if (pn.cap < pane->n) {  // grow: the stream may still read the old buffers (an earlier window)
      GF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
      if (pn.bitmap) GF_HIP_CHECK(ctx, hipFree(pn.bitmap));
      if (pn.list) GF_HIP_CHECK(ctx, hipFree(pn.list));
      pn.bitmap = nullptr;
      pn.list = nullptr;
      pn.cap = 0;
      const int64_t c = std::max<int64_t>(pane->n + pane->n / 4, 4096);
      GF_HIP_CHECK(ctx, hipMalloc(&pn.bitmap, sizeof(uint64_t) * (size_t)((c + 63) / 64)));
      GF_HIP_CHECK(ctx, hipMalloc(&pn.list, sizeof(uint32_t) * (size_t)c));
      pn.cap = c;
    }
    int64_t* cnt = s->counts + floor_mod(pane_index, s->W);
    if ((st = gf_range_run(s->plan, pane, pn.bitmap, nullptr, nullptr))) return st;
    if ((st = gf_bitmap_to_indices_async(ctx, pn.bitmap, pane->n, pn.list, pane->n, cnt))) return st;
  }
  s->started = true;
  s->last = pane_index;
  if (closes && wn > 0) {  // a window with no point never fires
    RangeGatherArgs a{};
    int64_t base = 0;
    for (int64_t q = pane_index - s->W + 1; q <= pane_index; ++q) {
      const gf_range_sliding::Pane& w = rslot(s, q);
      if (w.index != q || w.n == 0) continue;
      a.list[a.npanes] = w.list;
      a.cnt[a.npanes] = s->counts + floor_mod(q, s->W);
      a.base[a.npanes] = base;
      ++a.npanes;
      base += w.n;
    }
    a.total = base;
    a.out = idx;
    a.count = count;
    GF_HIP_CHECK(ctx, launch_range_window_gather(ctx->stream, a));
    *closed = 1;
    if (window_end) *window_end = (pane_index + 1) * s->pane_ms;
  }
  return GF_OK;
}
