/*
 * asan_driver.c -- host AddressSanitizer / UBSan coverage of the product's host code that handles
 * caller data: the objID dictionary (objid.cpp: intern, arena growth, decode
 * with short buffers, string records), the sliding pane ring (sliding.cpp: pushes, empty panes,
 * window closing, decode), the CSV / GeoJSON host sides (csv.cpp) and the JNI shim core's host
 * paths (geoflink_shim.c: cached windows, pinned staging, the sharded kNN's exact re-exchange).
 *
 * Built by `make asan-gpu` against a HOST-sanitized build of the library (every source compiled
 * with -Xarch_host -fsanitize=address,undefined: the device code is the ordinary gfx950 code) and
 * the C oracle, and run on the GPU box by tools/gpu_asan.sh.  Every result is checked against the
 * oracle; any sanitizer report aborts the run (halt_on_error).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../integration/jni/geoflink_shim.h"
#include "../../oracle/geoflink_oracle.h"

#define BX0 115.5
#define BX1 117.6
#define BY0 39.6
#define BY1 41.1
#define QX 116.414899
#define QY 39.920374

static int failures = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                    \
      fputc('\n', stderr);                             \
      ++failures;                                      \
    }                                                  \
  } while (0)
#define OK(st, c, what) CHECK((st) == 0, "%s: status %d (%s)", what, (int)(st), shim_last_error(c))

static void points(int64_t seed, int64_t n, double* x, double* y) {
  orc_java_random_points(seed, n, BX0, BX1, BY0, BY1, x, y);
}

/* ---- objID dictionary: intern / decode round trip, arena growth, short decode buffers ---- */
static void test_objid(shim_ctx* c) {
  const int64_t n = 20000;
  int64_t* offs = calloc(n + 1, sizeof(int64_t));
  char* bytes = malloc(n * 64);
  int64_t at = 0;
  for (int64_t i = 0; i < n; ++i) {
    offs[i] = at;
    int len;
    if (i % 7 == 0) len = snprintf(bytes + at, 64, "%lld", (long long)(i * 31 - 5000));  /* canonical decimal */
    else if (i % 7 == 1) len = snprintf(bytes + at, 64, "00%lld", (long long)i);        /* non-canonical */
    else if (i % 7 == 2) len = 0;                                                          /* empty String */
    else len = snprintf(bytes + at, 64, "veh-%lld-%s", (long long)(i % 5000), i % 3 ? "abcdefghijklmnopqrstuvwxyz" : "x");
    at += len;
  }
  offs[n] = at;
  int64_t* keys = malloc(n * sizeof(int64_t));
  OK(shim_objid_intern(c, bytes, offs, n, keys), c, "objidIntern");
  int64_t* k2 = malloc(n * sizeof(int64_t));
  OK(shim_objid_intern(c, bytes, offs, n, k2), c, "objidIntern again");
  CHECK(memcmp(keys, k2, n * sizeof(int64_t)) == 0, "keys differ between two interns of the same Strings");
  int64_t* doffs = calloc(n + 1, sizeof(int64_t));
  char small[16];
  int st = shim_objid_decode(c, keys, n, small, (int64_t)sizeof small, doffs);
  CHECK(st == GF_ERR_CAPACITY && doffs[n] == at, "short decode buffer: status %d, needed %lld of %lld", st,
        (long long)doffs[n], (long long)at);
  char* back = malloc(at + 1);
  OK(shim_objid_decode(c, keys, n, back, at, doffs), c, "objidDecode");
  for (int64_t i = 0; i < n; ++i) {
    const int64_t l0 = offs[i + 1] - offs[i], l1 = doffs[i + 1] - doffs[i];
    if (l0 != l1 || memcmp(bytes + offs[i], back + doffs[i], (size_t)l0) != 0) {
      CHECK(0, "String %lld did not round-trip", (long long)i);
      break;
    }
  }
  free(offs); free(bytes); free(keys); free(k2); free(doffs); free(back);
}

static int32_t oracle_knn(const orc_grid* og, int64_t n, const double* x, const double* y, const int64_t* o,
                          int32_t k, int64_t* eo, double* ed, int64_t* ei) {
  return orc_knn_contract(og, n, x, y, o, QX, QY, 0.5, k, 0, eo, ed, ei);
}

/* ---- kNN windows through the shim (cached window growth, pinned objID column) ---- */
static void test_knn(shim_ctx* c) {
  gf_grid g;
  orc_grid og;
  gf_grid_make(500, BX0, BX1, BY0, BY1, &g);
  orc_grid_make(500, BX0, BX1, BY0, BY1, &og);
  shim_knn* h = NULL;
  OK(shim_knn_plan(c, &g, QX, QY, 0.5, 50, &h), c, "knnPlan");
  if (!h) return;
  const int64_t sizes[] = {300000, 0, 5, 1200000, 64};
  for (int j = 0; j < 5; ++j) {
    const int64_t n = sizes[j];
    double* x = malloc((n + 1) * 8);
    double* y = malloc((n + 1) * 8);
    int64_t* o = malloc((n + 1) * 8);
    points(100 + j, n, x, y);
    for (int64_t i = 0; i < n; ++i) o[i] = (i * 7919) % (n / 2 + 1);
    int64_t oo[50], oi[50], eo[50], ei[50];
    double od[50], ed[50];
    int32_t m = -1;
    OK(shim_knn_window(h, x, y, o, n, oo, od, oi, &m), c, "knnWindow");
    const int32_t em = oracle_knn(&og, n, x, y, o, 50, eo, ed, ei);
    CHECK(m == em && memcmp(oo, eo, 8 * (size_t)m) == 0 && memcmp(od, ed, 8 * (size_t)m) == 0 &&
              memcmp(oi, ei, 8 * (size_t)m) == 0,
          "kNN window %d: %d vs %d entries", j, m, em);
    free(x); free(y); free(o);
  }
  /* the objID column in pinned memory (read in place by the kernels) */
  const int64_t n = 700000;
  void* pin = NULL;
  OK(shim_pinned_alloc(8 * n, &pin), c, "pinnedAlloc");
  double* x = malloc(n * 8);
  double* y = malloc(n * 8);
  int64_t* o = (int64_t*)pin;
  points(777, n, x, y);
  for (int64_t i = 0; i < n; ++i) o[i] = n - i;
  int64_t oo[50], oi[50], eo[50], ei[50];
  double od[50], ed[50];
  int32_t m = -1;
  OK(shim_knn_window(h, x, y, o, n, oo, od, oi, &m), c, "knnWindow pinned");
  const int32_t em = oracle_knn(&og, n, x, y, o, 50, eo, ed, ei);
  CHECK(m == em && memcmp(oo, eo, 8 * (size_t)m) == 0 && memcmp(oi, ei, 8 * (size_t)m) == 0, "pinned kNN");
  /* the sharded form on a one-rank communicator, with a window that overflows the candidate
   * buffer (1.1M points on the query point): the exact re-exchange path */
  uint8_t id[GF_COMM_ID_BYTES];
  shim_comm* comm = NULL;
  if (shim_comm_unique_id(id) == 0 && shim_comm_create(c, id, 1, 0, &comm) == 0) {
    const int64_t ns = 1100000 + 1000;
    double* sx = malloc(ns * 8);
    double* sy = malloc(ns * 8);
    int64_t* so = malloc(ns * 8);
    points(31, 1000, sx, sy);
    for (int64_t i = 1000; i < ns; ++i) { sx[i] = QX; sy[i] = QY; }
    for (int64_t i = 0; i < ns; ++i) so[i] = (i * 104729) % 900001;
    m = -1;
    OK(shim_knn_window_sharded(h, comm, sx, sy, so, ns, 17, oo, od, oi, &m), c, "knnWindowSharded");
    const int32_t es = oracle_knn(&og, ns, sx, sy, so, 50, eo, ed, ei);
    for (int i = 0; i < es; ++i) ei[i] += 17;
    CHECK(m == es && memcmp(oo, eo, 8 * (size_t)m) == 0 && memcmp(oi, ei, 8 * (size_t)m) == 0, "sharded kNN");
    shim_comm_destroy(comm);
    free(sx); free(sy); free(so);
  } else {
    CHECK(0, "one-rank communicator: %s", gf_comm_last_error(NULL));
  }
  shim_knn_destroy(h);
  shim_pinned_free(pin);
  free(x); free(y);
}

/* ---- sliding kNN: the pane ring (pushes, an empty pane, decode of every fired window) ---- */
static void test_sliding(shim_ctx* c) {
  gf_grid g;
  orc_grid og;
  gf_grid_make(1000, BX0, BX1, BY0, BY1, &g);
  orc_grid_make(1000, BX0, BX1, BY0, BY1, &og);
  const int32_t k = 100;
  shim_knn* h = NULL;
  shim_sliding* s = NULL;
  OK(shim_knn_plan(c, &g, QX, QY, 0.5, k, &h), c, "knnPlan");
  if (!h) return;
  OK(shim_sliding_create(h, 2000, 1000, &s), c, "slidingCreate");
  const int64_t npane = 9, per = 60000;
  double* x = malloc(npane * per * 8);
  double* y = malloc(npane * per * 8);
  int64_t* o = malloc(npane * per * 8);
  points(55, npane * per, x, y);
  for (int64_t i = 0; i < npane * per; ++i) o[i] = (i * 31) % (npane * per / 2);
  int64_t pend[4] = {-1, -1, -1, -1};
  int fired = 0;
  for (int64_t p = 0; p < npane && s; ++p) {
    const int64_t n = p == 4 ? 0 : per;  /* pane 4 empty */
    int32_t closed = 0;
    int64_t end = -1;
    OK(shim_sliding_push(s, p, x + p * per, y + p * per, o + p * per, n, &closed, &end), c, "slidingPush");
    for (int i = 0; i < 4; ++i) {
      if (pend[i] < 0) continue;
      const int64_t e = pend[i];
      pend[i] = -1;
      /* window [e - 2000, e): panes e/1000 - 2 and e/1000 - 1 (pane 4 holds nothing; the first
       * window, [-1000, 1000), holds pane 0 only) */
      const int64_t p0 = e / 1000 - 2;
      double* wx = malloc(2 * per * 8);
      double* wy = malloc(2 * per * 8);
      int64_t* wo = malloc(2 * per * 8);
      int64_t m2 = 0;
      for (int64_t q = p0; q < p0 + 2; ++q)
        if (q >= 0 && q < npane && q != 4)
          for (int64_t t = q * per; t < (q + 1) * per; ++t) { wx[m2] = x[t]; wy[m2] = y[t]; wo[m2] = o[t]; ++m2; }
      int64_t oo[100], oi[100], eo[100], ei[100];
      double od[100], ed[100];
      int32_t m = -1;
      OK(shim_sliding_decode(s, e, oo, od, oi, &m), c, "slidingDecode");
      const int32_t em = orc_knn_contract(&og, m2, wx, wy, wo, QX, QY, 0.5, k, 0, eo, ed, ei);
      CHECK(m == em && memcmp(oo, eo, 8 * (size_t)m) == 0 && memcmp(od, ed, 8 * (size_t)m) == 0,
            "sliding window ending %lld: %d vs %d", (long long)e, m, em);
      ++fired;
      free(wx); free(wy); free(wo);
    }
    if (closed) pend[0] = end;
  }
  if (s && pend[0] >= 0) {
    OK(shim_sliding_flush(s), c, "slidingFlush");
    int64_t oo[100], oi[100];
    double od[100];
    int32_t m = -1;
    OK(shim_sliding_decode(s, pend[0], oo, od, oi, &m), c, "slidingDecode last");
  }
  CHECK(fired >= 5, "only %d sliding windows fired", fired);
  shim_sliding_destroy(s);
  shim_knn_destroy(h);
  free(x); free(y); free(o);
}

/* ---- range windows (capacity answer) and the point-point join through the shim ---- */
static void test_range_join(shim_ctx* c) {
  gf_grid g;
  orc_grid og;
  gf_grid_make(100, BX0, BX1, BY0, BY1, &g);
  orc_grid_make(100, BX0, BX1, BY0, BY1, &og);
  double qx[2] = {QX, 117.0}, qy[2] = {QY, 40.5};
  shim_range* h = NULL;
  OK(shim_range_plan(c, &g, qx, qy, 2, 0.05, 0, &h), c, "rangePlan");
  const int64_t n = 400000;
  double* x = malloc(n * 8);
  double* y = malloc(n * 8);
  points(9, n, x, y);
  int64_t* exp = malloc(n * 8);
  const int64_t ne = orc_range_pp(&og, n, x, y, 2, qx, qy, 0.05, 0, 0, exp, n);
  int32_t* out = malloc(n * 4);
  int64_t cnt = -1;
  int st = shim_range_window(h, x, y, n, out, 10, &cnt);
  CHECK(st == GF_ERR_CAPACITY && cnt == ne, "range capacity answer: %d, %lld vs %lld", st, (long long)cnt,
        (long long)ne);
  OK(shim_range_window(h, x, y, n, out, n, &cnt), c, "rangeWindow");
  int same = cnt == ne;
  for (int64_t i = 0; same && i < ne; ++i) same = out[i] == exp[i];
  CHECK(same, "range window: %lld vs %lld hits", (long long)cnt, (long long)ne);
  shim_range_destroy(h);
  /* join: 200K ordinary x 20K query points, r = 0.001 on 1000^2 */
  gf_grid gj;
  orc_grid oj;
  gf_grid_make(1000, BX0, BX1, BY0, BY1, &gj);
  orc_grid_make(1000, BX0, BX1, BY0, BY1, &oj);
  const int64_t no = 200000, nq = 20000;
  double* ox = malloc(no * 8);
  double* oy = malloc(no * 8);
  double* jx = malloc(nq * 8);
  double* jy = malloc(nq * 8);
  orc_java_random_points(5, no, 116.0, 116.3, 39.8, 40.0, ox, oy);
  orc_java_random_points(6, nq, 116.0, 116.3, 39.8, 40.0, jx, jy);
  const uint32_t* pairs = NULL;
  int64_t m = -1;
  OK(shim_join_window(c, &gj, &gj, ox, oy, no, jx, jy, nq, 0.001, 0, &pairs, &m), c, "joinWindow");
  const int64_t cap = 4 * no;
  int64_t* ep = malloc(cap * 2 * 8);
  const int64_t em = orc_join_pp(&oj, &oj, no, ox, oy, nq, jx, jy, 0.001, 0, 0, ep, cap);
  CHECK(m == em, "join: %lld vs %lld pairs", (long long)m, (long long)em);
  free(x); free(y); free(exp); free(out); free(ox); free(oy); free(jx); free(jy); free(ep);
}

/* ---- CSV ingest through the shim: a good chunk and a chunk with a bad line ---- */
static void test_csv(shim_ctx* c) {
  const int64_t n = 50000;
  char* text = malloc(n * 96);
  int64_t len = 0;
  double* x = malloc(n * 8);
  double* y = malloc(n * 8);
  points(3, n, x, y);
  for (int64_t i = 0; i < n; ++i)
    len += sprintf(text + len, "%s%lld, %lld ,%.17g,%.17g\n", i % 3 ? "veh" : "", (long long)(i % 999),
                   (long long)(1000 + i), x[i], y[i]);
  gf_csv_schema sc;
  memset(&sc, 0, sizeof sc);
  sc.delimiter = ',';
  sc.objid_field = 0; sc.time_field = 1; sc.x_field = 2; sc.y_field = 3;
  double* px = malloc(n * 8);
  double* py = malloc(n * 8);
  int64_t* po = malloc(n * 8);
  int64_t* pt = malloc(n * 8);
  int64_t got = -1, bad = -1;
  int32_t kind = -1;
  OK(shim_csv_parse(c, text, len, &sc, px, py, po, pt, n, &got, &bad, &kind), c, "csvParse");
  CHECK(got == n && memcmp(px, x, n * 8) == 0 && memcmp(py, y, n * 8) == 0, "csv: %lld lines", (long long)got);
  int same = 1;
  for (int64_t i = 0; same && i < n; ++i) same = pt[i] == 1000 + i;
  CHECK(same, "csv timestamps");
  /* a short output capacity, then a chunk whose line 7 has a malformed x */
  int st = shim_csv_parse(c, text, len, &sc, px, py, po, pt, 10, &got, &bad, &kind);
  CHECK(st == GF_ERR_CAPACITY && got == n, "csv capacity answer %d %lld", st, (long long)got);
  char* t2 = malloc(4096);
  int64_t l2 = 0;
  for (int i = 0; i < 10; ++i)
    l2 += sprintf(t2 + l2, i == 7 ? "a%d,5,11x6.5,40.1\n" : "a%d,5,116.5,40.1\n", i);
  st = shim_csv_parse(c, t2, l2, &sc, px, py, po, pt, n, &got, &bad, &kind);
  CHECK(st == GF_ERR_ARG && bad == 7 && kind == GF_CSV_NUMBER_FORMAT, "csv bad line: %d %lld %d", st,
        (long long)bad, kind);
  free(text); free(x); free(y); free(px); free(py); free(po); free(pt); free(t2);
}

int main(void) {
  shim_ctx* c = NULL;
  if (shim_ctx_create(0, &c) != 0) {
    fprintf(stderr, "no GPU context\n");
    return 2;
  }
  test_objid(c);
  test_knn(c);
  test_sliding(c);
  test_range_join(c);
  test_csv(c);
  shim_ctx_destroy(c);
  if (failures) {
    fprintf(stderr, "asan_driver: %d failures\n", failures);
    return 1;
  }
  printf("asan_driver: ok (objID dictionary, kNN windows + pinned objIDs + sharded re-exchange, sliding pane ring, "
         "range capacity, join, CSV)\n");
  return 0;
}
