/*
 * geoflink_oracle.c -- TEST INFRASTRUCTURE ONLY.  See geoflink_oracle.h.
 *
 * Plain-C restatement of the GeoFlink window-evaluation hot path, "reference-shaped":
 * string cell IDs, string hash sets for the guaranteed/candidate cells, per-cell
 * java.util.PriorityQueue heaps and the single-threaded windowAll merge.  Parity is
 * UNPINNED (no reference fixtures exist and no JVM/JTS is available); every function
 * cites the reference file:line it restates.  Build: oracle/Makefile (gcc -O2
 * -ffp-contract=off: Java never fuses a*b+c).
 */
#define _POSIX_C_SOURCE 200809L
#include "geoflink_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* Java primitives                                                                      */
/* ------------------------------------------------------------------------------------ */

/* JLS 5.1.3 narrowing double -> int: NaN -> 0, saturate, else round toward zero. */
int32_t orc_jint(double v) {
  if (v != v) return 0;
  if (v >= 2147483647.0) return 2147483647;
  if (v <= -2147483648.0) return (int32_t)(-2147483647 - 1);
  return (int32_t)v;
}

/* UniformGrid(int uniformGridRows, ...) -- UniformGrid.java:74-85: no squaring of bounds */
int orc_grid_make(int32_t n, double minX, double maxX, double minY, double maxY, orc_grid* g) {
  if (!g || n <= 0) return ORC_ERR_ARG;
  g->n = n;
  g->minX = minX; g->maxX = maxX; g->minY = minY; g->maxY = maxY;
  g->cellLength = (maxX - minX) / n;
  return ORC_OK;
}

/* HelperClass.assignGridCellID -- HelperClass.java:109-110 */
void orc_cell_of(const orc_grid* g, double x, double y, int32_t* cx, int32_t* cy) {
  *cx = orc_jint(floor((x - g->minX) / g->cellLength));
  *cy = orc_jint(floor((y - g->minY) / g->cellLength));
}

/* String.format("%05d", i) + String.format("%05d", j) -- HelperClass.java:54-57,118-120.
 * C printf("%05d") renders negatives as Java does ("-0001"). */
void orc_cell_id(int32_t cx, int32_t cy, char* buf) { sprintf(buf, "%05d%05d", cx, cy); }

/* removeLeadingZeroesFromString -- HelperClass.java:60-63: replaceFirst("^0+(?!$)","") then
 * Integer.parseInt.  parseInt of the remainder (optional sign, digits). */
static int32_t parse_java_int(const char* s, size_t len) {
  size_t i = 0;
  /* strip leading zeros but keep the last character */
  while (i + 1 < len && s[i] == '0') i++;
  int neg = 0;
  long long v = 0;
  if (i < len && (s[i] == '-' || s[i] == '+')) { neg = s[i] == '-'; i++; }
  for (; i < len; i++) v = v * 10 + (s[i] - '0');
  return (int32_t)(neg ? -v : v);
}

/* HelperClass.getIntCellIndices -- HelperClass.java:263-276 */
void orc_parse_cell_id(const char* id, int32_t* cx, int32_t* cy) {
  size_t len = strlen(id);
  *cx = parse_java_int(id, len < 5 ? len : 5);
  *cy = len > 5 ? parse_java_int(id + 5, len - 5) : 0;
}

void orc_assign_cells(const orc_grid* g, int64_t n, const double* x, const double* y,
                      int32_t* cx, int32_t* cy) {
  for (int64_t i = 0; i < n; i++) orc_cell_of(g, x[i], y[i], &cx[i], &cy[i]);
}

/* UniformGrid.getGuaranteedNeighboringLayers -- UniformGrid.java:428-439 */
int32_t orc_guaranteed_layers(const orc_grid* g, double r) {
  double cellDiagonal = g->cellLength * sqrt(2.0);
  return orc_jint(floor((r / cellDiagonal) - 1));
}

/* UniformGrid.getCandidateNeighboringLayers -- UniformGrid.java:441-445 */
int32_t orc_candidate_layers(const orc_grid* g, double r) { return orc_jint(ceil(r / g->cellLength)); }

/* UniformGrid.validKey -- UniformGrid.java:224-229 */
static int valid_key(const orc_grid* g, int64_t x, int64_t y) {
  return x >= 0 && y >= 0 && x < g->n && y < g->n;
}

/* ------------------------------------------------------------------------------------ */
/* JTS 1.16.1 numerics (restated; third-party, absent from the reference tree)         */
/* ------------------------------------------------------------------------------------ */

typedef union { double d; uint64_t u; } dbits;
static uint32_t hi_word(double x) { dbits b; b.d = x; return (uint32_t)(b.u >> 32); }
static uint32_t lo_word(double x) { dbits b; b.d = x; return (uint32_t)b.u; }
static double with_hi(double x, uint32_t hi) {
  dbits b; b.d = x; b.u = ((uint64_t)hi << 32) | (b.u & 0xffffffffULL); return b.d;
}

/* fdlibm 5.3 e_hypot.c, which JDK 8 StrictMath.hypot (and Math.hypot) executes. */
double orc_hypot(double x, double y) {
  double a, b, t1, t2, y1, y2, w;
  int32_t j, k, ha, hb;
  ha = (int32_t)(hi_word(x) & 0x7fffffff);
  hb = (int32_t)(hi_word(y) & 0x7fffffff);
  if (hb > ha) { a = y; b = x; j = ha; ha = hb; hb = j; } else { a = x; b = y; }
  a = with_hi(a, (uint32_t)ha);
  b = with_hi(b, (uint32_t)hb);
  if ((ha - hb) > 0x3c00000) return a + b; /* x/y > 2**60 */
  k = 0;
  if (ha > 0x5f300000) {                  /* a > 2**500 */
    if (ha >= 0x7ff00000) {               /* Inf or NaN */
      w = a + b;
      if (((ha & 0xfffff) | lo_word(a)) == 0) w = a;
      if (((hb ^ 0x7ff00000) | lo_word(b)) == 0) w = b;
      return w;
    }
    ha -= 0x25800000; hb -= 0x25800000; k += 600;
    a = with_hi(a, (uint32_t)ha);
    b = with_hi(b, (uint32_t)hb);
  }
  if (hb < 0x20b00000) {                  /* b < 2**-500 */
    if (hb <= 0x000fffff) {               /* subnormal b or 0 */
      if ((hb | lo_word(b)) == 0) return a;
      t1 = with_hi(0.0, 0x7fd00000);      /* t1 = 2^1022 */
      b *= t1; a *= t1; k -= 1022;
    } else {
      ha += 0x25800000; hb += 0x25800000; k -= 600;
      a = with_hi(a, (uint32_t)ha);
      b = with_hi(b, (uint32_t)hb);
    }
  }
  w = a - b;
  if (w > b) {
    t1 = with_hi(0.0, (uint32_t)ha);
    t2 = a - t1;
    w = sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)));
  } else {
    a = a + a;
    y1 = with_hi(0.0, (uint32_t)hb);
    y2 = b - y1;
    t1 = with_hi(0.0, (uint32_t)(ha + 0x00100000));
    t2 = a - t1;
    w = sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)));
  }
  if (k != 0) {
    t1 = with_hi(1.0, hi_word(1.0) + ((uint32_t)k << 20));
    return t1 * w;
  }
  return w;
}

/* JTS Coordinate.distance(c): dx = x - c.x; dy = y - c.y; sqrt or hypot */
double orc_distance(double x1, double y1, double x2, double y2, int metric) {
  double dx = x1 - x2, dy = y1 - y2;
  if (metric == ORC_METRIC_HYPOT) return orc_hypot(dx, dy);
  return sqrt(dx * dx + dy * dy);
}

/* JTS algorithm.Distance.pointToSegment(p, A, B) */
static double point_to_segment(double px, double py, double ax, double ay, double bx, double by,
                               int metric) {
  if (ax == bx && ay == by) return orc_distance(px, py, ax, ay, metric);
  double len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay);
  double r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2;
  if (r <= 0.0) return orc_distance(px, py, ax, ay, metric);
  if (r >= 1.0) return orc_distance(px, py, bx, by, metric);
  double s = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2;
  return fabs(s) * sqrt(len2);
}

/* Exact sign of x1*y2 - y1*x2 for the given doubles (what JTS RobustDeterminant.signOfDet2x2
 * returns).  Products split exactly with fma, the four-term sum grown as a Shewchuk
 * nonoverlapping expansion; its sign is the sign of the top nonzero component. */
static void two_sum(double a, double b, double* s, double* e) {
  double x = a + b, bv = x - a, av = x - bv;
  *s = x; *e = (a - av) + (b - bv);
}
static int sign_det2x2(double x1, double y1, double x2, double y2) {
  double p1 = x1 * y2, e1 = fma(x1, y2, -p1);
  double p2 = y1 * x2, e2 = fma(y1, x2, -p2);
  double terms[4] = {e1, -e2, p1, -p2};
  double h[4];
  int m = 1;
  h[0] = terms[0];
  for (int t = 1; t < 4; t++) {
    double q = terms[t];
    for (int i = 0; i < m; i++) { double s, e; two_sum(q, h[i], &s, &e); h[i] = e; q = s; }
    h[m++] = q;
  }
  for (int i = m - 1; i >= 0; i--) {
    if (h[i] > 0) return 1;
    if (h[i] < 0) return -1;
  }
  return 0;
}

#define LOC_INTERIOR 0
#define LOC_BOUNDARY 1
#define LOC_EXTERIOR 2

/* JTS RayCrossingCounter.locatePointInRing / countSegment (1.16: RobustDeterminant on the
 * translated segment). */
static int locate_in_ring(double px, double py, const double* vx, const double* vy, int32_t nv) {
  int crossings = 0;
  for (int32_t i = 1; i < nv; i++) {
    double p1x = vx[i], p1y = vy[i], p2x = vx[i - 1], p2y = vy[i - 1];
    if (p1x < px && p2x < px) continue;
    if (px == p2x && py == p2y) return LOC_BOUNDARY;
    if (p1y == py && p2y == py) {
      double minx = p1x, maxx = p2x;
      if (minx > maxx) { minx = p2x; maxx = p1x; }
      if (px >= minx && px <= maxx) return LOC_BOUNDARY;
      continue;
    }
    if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
      double x1 = p1x - px, y1 = p1y - py, x2 = p2x - px, y2 = p2y - py;
      int sgn = sign_det2x2(x1, y1, x2, y2);
      if (sgn == 0) return LOC_BOUNDARY;
      if (y2 < y1) sgn = -sgn;
      if (sgn > 0) crossings++;
    }
  }
  return (crossings & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

typedef struct { double minx, maxx, miny, maxy; } env_t;
static env_t ring_env(const double* vx, const double* vy, int32_t nv) {
  env_t e = {vx[0], vx[0], vy[0], vy[0]};
  for (int32_t i = 1; i < nv; i++) {
    if (vx[i] < e.minx) e.minx = vx[i];
    if (vx[i] > e.maxx) e.maxx = vx[i];
    if (vy[i] < e.miny) e.miny = vy[i];
    if (vy[i] > e.maxy) e.maxy = vy[i];
  }
  return e;
}

/* JTS PointLocator.locateInPolygonRing: envelope test, then ring location */
static int locate_in_polygon_ring(double px, double py, const double* vx, const double* vy,
                                  int32_t nv) {
  env_t e = ring_env(vx, vy, nv);
  if (px > e.maxx || px < e.minx || py > e.maxy || py < e.miny) return LOC_EXTERIOR;
  return locate_in_ring(px, py, vx, vy, nv);
}

/* JTS Envelope.distance(point envelope) */
static double env_point_distance(env_t e, double px, double py) {
  if (!(px > e.maxx || px < e.minx || py > e.maxy || py < e.miny)) return 0.0;
  double dx = 0.0, dy = 0.0;
  if (e.maxx < px) dx = px - e.maxx; else if (e.minx > px) dx = e.minx - px;
  if (e.maxy < py) dy = py - e.maxy; else if (e.miny > py) dy = e.miny - py;
  if (dx == 0.0) return dy;
  if (dy == 0.0) return dx;
  return sqrt(dx * dx + dy * dy);
}

/* JTS DistanceOp(point, polygon).distance(): containment (PointLocator) then facet
 * distance over shell then holes (computeMinDistanceLinesPoints). */
double orc_point_polygon_distance(double px, double py, const orc_polygons* P, int32_t p,
                                  int metric) {
  int32_t r0 = P->ring_off[p], r1 = P->ring_off[p + 1];
  /* computeContainmentDistance: PointLocator.locate(pt, poly) != EXTERIOR -> 0.
   * Deliberate, documented deviation: a NaN x skips the containment test (JTS would feed
   * NaN into RobustDeterminant's branch ladder, which is not restated). */
  if (px == px) {
    int32_t v0 = P->vert_off[r0], nv = P->vert_off[r0 + 1] - v0;
    int loc = locate_in_polygon_ring(px, py, P->vx + v0, P->vy + v0, nv);
    if (loc == LOC_BOUNDARY) return 0.0;
    if (loc == LOC_INTERIOR) {
      int inside = 1;
      for (int32_t h = r0 + 1; h < r1; h++) {
        int32_t hv0 = P->vert_off[h], hnv = P->vert_off[h + 1] - hv0;
        int hl = locate_in_polygon_ring(px, py, P->vx + hv0, P->vy + hv0, hnv);
        if (hl == LOC_INTERIOR) { inside = 0; break; }
        if (hl == LOC_BOUNDARY) return 0.0;
      }
      if (inside) return 0.0;
    }
  }
  /* computeFacetDistance -> computeMinDistance(line, pt) per ring */
  double minDistance = DBL_MAX;
  for (int32_t rg = r0; rg < r1; rg++) {
    int32_t v0 = P->vert_off[rg], nv = P->vert_off[rg + 1] - v0;
    const double* vx = P->vx + v0;
    const double* vy = P->vy + v0;
    if (env_point_distance(ring_env(vx, vy, nv), px, py) > minDistance) continue;
    for (int32_t i = 0; i < nv - 1; i++) {
      double dist = point_to_segment(px, py, vx[i], vy[i], vx[i + 1], vy[i + 1], metric);
      if (dist < minDistance) minDistance = dist;
      if (minDistance <= 0.0) return minDistance;
    }
  }
  return minDistance;
}

/* DistanceFunctions.getPointPointEuclideanDistance(lon, lat, lon1, lat1) -- :60-63 */
static double pp_euclid(double lon, double lat, double lon1, double lat1) {
  double a = lat1 - lat, b = lon1 - lon;
  return sqrt(a * a + b * b); /* Math.pow(v, 2) == v*v (fdlibm e_pow special case y==2) */
}
/* DistanceFunctions.getPointLineStringNearestBBoxBorderMinEuclideanDistance -- :133-146 */
static double bbox_border(double x, double y, double x1, double y1, double x2, double y2) {
  if (x1 == x2) return pp_euclid(x, y, x1, y);
  else if (y1 == y2) return pp_euclid(x, y, x, y1);
  return 4.9e-324; /* Double.MIN_VALUE */
}
/* DistanceFunctions.getPointPolygonBBoxMinEuclideanDistance -- :150-200 */
double orc_point_bbox_distance(double x, double y, double x1, double y1, double x2, double y2) {
  if (x <= x1) {
    if (y <= y1) return pp_euclid(x, y, x1, y1);
    else if (y >= y2) return pp_euclid(x, y, x1, y2);
    else return bbox_border(x, y, x1, y1, x1, y2);
  } else if (x >= x2) {
    if (y <= y1) return pp_euclid(x, y, x2, y1);
    else if (y >= y2) return pp_euclid(x, y, x2, y2);
    else return bbox_border(x, y, x2, y1, x2, y2);
  } else {
    if (y <= y1) return bbox_border(x, y, x1, y1, x2, y1);
    else if (y >= y2) return bbox_border(x, y, x1, y2, x2, y2);
    else return 0.0;
  }
}

/* ------------------------------------------------------------------------------------ */
/* String hash set (java.util.HashSet<String> stand-in; iteration order never matters)  */
/* ------------------------------------------------------------------------------------ */

#define KEYLEN 24
typedef struct {
  char* keys;      /* cap * KEYLEN, "" = empty slot */
  int64_t cap, size;
} strset;

static uint64_t str_hash(const char* s) {
  uint64_t h = 1469598103934665603ULL;
  while (*s) { h ^= (unsigned char)*s++; h *= 1099511628211ULL; }
  return h;
}
static void ss_init(strset* s, int64_t hint) {
  int64_t cap = 16;
  while (cap < 2 * hint) cap <<= 1;
  s->keys = (char*)calloc((size_t)cap, KEYLEN);
  s->cap = cap; s->size = 0;
}
static void ss_free(strset* s) { free(s->keys); s->keys = NULL; s->cap = s->size = 0; }
static int64_t ss_find(const strset* s, const char* k) {
  uint64_t m = (uint64_t)s->cap - 1, i = str_hash(k) & m;
  for (;;) {
    const char* slot = s->keys + i * KEYLEN;
    if (!slot[0]) return -1;
    if (!strcmp(slot, k)) return (int64_t)i;
    i = (i + 1) & m;
  }
}
static int ss_contains(const strset* s, const char* k) { return ss_find(s, k) >= 0; }
static int64_t ss_add(strset* s, const char* k);
static void ss_grow(strset* s) {
  strset t;
  ss_init(&t, s->cap);
  for (int64_t i = 0; i < s->cap; i++)
    if (s->keys[i * KEYLEN]) ss_add(&t, s->keys + i * KEYLEN);
  free(s->keys);
  *s = t;
}
/* returns slot index (new or existing) */
static int64_t ss_add(strset* s, const char* k) {
  if (2 * (s->size + 1) > s->cap) ss_grow(s);
  uint64_t m = (uint64_t)s->cap - 1, i = str_hash(k) & m;
  for (;;) {
    char* slot = s->keys + i * KEYLEN;
    if (!slot[0]) { strncpy(slot, k, KEYLEN - 1); s->size++; return (int64_t)i; }
    if (!strcmp(slot, k)) return (int64_t)i;
    i = (i + 1) & m;
  }
}
static void ss_add_all(strset* dst, const strset* src) {
  for (int64_t i = 0; i < src->cap; i++)
    if (src->keys[i * KEYLEN]) ss_add(dst, src->keys + i * KEYLEN);
}

/* ------------------------------------------------------------------------------------ */
/* Guaranteed / candidate cell sets -- UniformGrid.java:165-206, 368-411                */
/* ------------------------------------------------------------------------------------ */

static int64_t lmax(int64_t a, int64_t b) { return a > b ? a : b; }
static int64_t lmin(int64_t a, int64_t b) { return a < b ? a : b; }

/* getGuaranteedNeighboringCells(r, String queryGridCellID) -- UniformGrid.java:165-190.
 * Loop bounds are clipped to the grid (validKey rejects everything outside). */
static void g_cells_of(const orc_grid* g, double r, const char* cellID, strset* out) {
  int32_t gl = orc_guaranteed_layers(g, r);
  char id[32];
  if (gl == 0) {
    ss_add(out, cellID);
  } else if (gl > 0) {
    int32_t qx, qy;
    orc_parse_cell_id(cellID, &qx, &qy);
    for (int64_t i = lmax((int64_t)qx - gl, 0); i <= lmin((int64_t)qx + gl, g->n - 1); i++)
      for (int64_t j = lmax((int64_t)qy - gl, 0); j <= lmin((int64_t)qy + gl, g->n - 1); j++)
        if (valid_key(g, i, j)) { orc_cell_id((int32_t)i, (int32_t)j, id); ss_add(out, id); }
  }
}

/* getCandidateNeighboringCells(r, String, Set G) -- UniformGrid.java:368-395 */
static void c_cells_of(const orc_grid* g, double r, const char* cellID, const strset* G,
                       strset* out) {
  int32_t cl = orc_candidate_layers(g, r);
  char id[32];
  if (cl > 0) {
    int32_t qx, qy;
    orc_parse_cell_id(cellID, &qx, &qy);
    for (int64_t i = lmax((int64_t)qx - cl, 0); i <= lmin((int64_t)qx + cl, g->n - 1); i++)
      for (int64_t j = lmax((int64_t)qy - cl, 0); j <= lmin((int64_t)qy + cl, g->n - 1); j++)
        if (valid_key(g, i, j)) {
          orc_cell_id((int32_t)i, (int32_t)j, id);
          if (!ss_contains(G, id)) ss_add(out, id);
        }
  }
}

int64_t orc_gc_sets_point(const orc_grid* g, double r, int32_t qcx, int32_t qcy,
                          int32_t* g_cells, int64_t capG, int64_t* nG,
                          int32_t* c_cells, int64_t capC, int64_t* nC) {
  char qid[32];
  strset G, C;
  orc_cell_id(qcx, qcy, qid);
  ss_init(&G, 64); ss_init(&C, 64);
  g_cells_of(g, r, qid, &G);
  c_cells_of(g, r, qid, &G, &C);
  *nG = G.size; *nC = C.size;
  int64_t w = 0;
  for (int64_t i = 0; i < G.cap && g_cells; i++)
    if (G.keys[i * KEYLEN] && w < capG) {
      orc_parse_cell_id(G.keys + i * KEYLEN, &g_cells[2 * w], &g_cells[2 * w + 1]); w++;
    }
  w = 0;
  for (int64_t i = 0; i < C.cap && c_cells; i++)
    if (C.keys[i * KEYLEN] && w < capC) {
      orc_parse_cell_id(C.keys + i * KEYLEN, &c_cells[2 * w], &c_cells[2 * w + 1]); w++;
    }
  ss_free(&G); ss_free(&C);
  return ORC_OK;
}

/* ------------------------------------------------------------------------------------ */
/* Range queries                                                                        */
/* ------------------------------------------------------------------------------------ */

static int64_t emit(int64_t* out, int64_t cap, int64_t cnt, int64_t v) {
  if (cnt < cap) out[cnt] = v;
  return cnt + 1;
}

/* PointPointRangeQuery.run, WindowBased -- PointPointRangeQuery.java:111-187 */
int64_t orc_range_pp(const orc_grid* g, int64_t n, const double* x, const double* y,
                     int32_t nq, const double* qx, const double* qy, double r,
                     int approximate, int metric, int64_t* out_idx, int64_t cap) {
  strset G, C;
  char id[32];
  ss_init(&G, 64); ss_init(&C, 64);
  /* :122-125 -- sets accumulated query by query */
  for (int32_t q = 0; q < nq; q++) {
    int32_t cx, cy;
    strset Gq, Cq;
    orc_cell_of(g, qx[q], qy[q], &cx, &cy); /* Point(x, y, uGrid), Point.java:60-67 */
    orc_cell_id(cx, cy, id);
    ss_init(&Gq, 64);
    g_cells_of(g, r, id, &Gq);
    ss_add_all(&G, &Gq);
    ss_free(&Gq);
    ss_init(&Cq, 64);
    c_cells_of(g, r, id, &G, &Cq);
    ss_add_all(&C, &Cq);
    ss_free(&Cq);
  }
  int64_t cnt = 0;
  for (int64_t i = 0; i < n; i++) {
    int32_t cx, cy;
    orc_cell_of(g, x[i], y[i], &cx, &cy); /* ingest: Point.java:91-100 */
    orc_cell_id(cx, cy, id);
    int inG = ss_contains(&G, id);
    if (!(ss_contains(&C, id) || inG)) continue; /* filter :135-140 */
    if (inG) { cnt = emit(out_idx, cap, cnt, i); continue; } /* :154-155 */
    for (int32_t q = 0; q < nq; q++) {                        /* :158-183 */
      if (approximate) {
        cnt = emit(out_idx, cap, cnt, i);
      } else {
        double d = orc_distance(qx[q], qy[q], x[i], y[i], metric);
        if (d <= r) { cnt = emit(out_idx, cap, cnt, i); break; }
      }
    }
  }
  ss_free(&G); ss_free(&C);
  return cnt;
}

/* Polygon(List<List<Coordinate>>, UniformGrid) -- Polygon.java:52-66: bbox of the shell
 * (HelperClass.getBoundingBox :76-80) and gridIDsSet = every cell under the bbox
 * (HelperClass.assignGridCellID(bBox) :123-143, no validKey). */
static void polygon_bbox(const orc_polygons* P, int32_t p, double* x1, double* y1,
                         double* x2, double* y2) {
  int32_t r0 = P->ring_off[p];
  int32_t v0 = P->vert_off[r0], nv = P->vert_off[r0 + 1] - v0;
  env_t e = ring_env(P->vx + v0, P->vy + v0, nv);
  *x1 = e.minx; *y1 = e.miny; *x2 = e.maxx; *y2 = e.maxy;
}

/* PointPolygonRangeQuery.run, WindowBased -- PointPolygonRangeQuery.java:134-205 */
int64_t orc_range_ppoly(const orc_grid* g, int64_t n, const double* x, const double* y,
                        const orc_polygons* P, double r, int approximate, int metric,
                        int64_t* out_idx, int64_t cap) {
  strset G, C;
  char id[32];
  ss_init(&G, 64); ss_init(&C, 64);
  double* bb = (double*)malloc(sizeof(double) * 4 * (size_t)(P->npoly > 0 ? P->npoly : 1));
  for (int32_t p = 0; p < P->npoly; p++) {
    double x1, y1, x2, y2;
    polygon_bbox(P, p, &x1, &y1, &x2, &y2);
    bb[4 * p] = x1; bb[4 * p + 1] = y1; bb[4 * p + 2] = x2; bb[4 * p + 3] = y2;
    int32_t xi1, yi1, xi2, yi2;
    orc_cell_of(g, x1, y1, &xi1, &yi1);
    orc_cell_of(g, x2, y2, &xi2, &yi2);
    /* getGuaranteedNeighboringCells(r, Polygon) -- UniformGrid.java:193-206 */
    strset Gp, Cp;
    ss_init(&Gp, 64);
    for (int64_t a = xi1; a <= xi2; a++)
      for (int64_t b = yi1; b <= yi2; b++) {
        orc_cell_id((int32_t)a, (int32_t)b, id);
        g_cells_of(g, r, id, &Gp);
      }
    ss_add_all(&G, &Gp);
    ss_free(&Gp);
    /* getCandidateNeighboringCells(r, Polygon, G) -- UniformGrid.java:399-411 */
    ss_init(&Cp, 64);
    for (int64_t a = xi1; a <= xi2; a++)
      for (int64_t b = yi1; b <= yi2; b++) {
        orc_cell_id((int32_t)a, (int32_t)b, id);
        c_cells_of(g, r, id, &G, &Cp);
      }
    ss_add_all(&C, &Cp);
    ss_free(&Cp);
  }
  int64_t cnt = 0;
  for (int64_t i = 0; i < n; i++) {
    int32_t cx, cy;
    orc_cell_of(g, x[i], y[i], &cx, &cy);
    orc_cell_id(cx, cy, id);
    int inG = ss_contains(&G, id);
    if (!(ss_contains(&C, id) || inG)) continue; /* :157-162 */
    if (inG) { cnt = emit(out_idx, cap, cnt, i); continue; }
    for (int32_t p = 0; p < P->npoly; p++) { /* :179-201 */
      double d = approximate
                     ? orc_point_bbox_distance(x[i], y[i], bb[4 * p], bb[4 * p + 1], bb[4 * p + 2],
                                               bb[4 * p + 3])
                     : orc_point_polygon_distance(x[i], y[i], P, p, metric);
      if (d <= r) { cnt = emit(out_idx, cap, cnt, i); break; }
    }
  }
  free(bb);
  ss_free(&G); ss_free(&C);
  return cnt;
}

/* ------------------------------------------------------------------------------------ */
/* kNN                                                                                  */
/* ------------------------------------------------------------------------------------ */

typedef struct { double d; int64_t obj; int64_t idx; } tup; /* Tuple2<Point, Double> */

/* kNN candidates: cell in C u G and d <= r -- PointPointKNNQuery.java:134-150,167-186 */
static int64_t knn_candidates(const orc_grid* g, int64_t n, const double* x, const double* y,
                              const int64_t* objID, double qx, double qy, double r, int metric,
                              tup** out, int64_t** cell_slot, strset* cells_seen) {
  strset G, C;
  char id[32];
  int32_t qcx, qcy;
  orc_cell_of(g, qx, qy, &qcx, &qcy);
  orc_cell_id(qcx, qcy, id);
  ss_init(&G, 64); ss_init(&C, 64);
  g_cells_of(g, r, id, &G);
  c_cells_of(g, r, id, &G, &C);
  tup* c = (tup*)malloc(sizeof(tup) * (size_t)(n > 0 ? n : 1));
  int64_t* slot = cell_slot ? (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1)) : NULL;
  int64_t m = 0;
  for (int64_t i = 0; i < n; i++) {
    int32_t cx, cy;
    orc_cell_of(g, x[i], y[i], &cx, &cy);
    orc_cell_id(cx, cy, id);
    if (!(ss_contains(&C, id) || ss_contains(&G, id))) continue;
    double d = orc_distance(qx, qy, x[i], y[i], metric);
    if (slot) slot[m] = ss_add(cells_seen, id);
    if (!(d <= r)) {
      if (slot) { c[m].d = NAN; c[m].obj = objID[i]; c[m].idx = i; m++; }
      continue;
    }
    c[m].d = d; c[m].obj = objID[i]; c[m].idx = i; m++;
  }
  ss_free(&G); ss_free(&C);
  *out = c;
  if (cell_slot) *cell_slot = slot;
  return m;
}

static int cmp_obj_d_idx(const void* a, const void* b) {
  const tup* p = (const tup*)a; const tup* q = (const tup*)b;
  if (p->obj != q->obj) return p->obj < q->obj ? -1 : 1;
  if (p->d != q->d) return p->d < q->d ? -1 : 1;
  return p->idx < q->idx ? -1 : (p->idx > q->idx);
}
static int cmp_d_obj(const void* a, const void* b) {
  const tup* p = (const tup*)a; const tup* q = (const tup*)b;
  if (p->d != q->d) return p->d < q->d ? -1 : 1;
  if (p->obj != q->obj) return p->obj < q->obj ? -1 : 1;
  return p->idx < q->idx ? -1 : (p->idx > q->idx);
}

/* Build contract */
int32_t orc_knn_contract(const orc_grid* g, int64_t n, const double* x, const double* y,
                         const int64_t* objID, double qx, double qy, double r, int32_t k,
                         int metric, int64_t* out_objID, double* out_d, int64_t* out_idx) {
  if (k <= 0) return ORC_ERR_ARG;
  tup* c;
  int64_t m = knn_candidates(g, n, x, y, objID, qx, qy, r, metric, &c, NULL, NULL);
  qsort(c, (size_t)m, sizeof(tup), cmp_obj_d_idx);
  int64_t u = 0;
  for (int64_t i = 0; i < m; i++)
    if (u == 0 || c[u - 1].obj != c[i].obj) c[u++] = c[i];
  qsort(c, (size_t)u, sizeof(tup), cmp_d_obj);
  int32_t nout = (int32_t)(u < k ? u : k);
  for (int32_t i = 0; i < nout; i++) {
    out_objID[i] = c[i].obj; out_d[i] = c[i].d; out_idx[i] = c[i].idx;
  }
  free(c);
  return nout;
}

/* PointPolygonKNNQuery.windowBased -- knn/PointPolygonKNNQuery.java:245-317: cell filter with the
 * polygon's guaranteed / candidate sets (UniformGrid.java:193-206,399-411, as orc_range_ppoly),
 * d = JTS point-polygon distance (DistanceFunctions.java:33-36) or, approximate, the bbox
 * distance (:150-200); d <= r; then the build contract of orc_knn_contract (one entry per objID,
 * (d, objID) order, first k). */
int32_t orc_knn_ppoly_contract(const orc_grid* g, int64_t n, const double* x, const double* y,
                               const int64_t* objID, const orc_polygons* P, double r, int32_t k,
                               int approximate, int metric, int64_t* out_objID, double* out_d,
                               int64_t* out_idx) {
  strset G, C;
  char id[32];
  double x1, y1, x2, y2;
  int32_t xi1, yi1, xi2, yi2;
  if (k <= 0 || P->npoly != 1) return ORC_ERR_ARG;
  ss_init(&G, 64); ss_init(&C, 64);
  polygon_bbox(P, 0, &x1, &y1, &x2, &y2);
  orc_cell_of(g, x1, y1, &xi1, &yi1);
  orc_cell_of(g, x2, y2, &xi2, &yi2);
  for (int64_t a = xi1; a <= xi2; a++)
    for (int64_t b = yi1; b <= yi2; b++) {
      orc_cell_id((int32_t)a, (int32_t)b, id);
      g_cells_of(g, r, id, &G);
    }
  for (int64_t a = xi1; a <= xi2; a++)
    for (int64_t b = yi1; b <= yi2; b++) {
      orc_cell_id((int32_t)a, (int32_t)b, id);
      c_cells_of(g, r, id, &G, &C);
    }
  tup* c = (tup*)malloc(sizeof(tup) * (size_t)(n > 0 ? n : 1));
  int64_t m = 0;
  for (int64_t i = 0; i < n; i++) {
    int32_t cx, cy;
    orc_cell_of(g, x[i], y[i], &cx, &cy);
    orc_cell_id(cx, cy, id);
    if (!(ss_contains(&C, id) || ss_contains(&G, id))) continue; /* :279-284 */
    double d = approximate ? orc_point_bbox_distance(x[i], y[i], x1, y1, x2, y2)
                           : orc_point_polygon_distance(x[i], y[i], P, 0, metric);
    if (!(d <= r)) continue;
    c[m].d = d; c[m].obj = objID[i]; c[m].idx = i; m++;
  }
  ss_free(&G); ss_free(&C);
  qsort(c, (size_t)m, sizeof(tup), cmp_obj_d_idx);
  int64_t u = 0;
  for (int64_t i = 0; i < m; i++)
    if (u == 0 || c[u - 1].obj != c[i].obj) c[u++] = c[i];
  qsort(c, (size_t)u, sizeof(tup), cmp_d_obj);
  int32_t nout = (int32_t)(u < k ? u : k);
  for (int32_t i = 0; i < nout; i++) {
    out_objID[i] = c[i].obj; out_d[i] = c[i].d; out_idx[i] = c[i].idx;
  }
  free(c);
  return nout;
}

/* ---- java.util.PriorityQueue<Tuple2<Point,Double>> with
 *      Comparators.inTuplePointDistanceComparator (utils/Comparators.java:14-32) ---- */
typedef struct { tup* q; int32_t size, cap; } jpq;
static int jcmp(const tup* a, const tup* b) { /* max-heap on distance */
  if (a->d > b->d) return -1;
  else if (a->d == b->d) return 0;
  return 1;
}
static void jpq_init(jpq* p, int32_t cap) {
  p->cap = cap > 0 ? cap : 1; p->size = 0; p->q = (tup*)malloc(sizeof(tup) * (size_t)p->cap);
}
static void jpq_free(jpq* p) { free(p->q); p->q = NULL; }
static void jpq_sift_up(jpq* p, int32_t k, tup x) {
  while (k > 0) {
    int32_t parent = (k - 1) >> 1;
    tup e = p->q[parent];
    if (jcmp(&x, &e) >= 0) break;
    p->q[k] = e; k = parent;
  }
  p->q[k] = x;
}
static void jpq_sift_down(jpq* p, int32_t k, tup x) {
  int32_t half = p->size >> 1;
  while (k < half) {
    int32_t child = (k << 1) + 1;
    tup c = p->q[child];
    int32_t right = child + 1;
    if (right < p->size && jcmp(&c, &p->q[right]) > 0) c = p->q[child = right];
    if (jcmp(&x, &c) <= 0) break;
    p->q[k] = c; k = child;
  }
  p->q[k] = x;
}
static void jpq_offer(jpq* p, tup e) {
  if (p->size >= p->cap) { p->cap *= 2; p->q = (tup*)realloc(p->q, sizeof(tup) * (size_t)p->cap); }
  int32_t i = p->size++;
  if (i == 0) p->q[0] = e; else jpq_sift_up(p, i, e);
}
static tup jpq_poll(jpq* p) {
  int32_t s = --p->size;
  tup result = p->q[0];
  tup x = p->q[s];
  if (s != 0) jpq_sift_down(p, 0, x);
  return result;
}
/* remove(Object) -> removeAt(indexOf), identity = point index */
static void jpq_remove_idx(jpq* p, int64_t idx) {
  int32_t i = -1;
  for (int32_t j = 0; j < p->size; j++) if (p->q[j].idx == idx) { i = j; break; }
  if (i < 0) return;
  int32_t s = --p->size;
  if (s == i) return;
  tup moved = p->q[s];
  jpq_sift_down(p, i, moved);
  if (p->q[i].idx == moved.idx) jpq_sift_up(p, i, moved);
}

typedef struct { int64_t* v; int64_t n, cap; } i64set; /* HashSet<String> objIDs (linear) */
static int i64_contains(const i64set* s, int64_t v) {
  for (int64_t i = 0; i < s->n; i++) if (s->v[i] == v) return 1;
  return 0;
}
static void i64_add(i64set* s, int64_t v) {
  if (i64_contains(s, v)) return;
  if (s->n == s->cap) { s->cap = s->cap ? 2 * s->cap : 64; s->v = (int64_t*)realloc(s->v, 8 * (size_t)s->cap); }
  s->v[s->n++] = v;
}
static void i64_remove(i64set* s, int64_t v) {
  for (int64_t i = 0; i < s->n; i++) if (s->v[i] == v) { s->v[i] = s->v[--s->n]; return; }
}

/* Per-cell apply of PointPointKNNQuery.windowBased (:159-192) on one cell's candidates in
 * arrival order: a bounded max-heap of (Point, d) over d <= r, replaced iff peek.d > d.  The
 * heap (array order) is written to out[0 .. return). */
static int32_t knn_cell_apply(const tup* c, int64_t m, int32_t k, tup* out) {
  jpq pq;
  jpq_init(&pq, k);
  for (int64_t i = 0; i < m; i++) {
    double d = c[i].d; /* NaN marks d > r (distance already tested) */
    if (pq.size < k) {
      if (d == d) jpq_offer(&pq, c[i]);
    } else if (d == d) {
      double largest = pq.q[0].d;
      if (largest > d) { jpq_poll(&pq); jpq_offer(&pq, c[i]); }
    }
  }
  int32_t n = pq.size;
  if (n > 0) memcpy(out, pq.q, sizeof(tup) * (size_t)n);
  jpq_free(&pq);
  return n;
}

/* KNNQuery.kNNWinAllEvaluationPointStream (:213-272): merge the per-cell heaps (cells in the
 * given order) into one k-heap with the objID set, its eviction bug included. */
static int32_t knn_winall_merge(const tup* heaps, const int64_t* heap_off, int64_t ncell, int32_t k,
                                int64_t* out_objID, double* out_d, int64_t* out_idx) {
  jpq W;
  i64set objIDs = {0};
  jpq_init(&W, k);
  int status = ORC_OK;
  for (int64_t ci = 0; ci < ncell && status == ORC_OK; ci++) {
    for (int64_t t = heap_off[ci]; t < heap_off[ci + 1]; t++) {
      tup cand = heaps[t];
      if (W.size < k) {
        if (!i64_contains(&objIDs, cand.obj)) {
          jpq_offer(&W, cand); i64_add(&objIDs, cand.obj);
        } else {
          for (int32_t e = 0; e < W.size; e++)
            if (W.q[e].obj == cand.obj && W.q[e].d > cand.d) {
              jpq_remove_idx(&W, W.q[e].idx); jpq_offer(&W, cand); break;
            }
        }
      } else {
        double largest = W.q[0].d;
        if (largest > cand.d) {
          if (!i64_contains(&objIDs, cand.obj)) {
            jpq_poll(&W);
            if (W.size == 0) { status = ORC_ERR_NPE; break; } /* peek() == null -> NPE */
            i64_remove(&objIDs, W.q[0].obj); /* the reference's bug: removes the NEW peek */
            jpq_offer(&W, cand); i64_add(&objIDs, cand.obj);
          } else {
            for (int32_t e = 0; e < W.size; e++)
              if (W.q[e].obj == cand.obj && W.q[e].d > cand.d) {
                jpq_remove_idx(&W, W.q[e].idx); jpq_offer(&W, cand); break;
              }
          }
        }
      }
    }
  }
  int32_t nout = W.size;
  if (status == ORC_OK)
    for (int32_t i = 0; i < nout; i++) {
      out_objID[i] = W.q[i].obj; out_d[i] = W.q[i].d; out_idx[i] = W.q[i].idx;
    }
  jpq_free(&W);
  free(objIDs.v);
  return status == ORC_OK ? nout : status;
}

/* PointPointKNNQuery.windowBased apply (:159-192) + KNNQuery.kNNWinAllEvaluationPointStream
 * (:213-272).  Cells visited in first-appearance order; each cell's candidates in arrival
 * order (the keyed window buffer), grouped by a stable counting sort on the cell slot. */
int32_t orc_knn_reference(const orc_grid* g, int64_t n, const double* x, const double* y,
                          const int64_t* objID, double qx, double qy, double r, int32_t k,
                          int metric, int64_t* out_objID, double* out_d, int64_t* out_idx) {
  if (k <= 0) return ORC_ERR_ARG; /* new PriorityQueue(k<1) throws */
  strset cells;
  ss_init(&cells, n + 16); /* sized so it never rehashes: slot indices stay valid */
  tup* c;
  int64_t* slot;
  int64_t m = knn_candidates(g, n, x, y, objID, qx, qy, r, metric, &c, &slot, &cells);
  /* cell rank in first-appearance order, then a stable counting sort of the candidates */
  int64_t* rank = (int64_t*)malloc(sizeof(int64_t) * (size_t)cells.cap);
  int64_t ncell = 0;
  for (int64_t i = 0; i < cells.cap; i++) rank[i] = -1;
  for (int64_t i = 0; i < m; i++)
    if (rank[slot[i]] < 0) rank[slot[i]] = ncell++;
  int64_t* off = (int64_t*)calloc((size_t)ncell + 1, sizeof(int64_t));
  for (int64_t i = 0; i < m; i++) off[rank[slot[i]] + 1]++;
  for (int64_t ci = 0; ci < ncell; ci++) off[ci + 1] += off[ci];
  tup* grouped = (tup*)malloc(sizeof(tup) * (size_t)(m > 0 ? m : 1));
  int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ncell > 0 ? ncell : 1));
  for (int64_t ci = 0; ci < ncell; ci++) cur[ci] = off[ci];
  for (int64_t i = 0; i < m; i++) grouped[cur[rank[slot[i]]]++] = c[i];
  /* per-cell heaps, concatenated in cell order */
  tup* heaps = (tup*)malloc(sizeof(tup) * (size_t)(m > 0 ? m : 1));
  int64_t* hoff = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ncell + 1));
  hoff[0] = 0;
  for (int64_t ci = 0; ci < ncell; ci++)
    hoff[ci + 1] = hoff[ci] + knn_cell_apply(grouped + off[ci], off[ci + 1] - off[ci], k, heaps + hoff[ci]);
  int32_t st = knn_winall_merge(heaps, hoff, ncell, k, out_objID, out_d, out_idx);
  free(rank); free(off); free(grouped); free(cur); free(heaps); free(hoff); free(c); free(slot);
  ss_free(&cells);
  return st;
}

/* ---- the same operator on T host threads, shaped as Flink runs it with parallelism T
 * (conf/geoflink-conf.yml:55; keyBy(gridID) over subtasks, PointPointKNNQuery.java:144-158):
 *   source subtasks   contiguous point ranges: cell-ID string, HashSet C/G filter, JTS distance;
 *                     each candidate goes to key subtask hash(gridID) % T (the shuffle)
 *   key subtasks      group their candidates by cell string (arrival order kept: sources are
 *                     drained in order), per-cell bounded heap (:159-192)
 *   windowAll         one thread merges every cell's heap (KNNQuery.java:213-272), cells in
 *                     first-appearance order -- so the result equals orc_knn_reference. */
#include <pthread.h>

typedef struct { tup t; uint64_t h; int32_t cx, cy; } cand_t;
typedef struct { cand_t* v; int64_t n, cap; } cvec;
static void cvec_push(cvec* a, cand_t c) {
  if (a->n == a->cap) { a->cap = a->cap ? 2 * a->cap : 1024; a->v = (cand_t*)realloc(a->v, sizeof(cand_t) * (size_t)a->cap); }
  a->v[a->n++] = c;
}
typedef struct { int64_t first; int64_t off, cnt; const tup* h; } cellrun;
typedef struct {
  int T, tid;
  const orc_grid* g;
  int64_t n;
  const double *x, *y;
  const int64_t* objID;
  double qx, qy, r;
  int32_t k;
  int metric;
  const strset *G, *C;
  cvec* out;            /* [T * T]: out[src * T + dst] */
  /* key phase results */
  tup* heaps;
  cellrun* runs;
  int64_t nruns;
  pthread_barrier_t* bar;
} mt_arg;

static void* knn_mt_worker(void* p) {
  mt_arg* a = (mt_arg*)p;
  const int T = a->T, t = a->tid;
  char id[32];
  /* source subtask: points [lo, hi) */
  const int64_t lo = a->n * t / T, hi = a->n * (t + 1) / T;
  for (int64_t i = lo; i < hi; i++) {
    int32_t cx, cy;
    orc_cell_of(a->g, a->x[i], a->y[i], &cx, &cy);
    orc_cell_id(cx, cy, id);
    if (!(ss_contains(a->C, id) || ss_contains(a->G, id))) continue;
    double d = orc_distance(a->qx, a->qy, a->x[i], a->y[i], a->metric);
    cand_t c;
    c.t.d = d <= a->r ? d : NAN; c.t.obj = a->objID[i]; c.t.idx = i;
    c.h = str_hash(id); c.cx = cx; c.cy = cy;
    cvec_push(&a->out[(int64_t)t * T + (int64_t)(c.h % (uint64_t)T)], c);
  }
  pthread_barrier_wait(a->bar);
  /* key subtask t: its candidates from every source, in source (= arrival) order */
  int64_t m = 0;
  for (int s = 0; s < T; s++) m += a->out[(int64_t)s * T + t].n;
  strset keys;
  ss_init(&keys, m + 16);
  int64_t* rank = (int64_t*)malloc(sizeof(int64_t) * (size_t)keys.cap);
  for (int64_t i = 0; i < keys.cap; i++) rank[i] = -1;
  int64_t* slot = (int64_t*)malloc(sizeof(int64_t) * (size_t)(m > 0 ? m : 1));
  cellrun* runs = (cellrun*)malloc(sizeof(cellrun) * (size_t)(m > 0 ? m : 1));
  int64_t nr = 0, j = 0;
  for (int s = 0; s < T; s++) {
    const cvec* v = &a->out[(int64_t)s * T + t];
    for (int64_t i = 0; i < v->n; i++, j++) {
      orc_cell_id(v->v[i].cx, v->v[i].cy, id);
      int64_t sl = ss_add(&keys, id);
      if (rank[sl] < 0) { rank[sl] = nr; runs[nr].first = v->v[i].t.idx; runs[nr].cnt = 0; nr++; }
      slot[j] = rank[sl];
      runs[slot[j]].cnt++;
    }
  }
  int64_t acc = 0;
  for (int64_t ri = 0; ri < nr; ri++) { runs[ri].off = acc; acc += runs[ri].cnt; runs[ri].cnt = 0; }
  tup* grouped = (tup*)malloc(sizeof(tup) * (size_t)(m > 0 ? m : 1));
  j = 0;
  for (int s = 0; s < T; s++) {
    const cvec* v = &a->out[(int64_t)s * T + t];
    for (int64_t i = 0; i < v->n; i++, j++) {
      cellrun* R = &runs[slot[j]];
      grouped[R->off + R->cnt++] = v->v[i].t;
    }
  }
  /* per-cell heaps: heap of run ri replaces its candidates at the same offset */
  a->heaps = (tup*)malloc(sizeof(tup) * (size_t)(m > 0 ? m : 1));
  for (int64_t ri = 0; ri < nr; ri++) {
    int32_t h = knn_cell_apply(grouped + runs[ri].off, runs[ri].cnt, a->k, a->heaps + runs[ri].off);
    runs[ri].cnt = h;
    runs[ri].h = a->heaps + runs[ri].off;
  }
  a->runs = runs;
  a->nruns = nr;
  free(grouped); free(slot); free(rank);
  ss_free(&keys);
  return NULL;
}

static int cmp_run_first(const void* p, const void* q) {
  const cellrun* a = *(const cellrun* const*)p; const cellrun* b = *(const cellrun* const*)q;
  return a->first < b->first ? -1 : (a->first > b->first);
}

int32_t orc_knn_reference_mt(const orc_grid* g, int64_t n, const double* x, const double* y,
                             const int64_t* objID, double qx, double qy, double r, int32_t k,
                             int metric, int nthreads, int64_t* out_objID, double* out_d, int64_t* out_idx) {
  if (k <= 0) return ORC_ERR_ARG;
  const int T = nthreads < 1 ? 1 : nthreads;
  strset G, C;
  char id[32];
  int32_t qcx, qcy;
  orc_cell_of(g, qx, qy, &qcx, &qcy);
  orc_cell_id(qcx, qcy, id);
  ss_init(&G, 64); ss_init(&C, 64);
  g_cells_of(g, r, id, &G);
  c_cells_of(g, r, id, &G, &C);
  cvec* out = (cvec*)calloc((size_t)T * (size_t)T, sizeof(cvec));
  mt_arg* args = (mt_arg*)calloc((size_t)T, sizeof(mt_arg));
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)T);
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)T);
  for (int t = 0; t < T; t++) {
    mt_arg* a = &args[t];
    a->T = T; a->tid = t; a->g = g; a->n = n; a->x = x; a->y = y; a->objID = objID;
    a->qx = qx; a->qy = qy; a->r = r; a->k = k; a->metric = metric; a->G = &G; a->C = &C;
    a->out = out; a->bar = &bar;
    if (t > 0) pthread_create(&th[t], NULL, knn_mt_worker, a);
  }
  knn_mt_worker(&args[0]);
  for (int t = 1; t < T; t++) pthread_join(th[t], NULL);
  pthread_barrier_destroy(&bar);
  /* windowAll: every cell's heap, cells in first-appearance order */
  int64_t ncell = 0, total = 0;
  for (int t = 0; t < T; t++) ncell += args[t].nruns;
  cellrun** order = (cellrun**)malloc(sizeof(cellrun*) * (size_t)(ncell > 0 ? ncell : 1));
  int64_t w = 0;
  for (int t = 0; t < T; t++)
    for (int64_t ri = 0; ri < args[t].nruns; ri++) order[w++] = &args[t].runs[ri];
  qsort(order, (size_t)ncell, sizeof(cellrun*), cmp_run_first);
  for (int64_t ci = 0; ci < ncell; ci++) total += order[ci]->cnt;
  tup* heaps = (tup*)malloc(sizeof(tup) * (size_t)(total > 0 ? total : 1));
  int64_t* hoff = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ncell + 1));
  hoff[0] = 0;
  for (int64_t ci = 0; ci < ncell; ci++) {
    const cellrun* R = order[ci];
    if (R->cnt) memcpy(heaps + hoff[ci], R->h, sizeof(tup) * (size_t)R->cnt);
    hoff[ci + 1] = hoff[ci] + R->cnt;
  }
  int32_t st = knn_winall_merge(heaps, hoff, ncell, k, out_objID, out_d, out_idx);
  for (int t = 0; t < T; t++) { free(args[t].heaps); free(args[t].runs); }
  for (int64_t i = 0; i < (int64_t)T * T; i++) free(out[i].v);
  free(out); free(args); free(th); free(order); free(heaps); free(hoff);
  ss_free(&G); ss_free(&C);
  return st;
}

/* ------------------------------------------------------------------------------------ */
/* Join -- JoinQuery.getReplicatedPointQueryStream (:73-90) + PointPointJoinQuery (:124-183) */
/* ------------------------------------------------------------------------------------ */

int64_t orc_join_pp(const orc_grid* ugrid, const orc_grid* qgrid,
                    int64_t no, const double* ox, const double* oy,
                    int64_t nq, const double* qx, const double* qy,
                    double r, int approximate, int metric, int64_t* out_pairs, int64_t cap) {
  char id[32];
  int32_t cl = 0;
  if (!(r == 0)) {
    cl = orc_candidate_layers(qgrid, r);
    if (cl <= 0) return ORC_ERR_LAYERS; /* UniformGrid.java:272-276 System.exit(1) */
  }
  /* replicate: cell string -> list of query indices */
  strset cells;
  ss_init(&cells, 1024);
  int64_t nrep = 0, repcap = 1024;
  int64_t* rep_slot = (int64_t*)malloc(8 * (size_t)repcap);
  int64_t* rep_q = (int64_t*)malloc(8 * (size_t)repcap);
  for (int64_t q = 0; q < nq; q++) {
    int64_t i0, i1, j0, j1;
    if (r == 0) { /* getNeighboringCells: return girdCellsSet (UniformGrid.java:264-266) */
      i0 = 0; i1 = qgrid->n - 1; j0 = 0; j1 = qgrid->n - 1;
    } else {
      int32_t cx, cy, px, py;
      orc_cell_of(qgrid, qx[q], qy[q], &cx, &cy);
      orc_cell_id(cx, cy, id);
      orc_parse_cell_id(id, &px, &py); /* :279 getIntCellIndices(queryCellID) */
      i0 = lmax((int64_t)px - cl, 0); i1 = lmin((int64_t)px + cl, qgrid->n - 1);
      j0 = lmax((int64_t)py - cl, 0); j1 = lmin((int64_t)py + cl, qgrid->n - 1);
    }
    for (int64_t i = i0; i <= i1; i++)
      for (int64_t j = j0; j <= j1; j++) {
        if (!valid_key(qgrid, i, j)) continue;
        orc_cell_id((int32_t)i, (int32_t)j, id);
        if (nrep == repcap) {
          repcap *= 2;
          rep_slot = (int64_t*)realloc(rep_slot, 8 * (size_t)repcap);
          rep_q = (int64_t*)realloc(rep_q, 8 * (size_t)repcap);
        }
        rep_slot[nrep] = -1; /* slot assigned after all insertions (set may grow) */
        rep_q[nrep] = q;
        ss_add(&cells, id);
        nrep++;
      }
  }
  /* resolve slots now that the set is final; regenerate ids in the same order */
  {
    int64_t t = 0;
    for (int64_t q = 0; q < nq; q++) {
      int64_t i0, i1, j0, j1;
      if (r == 0) { i0 = 0; i1 = qgrid->n - 1; j0 = 0; j1 = qgrid->n - 1; }
      else {
        int32_t cx, cy, px, py;
        orc_cell_of(qgrid, qx[q], qy[q], &cx, &cy);
        orc_cell_id(cx, cy, id);
        orc_parse_cell_id(id, &px, &py);
        i0 = lmax((int64_t)px - cl, 0); i1 = lmin((int64_t)px + cl, qgrid->n - 1);
        j0 = lmax((int64_t)py - cl, 0); j1 = lmin((int64_t)py + cl, qgrid->n - 1);
      }
      for (int64_t i = i0; i <= i1; i++)
        for (int64_t j = j0; j <= j1; j++) {
          if (!valid_key(qgrid, i, j)) continue;
          orc_cell_id((int32_t)i, (int32_t)j, id);
          rep_slot[t++] = ss_find(&cells, id);
        }
    }
  }
  /* bucket replicated queries by slot (CSR) */
  int64_t* off = (int64_t*)calloc((size_t)cells.cap + 1, 8);
  int64_t* lst = (int64_t*)malloc(8 * (size_t)(nrep > 0 ? nrep : 1));
  for (int64_t t = 0; t < nrep; t++) off[rep_slot[t] + 1]++;
  for (int64_t s = 0; s < cells.cap; s++) off[s + 1] += off[s];
  {
    int64_t* cur = (int64_t*)malloc(8 * (size_t)cells.cap);
    memcpy(cur, off, 8 * (size_t)cells.cap);
    for (int64_t t = 0; t < nrep; t++) lst[cur[rep_slot[t]]++] = rep_q[t];
    free(cur);
  }
  /* window join on gridID: JoinFunction.join per co-located pair (:160-175) */
  int64_t cnt = 0;
  for (int64_t p = 0; p < no; p++) {
    int32_t cx, cy;
    orc_cell_of(ugrid, ox[p], oy[p], &cx, &cy);
    orc_cell_id(cx, cy, id);
    int64_t s = ss_find(&cells, id);
    if (s < 0) continue;
    for (int64_t t = off[s]; t < off[s + 1]; t++) {
      int64_t q = lst[t];
      if (approximate || orc_distance(ox[p], oy[p], qx[q], qy[q], metric) <= r) {
        if (cnt < cap) { out_pairs[2 * cnt] = p; out_pairs[2 * cnt + 1] = q; }
        cnt++;
      }
    }
  }
  free(off); free(lst); free(rep_slot); free(rep_q);
  ss_free(&cells);
  return cnt;
}

/* PointPolygonJoinQuery.windowBased -- PointPolygonJoinQuery.java:154-213, with the query
 * polygons replicated by JoinQuery.getReplicatedPolygonQueryStream (JoinQuery.java:93-115):
 * polygon q goes to every key of getGuaranteedNeighboringCells(r, q) (UniformGrid.java:193-206)
 * and of getCandidateNeighboringCells(r, q, G_q) (:399-411) -- its OWN G, not a global one.
 * The window join on gridID pairs point p (key = p.gridID on ugrid) with each replica whose key
 * equals it; JoinFunction.join keeps (p, q) if approximate or getDistance(p, q) <= r
 * (DistanceFunctions.java:33-36).  A polygon's keys form a set, so a pair appears at most once.
 * Pairs come out grouped by point, polygons in replication order. */
/* The polygon side's replication (JoinQuery.getReplicatedPolygonQueryStream) as a key -> polygon
 * CSR: cells holds every replicated key; the replicas of key slot s are lst[off[s] .. off[s+1]),
 * in replication order. */
static void ppoly_replicate(const orc_grid* qgrid, const orc_polygons* P, double r, strset* cells_out,
                            int64_t** off_out, int64_t** lst_out) {
  char id[32];
  strset cells; /* every replicated key */
  ss_init(&cells, 1024);
  int64_t nrep = 0, repcap = 1024;
  char* rep_key = (char*)malloc(KEYLEN * (size_t)repcap);
  int64_t* rep_q = (int64_t*)malloc(8 * (size_t)repcap);
  for (int32_t q = 0; q < P->npoly; q++) {
    double x1, y1, x2, y2;
    polygon_bbox(P, q, &x1, &y1, &x2, &y2);
    int32_t xi1, yi1, xi2, yi2;
    orc_cell_of(qgrid, x1, y1, &xi1, &yi1); /* Polygon.gridIDsSet: cells under the bbox */
    orc_cell_of(qgrid, x2, y2, &xi2, &yi2);
    strset Gq, Cq;
    ss_init(&Gq, 64);
    ss_init(&Cq, 64);
    for (int64_t a = xi1; a <= xi2; a++)
      for (int64_t b = yi1; b <= yi2; b++) {
        orc_cell_id((int32_t)a, (int32_t)b, id);
        g_cells_of(qgrid, r, id, &Gq);
      }
    for (int64_t a = xi1; a <= xi2; a++)
      for (int64_t b = yi1; b <= yi2; b++) {
        orc_cell_id((int32_t)a, (int32_t)b, id);
        c_cells_of(qgrid, r, id, &Gq, &Cq);
      }
    const strset* sets[2] = {&Gq, &Cq};
    for (int k = 0; k < 2; k++)
      for (int64_t i = 0; i < sets[k]->cap; i++) {
        const char* key = sets[k]->keys + i * KEYLEN;
        if (!key[0]) continue;
        if (nrep == repcap) {
          repcap *= 2;
          rep_key = (char*)realloc(rep_key, KEYLEN * (size_t)repcap);
          rep_q = (int64_t*)realloc(rep_q, 8 * (size_t)repcap);
        }
        memcpy(rep_key + nrep * KEYLEN, key, KEYLEN);
        rep_q[nrep++] = q;
        ss_add(&cells, key);
      }
    ss_free(&Gq);
    ss_free(&Cq);
  }
  /* bucket the replicas by key slot (CSR), replication order kept inside a key */
  int64_t* off = (int64_t*)calloc((size_t)cells.cap + 1, 8);
  int64_t* slot = (int64_t*)malloc(8 * (size_t)(nrep > 0 ? nrep : 1));
  int64_t* lst = (int64_t*)malloc(8 * (size_t)(nrep > 0 ? nrep : 1));
  for (int64_t t = 0; t < nrep; t++) { slot[t] = ss_find(&cells, rep_key + t * KEYLEN); off[slot[t] + 1]++; }
  for (int64_t s2 = 0; s2 < cells.cap; s2++) off[s2 + 1] += off[s2];
  {
    int64_t* cur = (int64_t*)malloc(8 * (size_t)(cells.cap > 0 ? cells.cap : 1));
    memcpy(cur, off, 8 * (size_t)cells.cap);
    for (int64_t t = 0; t < nrep; t++) lst[cur[slot[t]]++] = rep_q[t];
    free(cur);
  }
  free(slot); free(rep_key); free(rep_q);
  *cells_out = cells;
  *off_out = off;
  *lst_out = lst;
}

int64_t orc_join_ppoly(const orc_grid* ugrid, const orc_grid* qgrid, int64_t no, const double* ox,
                       const double* oy, const orc_polygons* P, double r, int approximate, int metric,
                       int64_t* out_pairs, int64_t cap) {
  char id[32];
  strset cells;
  int64_t *off, *lst;
  ppoly_replicate(qgrid, P, r, &cells, &off, &lst);
  int64_t cnt = 0;
  for (int64_t p = 0; p < no; p++) {
    int32_t cx, cy;
    orc_cell_of(ugrid, ox[p], oy[p], &cx, &cy);
    orc_cell_id(cx, cy, id);
    int64_t s2 = ss_find(&cells, id);
    if (s2 < 0) continue;
    for (int64_t t = off[s2]; t < off[s2 + 1]; t++) {
      int64_t q = lst[t];
      if (approximate || orc_point_polygon_distance(ox[p], oy[p], P, (int32_t)q, metric) <= r) {
        if (cnt < cap) { out_pairs[2 * cnt] = p; out_pairs[2 * cnt + 1] = q; }
        cnt++;
      }
    }
  }
  free(off); free(lst);
  ss_free(&cells);
  return cnt;
}

/* ------------------------------------------------------------------------------------ */
/* Generators                                                                           */
/* ------------------------------------------------------------------------------------ */

/* HelperClass.generateQueryPolygons -- HelperClass.java:387-421 */
int32_t orc_generate_query_polygons(int32_t numQueryPolygons, double minX, double minY,
                                    double maxX, double maxY, double* vx, double* vy, int32_t cap) {
  int gridSize = 100;
  double polyLength1 = (maxX - minX) / gridSize;
  double polyLength2 = (maxY - minY) / gridSize;
  double polyLength = polyLength2 < polyLength1 ? polyLength2 : polyLength1;
  int32_t count = 0;
  for (double i = minX; i < maxX; i += polyLength) {
    if (count >= numQueryPolygons) break;
    for (double j = minY; j < maxY; j += polyLength) {
      if (count < cap) {
        double* px = vx + 5 * count;
        double* py = vy + 5 * count;
        px[0] = i;              py[0] = j;
        px[1] = i + polyLength; py[1] = j;
        px[2] = i + polyLength; py[2] = j + polyLength;
        px[3] = i;              py[3] = j + polyLength;
        px[4] = i;              py[4] = j;
      }
      count++;
    }
  }
  return count;
}

/* java.util.Random(seed): 48-bit LCG, nextDouble() = ((next(26) << 27) + next(27)) * 2^-53 */
typedef struct { uint64_t seed; } jrandom;
static void jr_init(jrandom* r, int64_t seed) {
  r->seed = ((uint64_t)seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1);
}
static int32_t jr_next(jrandom* r, int bits) {
  r->seed = (r->seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
  return (int32_t)(r->seed >> (48 - bits));
}
static double jr_next_double(jrandom* r) {
  int64_t hi = jr_next(r, 26);
  int64_t lo = jr_next(r, 27);
  return (double)((hi << 27) + lo) * 0x1.0p-53;
}

void orc_java_random_points(int64_t seed, int64_t n, double minX, double maxX,
                            double minY, double maxY, double* x, double* y) {
  jrandom r;
  jr_init(&r, seed);
  for (int64_t i = 0; i < n; i++) {
    x[i] = minX + jr_next_double(&r) * (maxX - minX);
    y[i] = minY + jr_next_double(&r) * (maxY - minY);
  }
}

/* ------------------------------------------------------------------------------------
 * CSV / TSV ingest -- Deserialization.CSVTSVToTSpatial.map (Deserialization.java:314-322):
 *   strArrayList = Arrays.asList(str.replace("\"", "").split("\\s*" + delimiter + "\\s*"));
 *   String strOId = get(objid)   (the field itself: any String, whitespace kept, :317)
 *   long time = Long.valueOf(get(time))     (:318)
 *   double x = Double.valueOf(get(x)), y = Double.valueOf(get(y))   (:319-320; JDK
 *   FloatingDecimal: trim, Java literal grammar, correctly rounded; glibc strtod is correctly
 *   rounded too).  Evaluated in that order: the first get() past the fields
 *   (IndexOutOfBoundsException) or malformed number (NumberFormatException) is the error.
 *   Lines come from Flink's TextInputFormat: split on '\n', a trailing '\r' dropped.
 * ------------------------------------------------------------------------------------ */
static int orc_java_s(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\x0B' || c == '\f' || c == '\r'; }

/* String.split(regex "\s*D\s*") with limit 0: returns field count, fields as [fb, fe) */
static int orc_java_split(const char* s, int n, char D, int* fb, int* fe, int maxf) {
  int nf = 0, start = 0, pos = 0;
  while (pos < n) {
    int p, mb = -1, me = -1;
    for (p = pos; p < n; ++p) {  /* leftmost match */
      int q = p;
      while (q < n && orc_java_s(s[q])) ++q;
      if (orc_java_s(D)) {
        int r, has = 0;
        for (r = p; r < q; ++r) has |= s[r] == D;
        if (q > p && has) { mb = p; me = q; break; }
      } else if (q < n && s[q] == D) {
        int r = q + 1;
        while (r < n && orc_java_s(s[r])) ++r;
        mb = p; me = r;
        break;
      }
    }
    if (mb < 0) break;
    if (nf < maxf) { fb[nf] = start; fe[nf] = mb; }
    ++nf;
    start = me;
    pos = me;
  }
  if (nf < maxf) { fb[nf] = start; fe[nf] = n; }
  ++nf;
  while (nf > 0 && nf <= maxf && fe[nf - 1] == fb[nf - 1]) --nf;  /* trailing empty strings removed */
  return nf;
}

/* Long.valueOf: [+-]digits, no whitespace, overflow -> NumberFormatException */
static int orc_java_long(const char* s, int n, int64_t* out) {
  int i = 0, neg = 0;
  uint64_t v = 0, lim;
  if (n == 0) return 1;
  if (s[0] == '-' || s[0] == '+') { neg = s[0] == '-'; i = 1; }
  if (i == n) return 1;
  lim = neg ? 9223372036854775808ull : 9223372036854775807ull;
  for (; i < n; ++i) {
    uint64_t d;
    if (s[i] < '0' || s[i] > '9') return 1;
    d = (uint64_t)(s[i] - '0');
    if (v > (lim - d) / 10) return 1;
    v = v * 10 + d;
  }
  *out = neg ? (int64_t)(0ull - v) : (int64_t)v;
  return 0;
}

static int orc_isdig(char c) { return c >= '0' && c <= '9'; }
static int orc_ishex(char c) { return orc_isdig(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

/* Double.valueOf: 0 ok, 1 NumberFormatException; *hex = 1 for a hexadecimal literal */
static int orc_java_double(const char* s0, int n, double* out, int* hex) {
  char buf[512];
  int b = 0, e = n, i, neg = 0, nd = 0;
  *hex = 0;
  while (b < e && (unsigned char)s0[b] <= ' ') ++b;  /* String.trim() */
  while (e > b && (unsigned char)s0[e - 1] <= ' ') --e;
  if (e - b <= 0 || e - b >= (int)sizeof(buf)) return 1;
  memcpy(buf, s0 + b, (size_t)(e - b));
  n = e - b;
  buf[n] = 0;
  i = 0;
  if (buf[0] == '+' || buf[0] == '-') { neg = buf[0] == '-'; i = 1; }
  if (!strcmp(buf + i, "NaN")) { *out = NAN; return 0; }
  if (!strcmp(buf + i, "Infinity")) { *out = neg ? -INFINITY : INFINITY; return 0; }
  if (n > 0 && (buf[n - 1] == 'f' || buf[n - 1] == 'F' || buf[n - 1] == 'd' || buf[n - 1] == 'D')) buf[--n] = 0;
  if (buf[i] == '0' && (buf[i + 1] == 'x' || buf[i + 1] == 'X')) {  /* 0x h* [. h*] p [+-] d+ */
    int j = i + 2, nh = 0;
    while (orc_ishex(buf[j])) { ++j; ++nh; }
    if (buf[j] == '.') { ++j; while (orc_ishex(buf[j])) { ++j; ++nh; } }
    if (!nh || (buf[j] != 'p' && buf[j] != 'P')) return 1;
    ++j;
    if (buf[j] == '+' || buf[j] == '-') ++j;
    if (!orc_isdig(buf[j])) return 1;
    while (orc_isdig(buf[j])) ++j;
    if (j != n) return 1;
    *hex = 1;
    *out = strtod(buf, NULL);
    return 0;
  }
  {
    int j = i;
    while (orc_isdig(buf[j])) { ++j; ++nd; }
    if (buf[j] == '.') { ++j; while (orc_isdig(buf[j])) { ++j; ++nd; } }
    if (!nd) return 1;
    if (buf[j] == 'e' || buf[j] == 'E') {
      ++j;
      if (buf[j] == '+' || buf[j] == '-') ++j;
      if (!orc_isdig(buf[j])) return 1;
      while (orc_isdig(buf[j])) ++j;
    }
    if (j != n) return 1;
  }
  *out = strtod(buf, NULL);
  return 0;
}

int64_t orc_csv_parse(const char* text, int64_t len, char delim, const int32_t* want, double* x, double* y,
                      char* oid, int64_t oid_cap, int64_t* oid_off, int64_t* oid_len, int64_t* ts, int64_t cap,
                      int64_t* bad_line, int32_t* bad_kind) {
  int64_t pos = 0, line = 0, ob = 0;
  char* buf = NULL;
  int bufcap = 0, *fidx = NULL;
  *bad_line = -1;
  *bad_kind = 0;
  while (pos < len) {
    int64_t e = pos, le;
    int n = 0, nf = 0, kind = 0, *fb, *fe;
    int64_t t = 0;
    double vx = 0, vy = 0;
    int hx = 0, hy = 0;
    while (e < len && text[e] != '\n') ++e;
    le = e;
    if (le > pos && text[le - 1] == '\r') --le;
    if (le - pos + 1 > bufcap) {
      bufcap = (int)(le - pos + 1) * 2;
      buf = (char*)realloc(buf, (size_t)bufcap);
      fidx = (int*)realloc(fidx, sizeof(int) * 2 * (size_t)(bufcap + 2));
    }
    fb = fidx;
    fe = fidx + bufcap + 2;
    for (int64_t i = pos; i < le; ++i)
      if (text[i] != '"') buf[n++] = text[i];  /* str.replace("\"", "") */
    if (oid_off && line < cap) oid_off[line] = ob;
    if (le == pos) kind = 4;
    else {
      nf = orc_java_split(buf, n, delim, fb, fe, bufcap + 2);
      if (want[0] >= nf) kind = 3;                                   /* get(objid) */
      else {
        const int ol = fe[want[0]] - fb[want[0]];
        if (oid && ob + ol <= oid_cap) memcpy(oid + ob, buf + fb[want[0]], (size_t)ol);
        ob += ol;
      }
      if (!kind && want[1] >= nf) kind = 3;                          /* Long.valueOf(get(time)) */
      if (!kind && orc_java_long(buf + fb[want[1]], fe[want[1]] - fb[want[1]], &t)) kind = 1;
      if (!kind && want[2] >= nf) kind = 3;                          /* Double.valueOf(get(x)) */
      if (!kind && orc_java_double(buf + fb[want[2]], fe[want[2]] - fb[want[2]], &vx, &hx)) kind = 1;
      if (!kind && want[3] >= nf) kind = 3;                          /* Double.valueOf(get(y)) */
      if (!kind && orc_java_double(buf + fb[want[3]], fe[want[3]] - fb[want[3]], &vy, &hy)) kind = 1;
      if (!kind && line < cap) { x[line] = vx; y[line] = vy; ts[line] = t; }
      if (!kind && (hx || hy)) kind = 2;  /* valid Java; reported so tests can pin the device's answer */
    }
    if (kind && *bad_line < 0) { *bad_line = line; *bad_kind = kind; }
    ++line;
    pos = e + 1;
  }
  if (oid_off && line <= cap) oid_off[line] = ob;
  *oid_len = ob;
  free(buf);
  free(fidx);
  return line;
}

/* ------------------------------------------------------------------------------------ */
/* Multi-core CPU baselines (bench only; TEST / BASELINE INFRASTRUCTURE).  The reference  */
/* operators as Flink runs them with parallelism T (conf/geoflink-conf.yml:55): source    */
/* subtasks evaluate the per-point work up to the keyBy(gridID) (string cell ID, HashSet  */
/* membership), survivors are shuffled to key subtask hash(gridID) % T, and the key        */
/* subtasks run the window apply; results are concatenated.  Same outputs as the serial    */
/* restatements above (ascending indices / the same pair set).                            */
/* ------------------------------------------------------------------------------------ */
#include <omp.h>

typedef struct { int64_t* v; int64_t n, cap; } lvec;
static void lvec_push(lvec* a, int64_t x) {
  if (a->n == a->cap) { a->cap = a->cap ? 2 * a->cap : 256; a->v = (int64_t*)realloc(a->v, 8 * (size_t)a->cap); }
  a->v[a->n++] = x;
}
static int cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return x < y ? -1 : (x > y);
}
static int cmp_pair(const void* a, const void* b) {
  const int64_t* x = (const int64_t*)a; const int64_t* y = (const int64_t*)b;
  if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
  return x[1] < y[1] ? -1 : (x[1] > y[1]);
}
/* concatenation of per-thread results (sorted ascending) into out[cap]; returns the count */
static int64_t gather_sorted(lvec* res, int T, int64_t* out, int64_t cap, int width) {
  int64_t tot = 0;
  for (int t = 0; t < T; t++) tot += res[t].n;
  int64_t* all = (int64_t*)malloc(8 * (size_t)(tot > 0 ? tot : 1));
  int64_t w = 0;
  for (int t = 0; t < T; t++) {
    if (res[t].n) memcpy(all + w, res[t].v, 8 * (size_t)res[t].n);
    w += res[t].n;
    free(res[t].v);
  }
  qsort(all, (size_t)(tot / width), 8 * (size_t)width, width == 1 ? cmp_i64 : cmp_pair);
  const int64_t keep = tot < cap * width ? tot : cap * width;
  if (keep > 0) memcpy(out, all, 8 * (size_t)keep);
  free(all);
  return tot / width;
}

/* shared shape of the range operators: G / C built by the driver, then T subtasks */
static int64_t range_mt(const orc_grid* g, int64_t n, const double* x, const double* y, const strset* G,
                        const strset* C, int nthreads, int64_t* out_idx, int64_t cap,
                        int (*apply)(const void* ctx, int64_t i, int64_t* reps), const void* actx) {
  const int T = nthreads < 1 ? 1 : nthreads;
  lvec* box = (lvec*)calloc((size_t)T * (size_t)T, sizeof(lvec)); /* survivors: i << 1 | inG */
  lvec* res = (lvec*)calloc((size_t)T, sizeof(lvec));
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    char id[32];
    for (int64_t i = n * t / T; i < n * (t + 1) / T; i++) { /* source subtask: filter, keyBy */
      int32_t cx, cy;
      orc_cell_of(g, x[i], y[i], &cx, &cy);
      orc_cell_id(cx, cy, id);
      const int inG = ss_contains(G, id);
      if (!(inG || ss_contains(C, id))) continue;
      lvec_push(&box[(int64_t)t * T + (int64_t)(str_hash(id) % (uint64_t)T)], i << 1 | inG);
    }
#pragma omp barrier
    for (int s = 0; s < T; s++) { /* key subtask t: the window apply per point */
      const lvec* b = &box[(int64_t)s * T + t];
      for (int64_t j = 0; j < b->n; j++) {
        const int64_t i = b->v[j] >> 1;
        if (b->v[j] & 1) { lvec_push(&res[t], i); continue; }
        int64_t reps = 0;
        if (apply(actx, i, &reps))
          for (int64_t k = 0; k < reps; k++) lvec_push(&res[t], i);
      }
    }
  }
  for (int64_t i = 0; i < (int64_t)T * T; i++) free(box[i].v);
  free(box);
  int64_t cnt = gather_sorted(res, T, out_idx, cap, 1);
  free(res);
  return cnt;
}

typedef struct { const double *x, *y, *qx, *qy; int32_t nq; double r; int approx, metric; } pp_ctx;
static int pp_apply(const void* c_, int64_t i, int64_t* reps) { /* PointPointRangeQuery.java:158-183 */
  const pp_ctx* c = (const pp_ctx*)c_;
  if (c->approx) { *reps = c->nq; return c->nq > 0; }
  for (int32_t q = 0; q < c->nq; q++)
    if (orc_distance(c->qx[q], c->qy[q], c->x[i], c->y[i], c->metric) <= c->r) { *reps = 1; return 1; }
  return 0;
}
int64_t orc_range_pp_mt(const orc_grid* g, int64_t n, const double* x, const double* y, int32_t nq,
                        const double* qx, const double* qy, double r, int approximate, int metric, int nthreads,
                        int64_t* out_idx, int64_t cap) {
  strset G, C;
  char id[32];
  ss_init(&G, 64); ss_init(&C, 64);
  for (int32_t q = 0; q < nq; q++) {
    int32_t cx, cy;
    strset Gq, Cq;
    orc_cell_of(g, qx[q], qy[q], &cx, &cy);
    orc_cell_id(cx, cy, id);
    ss_init(&Gq, 64); g_cells_of(g, r, id, &Gq); ss_add_all(&G, &Gq); ss_free(&Gq);
    ss_init(&Cq, 64); c_cells_of(g, r, id, &G, &Cq); ss_add_all(&C, &Cq); ss_free(&Cq);
  }
  pp_ctx c = {x, y, qx, qy, nq, r, approximate, metric};
  int64_t cnt = range_mt(g, n, x, y, &G, &C, nthreads, out_idx, cap, pp_apply, &c);
  ss_free(&G); ss_free(&C);
  return cnt;
}

typedef struct { const double *x, *y, *bb; const orc_polygons* P; double r; int approx, metric; } ppoly_ctx;
static int ppoly_apply(const void* c_, int64_t i, int64_t* reps) { /* PointPolygonRangeQuery.java:179-201 */
  const ppoly_ctx* c = (const ppoly_ctx*)c_;
  for (int32_t p = 0; p < c->P->npoly; p++) {
    const double* b = c->bb + 4 * p;
    double d = c->approx ? orc_point_bbox_distance(c->x[i], c->y[i], b[0], b[1], b[2], b[3])
                         : orc_point_polygon_distance(c->x[i], c->y[i], c->P, p, c->metric);
    if (d <= c->r) { *reps = 1; return 1; }
  }
  return 0;
}
int64_t orc_range_ppoly_mt(const orc_grid* g, int64_t n, const double* x, const double* y, const orc_polygons* P,
                           double r, int approximate, int metric, int nthreads, int64_t* out_idx, int64_t cap) {
  strset G, C;
  char id[32];
  ss_init(&G, 64); ss_init(&C, 64);
  double* bb = (double*)malloc(sizeof(double) * 4 * (size_t)(P->npoly > 0 ? P->npoly : 1));
  for (int32_t p = 0; p < P->npoly; p++) {
    double x1, y1, x2, y2;
    polygon_bbox(P, p, &x1, &y1, &x2, &y2);
    bb[4 * p] = x1; bb[4 * p + 1] = y1; bb[4 * p + 2] = x2; bb[4 * p + 3] = y2;
    int32_t xi1, yi1, xi2, yi2;
    orc_cell_of(g, x1, y1, &xi1, &yi1);
    orc_cell_of(g, x2, y2, &xi2, &yi2);
    strset Gp, Cp;
    ss_init(&Gp, 64);
    for (int64_t a = xi1; a <= xi2; a++)
      for (int64_t b = yi1; b <= yi2; b++) { orc_cell_id((int32_t)a, (int32_t)b, id); g_cells_of(g, r, id, &Gp); }
    ss_add_all(&G, &Gp); ss_free(&Gp);
    ss_init(&Cp, 64);
    for (int64_t a = xi1; a <= xi2; a++)
      for (int64_t b = yi1; b <= yi2; b++) { orc_cell_id((int32_t)a, (int32_t)b, id); c_cells_of(g, r, id, &G, &Cp); }
    ss_add_all(&C, &Cp); ss_free(&Cp);
  }
  ppoly_ctx c = {x, y, bb, P, r, approximate, metric};
  int64_t cnt = range_mt(g, n, x, y, &G, &C, nthreads, out_idx, cap, ppoly_apply, &c);
  free(bb);
  ss_free(&G); ss_free(&C);
  return cnt;
}

/* PointPointJoinQuery with parallelism T: the query stream's replication (JoinQuery.java:73-90)
 * by the driver-side restatement above (orc_join_pp's first half), the ordinary points keyed by
 * gridID over T subtasks, each joining its keys' co-located pairs.  Pairs (sorted) out. */
int64_t orc_join_pp_mt(const orc_grid* ugrid, const orc_grid* qgrid, int64_t no, const double* ox, const double* oy,
                       int64_t nq, const double* qx, const double* qy, double r, int approximate, int metric,
                       int nthreads, int64_t* out_pairs, int64_t cap) {
  const int T = nthreads < 1 ? 1 : nthreads;
  char id[32];
  int32_t cl = 0;
  if (!(r == 0)) {
    cl = orc_candidate_layers(qgrid, r);
    if (cl <= 0) return ORC_ERR_LAYERS;
  }
  strset cells;
  ss_init(&cells, 1024);
  lvec rq = {0, 0, 0}, rk = {0, 0, 0};  /* replica: query index, key hash */
  for (int64_t q = 0; q < nq; q++) {
    int64_t i0, i1, j0, j1;
    if (r == 0) { i0 = 0; i1 = qgrid->n - 1; j0 = 0; j1 = qgrid->n - 1; }
    else {
      int32_t cx, cy, px, py;
      orc_cell_of(qgrid, qx[q], qy[q], &cx, &cy);
      orc_cell_id(cx, cy, id);
      orc_parse_cell_id(id, &px, &py);
      i0 = lmax((int64_t)px - cl, 0); i1 = lmin((int64_t)px + cl, qgrid->n - 1);
      j0 = lmax((int64_t)py - cl, 0); j1 = lmin((int64_t)py + cl, qgrid->n - 1);
    }
    for (int64_t i = i0; i <= i1; i++)
      for (int64_t j = j0; j <= j1; j++) {
        if (!valid_key(qgrid, i, j)) continue;
        orc_cell_id((int32_t)i, (int32_t)j, id);
        ss_add(&cells, id);
        lvec_push(&rq, q);
        lvec_push(&rk, (int64_t)(((uint64_t)i << 32) | (uint64_t)j));
      }
  }
  int64_t* off = (int64_t*)calloc((size_t)cells.cap + 1, 8);
  int64_t* slot = (int64_t*)malloc(8 * (size_t)(rq.n > 0 ? rq.n : 1));
  for (int64_t t = 0; t < rq.n; t++) {
    orc_cell_id((int32_t)(rk.v[t] >> 32), (int32_t)(rk.v[t] & 0xffffffff), id);
    slot[t] = ss_find(&cells, id);
    off[slot[t] + 1]++;
  }
  for (int64_t s = 0; s < cells.cap; s++) off[s + 1] += off[s];
  int64_t* lst = (int64_t*)malloc(8 * (size_t)(rq.n > 0 ? rq.n : 1));
  {
    int64_t* cur = (int64_t*)malloc(8 * (size_t)(cells.cap > 0 ? cells.cap : 1));
    memcpy(cur, off, 8 * (size_t)cells.cap);
    for (int64_t t = 0; t < rq.n; t++) lst[cur[slot[t]]++] = rq.v[t];
    free(cur);
  }
  lvec* box = (lvec*)calloc((size_t)T * (size_t)T, sizeof(lvec));  /* (p, key slot) */
  lvec* res = (lvec*)calloc((size_t)T, sizeof(lvec));
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    char pid[32];
    for (int64_t p = no * t / T; p < no * (t + 1) / T; p++) {  /* ordinary stream: keyBy(gridID) */
      int32_t cx, cy;
      orc_cell_of(ugrid, ox[p], oy[p], &cx, &cy);
      orc_cell_id(cx, cy, pid);
      const int64_t s = ss_find(&cells, pid);
      if (s < 0) continue;  /* no replica carries this key: the coGroup emits nothing */
      lvec* b = &box[(int64_t)t * T + (int64_t)(str_hash(pid) % (uint64_t)T)];
      lvec_push(b, p);
      lvec_push(b, s);
    }
#pragma omp barrier
    for (int s_ = 0; s_ < T; s_++) {  /* key subtask: JoinFunction.join per co-located pair */
      const lvec* b = &box[(int64_t)s_ * T + t];
      for (int64_t j = 0; j < b->n; j += 2) {
        const int64_t p = b->v[j], s = b->v[j + 1];
        for (int64_t k = off[s]; k < off[s + 1]; k++) {
          const int64_t q = lst[k];
          if (approximate || orc_distance(ox[p], oy[p], qx[q], qy[q], metric) <= r) {
            lvec_push(&res[t], p);
            lvec_push(&res[t], q);
          }
        }
      }
    }
  }
  for (int64_t i = 0; i < (int64_t)T * T; i++) free(box[i].v);
  free(box);
  int64_t cnt = gather_sorted(res, T, out_pairs, cap, 2);
  free(res); free(off); free(slot); free(lst); free(rq.v); free(rk.v);
  ss_free(&cells);
  return cnt;
}

/* PointPolygonJoinQuery with parallelism T: the polygon stream's replication (serial, as the
 * driver-side restatement in orc_join_ppoly), the points split into T contiguous parts -- each
 * part's points keyed by gridID and joined with their key's replicas (JoinFunction.join: JTS
 * distance per co-located pair).  Pairs (sorted by point, then polygon) out. */
int64_t orc_join_ppoly_mt(const orc_grid* ugrid, const orc_grid* qgrid, int64_t no, const double* ox,
                          const double* oy, const orc_polygons* P, double r, int approximate, int metric,
                          int nthreads, int64_t* out_pairs, int64_t cap) {
  const int T = nthreads < 1 ? 1 : nthreads;
  strset cells;
  int64_t *off, *lst;
  ppoly_replicate(qgrid, P, r, &cells, &off, &lst);
  lvec* res = (lvec*)calloc((size_t)T, sizeof(lvec));
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    char id[32];
    for (int64_t p = no * t / T; p < no * (t + 1) / T; p++) {
      int32_t cx, cy;
      orc_cell_of(ugrid, ox[p], oy[p], &cx, &cy);
      orc_cell_id(cx, cy, id);
      const int64_t s2 = ss_find(&cells, id);
      if (s2 < 0) continue;
      for (int64_t k = off[s2]; k < off[s2 + 1]; k++) {
        const int64_t q = lst[k];
        if (approximate || orc_point_polygon_distance(ox[p], oy[p], P, (int32_t)q, metric) <= r) {
          lvec_push(&res[t], p);
          lvec_push(&res[t], q);
        }
      }
    }
  }
  int64_t cnt = gather_sorted(res, T, out_pairs, cap, 2);
  free(res); free(off); free(lst);
  ss_free(&cells);
  return cnt;
}

/* PointPolygonKNNQuery with parallelism T: the polygon's G / C key sets built once, the window's
 * points split into T contiguous parts (cell filter + JTS distance per point, as
 * orc_knn_ppoly_contract), the parts' candidates concatenated and merged by the same contract
 * (one entry per objID, (d, objID) order, first k): identical output. */
int32_t orc_knn_ppoly_mt(const orc_grid* g, int64_t n, const double* x, const double* y, const int64_t* objID,
                         const orc_polygons* P, double r, int32_t k, int approximate, int metric, int nthreads,
                         int64_t* out_objID, double* out_d, int64_t* out_idx) {
  const int T = nthreads < 1 ? 1 : nthreads;
  strset G, C;
  char id[32];
  double x1, y1, x2, y2;
  int32_t xi1, yi1, xi2, yi2;
  if (k <= 0 || P->npoly != 1) return ORC_ERR_ARG;
  ss_init(&G, 64); ss_init(&C, 64);
  polygon_bbox(P, 0, &x1, &y1, &x2, &y2);
  orc_cell_of(g, x1, y1, &xi1, &yi1);
  orc_cell_of(g, x2, y2, &xi2, &yi2);
  for (int64_t a = xi1; a <= xi2; a++)
    for (int64_t b = yi1; b <= yi2; b++) { orc_cell_id((int32_t)a, (int32_t)b, id); g_cells_of(g, r, id, &G); }
  for (int64_t a = xi1; a <= xi2; a++)
    for (int64_t b = yi1; b <= yi2; b++) { orc_cell_id((int32_t)a, (int32_t)b, id); c_cells_of(g, r, id, &G, &C); }
  tup* c = (tup*)malloc(sizeof(tup) * (size_t)(n > 0 ? n : 1));
  int64_t* cnt = (int64_t*)calloc((size_t)T + 1, 8);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    char cid[32];
    const int64_t b = n * t / T, e = n * (t + 1) / T;
    int64_t m = b;  /* this part's candidates at c[b ..) */
    for (int64_t i = b; i < e; i++) {
      int32_t cx, cy;
      orc_cell_of(g, x[i], y[i], &cx, &cy);
      orc_cell_id(cx, cy, cid);
      if (!(ss_contains(&C, cid) || ss_contains(&G, cid))) continue;
      const double d = approximate ? orc_point_bbox_distance(x[i], y[i], x1, y1, x2, y2)
                                   : orc_point_polygon_distance(x[i], y[i], P, 0, metric);
      if (!(d <= r)) continue;
      c[m].d = d; c[m].obj = objID[i]; c[m].idx = i; m++;
    }
    cnt[t] = m - b;
  }
  int64_t m = 0;
  for (int t = 0; t < T; t++) {  /* compact the parts */
    const int64_t b = n * t / T;
    memmove(c + m, c + b, sizeof(tup) * (size_t)cnt[t]);
    m += cnt[t];
  }
  free(cnt);
  ss_free(&G); ss_free(&C);
  qsort(c, (size_t)m, sizeof(tup), cmp_obj_d_idx);
  int64_t u = 0;
  for (int64_t i = 0; i < m; i++)
    if (u == 0 || c[u - 1].obj != c[i].obj) c[u++] = c[i];
  qsort(c, (size_t)u, sizeof(tup), cmp_d_obj);
  const int32_t nout = (int32_t)(u < k ? u : k);
  for (int32_t i = 0; i < nout; i++) {
    out_objID[i] = c[i].obj; out_d[i] = c[i].d; out_idx[i] = c[i].idx;
  }
  free(c);
  return nout;
}

/* CSVTSVToTSpatial.map on T threads: the chunk's lines split into T contiguous parts (the
 * source parallelism of a Flink map), each parsed by orc_csv_parse into its own buffers.
 * Fills x, y, ts in line order; returns the line count (bad lines: first one reported). */
int64_t orc_csv_parse_mt(const char* text, int64_t len, char delim, const int32_t* want, double* x, double* y,
                         int64_t* ts, int64_t cap, int nthreads, int64_t* bad_line, int32_t* bad_kind) {
  const int T = nthreads < 1 ? 1 : nthreads;
  int64_t* cut = (int64_t*)malloc(8 * (size_t)(T + 1));
  cut[0] = 0;
  for (int t = 1; t < T; t++) {  /* part boundaries after a '\n' */
    int64_t p = len * t / T;
    if (p < cut[t - 1]) p = cut[t - 1];
    if (p > 0)
      while (p < len && text[p - 1] != '\n') ++p;
    cut[t] = p;
  }
  cut[T] = len;
  int64_t* nl = (int64_t*)calloc((size_t)T + 1, 8);
  int64_t* bl = (int64_t*)malloc(8 * (size_t)T);
  int32_t* bk = (int32_t*)malloc(4 * (size_t)T);
#pragma omp parallel num_threads(T)
  {  /* count lines per part, then parse into the part's slice */
    const int t = omp_get_thread_num();
    int64_t c = 0;
    for (int64_t i = cut[t]; i < cut[t + 1]; i++) c += text[i] == '\n';
    if (cut[t + 1] > cut[t] && text[cut[t + 1] - 1] != '\n') c++;
    nl[t + 1] = c;
#pragma omp barrier
#pragma omp single
    for (int u = 0; u < T; u++) nl[u + 1] += nl[u];
    const int64_t o = nl[t], m = nl[t + 1] - nl[t];
    if (m > 0 && o + m <= cap) {
      char* oid = (char*)malloc((size_t)(cut[t + 1] - cut[t]) + 16);
      int64_t* off = (int64_t*)malloc(8 * (size_t)(m + 1));
      int64_t ol = 0;
      orc_csv_parse(text + cut[t], cut[t + 1] - cut[t], delim, want, x + o, y + o, oid, cut[t + 1] - cut[t] + 16, off,
                    &ol, ts + o, m, &bl[t], &bk[t]);
      free(oid); free(off);
    } else {
      bl[t] = -1; bk[t] = 0;
    }
  }
  *bad_line = -1; *bad_kind = 0;
  for (int t = 0; t < T; t++)
    if (bl[t] >= 0) { *bad_line = nl[t] + bl[t]; *bad_kind = bk[t]; break; }
  const int64_t lines = nl[T];
  free(cut); free(nl); free(bl); free(bk);
  return lines;
}
