// k_range.hip -- window apply of the range queries:
//   PointPointRangeQuery.java:150-186   (guaranteed cell -> emit; candidate cell -> emit once
//                                         if some query point is within r; approximate: once
//                                         per query point)
//   PointPolygonRangeQuery.java:170-204 (same with JTS point-polygon distance, or the polygon
//                                         bounding-box distance in approximate mode)
// One fused HBM-bound pass: 16 B/point in (x, y), 1 bit/point out (selection bitmap, built
// from two wave ballots per 128 points), per-block hit counts (no global atomics).
//
// Classification (guaranteed / candidate / none):
//   ARITH  single query point: exact per-axis double intervals precomputed on the host from
//          the cell thresholds, so no per-point division at all.
//   TABLE  many query objects: exact cell (two fp64 divisions) + one byte from a per-cell
//          class table (L1/L2 resident), out-of-grid cells against the g == 0 extra rects.
// Testing a candidate-cell point walks that cell's object list (CSR built on the host over a
// (c+2)-cell reach, a superset of every object that can be within r).
#include "gf_internal.hpp"

namespace gf {

// ---------------- JTS point-polygon distance (device restatement) ----------------------
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  const double x = a + b, bv = x - a, av = x - bv;
  s = x;
  e = (a - av) + (b - bv);
}
// exact sign of x1*y2 - y1*x2 (what JTS RobustDeterminant.signOfDet2x2 returns)
__device__ int sign_det2x2(double x1, double y1, double x2, double y2) {
  const double p1 = x1 * y2, e1 = fma(x1, y2, -p1);
  const double p2 = y1 * x2, e2 = fma(y1, x2, -p2);
  const double terms[4] = {e1, -e2, p1, -p2};
  double h[4];
  int m = 1;
  h[0] = terms[0];
#pragma unroll
  for (int t = 1; t < 4; ++t) {
    double q = terms[t];
    for (int i = 0; i < m; ++i) {
      double s, e;
      two_sum(q, h[i], s, e);
      h[i] = e;
      q = s;
    }
    h[m++] = q;
  }
  for (int i = m - 1; i >= 0; --i) {
    if (h[i] > 0) return 1;
    if (h[i] < 0) return -1;
  }
  return 0;
}

constexpr int kLocInterior = 0, kLocBoundary = 1, kLocExterior = 2;

// RayCrossingCounter.locatePointInRing (JTS 1.16) behind PointLocator's envelope test
__device__ int locate_in_ring(double px, double py, const double* vx, const double* vy, int nv,
                              const double* env) {
  if (px > env[1] || px < env[0] || py > env[3] || py < env[2]) return kLocExterior;
  int crossings = 0;
  for (int i = 1; i < nv; ++i) {
    const double p1x = vx[i], p1y = vy[i], p2x = vx[i - 1], p2y = vy[i - 1];
    if (p1x < px && p2x < px) continue;
    if (px == p2x && py == p2y) return kLocBoundary;
    if (p1y == py && p2y == py) {
      double mn = p1x, mx = p2x;
      if (mn > mx) { mn = p2x; mx = p1x; }
      if (px >= mn && px <= mx) return kLocBoundary;
      continue;
    }
    if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
      const double x1 = p1x - px, y1 = p1y - py, x2 = p2x - px, y2 = p2y - py;
      int sgn = sign_det2x2(x1, y1, x2, y2);
      if (sgn == 0) return kLocBoundary;
      if (y2 < y1) sgn = -sgn;
      if (sgn > 0) ++crossings;
    }
  }
  return (crossings & 1) ? kLocInterior : kLocExterior;
}

__device__ double point_to_segment(double px, double py, double ax, double ay, double bx, double by, int metric) {
  if (ax == bx && ay == by) return distance(px, py, ax, ay, metric);
  const double len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay);
  const double r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2;
  if (r <= 0.0) return distance(px, py, ax, ay, metric);
  if (r >= 1.0) return distance(px, py, bx, by, metric);
  const double s = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2;
  return fabs(s) * sqrt(len2);
}

// JTS Envelope.distance against a point envelope
__device__ double env_point_distance(const double* e, double px, double py) {
  if (!(px > e[1] || px < e[0] || py > e[3] || py < e[2])) return 0.0;
  double dx = 0.0, dy = 0.0;
  if (e[1] < px) dx = px - e[1]; else if (e[0] > px) dx = e[0] - px;
  if (e[3] < py) dy = py - e[3]; else if (e[2] > py) dy = e[2] - py;
  if (dx == 0.0) return dy;
  if (dy == 0.0) return dx;
  return sqrt(dx * dx + dy * dy);
}

// DistanceOp(point, polygon): containment (shell, holes), then min facet distance
__device__ double point_polygon_distance(double px, double py, const RangeArgs& a, int p) {
  const int r0 = a.ring_off[p], r1 = a.ring_off[p + 1];
  if (px == px) {  // NaN x: containment skipped (documented; matches the oracle)
    const int v0 = a.vert_off[r0], nv = a.vert_off[r0 + 1] - v0;
    const int loc = locate_in_ring(px, py, a.vx + v0, a.vy + v0, nv, a.ring_env + 4 * r0);
    if (loc == kLocBoundary) return 0.0;
    if (loc == kLocInterior) {
      bool inside = true;
      for (int h = r0 + 1; h < r1; ++h) {
        const int hv0 = a.vert_off[h], hnv = a.vert_off[h + 1] - hv0;
        const int hl = locate_in_ring(px, py, a.vx + hv0, a.vy + hv0, hnv, a.ring_env + 4 * h);
        if (hl == kLocInterior) { inside = false; break; }
        if (hl == kLocBoundary) return 0.0;
      }
      if (inside) return 0.0;
    }
  }
  double md = 1.7976931348623157e308;
  for (int rg = r0; rg < r1; ++rg) {
    const int v0 = a.vert_off[rg], nv = a.vert_off[rg + 1] - v0;
    if (env_point_distance(a.ring_env + 4 * rg, px, py) > md) continue;
    for (int i = 0; i < nv - 1; ++i) {
      const double d = point_to_segment(px, py, a.vx[v0 + i], a.vy[v0 + i], a.vx[v0 + i + 1], a.vy[v0 + i + 1],
                                        a.metric);
      if (d < md) md = d;
      if (md <= 0.0) return md;
    }
  }
  return md;
}

// DistanceFunctions.getPointPolygonBBoxMinEuclideanDistance -- DistanceFunctions.java:150-200
__device__ __forceinline__ double pp_euclid(double lon, double lat, double lon1, double lat1) {
  const double a = lat1 - lat, b = lon1 - lon;
  return sqrt(a * a + b * b);
}
__device__ __forceinline__ double bbox_border(double x, double y, double x1, double y1, double x2, double y2) {
  if (x1 == x2) return pp_euclid(x, y, x1, y);
  if (y1 == y2) return pp_euclid(x, y, x, y1);
  return 4.9e-324;
}
__device__ double point_bbox_distance(double x, double y, const double* bb) {
  const double x1 = bb[0], y1 = bb[1], x2 = bb[2], y2 = bb[3];
  if (x <= x1) {
    if (y <= y1) return pp_euclid(x, y, x1, y1);
    if (y >= y2) return pp_euclid(x, y, x1, y2);
    return bbox_border(x, y, x1, y1, x1, y2);
  } else if (x >= x2) {
    if (y <= y1) return pp_euclid(x, y, x2, y1);
    if (y >= y2) return pp_euclid(x, y, x2, y2);
    return bbox_border(x, y, x2, y1, x2, y2);
  }
  if (y <= y1) return bbox_border(x, y, x1, y1, x2, y1);
  if (y >= y2) return bbox_border(x, y, x1, y2, x2, y2);
  return 0.0;
}

// ---------------- classification --------------------------------------------------------
constexpr int kNone = 0, kTest = 1, kAccept = 2;

template <int TABLE>
__device__ __forceinline__ int classify(const RangeArgs& a, double px, double py, int32_t& cell) {
  if (!TABLE) {
    const double xs = (px == px) ? px : a.qr.minX;
    const double ys = (py == py) ? py : a.qr.minY;
    if (a.qr.g_any && in_iv(a.qr.gx, xs) && in_iv(a.qr.gy, ys)) return kAccept;
    return (in_iv(a.qr.cgx, xs) && in_iv(a.qr.cgy, ys)) ? kTest : kNone;
  }
  const int32_t cx = cell_index(px, a.minX, a.cl);
  const int32_t cy = cell_index(py, a.minY, a.cl);
  if (cx >= 0 && cy >= 0 && cx < a.grid_n && cy < a.grid_n) {
    cell = cy * a.grid_n + cx;
    return a.table[cell];
  }
  for (int e = 0; e < a.n_extra; ++e) {
    const int32_t* r = a.extra + 4 * e;
    if (cx >= r[0] && cx <= r[1] && cy >= r[2] && cy <= r[3]) return kAccept;
  }
  return kNone;
}

// candidate-cell test: exists object within r (first hit wins, emitted once)
template <int TABLE, int POLY>
__device__ __forceinline__ bool test_point(const RangeArgs& a, double px, double py, int32_t cell) {
  if (!POLY && !TABLE) {  // single query point: exact s <= smax(r) for the sqrt metric
    const double dx = a.qx0 - px, dy = a.qy0 - py;
    if (a.metric == 0) return dx * dx + dy * dy <= a.s_r;
    return fdlibm_hypot(dx, dy) <= a.r;
  }
  int32_t b = 0, e = POLY ? a.npoly : a.nq;
  const int32_t* lst = nullptr;
  if (a.cand_off) {
    b = a.cand_off[cell];
    e = a.cand_off[cell + 1];
    lst = a.cand_list;
  }
  for (int32_t t = b; t < e; ++t) {
    const int32_t o = lst ? lst[t] : t;
    if (POLY) {
      const double d = a.approx ? point_bbox_distance(px, py, a.bbox + 4 * o) : point_polygon_distance(px, py, a, o);
      if (d <= a.r) return true;
    } else {
      if (distance(a.qx[o], a.qy[o], px, py, a.metric) <= a.r) return true;
    }
  }
  return false;
}

__device__ __forceinline__ uint64_t spread32(uint32_t v) {
  uint64_t x = v;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}

template <int TABLE, int POLY>
__device__ __forceinline__ void eval_point(const RangeArgs& a, double px, double py, bool valid, bool& hit,
                                           bool& multi) {
  hit = false;
  multi = false;
  if (!valid) return;
  int32_t cell = 0;
  const int cls = classify<TABLE>(a, px, py, cell);
  if (cls == kAccept) {
    hit = true;
  } else if (cls == kTest) {
    if (!POLY && a.approx) {  // approximate point-point: emitted once per query point
      hit = true;
      multi = a.nq > 1;
    } else {
      hit = test_point<TABLE, POLY>(a, px, py, cell);
    }
  }
}

template <int TABLE, int POLY>
__global__ __launch_bounds__(kBlock) void range_kernel(RangeArgs a) {
  const int64_t npairs = (a.n + 1) >> 1;
  const int64_t words = (a.n + 63) >> 6;
  const int lane = threadIdx.x & 63;
  uint64_t hits = 0, mult = 0;
  for (int64_t base = (int64_t)blockIdx.x * kBlock + (threadIdx.x & ~63); base < npairs;
       base += (int64_t)gridDim.x * kBlock) {
    const int64_t i = 2 * (base + lane);
    double2 xv, yv;
    const bool v0 = i < a.n, v1 = i + 1 < a.n;
    if (v1) {
      xv = *reinterpret_cast<const double2*>(a.x + i);
      yv = *reinterpret_cast<const double2*>(a.y + i);
    } else if (v0) {
      xv.x = a.x[i]; yv.x = a.y[i]; xv.y = yv.y = 0.0;
    } else {
      xv.x = xv.y = yv.x = yv.y = 0.0;
    }
    bool h0, h1, m0, m1;
    eval_point<TABLE, POLY>(a, xv.x, yv.x, v0, h0, m0);
    eval_point<TABLE, POLY>(a, xv.y, yv.y, v1, h1, m1);
    const uint64_t b0 = __ballot(h0), b1 = __ballot(h1);
    const int64_t w = base >> 5;  // 128 points per wave = 2 words
    if (lane < 2 && w + lane < words) {
      const uint32_t s0 = lane ? (uint32_t)(b0 >> 32) : (uint32_t)b0;
      const uint32_t s1 = lane ? (uint32_t)(b1 >> 32) : (uint32_t)b1;
      a.bitmap[w + lane] = spread32(s0) | (spread32(s1) << 1);
    }
    if (a.multi) {
      const uint64_t c0 = __ballot(m0), c1 = __ballot(m1);
      if (lane < 2 && w + lane < words) {
        const uint32_t s0 = lane ? (uint32_t)(c0 >> 32) : (uint32_t)c0;
        const uint32_t s1 = lane ? (uint32_t)(c1 >> 32) : (uint32_t)c1;
        a.multi[w + lane] = spread32(s0) | (spread32(s1) << 1);
      }
      mult += (uint64_t)(__popcll(c0) + __popcll(c1));
    }
    hits += (uint64_t)(__popcll(b0) + __popcll(b1));
  }
  // per-block partial counts (plain stores; summed by range_finalize)
  __shared__ uint64_t sh[kBlock / 64], sm[kBlock / 64];
  const int wid = threadIdx.x >> 6;
  if (lane == 0) { sh[wid] = hits; sm[wid] = mult; }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t th = 0, tm = 0;
    for (int w = 0; w < kBlock / 64; ++w) { th += sh[w]; tm += sm[w]; }
    a.partials[2 * blockIdx.x] = th;
    a.partials[2 * blockIdx.x + 1] = th + tm * (uint64_t)(a.nq > 1 ? a.nq - 1 : 0);
  }
}

hipError_t launch_range(gf_ctx* ctx, const RangeArgs& a, int table_mode, int poly, int blocks) {
  KTimer t(ctx, GF_K_RANGE_SCAN);
  const dim3 g(blocks), b(kBlock);
  if (!table_mode && !poly) hipLaunchKernelGGL((range_kernel<0, 0>), g, b, 0, ctx->stream, a);
  else if (table_mode && !poly) hipLaunchKernelGGL((range_kernel<1, 0>), g, b, 0, ctx->stream, a);
  else hipLaunchKernelGGL((range_kernel<1, 1>), g, b, 0, ctx->stream, a);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void range_finalize_kernel(const uint64_t* __restrict__ partials, int blocks,
                                                                int64_t* counts) {
  uint64_t h = 0, m = 0;
  for (int b = threadIdx.x; b < blocks; b += kBlock) { h += partials[2 * b]; m += partials[2 * b + 1]; }
  __shared__ uint64_t sh[kBlock], sm[kBlock];
  sh[threadIdx.x] = h; sm[threadIdx.x] = m;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) { sh[threadIdx.x] += sh[threadIdx.x + s]; sm[threadIdx.x] += sm[threadIdx.x + s]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) { counts[0] = (int64_t)sh[0]; counts[1] = (int64_t)sm[0]; }
}

hipError_t launch_range_finalize(hipStream_t s, const uint64_t* partials, int blocks, int64_t* counts) {
  hipLaunchKernelGGL(range_finalize_kernel, dim3(1), dim3(kBlock), 0, s, partials, blocks, counts);
  return hipGetLastError();
}

}  // namespace gf
