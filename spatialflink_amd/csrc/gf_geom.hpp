// gf_geom.hpp -- device restatements of the JTS 1.16.1 point-polygon geometry the reference
// calls through DistanceFunctions.getDistance(Point, Polygon) (DistanceFunctions.java:33-36:
// DistanceOp -> PointLocator / RayCrossingCounter / RobustDeterminant, Distance.pointToSegment)
// and of its own bbox distance (getPointPolygonBBoxMinEuclideanDistance, :150-200).  Shared by
// the range kernels (k_range.hip) and the polygon-query kNN (k_knn.hip).
#pragma once

#include "gf_internal.hpp"

namespace gf {


__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  const double x = a + b, bv = x - a, av = x - bv;
  s = x;
  e = (a - av) + (b - bv);
}
// exact sign of x1*y2 - y1*x2 (what JTS RobustDeterminant.signOfDet2x2 returns)
static __device__ __forceinline__ int sign_det2x2(double x1, double y1, double x2, double y2) {
  const double p1 = x1 * y2, e1 = fma(x1, y2, -p1);
  const double p2 = y1 * x2, e2 = fma(y1, x2, -p2);
  const double terms[4] = {e1, -e2, p1, -p2};
  double h[4];
  int m = 1;
  h[0] = terms[0];
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
static __device__ __forceinline__ int locate_in_ring(double px, double py, const double* vx, const double* vy, int nv,
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

static __device__ inline double point_to_segment(double px, double py, double ax, double ay, double bx, double by, int metric) {
  if (ax == bx && ay == by) return distance(px, py, ax, ay, metric);
  const double len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay);
  const double r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2;
  if (r <= 0.0) return distance(px, py, ax, ay, metric);
  if (r >= 1.0) return distance(px, py, bx, by, metric);
  const double s = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2;
  return fabs(s) * sqrt(len2);
}

// JTS Envelope.distance against a point envelope
static __device__ inline double env_point_distance(const double* e, double px, double py) {
  if (!(px > e[1] || px < e[0] || py > e[3] || py < e[2])) return 0.0;
  double dx = 0.0, dy = 0.0;
  if (e[1] < px) dx = px - e[1]; else if (e[0] > px) dx = e[0] - px;
  if (e[3] < py) dy = py - e[3]; else if (e[2] > py) dy = e[2] - py;
  if (dx == 0.0) return dy;
  if (dy == 0.0) return dx;
  return sqrt(dx * dx + dy * dy);
}

// DistanceOp(point, polygon): containment (shell, holes), then min facet distance.  Inlined
// like its helpers: as calls, the ABI's callee-saved registers and stack cost every kernel that
// tests polygons (the range scan with its deferred drain: 101 -> 87 VGPRs, 5 waves/SIMD).
static __device__ __forceinline__ double polygon_distance(double px, double py, const PolyView& a, int p) {
  const int r0 = a.ring_off[p], r1 = a.ring_off[p + 1];
  if (a.rect && a.rect[p]) {
    // one-ring axis-aligned rectangle: PointLocator's interior-or-boundary is exactly the
    // closed box (every orientation sign against an axis-aligned edge is a plain comparison);
    // outside it, the same facet loop as below (a NaN coordinate fails the box and lands there
    // too, as it does on the general path)
    const double* e = a.ring_env + 4 * r0;
    if (px >= e[0] && px <= e[1] && py >= e[2] && py <= e[3]) return 0.0;
  } else if (px == px) {  // NaN x: containment skipped (documented; matches the oracle)
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
static __device__ inline double point_bbox_distance(double x, double y, const double* bb) {
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

// Envelope prune for the exact point-polygon test.  The computed point-polygon distance of a
// point outside the (closed) shell envelope is a min of computed point-segment distances, each
// within ~16 eps x (coordinate scale) of a true distance >= the true envelope distance; the
// margin (1e-12 relative to the coordinates, 1e-9 relative to r) exceeds that by orders of
// magnitude, so a pruned polygon could never have tested <= r.
__device__ __forceinline__ bool env_far(const double* bb, double px, double py, double r) {
  const double dx = px < bb[0] ? bb[0] - px : (px > bb[2] ? px - bb[2] : 0.0);
  const double dy = py < bb[1] ? bb[1] - py : (py > bb[3] ? py - bb[3] : 0.0);
  const double scale = fabs(px) + fabs(py) + fabs(bb[0]) + fabs(bb[1]) + fabs(bb[2]) + fabs(bb[3]);
  const double rm = r + r * 1e-9 + scale * 1e-12;
  return dx > rm || dy > rm || dx * dx + dy * dy > rm * rm;
}
__device__ __forceinline__ bool env_holds(const double* bb, double px, double py) {
  return px >= bb[0] && px <= bb[2] && py >= bb[1] && py <= bb[3];
}

}  // namespace gf
