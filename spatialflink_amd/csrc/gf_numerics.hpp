// gf_numerics.hpp -- host + device fp64 numerics of the window-evaluation path (gfx950).
//
// Everything here must be bit-identical on the host (x86-64 SSE2) and on the GPU: the whole
// library is compiled with -ffp-contract=off (Java never fuses a*b+c) and without fast-math;
// gfx950 fp64 division (v_div_scale/fmas/fixup) and sqrt lowerings are IEEE correctly rounded.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#define GF_HD __host__ __device__ __forceinline__

namespace gf {

GF_HD uint64_t dbits(double d) { return __builtin_bit_cast(uint64_t, d); }
GF_HD double from_bits(uint64_t u) { return __builtin_bit_cast(double, u); }

// Java (int) narrowing of a double (JLS 5.1.3): NaN -> 0, saturate, else truncate.
// Device: the same cases as selects (r06): written as branches the compiler kept them as
// exec-mask branches, ~20 scalar + 5 vector instructions per conversion in the per-point loops.
// The clamped value is in range, so the conversion is one v_cvt_i32_f64; a NaN input is
// selected away (the conversion's value is unused then).
GF_HD int32_t jint(double v) {
#ifdef __HIP_DEVICE_COMPILE__
  const double c = v < -2147483648.0 ? -2147483648.0 : (v > 2147483647.0 ? 2147483647.0 : v);
  const int32_t r = (int32_t)c;
  return v == v ? r : 0;
#else
  if (v != v) return 0;
  if (v >= 2147483647.0) return INT32_MAX;
  if (v <= -2147483648.0) return INT32_MIN;
  return (int32_t)v;
#endif
}

// HelperClass.assignGridCellID, one axis -- HelperClass.java:109-110: (int) floor((v - mn) / cl).
// Device (r06): the quotient from a multiply by fl(1 / cl), exact whenever no integer lies near it.
// q = fl(t * fl(1/cl)) and Q = fl(t / cl) differ by at most |q| * 3.001 * 2^-53 (three
// roundings), so Q lies in [fl(q - e), fl(q + e)] for e = |q| 2^-48 (the two roundings of q -/+ e
// are below |q| 2^-53 each); when both ends floor to the same integer, that is floor(Q).  Otherwise
// -- Q within ~2^-48 |q| of a cell edge (points on or next to a cell bound, NaN, +-inf, a tiny
// or overflowing quotient) -- the correctly rounded division decides, as on the host.  Uniform
// points take the exact division with probability ~1e-11 per point; the per-point fp64 division
// (~11 vector instructions, a quarter-rate reciprocal among them) leaves the streaming loops.
GF_HD int32_t cell_index(double v, double mn, double cl) {
#ifdef __HIP_DEVICE_COMPILE__
  const double t = v - mn, q = t * (1.0 / cl);
  const double e = fabs(q) * 0x1p-48 + 0x1p-1000;
  const double lo = floor(q - e);
  if (lo == floor(q + e) && fabs(lo) < 2147483648.0) return (int32_t)lo;  // in range: no saturation
  return jint(floor(t / cl));
#else
  return jint(floor((v - mn) / cl));
#endif
}

// UniformGrid.getGuaranteedNeighboringLayers / getCandidateNeighboringLayers -- :428-445
GF_HD int32_t guaranteed_layers(double cl, double r) {
  return jint(floor((r / (cl * sqrt(2.0))) - 1));
}
GF_HD int32_t candidate_layers(double cl, double r) { return jint(ceil(r / cl)); }

// fdlibm 5.3 e_hypot.c (JDK 8 StrictMath.hypot == Math.hypot).
GF_HD uint32_t hi32(double x) { return (uint32_t)(dbits(x) >> 32); }
GF_HD uint32_t lo32(double x) { return (uint32_t)dbits(x); }
GF_HD double set_hi32(double x, uint32_t hi) {
  return from_bits(((uint64_t)hi << 32) | (dbits(x) & 0xffffffffull));
}
GF_HD double fdlibm_hypot(double x, double y) {
  double a, b, t1, t2, y1, y2, w;
  int32_t j, k, ha, hb;
  ha = (int32_t)(hi32(x) & 0x7fffffff);
  hb = (int32_t)(hi32(y) & 0x7fffffff);
  if (hb > ha) { a = y; b = x; j = ha; ha = hb; hb = j; } else { a = x; b = y; }
  a = set_hi32(a, (uint32_t)ha);
  b = set_hi32(b, (uint32_t)hb);
  if ((ha - hb) > 0x3c00000) return a + b;
  k = 0;
  if (ha > 0x5f300000) {
    if (ha >= 0x7ff00000) {
      w = a + b;
      if (((ha & 0xfffff) | lo32(a)) == 0) w = a;
      if (((hb ^ 0x7ff00000) | lo32(b)) == 0) w = b;
      return w;
    }
    ha -= 0x25800000; hb -= 0x25800000; k += 600;
    a = set_hi32(a, (uint32_t)ha);
    b = set_hi32(b, (uint32_t)hb);
  }
  if (hb < 0x20b00000) {
    if (hb <= 0x000fffff) {
      if ((hb | lo32(b)) == 0) return a;
      t1 = set_hi32(0.0, 0x7fd00000);
      b *= t1; a *= t1; k -= 1022;
    } else {
      ha += 0x25800000; hb += 0x25800000; k -= 600;
      a = set_hi32(a, (uint32_t)ha);
      b = set_hi32(b, (uint32_t)hb);
    }
  }
  w = a - b;
  if (w > b) {
    t1 = set_hi32(0.0, (uint32_t)ha);
    t2 = a - t1;
    w = sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)));
  } else {
    a = a + a;
    y1 = set_hi32(0.0, (uint32_t)hb);
    y2 = b - y1;
    t1 = set_hi32(0.0, (uint32_t)(ha + 0x00100000));
    t2 = a - t1;
    w = sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)));
  }
  if (k != 0) return set_hi32(1.0, hi32(1.0) + ((uint32_t)k << 20)) * w;
  return w;
}

// JTS Coordinate.distance -- DistanceFunctions.java:15-18 -> Geometry.distance -> DistanceOp.
GF_HD double distance(double x1, double y1, double x2, double y2, int metric) {
  double dx = x1 - x2, dy = y1 - y2;
  if (metric == 1) return fdlibm_hypot(dx, dy);
  return sqrt(dx * dx + dy * dy);
}

// Largest s >= 0 with fl(sqrt(s)) <= T.  Because correctly rounded sqrt is monotone,
// "sqrt(s) <= T" is exactly "s <= smax(T)": the scans test s = dx*dx + dy*dy against it and
// never take a sqrt for a rejected point.  Returns -1 when nothing qualifies (T < 0 or NaN).
GF_HD double next_up_pos(double s) { return from_bits(dbits(s) + 1); }   // s >= 0 finite
GF_HD double next_down_pos(double s) { return from_bits(dbits(s) - 1); } // s > 0
GF_HD double smax_for(double T) {
  if (!(T >= 0.0)) return -1.0;
  if (T == INFINITY) return INFINITY;
  double s = T * T;
  if (s == INFINITY) s = 1.7976931348623157e308;
  while (s > 0.0 && sqrt(s) > T) s = next_down_pos(s);
  for (;;) {
    double nx = next_up_pos(s);
    if (nx == INFINITY || sqrt(nx) > T) break;
    s = nx;
  }
  return s;
}
// Prefilter bound on s for a distance threshold T: exact for metric 0, generous for hypot
// (fdlibm hypot is within 1 ulp; survivors are re-tested with the exact distance).
GF_HD double s_prefilter(double T, int metric) {
  if (metric == 0) return smax_for(T);
  if (!(T >= 0.0)) return -1.0;
  double s = T * T * (1.0 + 0x1p-30);
  return s == s ? s : INFINITY;
}

// Half-open interval of doubles [lo, hi_excl): x is inside iff (x >= lo) && !(x >= hi_excl).
// lo == NaN: empty; hi_excl == NaN: unbounded above.  Built on the host from exact
// per-axis cell thresholds, so the test is identical to comparing cell_index(x) with
// integer bounds -- no per-point division.
struct AxisIv {
  double lo, hi_excl;
};
GF_HD bool in_iv(const AxisIv& iv, double v) { return (v >= iv.lo) && !(v >= iv.hi_excl); }

// Log-spaced distance buckets (11 exponent + 7 mantissa bits of d) over [0, T]: 4096 bins,
// 128 per binade, bin 4095 holds T.  Used by the kNN sample and select kernels.
constexpr int kDistBins = 4096;
GF_HD int64_t dist_bin_base(double T) {
  int64_t b = (int64_t)(dbits(T) >> 45) - (kDistBins - 1);
  return b < 0 ? 0 : b;
}
GF_HD int dist_bin(double d, int64_t base) {
  int64_t b = (int64_t)(dbits(d) >> 45) - base;
  return b < 0 ? 0 : (b > kDistBins - 1 ? kDistBins - 1 : (int)b);
}
// Largest double in bin b (inclusive upper edge).
GF_HD double dist_bin_upper(int b, int64_t base) {
  return from_bits((((uint64_t)(base + b + 1)) << 45) - 1);
}

}  // namespace gf
