// gf_decimal.hpp -- Java's Long.valueOf / Double.valueOf for the CSV ingest path
// (Deserialization.CSVTSVToTSpatial.map, Deserialization.java:314-322), __host__ __device__.
//
// Double.valueOf (JDK FloatingDecimal.readJavaFormatString) is correctly rounded, so the
// device must produce the correctly rounded binary64 of every decimal literal:
//   * Clinger's fast path: significand w <= 2^53 and |q| <= 22 -> one exact IEEE mul/div;
//   * otherwise Eisel-Lemire (Lemire 2021, "Number Parsing at a Gigabyte per Second"; the
//     128-bit 5^q table of tools/gen_pow5.py) on the first 19 significant digits; more than 19
//     digits: the result is final when w and w+1 round to the same double (the usual case);
//     otherwise the literal is reported as unsupported (kNumUnsupported) -- never guessed.
// Java grammar accepted: trim (chars <= ' '), [+-], NaN | Infinity | digits[.digits][e[+-]digits]
// with an optional [fFdD] suffix; hexadecimal literals are valid Java but reported unsupported.
#pragma once

#include <cstdint>

#include "gf_pow5.hpp"

#if defined(__HIPCC__)
#define GF_DHD __host__ __device__
#else
#define GF_DHD
#endif

namespace gf {

enum { kNumOk = 0, kNumBad = 1 /* NumberFormatException */, kNumUnsupported = 2 };

// a field of a CSV line: bytes [b, e) of the text, '"' characters skipped (the reference's
// str.replace("\"", "") runs before the split)
struct Field {
  int64_t b, e;
};

template <class Src>
GF_DHD inline int parse_java_long(const Src& s, Field f, int64_t* out) {
  int64_t i = f.b;
  while (i < f.e && s(i) == '"') ++i;
  if (i >= f.e) return kNumBad;
  bool neg = false;
  char c = s(i);
  if (c == '-' || c == '+') {
    neg = c == '-';
    ++i;
  }
  uint64_t v = 0;
  int nd = 0;
  const uint64_t lim = neg ? 9223372036854775808ull : 9223372036854775807ull;
  for (; i < f.e; ++i) {
    c = s(i);
    if (c == '"') continue;
    if (c < '0' || c > '9') return kNumBad;
    const uint64_t d = (uint64_t)(c - '0');
    if (v > (lim - d) / 10) return kNumBad;  // Long.parseLong overflow
    v = v * 10 + d;
    ++nd;
  }
  if (nd == 0) return kNumBad;
  *out = neg ? (int64_t)(0ull - v) : (int64_t)v;
  return kNumOk;
}

// objID keys (include/geoflink_hip.h, "objID keys"): the reference keeps the objID field as
// the String itself (Deserialization.java:317 strOId), so every distinct String must get its
// own key.  The numeric fast path takes a field only when the String IS Long.toString(v) of a
// v in [-2^62, 2^62) -- no sign '+', no leading zero, not "-0" -- so "7" -> 7 while "007",
// "+7", " 7" and "abc" go to the dictionary (keys INT64_MIN + id, below -2^62).
constexpr int64_t kObjKeyNumLo = -(int64_t(1) << 62);
constexpr int64_t kObjKeyNumHi = int64_t(1) << 62;  // exclusive
template <class Src>
GF_DHD inline bool canonical_objid_key(const Src& s, Field f, int64_t* out) {
  int64_t i = f.b;
  auto next = [&](int64_t j) {  // first non-quote position >= j
    while (j < f.e && s(j) == '"') ++j;
    return j;
  };
  i = next(i);
  if (i >= f.e) return false;
  bool neg = false;
  if (s(i) == '-') {
    neg = true;
    i = next(i + 1);
    if (i >= f.e) return false;
  }
  if (s(i) == '0') {  // "0" alone; "-0", "00", "05" are not Long.toString output
    if (neg) return false;
    if (next(i + 1) < f.e) return false;
    *out = 0;
    return true;
  }
  uint64_t v = 0;
  int nd = 0;
  for (; i < f.e; i = next(i + 1)) {
    const char c = s(i);
    if (c < '0' || c > '9' || ++nd > 19) return false;
    v = v * 10 + (uint64_t)(c - '0');
  }
  if (nd == 0) return false;
  if (neg ? v > (uint64_t)1 << 62 : v >= (uint64_t)1 << 62) return false;
  *out = neg ? (int64_t)(0ull - v) : (int64_t)v;
  return true;
}

GF_DHD inline int clz64(uint64_t x) { return __builtin_clzll(x); }

// Eisel-Lemire for binary64 (w != 0): the correctly rounded bits of w * 10^q.
GF_DHD inline uint64_t eisel_lemire(uint64_t w, int32_t q, const uint64_t* T) {
  if (w == 0 || q < GF_POW5_MIN_Q) return 0ull;
  if (q > GF_POW5_MAX_Q) return 0x7FF0000000000000ull;
  const int lz = clz64(w);
  w <<= lz;
  const int idx = 2 * (q - GF_POW5_MIN_Q);
  unsigned __int128 p = (unsigned __int128)w * T[idx];
  uint64_t hi = (uint64_t)(p >> 64), lo = (uint64_t)p;
  if ((hi & 0x1FFull) == 0x1FFull) {  // 55 bits of precision not yet certain: add the low word
    const uint64_t h2 = (uint64_t)(((unsigned __int128)w * T[idx + 1]) >> 64);
    lo += h2;
    if (h2 > lo) ++hi;
  }
  const int upper = (int)(hi >> 63);
  const int shift = upper + 64 - 52 - 3;
  uint64_t mant = hi >> shift;
  int32_t p2 = (int32_t)((((152170 + 65536) * q) >> 16) + 63) + upper - lz + 1023;
  if (p2 <= 0) {  // subnormal
    if (-p2 + 1 >= 64) return 0ull;
    mant >>= -p2 + 1;
    mant += mant & 1ull;
    mant >>= 1;
    p2 = mant < (1ull << 52) ? 0 : 1;
    return (mant & ((1ull << 52) - 1)) | ((uint64_t)p2 << 52);
  }
  // exactly halfway between two doubles (only possible when 5^q fits 64 bits): round to even
  if (lo <= 1 && q >= -4 && q <= 23 && (mant & 3ull) == 1ull && (mant << shift) == hi) mant &= ~1ull;
  mant += mant & 1ull;
  mant >>= 1;
  if (mant >= (2ull << 52)) {
    mant = 1ull << 52;
    ++p2;
  }
  mant &= ~(1ull << 52);
  if (p2 >= 0x7FF) return 0x7FF0000000000000ull;
  return mant | ((uint64_t)p2 << 52);
}

constexpr double kExactP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

GF_DHD inline double bits_to_double(uint64_t b) {
  union {
    uint64_t u;
    double d;
  } v;
  v.u = b;
  return v.d;
}

GF_DHD inline bool java_ws(char c) { return (unsigned char)c <= ' '; }  // String.trim()

// Double.valueOf(field) -> *out.  T: the 5^q table (device or host copy of GF_POW5_TABLE).
template <class Src>
GF_DHD inline int parse_java_double(const Src& s, Field f, const uint64_t* T, double* out) {
  int64_t i = f.b, e = f.e;
  // trim, skipping quotes on the way
  while (i < e && (s(i) == '"' || java_ws(s(i)))) ++i;
  while (e > i && (s(e - 1) == '"' || java_ws(s(e - 1)))) --e;
  auto next = [&](int64_t j) {  // first non-quote position >= j
    while (j < e && s(j) == '"') ++j;
    return j;
  };
  i = next(i);
  if (i >= e) return kNumBad;
  bool neg = false;
  char c = s(i);
  if (c == '-' || c == '+') {
    neg = c == '-';
    i = next(i + 1);
    if (i >= e) return kNumBad;
    c = s(i);
  }
  if (c == 'N' || c == 'I') {  // "NaN" / "Infinity", nothing after
    const char* word = c == 'N' ? "NaN" : "Infinity";
    int k = 0;
    for (; word[k] && i < e; ++k, i = next(i + 1))
      if (s(i) != word[k]) return kNumBad;
    if (word[k] || i < e) return kNumBad;
    *out = c == 'N' ? bits_to_double(0x7FF8000000000000ull) : bits_to_double(neg ? 0xFFF0000000000000ull : 0x7FF0000000000000ull);
    return kNumOk;
  }
  if (c == '0' && next(i + 1) < e && (s(next(i + 1)) == 'x' || s(next(i + 1)) == 'X')) return kNumUnsupported;
  uint64_t w = 0;
  int nsig = 0;         // significant digits taken into w (<= 19)
  int64_t dexp = 0;     // decimal exponent adjustment
  bool any = false, trunc = false, dot = false;
  for (; i < e; i = next(i + 1)) {
    c = s(i);
    if (c == '.') {
      if (dot) return kNumBad;
      dot = true;
      continue;
    }
    if (c < '0' || c > '9') break;
    any = true;
    const int d = c - '0';
    if (nsig == 0 && d == 0) {  // leading zero
      if (dot) --dexp;
      continue;
    }
    if (nsig < 19) {
      w = w * 10 + (uint64_t)d;
      ++nsig;
      if (dot) --dexp;
    } else {
      if (!dot) ++dexp;
      if (d) trunc = true;
    }
  }
  if (!any) return kNumBad;
  int64_t ex = 0;
  if (i < e && (s(i) == 'e' || s(i) == 'E')) {
    i = next(i + 1);
    bool eneg = false;
    if (i < e && (s(i) == '-' || s(i) == '+')) {
      eneg = s(i) == '-';
      i = next(i + 1);
    }
    int nd = 0;
    for (; i < e && s(i) >= '0' && s(i) <= '9'; i = next(i + 1), ++nd)
      if (ex < 100000000) ex = ex * 10 + (s(i) - '0');
    if (nd == 0) return kNumBad;
    if (eneg) ex = -ex;
  }
  if (i < e && (s(i) == 'f' || s(i) == 'F' || s(i) == 'd' || s(i) == 'D')) i = next(i + 1);
  if (i < e) return kNumBad;
  int64_t q64 = dexp + ex;
  if (w == 0) {
    *out = neg ? -0.0 : 0.0;
    return kNumOk;
  }
  if (q64 < -400) q64 = -400;  // beyond both ends the result is 0 / infinity anyway
  if (q64 > 400) q64 = 400;
  const int32_t q = (int32_t)q64;
  uint64_t bits;
  if (!trunc && w <= (1ull << 53) && q >= -22 && q <= 22) {  // Clinger: one exact operation
    const double v = q < 0 ? (double)w / kExactP10[-q] : (double)w * kExactP10[q];
    *out = neg ? -v : v;
    return kNumOk;
  }
  bits = eisel_lemire(w, q, T);
  if (trunc && w != 0xFFFFFFFFFFFFFFFFull && eisel_lemire(w + 1, q, T) != bits) return kNumUnsupported;
  *out = bits_to_double(bits | (neg ? 0x8000000000000000ull : 0ull));
  return kNumOk;
}

}  // namespace gf
