// gf_text.hpp -- what the text ingest paths (CSV / TSV, GeoJSON) share between the device
// kernels (k_csv.hip) and their host test builds (tests/native/): status kinds, the line result,
// byte sources.  __host__ __device__, no HIP runtime dependency.
#pragma once

#include <cstdint>

#include "../../include/geoflink_hip.h"
#include "gf_decimal.hpp"

#if defined(__HIPCC__)
#define GF_NOINLINE __noinline__
#else
#define GF_NOINLINE __attribute__((noinline))
#endif

// A pointer into LDS.  In the device pass it carries address space 3, so the parsers' byte and
// table reads compile to ds_read (a generic pointer makes them FLAT instructions, whose waits
// cover every memory counter); the host test builds (tests/native/) see a plain pointer.
#if defined(__HIP_DEVICE_COMPILE__)
#define GF_LDS_PTR(T) const __attribute__((address_space(3))) T*
#else
#define GF_LDS_PTR(T) const T*
#endif

namespace gf {

enum { kCsvOk = 0, kCsvNumberFormat = 1, kCsvUnsupported = 2, kCsvMissingField = 3, kCsvEmptyLine = 4 };
constexpr int kGeoPropMax = 64;   // longest GeoJSON property name taken
constexpr int kDictLenBits = 20;  // objID dictionary slot meta = arena offset << 20 | String length
constexpr uint64_t kDictLenMask = (1ull << kDictLenBits) - 1;

// One line, in the reference's order: the point's fields; the objID is its canonical decimal key
// or (dict) the String bytes f_obj for the dictionary.
struct LineOut {
  int64_t obj, ts;
  double x, y;
  bool dict;        // objID is not a canonical decimal: f_obj goes to the dictionary
  Field f_obj;
};

// text bytes read from global memory
struct GBytes {
  const char* p;
  GF_DHD char operator()(int64_t i) const { return p[i]; }
};
// the bytes of a block's lines staged in LDS: text position i lives at p[i - base]
struct LBytes {
  GF_LDS_PTR(char) p;
  int64_t base;
  GF_DHD char operator()(int64_t i) const { return p[i - base]; }
};

}  // namespace gf
