// Test-only host build of the GeoJSON ingest's per-line evaluator (spatialflink_amd/csrc/
// gf_geojson.hpp): the very code the GPU parse kernel runs -- the one-pass locator over
// LDS-staged bytes and the walk -- compiled for the CPU, so tests/test_geojson_core.py can check
// both paths against the oracle (oracle.geojson_parse) on every line.  Not part of the product.
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "../../spatialflink_amd/csrc/gf_geojson.hpp"

static const uint64_t kPow5Host[] = {GF_POW5_TABLE};

// Per line j of buf[off[j], off[j+1]) (no '\n'): kind, x, y, ts, objID key (dict = 1: the objID
// String is buf[ob[j], oe[j])).  walk: every line takes the walk (else the locator first).
extern "C" void geojson_core_parse(const char* buf, const int64_t* off, int64_t n, const char* prop_obj,
                                   const char* prop_ts, int date_fmt, int tz_off_min, int value_lines, int walk,
                                   int32_t* kind, double* x, double* y, int64_t* ts, int64_t* obj, int32_t* dict,
                                   int64_t* ob, int64_t* oe) {
  static uint64_t tab[256], ttab[256];
  for (int b = 0; b < 256; ++b) gf::geo_tab_entry(b, tab + b, ttab + b);
  static char keys[gf::kGeoKeys * gf::kGeoPropMax];
  std::memset(keys, 0, sizeof keys);
  const char* names[5] = {"value", "geometry", "properties", "coordinates", "type"};
  for (int k = 0; k < 4; ++k) std::memcpy(keys + k * gf::kGeoPropMax, names[k], std::strlen(names[k]));
  std::memcpy(keys + 6 * gf::kGeoPropMax, names[4], 4);
  const int len_obj = prop_obj ? (int)std::strlen(prop_obj) : -1, len_ts = prop_ts ? (int)std::strlen(prop_ts) : -1;
  if (prop_ts) std::memcpy(keys + 4 * gf::kGeoPropMax, prop_ts, len_ts);
  if (prop_obj) std::memcpy(keys + 5 * gf::kGeoPropMax, prop_obj, len_obj);
  const gf::GeoTabs gt{tab, ttab, keys, {5, 8, 10, 11, len_ts, len_obj, 4},
                       gf::geo_pack16(keys + 4 * gf::kGeoPropMax, len_ts <= 16 ? len_ts : 0),
                       gf::geo_pack16(keys + 5 * gf::kGeoPropMax, len_obj <= 16 ? len_obj : 0)};
  const gf::GeoProps gp{keys + 4 * gf::kGeoPropMax, keys + 5 * gf::kGeoPropMax, len_ts, len_obj, date_fmt,
                        (int64_t)tz_off_min * 60000, kPow5Host};
  for (int64_t j = 0; j < n; ++j) {
    // the kernel's staging: the line's bytes at a 4-byte aligned base (the locator reads words)
    const int64_t b = off[j];
    int64_t e = off[j + 1];
    const int64_t a0 = b & ~(int64_t)15;
    const gf::LBytes s{buf + a0, a0};
    gf::LineOut o{0, 0, 0.0, 0.0, false, {0, 0}};
    int k;
    if (e > b && s(e - 1) == '\r') --e;
    if (e <= b) {
      k = gf::kCsvEmptyLine;
    } else {
      const int64_t p = gf::jskip(s, b, e);
      if (p >= e || s(p) != '{') k = gf::kCsvMissingField;
      else k = gf::geojson_line(gt, gp, s, p, e, value_lines, walk == 0, &o);
    }
    kind[j] = k;
    x[j] = o.x;
    y[j] = o.y;
    ts[j] = o.ts;
    obj[j] = o.obj;
    dict[j] = o.dict;
    ob[j] = o.f_obj.b;
    oe[j] = o.f_obj.e;
  }
}

// The wave-per-line scan's byte classes (gf_geojson.hpp wave_class), for a CPU check of the table.
extern "C" void geojson_core_wave_classes(uint32_t* out) {
  for (int b = 0; b < 256; ++b) out[b] = gf::wave_class(b);
}
