// Test-only host build of the CSV numeric core (spatialflink_amd/csrc/gf_decimal.hpp): the very
// code the GPU ingest kernel runs, compiled for the CPU so tests/test_csv_core.py can check it
// against Python's correctly rounded float() on millions of literals.  Not part of the product.
#include <cstdint>
#include <cstring>

#include "../../spatialflink_amd/csrc/gf_decimal.hpp"

static const uint64_t kPow5Host[] = {GF_POW5_TABLE};

struct Str {
  const char* p;
  char operator()(int64_t i) const { return p[i]; }
};

extern "C" int core_parse_double(const char* s, int64_t len, double* out) {
  return gf::parse_java_double(Str{s}, gf::Field{0, len}, kPow5Host, out);
}
extern "C" int core_parse_long(const char* s, int64_t len, int64_t* out) {
  return gf::parse_java_long(Str{s}, gf::Field{0, len}, out);
}
// many literals in one call: NUL-separated strings
extern "C" void core_parse_many(const char* buf, const int64_t* off, int64_t n, double* out, int32_t* st) {
  for (int64_t j = 0; j < n; ++j) st[j] = core_parse_double(buf + off[j], off[j + 1] - off[j], out + j);
}
// objID fast path: 1 + key when the String is a canonical decimal key, 0 when it needs the dictionary
extern "C" int core_objid_key(const char* s, int64_t len, int64_t* out) {
  return gf::canonical_objid_key(Str{s}, gf::Field{0, len}, out) ? 1 : 0;
}
