// k_csv.hip -- GPU CSV/TSV ingest: Deserialization.CSVTSVToTSpatial.map
// (Deserialization.java:291-325) for a whole chunk of text lines at once, fused with
// HelperClass.assignGridCellID (Point.java:98).  Three kernels over HBM-resident text:
//
//   csv_count   newline bytes per 64 KB segment (16-B loads, SWAR byte compare)
//   csv_index   the newline positions, in order (block-wide prefix of per-thread counts)
//   csv_parse   one lane per line: quotes dropped, fields split on the delimiter with the
//               surrounding whitespace (the reference's split("\\s*" + delim + "\\s*")),
//               the objID String as its key (canonical decimals directly, the rest queued for
//               the dictionary, k_objid.hip), Long.valueOf(time), Double.valueOf(x, y) correctly
//               rounded on the device (gf_decimal.hpp), cell (cx, cy), SoA stores.
#include "gf_decimal.hpp"
#include "gf_internal.hpp"

namespace gf {

__device__ const uint64_t kPow5Dev[] = {GF_POW5_TABLE};

// bytes equal to '\n' in a 64-bit word: high bit of each matching byte (exact, no carries)
__device__ __forceinline__ uint64_t nl_bytes(uint64_t x) {
  const uint64_t y = x ^ 0x0A0A0A0A0A0A0A0Aull;
  const uint64_t t = (y & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full;
  return ~(t | y | 0x7F7F7F7F7F7F7F7Full);
}
// 16-bit mask of '\n' bytes in 16 bytes (bit b = byte b)
__device__ __forceinline__ uint32_t nl_mask16(uint64_t lo, uint64_t hi) {
  uint32_t m = 0;
  const uint64_t a = nl_bytes(lo), b = nl_bytes(hi);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    m |= (uint32_t)((a >> (8 * k + 7)) & 1ull) << k;
    m |= (uint32_t)((b >> (8 * k + 7)) & 1ull) << (k + 8);
  }
  return m;
}

// this thread's 16 bytes at [off, off + 16) of the segment (bytewise past len)
__device__ __forceinline__ uint32_t chunk_mask(const char* text, int64_t len, int64_t off) {
  if (off + 16 <= len) {
    const uint4 v = *reinterpret_cast<const uint4*>(text + off);
    return nl_mask16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z);
  }
  uint32_t m = 0;
  for (int k = 0; k < 16 && off + k < len; ++k) m |= (uint32_t)(text[off + k] == '\n') << k;
  return m;
}

__global__ __launch_bounds__(kBlock) void csv_count_kernel(const char* __restrict__ text, int64_t len,
                                                           uint32_t* __restrict__ counts) {
  const int64_t s0 = (int64_t)blockIdx.x * kCsvSeg;
  const int64_t s1 = s0 + kCsvSeg < len ? s0 + kCsvSeg : len;
  uint32_t c = 0;
  for (int64_t off = s0 + 16 * threadIdx.x; off < s1; off += 16 * kBlock) c += __popc(chunk_mask(text, len, off));
  __shared__ uint32_t ws[kBlock / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(kBlock) void csv_index_kernel(const char* __restrict__ text, int64_t len,
                                                           const uint32_t* __restrict__ seg_off,
                                                           int64_t* __restrict__ nl) {
  const int64_t s0 = (int64_t)blockIdx.x * kCsvSeg;
  const int64_t s1 = s0 + kCsvSeg < len ? s0 + kCsvSeg : len;
  __shared__ uint32_t ws[kBlock / 64];
  uint32_t base = seg_off[blockIdx.x];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t it = s0; it < s1; it += 16 * kBlock) {  // block-uniform trip count
    const int64_t off = it + 16 * threadIdx.x;
    const uint32_t m = off < s1 ? chunk_mask(text, len, off) : 0u;
    const uint32_t c = __popc(m);
    uint32_t inc = c;  // inclusive wave prefix
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int v = 0; v < kBlock / 64; ++v) {
      wbase += v < w ? ws[v] : 0u;
      tot += ws[v];
    }
    uint32_t pos = base + wbase + inc - c;
    for (uint32_t mm = m; mm; mm &= mm - 1) nl[pos++] = off + __ffs(mm) - 1;
    base += tot;
    __syncthreads();
  }
}

struct GBytes {
  const char* p;
  __device__ char operator()(int64_t i) const { return p[i]; }
};

__device__ __forceinline__ bool java_s(char c) {  // regex \s: [ \t\n\x0B\f\r]
  return c == ' ' || c == '\t' || c == '\n' || c == '\x0B' || c == '\f' || c == '\r';
}

// the bytes of a block's lines staged in LDS: text position i lives at p[i - base]
struct LBytes {
  const char* p;
  int64_t base;
  __device__ char operator()(int64_t i) const { return p[i - base]; }
};

// Field ranges of the wanted columns of line [b, e).  Returns the number of fields.
template <class Src>
__device__ int split_line(const Src& s, int64_t b, int64_t e, char d, const int32_t* want, Field* got) {
  const bool wsd = java_s(d);
  int field = 0;
  int64_t fs = b;
  auto close = [&](int64_t fe, bool last) {
    int64_t x0 = fs, x1 = fe;
    if (!wsd) {  // whitespace next to a delimiter belongs to the delimiter
      if (field > 0)
        while (x0 < x1 && (java_s(s(x0)) || s(x0) == '"')) ++x0;
      if (!last)
        while (x1 > x0 && (java_s(s(x1 - 1)) || s(x1 - 1) == '"')) --x1;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (want[k] == field) got[k] = Field{x0, x1};
    ++field;
  };
  if (!wsd) {
    for (int64_t i = b; i < e; ++i)
      if (s(i) == d) {
        close(i, false);
        fs = i + 1;
      }
  } else {  // a run of whitespace (quotes are transparent) holding a delimiter is one separator
    int64_t i = b;
    while (i < e) {
      const char c = s(i);
      if (java_s(c) || c == '"') {
        int64_t j = i;
        bool hd = false;
        while (j < e && (java_s(s(j)) || s(j) == '"')) {
          hd |= s(j) == d;
          ++j;
        }
        if (hd) {
          close(i, false);
          fs = j;
        }
        i = j;
      } else {
        ++i;
      }
    }
  }
  close(e, true);
  return field;
}

// One line, in the reference's order: strOId = get(objid) (any String: canonical decimals become
// their key here, the rest is queued for the dictionary), time = Long.valueOf(get(time)),
// x = Double.valueOf(get(x)), y = Double.valueOf(get(y)); the first missing field
// (IndexOutOfBounds) or malformed number (NumberFormatException) is the line's error.
struct LineOut {
  int64_t obj, ts;
  double x, y;
  bool dict;        // objID is not a canonical decimal: f_obj goes to the dictionary
  Field f_obj;
};
template <class Src>
__device__ __forceinline__ int eval_csv_line(const CsvArgs& a, const Src& s, int64_t j, LineOut* o) {
  const int64_t b = j == 0 ? 0 : a.nl[j - 1] + 1;
  int64_t e = j < a.newlines ? a.nl[j] : a.len;
  if (e > b && s(e - 1) == '\r') --e;  // TextInputFormat drops the '\r' of "\r\n"
  if (e <= b) return kCsvEmptyLine;
  Field f[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
  const int nf = split_line(s, b, e, a.delim, a.want, f);
  if (a.want[0] >= nf) return kCsvMissingField;
  o->dict = !canonical_objid_key(s, f[0], &o->obj);
  o->f_obj = f[0];
  if (o->dict && f[0].e - f[0].b > (int64_t)kDictLenMask) return kCsvUnsupported;
  int st;
  if (a.want[1] >= nf) return kCsvMissingField;
  if ((st = parse_java_long(s, f[1], &o->ts))) return st == kNumUnsupported ? kCsvUnsupported : kCsvNumberFormat;
  if (a.want[2] >= nf) return kCsvMissingField;
  if ((st = parse_java_double(s, f[2], kPow5Dev, &o->x))) return st == kNumUnsupported ? kCsvUnsupported : kCsvNumberFormat;
  if (a.want[3] >= nf) return kCsvMissingField;
  if ((st = parse_java_double(s, f[3], kPow5Dev, &o->y))) return st == kNumUnsupported ? kCsvUnsupported : kCsvNumberFormat;
  return kCsvOk;
}

// ---------------------------------------------------------------------------------------
// GeoJSON lines (Deserialization.GeoJSONToTSpatial.map, Deserialization.java:149-211): a small
// JSON scanner over the line's bytes -- member lookup (last duplicate wins, as Jackson's
// ObjectNode), value skipping, and the three values the map reads: the geometry's first
// coordinate, the time property, the objID property.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool jws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
template <class Src>
__device__ __forceinline__ int64_t jskip(const Src& s, int64_t p, int64_t e) {
  while (p < e && jws(s(p))) ++p;
  return p;
}
// the string at p (s(p) == '"'): index past its closing quote, -1 if unterminated
template <class Src>
__device__ int64_t jstr_end(const Src& s, int64_t p, int64_t e, bool* esc) {
  for (++p; p < e; ++p) {
    const char c = s(p);
    if (c == '\\') {
      *esc = true;
      ++p;
    } else if (c == '"') {
      return p + 1;
    }
  }
  return -1;
}
// end of the value at p (p at its first byte), -1 if malformed
template <class Src>
__device__ int64_t jval_end(const Src& s, int64_t p, int64_t e) {
  char c = s(p);
  if (c == '"') {
    bool esc = false;
    return jstr_end(s, p, e, &esc);
  }
  if (c == '{' || c == '[') {
    int depth = 0;
    while (p < e) {
      c = s(p);
      if (c == '"') {
        bool esc = false;
        p = jstr_end(s, p, e, &esc);
        if (p < 0) return -1;
        continue;
      }
      if (c == '{' || c == '[') ++depth;
      else if ((c == '}' || c == ']') && --depth == 0) return p + 1;
      ++p;
    }
    return -1;
  }
  int64_t q = p;
  while (q < e && !(s(q) == ',' || s(q) == '}' || s(q) == ']' || jws(s(q)))) ++q;
  return q > p ? q : -1;
}
// the value of the LAST member `key` of the object at p (s(p) == '{'): its first byte, -1 when
// absent, -2 when the object is malformed
template <class Src>
__device__ int64_t jfind(const Src& s, int64_t p, int64_t e, const char* key, int klen) {
  int64_t found = -1;
  p = jskip(s, p + 1, e);
  if (p < e && s(p) == '}') return -1;
  while (p < e) {
    if (s(p) != '"') return -2;
    bool esc = false;
    const int64_t ke = jstr_end(s, p, e, &esc);
    if (ke < 0) return -2;
    bool match = !esc && ke - p - 2 == klen;
    for (int i = 0; match && i < klen; ++i) match = s(p + 1 + i) == key[i];
    p = jskip(s, ke, e);
    if (p >= e || s(p) != ':') return -2;
    p = jskip(s, p + 1, e);
    if (p >= e) return -2;
    const int64_t ve = jval_end(s, p, e);
    if (ve < 0) return -2;
    if (match) found = p;
    p = jskip(s, ve, e);
    if (p >= e) return -2;
    if (s(p) == ',') {
      p = jskip(s, p + 1, e);
      continue;
    }
    return s(p) == '}' ? found : -2;
  }
  return -2;
}
// JSON number token [p, q): -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?; *integral = no frac/exp
template <class Src>
__device__ bool jnumber(const Src& s, int64_t p, int64_t q, bool* integral) {
  int64_t i = p;
  if (i < q && s(i) == '-') ++i;
  if (i >= q) return false;
  if (s(i) == '0') ++i;
  else if (s(i) >= '1' && s(i) <= '9') while (i < q && s(i) >= '0' && s(i) <= '9') ++i;
  else return false;
  *integral = true;
  if (i < q && s(i) == '.') {
    *integral = false;
    const int64_t d = ++i;
    while (i < q && s(i) >= '0' && s(i) <= '9') ++i;
    if (i == d) return false;
  }
  if (i < q && (s(i) == 'e' || s(i) == 'E')) {
    *integral = false;
    ++i;
    if (i < q && (s(i) == '+' || s(i) == '-')) ++i;
    const int64_t d = i;
    while (i < q && s(i) >= '0' && s(i) <= '9') ++i;
    if (i == d) return false;
  }
  return i == q;
}
// days since 1970-01-01 of the proleptic Gregorian date (y, m 1..12, day 1)
__device__ __forceinline__ int64_t days_from_civil(int64_t y, int64_t m) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5;
  return era * 146097 + yoe * 365 + yoe / 4 - yoe / 100 + doy - 719468;
}
// SimpleDateFormat("yyyy-MM-dd HH:mm:ss").parse (lenient: fields roll over) of the string content
// [p, q): 0 = parsed, 1 = ParseException (time stays 0), 2 = unsupported (before 1583)
template <class Src>
__device__ int jdate(const Src& s, int64_t p, int64_t q, int64_t tz_off_ms, int64_t* ms) {
  const char sep[5] = {'-', '-', ' ', ':', ':'};
  int64_t f[6];
  for (int k = 0; k < 6; ++k) {
    int nd = 0;
    int64_t v = 0;
    while (p < q && s(p) >= '0' && s(p) <= '9' && nd < 10) {
      v = v * 10 + (s(p) - '0');
      ++p;
      ++nd;
    }
    if (nd == 0) return 1;
    if (nd == 10) return 2;  // int overflow territory of the lenient calendar: not restated
    f[k] = v;
    if (k < 5) {
      if (p >= q || s(p) != sep[k]) return 1;
      ++p;
    }
  }
  const int64_t m0 = f[1] - 1;
  const int64_t y = f[0] + (m0 >= 0 ? m0 / 12 : (m0 - 11) / 12);
  const int64_t m = m0 - 12 * (y - f[0]) + 1;
  const int64_t days = days_from_civil(y, m) + f[2] - 1;
  const int64_t secs = ((days * 24 + f[3]) * 60 + f[4]) * 60 + f[5];
  if (secs < -12219292800ll) return 2;  // before 1582-10-15: Java's Julian calendar
  *ms = secs * 1000 - tz_off_ms;
  return 0;
}

// the geometry's first coordinate pair: c at the coordinates array's '['
template <class Src>
__device__ __forceinline__ int geo_coords(const Src& s, int64_t c, int64_t e, LineOut* o) {
  while (c < e && s(c) == '[') c = jskip(s, c + 1, e);  // the first coordinate of any nesting
  double xy[2];
  for (int k = 0; k < 2; ++k) {
    if (c >= e) return kCsvMissingField;
    const int64_t ce = jval_end(s, c, e);
    bool integral;
    if (ce < 0 || !jnumber(s, c, ce, &integral)) return kCsvNumberFormat;
    const int st = parse_java_double(s, Field{c, ce}, kPow5Dev, &xy[k]);
    if (st) return st == kNumUnsupported ? kCsvUnsupported : kCsvNumberFormat;
    c = jskip(s, ce, e);
    if (k == 0) {
      if (c >= e || s(c) != ',') return kCsvMissingField;
      c = jskip(s, c + 1, e);
    }
  }
  o->x = xy[0];
  o->y = xy[1];
  o->ts = 0;
  o->obj = GF_OBJID_NULL;
  o->dict = false;
  return kCsvOk;
}

// what the property lookups need of CsvArgs (passed by value: a reference to the kernel's
// argument block in an outlined call would copy the whole block to scratch, per lane)
struct GeoProps {
  const char* kts;   // property names (the block's LDS copies)
  const char* kobj;
  int32_t len_ts, len_obj, date_fmt;
  int64_t tz_off_ms;
};

// the time and objID properties: t, q = their values' first bytes (-1 absent, -2 malformed object)
template <class Src>
__device__ __forceinline__ int geo_props(const GeoProps& a, const Src& s, int64_t e, int64_t t, int64_t q, LineOut* o) {
  if (a.len_ts >= 0) {
    if (t == -2) return kCsvMissingField;
    if (t >= 0) {
      const int64_t te = jval_end(s, t, e);
      if (a.date_fmt == 0) {  // Long.parseLong(String.valueOf(node)): a JSON integer only
        bool integral;
        if (!jnumber(s, t, te, &integral) || !integral) return kCsvNumberFormat;
        if (parse_java_long(s, Field{t, te}, &o->ts)) return kCsvNumberFormat;
      } else {  // dateFormat.parse(node.textValue()); ParseException -> 0
        if (s(t) != '"') return kCsvNumberFormat;  // textValue() null: the parse throws
        bool esc = false;
        jstr_end(s, t, e, &esc);
        if (esc) return kCsvUnsupported;
        int64_t ms = 0;
        const int st = jdate(s, t + 1, te - 1, a.tz_off_ms, &ms);
        if (st == 2) return kCsvUnsupported;
        if (st == 0) o->ts = ms;
      }
    }
  }
  if (a.len_obj >= 0) {
    if (q == -2) return kCsvMissingField;
    if (q >= 0) {  // nodeOId.toString() with every '"' removed
      const int64_t qe = jval_end(s, q, e);
      Field f{q, qe};
      const char c0 = s(q);
      if (c0 == '"') {
        bool esc = false;
        jstr_end(s, q, e, &esc);
        if (esc) return kCsvUnsupported;
        f = Field{q + 1, qe - 1};
      } else if (c0 == '{' || c0 == '[') {
        return kCsvUnsupported;
      } else if (c0 == '-' || (c0 >= '0' && c0 <= '9')) {
        bool integral;
        if (!jnumber(s, q, qe, &integral)) return kCsvMissingField;
        if (!integral) return kCsvUnsupported;  // Double.toString rendering: not restated
        if (qe - q == 2 && c0 == '-' && s(q + 1) == '0') {  // IntNode(0).toString() == "0"
          o->obj = 0;
          return kCsvOk;
        }
      } else {  // true / false / null print as themselves
        bool lit = false;
        const int64_t n = qe - q;
        if (n == 4) lit = (s(q) == 't' && s(q + 1) == 'r' && s(q + 2) == 'u' && s(q + 3) == 'e') ||
                          (s(q) == 'n' && s(q + 1) == 'u' && s(q + 2) == 'l' && s(q + 3) == 'l');
        if (n == 5) lit = s(q) == 'f' && s(q + 1) == 'a' && s(q + 2) == 'l' && s(q + 3) == 's' && s(q + 4) == 'e';
        if (!lit) return kCsvMissingField;
      }
      o->dict = !canonical_objid_key(s, f, &o->obj);
      o->f_obj = f;
      if (o->dict && f.e - f.b > (int64_t)kDictLenMask) return kCsvUnsupported;
    }
  }
  return kCsvOk;
}

// Member-by-member walk (jfind per looked-up member): exact on any line, malformed ones included.
// p: the line's first non-blank byte, a '{'.
template <class Src>
__device__ __noinline__ int eval_geojson_walk(GeoProps a, Src s, int64_t p, int64_t e, LineOut* o) {
  // the feature: the record's "value" object, or the line's object itself
  int64_t feat = p;
  const int64_t v = jfind(s, p, e, "value", 5);
  if (v == -2) return kCsvMissingField;
  if (v >= 0 && s(v) == '{') feat = v;
  const int64_t g = jfind(s, feat, e, "geometry", 8);
  if (g < 0 || s(g) != '{') return kCsvMissingField;
  const int64_t c = jfind(s, g, e, "coordinates", 11);
  if (c < 0 || s(c) != '[') return kCsvMissingField;
  int st = geo_coords(s, c, e, o);
  if (st) return st;
  const int64_t pr = jfind(s, feat, e, "properties", 10);
  if (pr == -2) return kCsvMissingField;
  if (pr < 0 || s(pr) != '{') return kCsvOk;
  const int64_t t = a.len_ts >= 0 ? jfind(s, pr, e, a.kts, a.len_ts) : -1;
  const int64_t q = a.len_obj >= 0 ? jfind(s, pr, e, a.kobj, a.len_obj) : -1;
  return geo_props(a, s, e, t, q, o);
}

// ---------------------------------------------------------------------------------------
// One-pass member location (the common case).  The walk above re-scans the feature once per
// member it looks up, with nested data-dependent loops per lane: with 64 lines per wave in
// different places of that loop nest the exec-mask bookkeeping dominated (~2.7 k scalar
// instructions per line).  Here each lane runs one automaton over its line, byte by byte: a
// strict JSON syntax check plus a small stack of container roles (the top object, the record's
// "value" object, the geometry and properties objects under either), noting the position of
// the LAST key of each member the walk would look up.  On a line that passes the check --
// strictly valid JSON, no backslash, nesting <= 63 -- every jfind of the walk returns exactly
// that last member's value (the walk's looser scanning agrees with JSON on valid input), so the
// results are the walk's.  Any other line (malformed, escapes, deeper nesting) takes the walk.
//
// The per-byte step: one 8-B LDS entry per byte value holds the (next state, action) pair of
// all 9 states (7 bits each), so the lookup does not wait on the state and the state update is
// a shift; only the actions (brackets, commas, key quotes) do more, and the key comparison runs
// only for keys of a looked-up length in a looked-up container.  (A select-only form of the
// actions measured slower: 1.82 vs 1.67 ms for the locator over 1M lines.)  Stale
// notes need no reset: a note is current when it lies after the note of its container's key
// (e.g. the coordinates key after the last geometry key).
// ---------------------------------------------------------------------------------------
enum : uint8_t { JS_VAL, JS_ARR0, JS_OBJ0, JS_KEY, JS_COLON, JS_AFT, JS_VSTR, JS_KSTR, JS_TOK, JS_N, JS_ERR = 9 };
enum : uint8_t { JC_WS, JC_LBRACE, JC_RBRACE, JC_LBRACK, JC_RBRACK, JC_QUOTE, JC_COMMA, JC_COLON, JC_BSL, JC_TOK, JC_OTHER };
enum : uint8_t { JA_NONE, JA_PUSH_OBJ, JA_PUSH_ARR, JA_POP_OBJ, JA_POP_ARR, JA_COMMA, JA_KEY_BEGIN, JA_KEY_END };
enum : int { JR_NONE, JR_TOP, JR_VAL, JR_GEO_T, JR_PROP_T, JR_GEO_V, JR_PROP_V };  // container roles
enum : int { JK_NONE, JK_VALUE, JK_GEO, JK_PROP };                                 // member kinds
constexpr int kGeoKeys = 6;  // value, geometry, properties, coordinates, time property, objID property

__device__ __forceinline__ uint8_t jclass(int c) {
  switch (c) {
    case ' ': case '\t': case '\n': case '\r': return JC_WS;
    case '{': return JC_LBRACE;
    case '}': return JC_RBRACE;
    case '[': return JC_LBRACK;
    case ']': return JC_RBRACK;
    case '"': return JC_QUOTE;
    case ',': return JC_COMMA;
    case ':': return JC_COLON;
    case '\\': return JC_BSL;
    default: break;
  }
  if ((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '+' || c == '-' || c == '.')
    return JC_TOK;
  return JC_OTHER;
}
// next state | action << 4.  After the top object closes the state is JS_AFT at depth 0, where
// a comma or a closer is an error (checked with the depth, geo_locate).
__device__ __forceinline__ uint8_t jtrans(int st, int cl) {
  auto E = [](int n, int act) { return (uint8_t)(n | act << 4); };
  if (st == JS_VSTR) return cl == JC_QUOTE ? E(JS_AFT, 0) : cl == JC_BSL ? E(JS_ERR, 0) : E(JS_VSTR, 0);
  if (st == JS_KSTR) return cl == JC_QUOTE ? E(JS_COLON, JA_KEY_END) : cl == JC_BSL ? E(JS_ERR, 0) : E(JS_KSTR, 0);
  if (st == JS_TOK) {
    if (cl == JC_TOK) return E(JS_TOK, 0);
    st = JS_AFT;  // the token ends here: the byte is read as after a value
  }
  if (cl == JC_WS) return E(st, 0);
  switch (st) {
    case JS_VAL: case JS_ARR0:
      if (cl == JC_LBRACE) return E(JS_OBJ0, JA_PUSH_OBJ);
      if (cl == JC_LBRACK) return E(JS_ARR0, JA_PUSH_ARR);
      if (cl == JC_QUOTE) return E(JS_VSTR, 0);
      if (cl == JC_TOK) return E(JS_TOK, 0);
      if (st == JS_ARR0 && cl == JC_RBRACK) return E(JS_AFT, JA_POP_ARR);
      return E(JS_ERR, 0);
    case JS_OBJ0:
      if (cl == JC_QUOTE) return E(JS_KSTR, JA_KEY_BEGIN);
      if (cl == JC_RBRACE) return E(JS_AFT, JA_POP_OBJ);
      return E(JS_ERR, 0);
    case JS_KEY: return cl == JC_QUOTE ? E(JS_KSTR, JA_KEY_BEGIN) : E(JS_ERR, 0);
    case JS_COLON: return cl == JC_COLON ? E(JS_VAL, 0) : E(JS_ERR, 0);
    case JS_AFT:
      if (cl == JC_COMMA) return E(JS_VAL, JA_COMMA);
      if (cl == JC_RBRACE) return E(JS_AFT, JA_POP_OBJ);
      if (cl == JC_RBRACK) return E(JS_AFT, JA_POP_ARR);
      return E(JS_ERR, 0);
    default: return E(JS_ERR, 0);
  }
}

// LDS tables of a block: per byte value the 9 states' entries; the looked-up member names
struct GeoTabs {
  const uint64_t* tab;  // [256]: entry of state s at bits 7s..7s+6
  const char* keys;     // kGeoKeys x kGeoPropMax
  int32_t klen[kGeoKeys];
};

__device__ void geo_tabs_fill(const CsvArgs& a, uint64_t* tab, char* keys) {
  for (int b = threadIdx.x; b < 256; b += blockDim.x) {
    const int cl = jclass(b);
    uint64_t t = 0;
    for (int st = 0; st < JS_N; ++st) t |= (uint64_t)jtrans(st, cl) << (7 * st);
    tab[b] = t;
  }
  for (int i = threadIdx.x; i < kGeoKeys * kGeoPropMax; i += blockDim.x) {
    const int k = i / kGeoPropMax, c = i % kGeoPropMax;
    const char* names[4] = {"value", "geometry", "properties", "coordinates"};
    char ch = 0;
    if (k < 4) {
      const int n = k == 0 ? 5 : k == 1 ? 8 : k == 2 ? 10 : 11;
      ch = c < n ? names[k][c] : 0;
    } else {
      ch = k == 4 ? a.prop_ts[c] : a.prop_obj[c];
    }
    keys[i] = ch;
  }
}

template <class Src>
__device__ __forceinline__ bool jkey_eq(const Src& s, int64_t ks, int len, const GeoTabs& gt, int k) {
  if (gt.klen[k] != len) return false;
  bool eq = true;
  for (int i = 0; eq && i < len; ++i) eq = s(ks + i) == gt.keys[k * kGeoPropMax + i];
  return eq;
}

// the value of the member whose key's closing quote is at k (valid JSON: '"' ws ':' ws value)
template <class Src>
__device__ __forceinline__ int64_t jmember_value(const Src& s, int64_t k, int64_t e) {
  return jskip(s, jskip(s, k + 1, e) + 1, e);
}

// The automaton over the line [p, e) (s(p) == '{'), staged in LDS (lds + (pos - base)).  Returns
// false when the line must take the walk; otherwise the feature's member values g, c
// (coordinates), pr, t, q: first byte, -1 when absent.
__device__ __forceinline__ bool geo_locate(const LBytes& s, int64_t p, int64_t e, const GeoTabs& gt, int64_t* loc) {
  if (e - p >= INT32_MAX) return false;
  int st = JS_VAL, depth = 0, pend = JK_NONE;
  bool bad = false;
  uint64_t kinds = 0;  // bit d: the container at depth d is an object
  uint32_t roles = 0;  // 4 bits per depth 1..7
  int32_t ks = 0;
  // closing-quote positions (from p) of the last keys noted: the record's "value"; per feature
  // (top object T / value object V) geometry, properties, coordinates, time, objID
  int32_t v = -1, gT = -1, prT = -1, cT = -1, tT = -1, qT = -1, gV = -1, prV = -1, cV = -1, tV = -1, qV = -1;
  // length filters of the keys looked up per container group (lengths < 64)
  const uint64_t lf_top = (1ull << 5) | (1ull << 8) | (1ull << 10), lf_geo = 1ull << 11;
  const uint64_t lf_prop = (gt.klen[4] >= 0 ? 1ull << gt.klen[4] : 0) | (gt.klen[5] >= 0 ? 1ull << gt.klen[5] : 0);
  const int32_t o0 = (int32_t)(p - s.base), o1 = (int32_t)(e - s.base);  // the line's LDS offsets
  for (int32_t w = o0 & ~3; w < o1 && !bad; w += 4) {
    const uint32_t word = *reinterpret_cast<const uint32_t*>(s.p + w);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int32_t i = w + k - o0;  // offset in the line
      const uint32_t byte = i < 0 || w + k >= o1 ? (uint32_t)' ' : (word >> (8 * k)) & 0xFFu;
      const uint32_t ent = (uint32_t)(gt.tab[byte] >> (7 * st)) & 0x7Fu;
      int nst = (int)(ent & 15u);
      const int act = (int)(ent >> 4);
      if (act) {
        const int role = (unsigned)depth <= 7u ? (int)(roles >> (4 * depth)) & 15 : JR_NONE;
        if (act == JA_PUSH_OBJ || act == JA_PUSH_ARR) {
          int child = depth == 0 ? JR_TOP
                    : role == JR_TOP ? (int)(0x4320u >> (4 * pend)) & 15   // value, geometry, properties
                    : role == JR_VAL ? (int)(0x6500u >> (4 * pend)) & 15   // geometry, properties
                    : JR_NONE;
          if (act == JA_PUSH_ARR) child = JR_NONE;
          ++depth;
          bad |= depth > 63;
          kinds = (kinds & ~(1ull << (depth & 63))) | ((uint64_t)(act == JA_PUSH_OBJ) << (depth & 63));
          if ((unsigned)depth <= 7u) roles = (roles & ~(15u << (4 * depth))) | ((uint32_t)child << (4 * depth));
        } else if (act == JA_POP_OBJ || act == JA_POP_ARR) {
          bad |= depth <= 0 || (int)((kinds >> (depth & 63)) & 1) != (act == JA_POP_OBJ);
          --depth;
        } else if (act == JA_COMMA) {
          bad |= depth <= 0;
          nst = (kinds >> (depth & 63)) & 1 ? JS_KEY : JS_VAL;
        } else if (act == JA_KEY_BEGIN) {
          ks = i + 1;
        } else {  // JA_KEY_END: note a looked-up member of a looked-up container
          const int len = i - ks;
          const uint64_t lf = role == JR_TOP || role == JR_VAL ? lf_top
                            : role == JR_GEO_T || role == JR_GEO_V ? lf_geo
                            : role == JR_PROP_T || role == JR_PROP_V ? lf_prop : 0;
          pend = JK_NONE;
          if (len < 64 && ((lf >> len) & 1)) {
            const int64_t kp = p + ks;
            if (role == JR_TOP || role == JR_VAL) {
              if (role == JR_TOP && jkey_eq(s, kp, len, gt, 0)) {
                pend = JK_VALUE;
                v = i;
              } else if (jkey_eq(s, kp, len, gt, 1)) {
                pend = JK_GEO;
                if (role == JR_TOP) gT = i; else gV = i;
              } else if (jkey_eq(s, kp, len, gt, 2)) {
                pend = JK_PROP;
                if (role == JR_TOP) prT = i; else prV = i;
              }
            } else if (role == JR_GEO_T || role == JR_GEO_V) {
              if (jkey_eq(s, kp, len, gt, 3)) {
                if (role == JR_GEO_T) cT = i; else cV = i;
              }
            } else {
              if (jkey_eq(s, kp, len, gt, 4)) {
                if (role == JR_PROP_T) tT = i; else tV = i;
              }
              if (jkey_eq(s, kp, len, gt, 5)) {
                if (role == JR_PROP_T) qT = i; else qV = i;
              }
            }
          }
        }
      }
      bad |= nst == JS_ERR;
      st = nst == JS_ERR ? JS_AFT : nst;
    }
  }
  if (bad || st != JS_AFT || depth != 0) return false;
  auto val = [&](int32_t k) { return k < 0 ? (int64_t)-1 : jmember_value(s, p + k, e); };
  const int64_t vv = val(v);
  int32_t g, c, pr, t, q;
  if (vv >= 0 && s(vv) == '{') {  // notes inside an earlier "value" object or member are stale
    g = gV > v ? gV : -1;
    pr = prV > v ? prV : -1;
    c = g >= 0 && cV > g ? cV : -1;
    t = pr >= 0 && tV > pr ? tV : -1;
    q = pr >= 0 && qV > pr ? qV : -1;
  } else {
    g = gT;
    pr = prT;
    c = g >= 0 && cT > g ? cT : -1;
    t = pr >= 0 && tT > pr ? tT : -1;
    q = pr >= 0 && qT > pr ? qT : -1;
  }
  loc[0] = val(g);
  loc[1] = val(c);
  loc[2] = val(pr);
  loc[3] = val(t);
  loc[4] = val(q);
  return true;
}

// FAST: try the one-pass locator first (the LDS-staged path); otherwise the walk
template <bool FAST, class Src>
__device__ __forceinline__ int eval_geojson_line(const CsvArgs& a, const Src& s, int64_t j, LineOut* o, const GeoTabs& gt) {
  const int64_t b = j == 0 ? 0 : a.nl[j - 1] + 1;
  int64_t e = j < a.newlines ? a.nl[j] : a.len;
  if (e > b && s(e - 1) == '\r') --e;
  if (e <= b) return kCsvEmptyLine;
  const int64_t p = jskip(s, b, e);
  if (p >= e || s(p) != '{') return kCsvMissingField;
  const GeoProps gp{gt.keys + 4 * kGeoPropMax, gt.keys + 5 * kGeoPropMax, a.len_ts, a.len_obj, a.date_fmt, a.tz_off_ms};
  int64_t loc[5];
  bool located = false;
  if constexpr (FAST) located = geo_locate(s, p, e, gt, loc);
  if (!located) return eval_geojson_walk(gp, s, p, e, o);
  const int64_t g = loc[0], c = loc[1], pr = loc[2];
  if (g < 0 || s(g) != '{') return kCsvMissingField;
  if (c < 0 || s(c) != '[') return kCsvMissingField;
  const int st = geo_coords(s, c, e, o);
  if (st) return st;
  if (pr < 0 || s(pr) != '{') return kCsvOk;
  return geo_props(gp, s, e, a.len_ts >= 0 ? loc[3] : -1, a.len_obj >= 0 ? loc[4] : -1, o);
}

// parse + store line j; returns true when its objID needs the dictionary (*w filled)
template <int FMT, bool FAST, class Src>
__device__ __forceinline__ bool parse_line(const CsvArgs& a, const Src& s, int64_t j, DictWork* w, const GeoTabs& gt) {
  LineOut o{0, 0, 0.0, 0.0, false, {0, 0}};
  int st;
  if constexpr (FMT == 1) st = eval_geojson_line<FAST>(a, s, j, &o, gt);
  else st = eval_csv_line(a, s, j, &o);
  if (st != kCsvOk) {
    atomicMin(&a.err->line, (unsigned long long)j);
    return false;
  }
  a.x[j] = o.x;
  a.y[j] = o.y;
  a.ts[j] = o.ts;
  if (!o.dict) a.objID[j] = o.obj;
  if (a.cx) {
    a.cx[j] = cell_index(o.x, a.minX, a.cl);
    a.cy[j] = cell_index(o.y, a.minY, a.cl);
  }
  if (o.dict) *w = DictWork{o.f_obj.b, (int32_t)(o.f_obj.e - o.f_obj.b), (uint32_t)j};
  return o.dict;
}

// A block takes 256 consecutive lines.  Their bytes are contiguous: when they fit the block's
// staging area (a.lds_cap bytes of dynamic LDS, sized from the mean line length) they are staged
// in LDS with coalesced 16-B loads first, so the per-byte reads of the split/parse state machines
// (a dependent chain per lane) hit LDS instead of waiting on L2 one byte at a time.  GeoJSON
// blocks also fill the one-pass locator's tables (geo_locate) in LDS.
// Dictionary objIDs are queued with one atomic per wave (the queue order is free: ids follow
// line order, k_objid.hip).
template <int FMT>  // 0: CSV / TSV, 1: GeoJSON (a.format)
__global__ __launch_bounds__(kBlock) void csv_parse_kernel(CsvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int64_t L0 = (int64_t)blockIdx.x * kBlock;
  const int64_t L1 = L0 + kBlock < a.lines ? L0 + kBlock : a.lines;  // exclusive
  const int64_t b0 = L0 == 0 ? 0 : a.nl[L0 - 1] + 1;
  const int64_t b1 = L1 - 1 < a.newlines ? a.nl[L1 - 1] : a.len;     // the last line's '\n' (or end)
  const int64_t a0 = b0 & ~(int64_t)15;
  const int64_t j = L0 + threadIdx.x;
  DictWork w{0, 0, 0};
  bool need = false;
  __shared__ uint64_t gtab[FMT == 1 ? 256 : 1];
  __shared__ char gkeys[FMT == 1 ? kGeoKeys * kGeoPropMax : 1];
  const GeoTabs gt{gtab, gkeys, {5, 8, 10, 11, a.len_ts, a.len_obj}};
  if (FMT == 1) {
    geo_tabs_fill(a, gtab, gkeys);
    __syncthreads();
  }
  if (b1 - a0 <= a.lds_cap) {  // block-uniform
    for (int64_t off = a0 + 16 * threadIdx.x; off < b1; off += 16 * kBlock) {
      if (off + 16 <= a.len) {
        *reinterpret_cast<uint4*>(lds + (off - a0)) = *reinterpret_cast<const uint4*>(a.text + off);
      } else {
        for (int k = 0; k < 16 && off + k < a.len; ++k) lds[off - a0 + k] = a.text[off + k];
      }
    }
    __syncthreads();
    if (j < L1) {
      if (a.geo_fast) need = parse_line<FMT, true>(a, LBytes{lds, a0}, j, &w, gt);
      else need = parse_line<FMT, false>(a, LBytes{lds, a0}, j, &w, gt);
    }
  } else if (j < L1) {
    need = parse_line<FMT, false>(a, GBytes{a.text}, j, &w, gt);
  }
  const uint64_t m = __ballot(need);
  if (m) {
    const int lane = threadIdx.x & 63;
    unsigned long long nb = need ? (unsigned long long)w.n : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nb += __shfl_xor(nb, o, 64);
    uint32_t base = 0;
    if (lane == 0) {
      base = atomicAdd(a.dict_n, (uint32_t)__popcll(m));
      atomicAdd(a.dict_bytes, nb);
    }
    base = __shfl(base, 0, 64);
    if (need) a.dict_work[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = w;
  }
}

// error kind of the first bad line (re-derived by a one-lane pass over that line)
__global__ void csv_error_kernel(CsvArgs a) {
  const unsigned long long j = a.err->line;
  if (j == ~0ull) return;  // block-uniform
  __shared__ uint64_t gtab[256];
  __shared__ char gkeys[kGeoKeys * kGeoPropMax];
  const GeoTabs gt{gtab, gkeys, {5, 8, 10, 11, a.len_ts, a.len_obj}};
  if (a.format == 1) geo_tabs_fill(a, gtab, gkeys);
  __syncthreads();
  if (threadIdx.x != 0) return;
  LineOut o{0, 0, 0.0, 0.0, false, {0, 0}};
  const GBytes s{a.text};
  a.err->kind = a.format == 1 ? eval_geojson_line<false>(a, s, (int64_t)j, &o, gt) : eval_csv_line(a, s, (int64_t)j, &o);
}

hipError_t launch_csv_count(hipStream_t st, const char* text, int64_t len, int64_t nseg, uint32_t* counts) {
  hipLaunchKernelGGL(csv_count_kernel, dim3((unsigned)nseg), dim3(kBlock), 0, st, text, len, counts);
  return hipGetLastError();
}

hipError_t launch_csv_index(hipStream_t st, const char* text, int64_t len, int64_t nseg, const uint32_t* seg_off,
                            int64_t* nl) {
  hipLaunchKernelGGL(csv_index_kernel, dim3((unsigned)nseg), dim3(kBlock), 0, st, text, len, seg_off, nl);
  return hipGetLastError();
}

// Staging size: 256 mean-length lines plus a tenth for the spread of a block's sum, in 1-KB
// steps between kCsvLds and kCsvLdsMax (CSV points ~55 B/line keep the 24 KB floor, so 6 blocks
// share a CU).  GeoJSON features (~183 B/line, ~47 KB a block) are held to 50 KB when a mean
// block fits it with 5% to spare, so that 3 blocks (with the locator's 2.4 KB of tables) share
// a CU.  A block whose lines exceed the staging area parses from global memory with the walk
// (same results, one dependent L2 read per byte).
hipError_t launch_csv_parse(gf_ctx* ctx, const CsvArgs& a0) {
  KTimer t(ctx, GF_K_CSV_PARSE);
  CsvArgs a = a0;
  const int64_t mean = a.lines > 0 ? (a.len + a.lines - 1) / a.lines : 0;
  const int64_t need = mean * kBlock;
  int64_t cap = (need * 11 / 10 + 1023) & ~(int64_t)1023;
  constexpr int64_t kGeoLds3 = 50 * 1024;
  if (a.format == 1 && cap > kGeoLds3 && need * 20 <= kGeoLds3 * 19) cap = kGeoLds3;
  a.lds_cap = (int32_t)(cap < kCsvLds ? kCsvLds : cap > kCsvLdsMax ? kCsvLdsMax : cap);
  if (a.lines > 0) {
    const unsigned blocks = (unsigned)((a.lines + kBlock - 1) / kBlock);
    if (a.format == 1)
      hipLaunchKernelGGL(csv_parse_kernel<1>, dim3(blocks), dim3(kBlock), (size_t)a.lds_cap, ctx->stream, a);
    else
      hipLaunchKernelGGL(csv_parse_kernel<0>, dim3(blocks), dim3(kBlock), (size_t)a.lds_cap, ctx->stream, a);
  }
  hipLaunchKernelGGL(csv_error_kernel, dim3(1), dim3(64), 0, ctx->stream, a);
  return hipGetLastError();
}

}  // namespace gf
