// gf_geojson.hpp -- the GeoJSON point ingest's per-line evaluator (Deserialization.GeoJSONToTSpatial.map,
// Deserialization.java:149-211), __host__ __device__: the GPU parse kernel (k_csv.hip) runs it
// per lane over LDS-staged lines, and tests/native/geojson_core.cpp builds the very same code for
// the host so the CPU suite can check both of its paths (the one-pass locator and the walk)
// against the oracle on every generated and hand-built line.
#pragma once

#include <cstdint>

#include "gf_text.hpp"

namespace gf {

// ---------------------------------------------------------------------------------------
// GeoJSON lines (Deserialization.GeoJSONToTSpatial.map, Deserialization.java:149-211).  A line
// is the ObjectNode the map receives -- the Kafka record {"key": .., "value": ..} that
// JSONKeyValueDeserializationSchema builds -- or, with gf_geojson_schema.value_lines, the
// record's value itself (a Feature as Serialization.PointToGeoJSONOutputSchema writes it).
// Per line, in the map's order:
//  1. Jackson reads the record: strict JSON (RFC 8259 grammar; no NaN / Infinity, leading zeros
//     or unescaped control bytes; UTF-8 checked structurally, as Jackson's UTF-8 reader does),
//     else the line fails (GF_CSV_MISSING_FIELD: malformed).  V = the "value" member (last
//     duplicate, Jackson ObjectNode); a missing or non-object V fails the line (the catch
//     branch's value.get("geometry") throws NullPointerException).
//  2. geometry = readGeoJSON(V.toString()) -- jts-io-common 1.18.0 GeoJsonReader (pom.xml:100-104,
//     a dependency absent from the reference tree; its published algorithm restated): V's
//     "type" "Point" takes V's own "coordinates".  On any failure -- and for "Feature" (whose
//     createFeature parses the same V.geometry), a missing, non-string or unknown "type" -- the
//     catch branch (:136-141, :172-178): readGeoJSON(V.get("geometry").toString()), whose failure
//     fails the line.  x, y = the point's ordinates 0 and 1 (geometry.getCoordinate()).
//  3. properties = V.get("properties") (absent or not an object: objID null, ts 0); the time
//     property, then the objID property (geo_props).
// Not restated, reported as GF_CSV_UNSUPPORTED (never guessed): geometry types other than Point
// (JTS builds and validates them: ring closure, point counts) and FeatureCollection; Point
// coordinates with fewer than two ordinates (JTS's defaults) or a non-number third one; a
// number Jackson would hand json-simple as text it cannot read back (a float literal that
// overflows to Infinity, an integer literal outside long) anywhere on the line; nesting deeper
// than 256; an escape in a taken string or in a member name of an object a value is looked up
// in; non-integer or structured objIDs; dates before 1583.
// ---------------------------------------------------------------------------------------
GF_DHD inline bool jws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
template <class Src>
GF_DHD inline int64_t jskip(const Src& s, int64_t p, int64_t e) {
  while (p < e && jws(s(p))) ++p;
  return p;
}
// the string at p (s(p) == '"'): index past its closing quote, -1 if unterminated
template <class Src>
GF_DHD inline int64_t jstr_end(const Src& s, int64_t p, int64_t e, bool* esc) {
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
// end of the (valid) value at p (p at its first byte)
template <class Src>
GF_DHD inline int64_t jval_end(const Src& s, int64_t p, int64_t e) {
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
// The value of the LAST member `key` of the (valid) object at p (s(p) == '{'): its first byte,
// -1 when absent, -3 when a member name of the object is written with an escape (Jackson
// decodes it, so it might be the name looked up: not restated).
template <class Src>
GF_DHD inline int64_t jfind(const Src& s, int64_t p, int64_t e, const char* key, int klen) {
  int64_t found = -1;
  bool esc_key = false;
  p = jskip(s, p + 1, e);
  if (p < e && s(p) == '}') return -1;
  while (p < e && s(p) == '"') {
    bool esc = false;
    const int64_t ke = jstr_end(s, p, e, &esc);
    if (ke < 0) return -3;
    esc_key |= esc;
    bool match = !esc && ke - p - 2 == klen;
    for (int i = 0; match && i < klen; ++i) match = s(p + 1 + i) == key[i];
    p = jskip(s, jskip(s, ke, e) + 1, e);  // past ':'
    const int64_t ve = jval_end(s, p, e);
    if (ve < 0) return -3;
    if (match) found = p;
    p = jskip(s, ve, e);
    if (p >= e || s(p) != ',') break;
    p = jskip(s, p + 1, e);
  }
  return esc_key ? -3 : found;
}
// JSON number token [p, q): -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?; *integral = no frac/exp
template <class Src>
GF_DHD inline bool jnumber(const Src& s, int64_t p, int64_t q, bool* integral) {
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
GF_DHD inline int64_t days_from_civil(int64_t y, int64_t m) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5;
  return era * 146097 + yoe * 365 + yoe / 4 - yoe / 100 + doy - 719468;
}
// SimpleDateFormat("yyyy-MM-dd HH:mm:ss").parse (lenient: fields roll over) of the string content
// [p, q): 0 = parsed, 1 = ParseException (time stays 0), 2 = unsupported (before 1583)
template <class Src>
GF_DHD inline int jdate(const Src& s, int64_t p, int64_t q, int64_t tz_off_ms, int64_t* ms) {
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

// ---- strict validation (the slow path; Jackson's reader) -----------------------------
constexpr int kGeoMaxDepth = 256;  // deeper nesting: not restated (GF_CSV_UNSUPPORTED)
GF_DHD inline bool jtok_char(char c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '+' || c == '-' || c == '.';
}
// nesting depth of [p, e) above kGeoMaxDepth (brackets outside strings; any input)
template <class Src>
GF_DHD inline bool jtoo_deep(const Src& s, int64_t p, int64_t e) {
  int d = 0;
  bool str = false;
  for (int64_t i = p; i < e; ++i) {
    const char c = s(i);
    if (str) {
      if (c == '\\') ++i;
      else if (c == '"') str = false;
    } else if (c == '"') {
      str = true;
    } else if (c == '{' || c == '[') {
      if (++d > kGeoMaxDepth) return true;
    } else if (c == '}' || c == ']') {
      --d;
    }
  }
  return false;
}
GF_DHD inline bool jhex(char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
// the string at p: past its closing quote, -1 if invalid (unescaped control byte, bad escape,
// structurally bad UTF-8: a lead byte 110xxxxx / 1110xxxx / 11110xxx followed by 1 / 2 / 3
// bytes 10xxxxxx, as Jackson's UTF-8 reader checks)
template <class Src>
GF_DHD inline int64_t jstr_valid(const Src& s, int64_t p, int64_t e) {
  for (++p; p < e; ++p) {
    const uint8_t c = (uint8_t)s(p);
    if (c == '"') return p + 1;
    if (c < 0x20) return -1;
    if (c == '\\') {
      if (++p >= e) return -1;
      const char x = s(p);
      if (x == 'u') {
        if (p + 4 >= e) return -1;
        for (int k = 1; k <= 4; ++k)
          if (!jhex(s(p + k))) return -1;
        p += 4;
      } else if (!(x == '"' || x == '\\' || x == '/' || x == 'b' || x == 'f' || x == 'n' || x == 'r' || x == 't')) {
        return -1;
      }
    } else if (c >= 0x80) {
      const int n = (c & 0xE0) == 0xC0 ? 1 : (c & 0xF0) == 0xE0 ? 2 : (c & 0xF8) == 0xF0 ? 3 : -1;
      if (n < 0) return -1;
      for (int k = 0; k < n; ++k)
        if (++p >= e || ((uint8_t)s(p) & 0xC0) != 0x80) return -1;
    }
  }
  return -1;
}
// a token [p, q): 0 true / false / null or a JSON number Jackson hands json-simple readably,
// 1 invalid, 2 a number json-simple cannot read back (Infinity; an integer outside long)
template <class Src>
GF_DHD inline int jtok_valid(const Src& s, int64_t p, int64_t q, const uint64_t* T) {
  const int64_t n = q - p;
  const char c = s(p);
  if (c == 't' || c == 'f' || c == 'n') {
    const char* w = c == 't' ? "true" : c == 'f' ? "false" : "null";
    const int wl = c == 'f' ? 5 : 4;
    if (n != wl) return 1;
    for (int k = 0; k < wl; ++k)
      if (s(p + k) != w[k]) return 1;
    return 0;
  }
  bool integral;
  if (!jnumber(s, p, q, &integral)) return 1;
  if (integral) {
    int64_t v;
    return n < 19 || parse_java_long(s, Field{p, q}, &v) == kNumOk ? 0 : 2;
  }
  double v;
  if (parse_java_double(s, Field{p, q}, T, &v) != kNumOk) return 2;
  return (v == v && v - v != 0.0) ? 2 : 0;  // +-Infinity
}
// Jackson's strict parse of the line [p, e) (s(p) == '{'): kCsvOk, kCsvMissingField (malformed;
// it wins over the rest), kCsvUnsupported (nesting > kGeoMaxDepth, or a number json-simple
// cannot read back).
template <class Src>
GF_DHD GF_NOINLINE int jvalidate(Src s, int64_t p, int64_t e, const uint64_t* T) {
  if (jtoo_deep(s, p, e)) return kCsvUnsupported;
  enum { V, A0, K0, K, CO, AF };  // value, value or ']', key or '}', key, ':', after a value
  uint64_t obj[kGeoMaxDepth / 64] = {0, 0, 0, 0};  // bit: the container at that depth is an object
  int depth = 0, st = V;
  bool poison = false;
  int64_t i = p;
  while (true) {
    i = jskip(s, i, e);
    if (i >= e) break;
    const char c = s(i);
    if (st == V || st == A0) {
      if (c == '{' || c == '[') {
        const int d = depth++;
        const uint64_t bit = 1ull << (d & 63);
        obj[d >> 6] = c == '{' ? obj[d >> 6] | bit : obj[d >> 6] & ~bit;
        st = c == '{' ? K0 : A0;
        ++i;
      } else if (c == '"') {
        if ((i = jstr_valid(s, i, e)) < 0) return kCsvMissingField;
        st = AF;
      } else if (jtok_char(c)) {
        int64_t q = i;
        while (q < e && jtok_char(s(q))) ++q;
        const int t = jtok_valid(s, i, q, T);
        if (t == 1) return kCsvMissingField;
        poison |= t == 2;
        i = q;
        st = AF;
      } else if (st == A0 && c == ']') {
        --depth;
        ++i;
        st = AF;
      } else {
        return kCsvMissingField;
      }
    } else if (st == K0 || st == K) {
      if (c == '"') {
        if ((i = jstr_valid(s, i, e)) < 0) return kCsvMissingField;
        st = CO;
      } else if (st == K0 && c == '}') {
        --depth;
        ++i;
        st = AF;
      } else {
        return kCsvMissingField;
      }
    } else if (st == CO) {
      if (c != ':') return kCsvMissingField;
      ++i;
      st = V;
    } else {  // AF
      if (depth == 0) return kCsvMissingField;  // content after the record
      const bool isobj = (obj[(depth - 1) >> 6] >> ((depth - 1) & 63)) & 1;
      if (c == ',') {
        st = isobj ? K : V;
      } else if (c == (isobj ? '}' : ']')) {
        --depth;
        st = AF;
      } else {
        return kCsvMissingField;
      }
      ++i;
    }
  }
  if (st != AF || depth != 0) return kCsvMissingField;
  return poison ? kCsvUnsupported : kCsvOk;
}

// ---- the map's evaluation over located members ------------------------------------------
// The members read, as the first byte of their value (-1 absent): V, V.type, V.coordinates,
// V.geometry, geometry.type, geometry.coordinates, V.properties, properties[time],
// properties[objID]; esc*: that object has a member name written with an escape (only the slow
// path sees escapes) -- unsupported once the map looks a member up in it.
struct GeoPos {
  int64_t V, tV, cV, gV, tG, cG, prV, tsP, qP;
  bool escV, escG, escP;
};
enum { kTyNone, kTyPoint, kTyOtherGeom, kTyFeature, kTyFeatureColl, kTyEscaped };
// a "type" member's value: JTS's geometry types ("Point" restated, the rest not), GeoJSON's
// Feature / FeatureCollection, anything else (absent, not a String, unknown) -> kTyNone
template <class Src>
GF_DHD inline int geo_type(const Src& s, int64_t t, int64_t e) {
  if (t < 0 || s(t) != '"') return kTyNone;
  bool esc = false;
  const int64_t te = jstr_end(s, t, e, &esc);
  if (esc) return kTyEscaped;
  const int n = (int)(te - t - 2);
  auto is = [&](const char* w, int wl) {
    if (n != wl) return false;
    for (int k = 0; k < wl; ++k)
      if (s(t + 1 + k) != w[k]) return false;
    return true;
  };
  if (is("Point", 5)) return kTyPoint;
  if (is("LineString", 10) || is("Polygon", 7) || is("MultiPoint", 10) || is("MultiLineString", 15) ||
      is("MultiPolygon", 12) || is("GeometryCollection", 18))
    return kTyOtherGeom;
  if (is("Feature", 7)) return kTyFeature;
  if (is("FeatureCollection", 17)) return kTyFeatureColl;
  return kTyNone;
}
// GeoJsonReader.createPoint: coordinates = a list whose ordinates 0, 1 (and 2, if present) are
// Numbers (ordinates.get(i).doubleValue(); anything else throws ClassCastException ->
// GF_CSV_NUMBER_FORMAT; not a list -> GF_CSV_MISSING_FIELD); fewer than two ordinates or a
// non-number third -> GF_CSV_UNSUPPORTED.  An integral literal is Jackson's IntNode / LongNode:
// (double) of the long, so "-0" is +0.0 (the correctly rounded decimal otherwise).
template <class Src>
GF_DHD inline int point_coords(const Src& s, int64_t c, int64_t e, const uint64_t* T, double* x, double* y) {
  if (c < 0 || s(c) != '[') return kCsvMissingField;
  int64_t i = jskip(s, c + 1, e);
  double x0 = 0.0, y0 = 0.0;
  int n = 0;
  while (i < e && s(i) != ']') {
    const int64_t ve = jval_end(s, i, e);
    if (n < 3) {
      const char c0 = s(i);
      if (c0 == '-' || (c0 >= '0' && c0 <= '9')) {
        if (n < 2) {
          bool integral = false;
          jnumber(s, i, ve, &integral);
          double v;
          const int st = parse_java_double(s, Field{i, ve}, T, &v);
          if (st) return st == kNumUnsupported ? kCsvUnsupported : kCsvNumberFormat;
          v = integral && v == 0.0 ? 0.0 : v;
          if (n == 0) x0 = v;
          else y0 = v;
        }
      } else {
        return n < 2 ? kCsvNumberFormat : kCsvUnsupported;
      }
    }
    ++n;
    i = jskip(s, ve, e);
    if (i < e && s(i) == ',') i = jskip(s, i + 1, e);
  }
  if (n < 2) return kCsvUnsupported;
  *x = x0;
  *y = y0;
  return kCsvOk;
}

// what the property lookups need of CsvArgs (passed by value: a reference to the kernel's
// argument block in an outlined call would copy the whole block to scratch, per lane)
struct GeoProps {
  const char* kts;   // property names (the block's LDS copies)
  const char* kobj;
  int32_t len_ts, len_obj, date_fmt;
  int64_t tz_off_ms;
  const uint64_t* pow5;  // the 5^q table of Double.valueOf (device or host copy of GF_POW5_TABLE)
};

// the time and objID properties: t, q = their values' first bytes (-1 absent)
template <class Src>
GF_DHD inline int geo_props(const GeoProps& a, const Src& s, int64_t e, int64_t t, int64_t q, LineOut* o) {
  if (a.len_ts >= 0 && t >= 0) {
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
  if (a.len_obj >= 0 && q >= 0) {  // nodeOId.toString() with every '"' removed
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
      jnumber(s, q, qe, &integral);
      if (!integral) return kCsvUnsupported;  // Double.toString rendering: not restated
      if (qe - q == 2 && c0 == '-' && s(q + 1) == '0') {  // IntNode(0).toString() == "0"
        o->obj = 0;
        return kCsvOk;
      }
    }  // true / false / null print as themselves
    o->dict = !canonical_objid_key(s, f, &o->obj);
    o->f_obj = f;
    if (o->dict && f.e - f.b > (int64_t)kDictLenMask) return kCsvUnsupported;
  }
  return kCsvOk;
}

// steps 2-3 of the map over located members (both paths), in the map's order.  The walk calls it
// outlined (geo_eval: inlined into the walk it trips an AMDGPU backend bug -- an illegal
// v_cmp_ne_u32_e32 against src_shared_base); the locator's path inlines the body (geo_eval_body):
// an outlined call there cost every line a stack frame in scratch -- GeoPos, LineOut and the
// saved registers, ~270 B of scratch writes per line (r04 PMC: 276 MB written per 1M lines).
template <class Src>
GF_DHD inline int geo_eval_body(const GeoProps& a, const Src& s, int64_t e, const GeoPos& g, LineOut* o) {
  if (g.V < 0 || s(g.V) != '{') return kCsvMissingField;  // value.toString() / .get("geometry"): NPE
  if (g.escV) return kCsvUnsupported;
  o->ts = 0;
  o->obj = GF_OBJID_NULL;
  o->dict = false;
  bool have = false;
  const int tv = geo_type(s, g.tV, e);
  if (tv == kTyOtherGeom || tv == kTyFeatureColl || tv == kTyEscaped) return kCsvUnsupported;
  if (tv == kTyPoint) {  // readGeoJSON(value.toString())
    const int st = point_coords(s, g.cV, e, a.pow5, &o->x, &o->y);
    if (st == kCsvUnsupported) return st;
    have = st == kCsvOk;
  }
  if (!have) {  // the catch branch: readGeoJSON(value.get("geometry").toString())
    if (g.gV < 0 || s(g.gV) != '{') return kCsvMissingField;
    if (g.escG) return kCsvUnsupported;
    const int tg = geo_type(s, g.tG, e);
    if (tg == kTyNone) return kCsvMissingField;
    if (tg != kTyPoint) return kCsvUnsupported;
    const int st = point_coords(s, g.cG, e, a.pow5, &o->x, &o->y);
    if (st) return st;
  }
  if (g.prV < 0 || s(g.prV) != '{') return kCsvOk;
  if (g.escP && (a.len_ts >= 0 || a.len_obj >= 0)) return kCsvUnsupported;
  return geo_props(a, s, e, g.tsP, g.qP, o);
}
template <class Src>
GF_DHD GF_NOINLINE int geo_eval(const GeoProps& a, const Src& s, int64_t e, const GeoPos& g, LineOut* o) {
  return geo_eval_body(a, s, e, g, o);
}

// The slow path: Jackson's strict parse, then member-by-member lookup (jfind) -- exact on any
// line (escapes, deep nesting, malformed ones).  p: the line's first non-blank byte, a '{'.
template <class Src>
GF_DHD GF_NOINLINE int eval_geojson_walk(GeoProps a, Src s, int64_t p, int64_t e, int vlines, LineOut* o) {
  const int vs = jvalidate(s, p, e, a.pow5);
  if (vs) return vs;
  GeoPos g{-1, -1, -1, -1, -1, -1, -1, -1, -1, false, false, false};
  // member `k` of the object at obj (when it is one); false: obj has an escaped member name
  auto find = [&](int64_t obj, const char* k, int kl, int64_t* out) {
    if (obj < 0 || s(obj) != '{') return true;
    const int64_t f = jfind(s, obj, e, k, kl);
    *out = f < 0 ? -1 : f;
    return f != -3;
  };
  if (vlines) g.V = p;
  else if (!find(p, "value", 5, &g.V)) return kCsvUnsupported;
  g.escV = !find(g.V, "type", 4, &g.tV);
  find(g.V, "coordinates", 11, &g.cV);
  find(g.V, "geometry", 8, &g.gV);
  find(g.V, "properties", 10, &g.prV);
  g.escG = !find(g.gV, "type", 4, &g.tG);
  find(g.gV, "coordinates", 11, &g.cG);
  g.escP = !find(g.prV, a.kts, a.len_ts >= 0 ? a.len_ts : 0, &g.tsP);
  find(g.prV, a.kobj, a.len_obj >= 0 ? a.len_obj : 0, &g.qP);
  return geo_eval(a, s, e, g, o);
}

// ---------------------------------------------------------------------------------------
// One-pass member location (the common case).  The walk re-scans an object once per member it
// looks up, with nested data-dependent loops per lane; with 64 lines per wave in different
// places of that loop nest the exec-mask bookkeeping dominated.  Here each lane runs one
// automaton over its line, byte by byte: Jackson's strict syntax (below) plus a small stack of
// container roles (the record, its "value" object V, V's geometry and properties), noting the
// position of the LAST key of each member the map looks up.  On a line that passes -- strictly
// valid, no backslash, nesting <= 63, every token a literal or a number json-simple reads back
// (lines with a number of >= 19 characters or a 3-digit exponent are checked by the walk) --
// every jfind of the walk returns exactly that last member, so the results are the walk's.
// Any other line takes the walk (which also decides whether it is malformed).
//
// The per-byte step: one 8-B LDS entry per byte value holds the (next state, action) pair of all
// 9 syntax states (7 bits each); a second holds the next state of a 16-state token / string
// automaton for each of its states (4 bits each): the JSON number grammar, literals, and the
// structure of UTF-8 sequences inside strings.  Neither lookup waits on a state.  Only the
// actions (brackets, commas, key quotes) and token ends do more, and the key comparison runs
// only for keys of a looked-up length in a looked-up container.  Stale notes need no reset: a
// note is current when it lies after the note of its container's key.
// ---------------------------------------------------------------------------------------
enum : uint8_t { JS_VAL, JS_ARR0, JS_OBJ0, JS_KEY, JS_COLON, JS_AFT, JS_VSTR, JS_KSTR, JS_TOK, JS_N, JS_ERR = 9 };
enum : uint8_t { JC_WS, JC_LBRACE, JC_RBRACE, JC_LBRACK, JC_RBRACK, JC_QUOTE, JC_COMMA, JC_COLON, JC_BSL, JC_TOK,
                 JC_OTHER, JC_WSC, JC_CTRL, JC_HIGH };
enum : uint8_t { JA_NONE, JA_PUSH_OBJ, JA_PUSH_ARR, JA_POP_OBJ, JA_POP_ARR, JA_COMMA, JA_KEY_BEGIN, JA_KEY_END };
enum : int { JR_NONE, JR_TOP, JR_VAL, JR_GEO, JR_PROP };  // container roles
enum : int { JK_NONE, JK_VALUE, JK_GEO, JK_PROP };        // member kinds (a child container's role)
// token / string automaton states (4 bits): IDLE outside; S0 / NEED1..3 inside a string (UTF-8
// continuation bytes pending); the number grammar; LIT (letters: checked at the token's end)
enum : uint8_t { TS_IDLE, TS_S0, TS_NEED1, TS_NEED2, TS_NEED3, TS_MINUS, TS_ZERO, TS_INT, TS_DOT, TS_FRAC, TS_E,
                 TS_ESIGN, TS_EXP1, TS_EXP2, TS_LIT, TS_ERR };
constexpr uint32_t kTsAccept = (1u << TS_ZERO) | (1u << TS_INT) | (1u << TS_FRAC) | (1u << TS_EXP1) | (1u << TS_EXP2);
constexpr int kGeoKeys = 7;  // value, geometry, properties, coordinates, time property, objID property, type

GF_DHD inline uint8_t jclass(int c) {
  switch (c) {
    case ' ': return JC_WS;
    case '\t': case '\n': case '\r': return JC_WSC;
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
  if (c < 0x20) return JC_CTRL;
  if (c >= 0x80) return JC_HIGH;
  if ((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '+' || c == '-' || c == '.')
    return JC_TOK;
  return JC_OTHER;
}
// next state | action << 4.  After the top object closes the state is JS_AFT at depth 0, where
// a comma or a closer is an error (checked with the depth, geo_locate).  A backslash, a control
// byte in a string or any error -> JS_ERR (the line takes the walk).
GF_DHD inline uint8_t jtrans(int st, int cl) {
  auto E = [](int n, int act) { return (uint8_t)(n | act << 4); };
  if (st == JS_VSTR || st == JS_KSTR) {
    if (cl == JC_QUOTE) return st == JS_VSTR ? E(JS_AFT, 0) : E(JS_COLON, JA_KEY_END);
    if (cl == JC_BSL || cl == JC_WSC || cl == JC_CTRL) return E(JS_ERR, 0);
    return E(st, 0);
  }
  if (st == JS_TOK) {
    if (cl == JC_TOK) return E(JS_TOK, 0);
    st = JS_AFT;  // the token ends here: the byte is read as after a value
  }
  if (cl == JC_WS || cl == JC_WSC) return E(st, 0);
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
// next token / string state from state t on byte b (only consulted inside a token or a string)
GF_DHD inline uint8_t jtok_trans(int t, int b) {
  const bool dig = b >= '0' && b <= '9', e = b == 'e' || b == 'E';
  const bool let = (b >= 'a' && b <= 'z') || (b >= 'A' && b <= 'Z');
  switch (t) {
    case TS_IDLE:  // a token's first byte, or a string's opening quote
      if (b == '"') return TS_S0;
      if (b == '-') return TS_MINUS;
      if (b == '0') return TS_ZERO;
      if (dig) return TS_INT;
      if (b == 't' || b == 'f' || b == 'n') return TS_LIT;
      return TS_ERR;
    case TS_S0:
      if (b < 0x80) return TS_S0;
      if ((b & 0xE0) == 0xC0) return TS_NEED1;
      if ((b & 0xF0) == 0xE0) return TS_NEED2;
      if ((b & 0xF8) == 0xF0) return TS_NEED3;
      return TS_ERR;
    case TS_NEED1: return (b & 0xC0) == 0x80 ? TS_S0 : TS_ERR;
    case TS_NEED2: return (b & 0xC0) == 0x80 ? TS_NEED1 : TS_ERR;
    case TS_NEED3: return (b & 0xC0) == 0x80 ? TS_NEED2 : TS_ERR;
    case TS_MINUS: return b == '0' ? TS_ZERO : dig ? TS_INT : TS_ERR;
    case TS_ZERO: return b == '.' ? TS_DOT : e ? TS_E : TS_ERR;
    case TS_INT: return dig ? TS_INT : b == '.' ? TS_DOT : e ? TS_E : TS_ERR;
    case TS_DOT: return dig ? TS_FRAC : TS_ERR;
    case TS_FRAC: return dig ? TS_FRAC : e ? TS_E : TS_ERR;
    case TS_E: return dig ? TS_EXP1 : (b == '+' || b == '-') ? TS_ESIGN : TS_ERR;
    case TS_ESIGN: return dig ? TS_EXP1 : TS_ERR;
    case TS_EXP1: return dig ? TS_EXP2 : TS_ERR;
    case TS_EXP2: return TS_ERR;  // a 3-digit exponent: the walk checks it for overflow
    case TS_LIT: return let ? TS_LIT : TS_ERR;
    default: return TS_ERR;
  }
}

// LDS tables of a block: per byte value the 9 syntax states' entries and the 16 token states'
// next states; the looked-up member names; the time / objID property names packed (geo_pack16)
struct K16 {  // up to 16 bytes, first byte most significant: (hi, lo) after shifting each byte in
  uint64_t hi, lo;
};
GF_DHD constexpr K16 geo_pack16(const char* s, int n) {
  uint64_t hi = 0, lo = 0;
  for (int i = 0; i < n; ++i) {
    hi = (hi << 8) | (lo >> 56);
    lo = (lo << 8) | (uint8_t)s[i];
  }
  return K16{hi, lo};
}
struct GeoTabs {  // (in LDS on the device)
  GF_LDS_PTR(uint64_t) tab;   // [256]: entry of state s at bits 7s..7s+6
  GF_LDS_PTR(uint64_t) ttab;  // [256]: next token state of state t at bits 4t..4t+3
  GF_LDS_PTR(char) keys;      // kGeoKeys x kGeoPropMax
  int32_t klen[kGeoKeys];
  K16 pts, pobj;              // the time / objID property names when <= 16 bytes (klen[4], klen[5])
};

template <class Src>
GF_DHD inline bool jkey_eq(const Src& s, int64_t ks, int len, const GeoTabs& gt, int k) {
  if (gt.klen[k] != len) return false;
  bool eq = true;
  for (int i = 0; eq && i < len; ++i) eq = s(ks + i) == gt.keys[k * kGeoPropMax + i];
  return eq;
}

// the value of the member whose key's closing quote is at k (valid JSON: '"' ws ':' ws value)
template <class Src>
GF_DHD inline int64_t jmember_value(const Src& s, int64_t k, int64_t e) {
  return jskip(s, jskip(s, k + 1, e) + 1, e);
}

// The automaton's state over one line.  n[]: closing-quote positions (from p) of the last keys
// noted: the record's "value"; in V: type, coordinates, geometry, properties; in V.geometry:
// type, coordinates; in V.properties: the time and objID properties (-1: none).
enum { GN_V, GN_TV, GN_CV, GN_GV, GN_PRV, GN_TG, GN_CG, GN_TP, GN_QP, kGeoNotes };
struct GeoLoc {
  int st, depth, pend;
  uint32_t ts;
  bool bad;
  uint64_t kinds;  // bit d: the container at depth d is an object
  uint32_t roles;  // 4 bits per depth 1..7
  int32_t ks, tb;
  uint64_t khi, klo;  // the current key's last 16 bytes
  int32_t n[kGeoNotes];
};
GF_DHD inline void geo_loc_init(GeoLoc& L) {
  L.st = JS_VAL;
  L.depth = 0;
  L.pend = JK_NONE;
  L.ts = TS_IDLE;
  L.bad = false;
  L.kinds = 0;
  L.roles = 0;
  L.ks = 0;
  L.tb = 0;
  L.khi = 0;
  L.klo = 0;
  for (int k = 0; k < kGeoNotes; ++k) L.n[k] = -1;
}
// One byte step: `byte` at offset i of the line [p, e) (a blank for the word's bytes outside it).
// top_role: JR_VAL for value lines, JR_TOP for Kafka records.
GF_DHD inline void geo_step(GeoLoc& L, uint32_t byte, int32_t i, const LBytes& s, int64_t p, const GeoTabs& gt,
                            int top_role) {
  constexpr K16 kValue = geo_pack16("value", 5), kGeom = geo_pack16("geometry", 8);
  constexpr K16 kProps = geo_pack16("properties", 10), kCoord = geo_pack16("coordinates", 11);
  constexpr K16 kType = geo_pack16("type", 4);
  const int32_t lts = gt.klen[4], lobj = gt.klen[5];
  const int st = L.st;
  const uint32_t ts = L.ts;
  const uint32_t ent = (uint32_t)(gt.tab[byte] >> (7 * st)) & 0x7Fu;
  const uint32_t nts = (uint32_t)(gt.ttab[byte] >> (4 * ts)) & 15u;
  int nst = (int)(ent & 15u);
  const int act = (int)(ent >> 4);
  const bool in_tok = nst == JS_TOK, in_str = nst == JS_VSTR || nst == JS_KSTR;
  // a token ended before this byte: its state decides (a literal's letters: the rare branch)
  const bool tok_end = st == JS_TOK && !in_tok;
  const bool lit = tok_end && ts == TS_LIT;
  bool bad = L.bad;
  bad |= tok_end && !lit && !(((kTsAccept >> ts) & 1u) && i - L.tb < 19);
  if (lit) {  // true / false / null
    const int n = i - L.tb;
    const char c0 = s(p + L.tb);
    bool ok = n == (c0 == 'f' ? 5 : 4);
    const char* wd = c0 == 't' ? "true" : c0 == 'f' ? "false" : "null";
    for (int q = 1; ok && q < n; ++q) ok = s(p + L.tb + q) == wd[q];
    bad |= !ok;
  }
  L.tb = in_tok && st != JS_TOK ? i : L.tb;
  // a string's bytes (its closing quote included) must leave the UTF-8 automaton accepting
  bad |= (in_str || st == JS_VSTR || st == JS_KSTR) && nts == TS_ERR;
  L.ts = in_tok || in_str ? nts : TS_IDLE;
  // the key's bytes (between its quotes) into the accumulator; its opening quote resets it
  const bool in_key = st == JS_KSTR && nst == JS_KSTR;
  const uint64_t khi = L.khi, klo = L.klo;
  const uint64_t nhi = (khi << 8) | (klo >> 56), nlo = (klo << 8) | byte;
  const bool kb = act == JA_KEY_BEGIN;
  L.khi = kb ? 0ull : in_key ? nhi : khi;
  L.klo = kb ? 0ull : in_key ? nlo : klo;
  L.ks = kb ? i + 1 : L.ks;
  // containers: the role of the one we are in, a push's child role, the kind bits
  const int depth = L.depth;
  const int role = (unsigned)depth <= 7u ? (int)(L.roles >> (4 * depth)) & 15 : JR_NONE;
  const bool push = act == JA_PUSH_OBJ || act == JA_PUSH_ARR, pop = act == JA_POP_OBJ || act == JA_POP_ARR;
  int child = depth == 0 ? top_role
            : role == JR_TOP ? (int)(0x0020u >> (4 * L.pend)) & 15   // value -> V
            : role == JR_VAL ? (int)(0x4300u >> (4 * L.pend)) & 15   // geometry, properties
            : JR_NONE;
  child = act == JA_PUSH_ARR ? JR_NONE : child;
  const int nd = depth + 1;
  const uint64_t nbit = 1ull << (nd & 63);
  L.kinds = push ? (act == JA_PUSH_OBJ ? L.kinds | nbit : L.kinds & ~nbit) : L.kinds;
  const uint32_t rsh = 4u * (uint32_t)(nd & 7);
  L.roles = push && nd <= 7 ? (L.roles & ~(15u << rsh)) | ((uint32_t)child << rsh) : L.roles;
  const bool kobj = (L.kinds >> (depth & 63)) & 1;  // (a pop or comma does not change kinds)
  bad |= push && nd > 63;
  bad |= pop && (depth <= 0 || kobj != (act == JA_POP_OBJ));
  bad |= act == JA_COMMA && depth <= 0;
  nst = act == JA_COMMA ? (kobj ? JS_KEY : JS_VAL) : nst;
  L.depth = depth + (int)push - (int)pop;
  // a key's closing quote: note a looked-up member of a looked-up container
  const bool kend = act == JA_KEY_END;
  const int len = i - L.ks;
  const uint64_t chi = L.khi, clo = L.klo;
  // (a key of <= 8 bytes leaves khi 0: the short names compare klo only)
  const bool e_type = len == 4 && clo == kType.lo, e_value = len == 5 && clo == kValue.lo;
  const bool e_geom = len == 8 && clo == kGeom.lo;
  const bool e_props = len == 10 && clo == kProps.lo && chi == kProps.hi;
  const bool e_coord = len == 11 && clo == kCoord.lo && chi == kCoord.hi;
  const bool top = kend && role == JR_TOP, val = kend && role == JR_VAL;
  const bool geo = kend && role == JR_GEO, prop = kend && role == JR_PROP;
  const bool m_value = top && e_value;
  const bool v_type = val && e_type, v_coord = val && e_coord;
  const bool v_geom = val && e_geom, v_props = val && e_props;
  bool p_ts = prop && len == lts && lts <= 16 && clo == gt.pts.lo && chi == gt.pts.hi;
  bool p_obj = prop && len == lobj && lobj <= 16 && clo == gt.pobj.lo && chi == gt.pobj.hi;
  if ((lts > 16 || lobj > 16) && prop && len > 16) {  // (rare: a property name longer than 16 bytes)
    p_ts = jkey_eq(s, p + L.ks, len, gt, 4);
    p_obj = jkey_eq(s, p + L.ks, len, gt, 5);
  }
  L.pend = kend ? (m_value ? JK_VALUE : v_geom ? JK_GEO : v_props ? JK_PROP : JK_NONE) : L.pend;
  L.n[GN_V] = m_value ? i : L.n[GN_V];
  L.n[GN_TV] = v_type ? i : L.n[GN_TV];
  L.n[GN_CV] = v_coord ? i : L.n[GN_CV];
  L.n[GN_GV] = v_geom ? i : L.n[GN_GV];
  L.n[GN_PRV] = v_props ? i : L.n[GN_PRV];
  L.n[GN_TG] = geo && e_type ? i : L.n[GN_TG];
  L.n[GN_CG] = geo && e_coord ? i : L.n[GN_CG];
  L.n[GN_TP] = p_ts ? i : L.n[GN_TP];
  L.n[GN_QP] = p_obj ? i : L.n[GN_QP];
  bad |= nst == JS_ERR;
  L.bad = bad;
  L.st = nst == JS_ERR ? JS_AFT : nst;
}
// the line passed the automaton (valid, nothing the walk must check)
GF_DHD inline bool geo_loc_ok(const GeoLoc& L) { return !L.bad && L.st == JS_AFT && L.depth == 0; }
// The members the map reads from a passing line's notes n[] (positions from p; -1 none).
template <class Src>
GF_DHD inline void geo_notes_pos(const Src& s, int64_t p, int64_t e, int vlines, const int32_t* n, GeoPos* g) {
  auto val = [&](int32_t k) { return k < 0 ? (int64_t)-1 : jmember_value(s, p + k, e); };
  // notes inside an earlier "value" object, geometry or properties member are stale
  const int32_t vb = vlines ? -1 : n[GN_V];
  g->V = vlines ? p : val(n[GN_V]);
  g->tV = val(n[GN_TV] > vb ? n[GN_TV] : -1);
  g->cV = val(n[GN_CV] > vb ? n[GN_CV] : -1);
  const int32_t gv = n[GN_GV] > vb ? n[GN_GV] : -1, pv = n[GN_PRV] > vb ? n[GN_PRV] : -1;
  g->gV = val(gv);
  g->tG = val(gv >= 0 && n[GN_TG] > gv ? n[GN_TG] : -1);
  g->cG = val(gv >= 0 && n[GN_CG] > gv ? n[GN_CG] : -1);
  g->prV = val(pv);
  g->tsP = val(pv >= 0 && n[GN_TP] > pv ? n[GN_TP] : -1);
  g->qP = val(pv >= 0 && n[GN_QP] > pv ? n[GN_QP] : -1);
  g->escV = g->escG = g->escP = false;
}
// One word (4 LDS bytes at offset w from the staging base) of the line whose LDS offsets are
// [o0, o1).  r05: the byte step is BRANCH-FREE (see geo_locate)
#ifndef GF_GEO_UNROLL
#define GF_GEO_UNROLL 2  // byte steps of a word unrolled (r05 A/B, parse us per 1M lines, 256-line blocks: 2 -> 3042-3048,
                         // 4 -> 3082-3086; 192-line blocks (tools/gpu_r05_geo5.sh): 1 -> 2967-2977, 2 -> 2894-2903, 4 -> 2862-2864)
#endif
GF_DHD inline void geo_word(GeoLoc& L, int32_t w, int32_t o0, int32_t o1, const LBytes& s, int64_t p, const GeoTabs& gt,
                            int top_role) {
  const uint32_t word = *reinterpret_cast<const uint32_t*>(s.p + w);
#pragma unroll GF_GEO_UNROLL
  for (int k = 0; k < 4; ++k) {
    const int32_t i = w + k - o0;  // offset in the line
    const uint32_t byte = i < 0 || w + k >= o1 ? (uint32_t)' ' : (word >> (8 * k)) & 0xFFu;
    geo_step(L, byte, i, s, p, gt, top_role);
  }
}

// The automaton over the line [p, e) (s(p) == '{'), staged in LDS (lds + (pos - base)).  Returns
// false when the line must take the walk; otherwise *g = the members the map reads.
// r05: the byte step is BRANCH-FREE.  64 lanes walk 64 different lines, so some lane meets an
// action (a bracket, a comma, a key's quotes, a token's end) at nearly every step: as branches,
// every step paid every case's exec-mask juggling (r04 PMC: ~210 vector + ~300 scalar
// instructions per lane-byte).  Now each step computes every case with selects -- pushes and pops
// update depth / kinds / roles arithmetically, the key's bytes are shifted into a 16-byte
// accumulator while it is read, and its closing quote compares (length, accumulator) with the
// looked-up names' packed constants.  Only literals (true / false / null) at a token's end and
// property names longer than 16 bytes branch (rare).
GF_DHD inline bool geo_locate_notes(const LBytes& s, int64_t p, int64_t e, const GeoTabs& gt, int vlines,
                                    int32_t* n) {
  if (e - p >= INT32_MAX) return false;
  GeoLoc L;
  geo_loc_init(L);
  const int top_role = vlines ? JR_VAL : JR_TOP;
  const int32_t o0 = (int32_t)(p - s.base), o1 = (int32_t)(e - s.base);  // the line's LDS offsets
  for (int32_t w = o0 & ~3; w < o1 && !L.bad; w += 4) geo_word(L, w, o0, o1, s, p, gt, top_role);
  if (!geo_loc_ok(L)) return false;
  for (int k = 0; k < kGeoNotes; ++k) n[k] = L.n[k];
  return true;
}
GF_DHD inline bool geo_locate(const LBytes& s, int64_t p, int64_t e, const GeoTabs& gt, int vlines,
                                           GeoPos* g) {
  int32_t n[kGeoNotes];
  if (!geo_locate_notes(s, p, e, gt, vlines, n)) return false;
  geo_notes_pos(s, p, e, vlines, n, g);
  return true;
}


// One line [p, e) (s(p) == '{', trailing '\r' removed): the one-pass locator when `fast` (an
// LBytes source) and the line passes it, else the walk.
template <class Src>
GF_DHD inline int geojson_line(const GeoTabs& gt, const GeoProps& gp, const Src& s, int64_t p, int64_t e, int vlines,
                               LineOut* o) {
  LineOut w{0, 0, 0.0, 0.0, false, {0, 0}};  // (the outlined walk's own: see below)
  const int st = eval_geojson_walk(gp, s, p, e, vlines, &w);
  *o = w;
  return st;
}
GF_DHD inline int geojson_line(const GeoTabs& gt, const GeoProps& gp, const LBytes& s, int64_t p, int64_t e,
                               int vlines, bool fast, LineOut* o) {
  if (fast) {
    GeoPos g;
    if (geo_locate(s, p, e, gt, vlines, &g)) return geo_eval_body(gp, s, e, g, o);
  }
  // the walk is outlined: it gets its own LineOut, so that the caller's (whose address would
  // otherwise escape into the call) stays in registers on the locator's path
  LineOut w{0, 0, 0.0, 0.0, false, {0, 0}};
  const int st = eval_geojson_walk(gp, s, p, e, vlines, &w);
  *o = w;
  return st;
}

// ---------------------------------------------------------------------------------------
// Byte classes of the wave-per-line scan (k_csv.hip geo_wave_scan): flags, and in bits 24..27 the
// element a byte starts outside strings (a quote: a string, read as a value until its key-ness is
// known; a token byte: a token, when the byte before it is not one).
// ---------------------------------------------------------------------------------------
enum : uint32_t {
  WB_Q = 1u << 0,      // '"'
  WB_BAD = 1u << 1,    // a backslash, a control byte other than \t \n \r, a byte >= 0x80: the walk decides
  WB_WSC = 1u << 2,    // \t \n \r: whitespace outside strings, an error inside
  WB_OTH = 1u << 3,    // no JSON token holds it (JC_OTHER): an error outside strings
  WB_OB = 1u << 4, WB_CB = 1u << 5, WB_OA = 1u << 6, WB_CA = 1u << 7, WB_CO = 1u << 8, WB_CM = 1u << 9,
  WB_TOK = 1u << 10,   // [0-9a-zA-Z+-.]
  WB_DOT = 1u << 11, WB_E = 1u << 12
};
enum : uint32_t { WT_NONE, WT_OB, WT_OA, WT_CB, WT_CA, WT_CO, WT_CM, WT_SK, WT_SV, WT_TK };
constexpr uint32_t kWtValueEnd = (1u << WT_CB) | (1u << WT_CA) | (1u << WT_SV) | (1u << WT_TK);
GF_DHD inline uint32_t wave_class(int b) {
  const int cl = jclass(b);
  uint32_t f = 0, t = WT_NONE;
  switch (cl) {
    case JC_QUOTE: f = WB_Q; t = WT_SV; break;
    case JC_BSL: case JC_CTRL: case JC_HIGH: f = WB_BAD; break;
    case JC_WSC: f = WB_WSC; break;
    case JC_OTHER: f = WB_OTH; break;
    case JC_LBRACE: f = WB_OB; t = WT_OB; break;
    case JC_RBRACE: f = WB_CB; t = WT_CB; break;
    case JC_LBRACK: f = WB_OA; t = WT_OA; break;
    case JC_RBRACK: f = WB_CA; t = WT_CA; break;
    case JC_COLON: f = WB_CO; t = WT_CO; break;
    case JC_COMMA: f = WB_CM; t = WT_CM; break;
    case JC_TOK:
      f = WB_TOK | (b == '.' ? WB_DOT : 0u) | (b == 'e' || b == 'E' ? WB_E : 0u);
      t = WT_TK;
      break;
    default: break;  // JC_WS
  }
  return f | t << 24;
}

// one entry of the locator's two per-byte tables (geo_tabs_fill)
GF_DHD inline void geo_tab_entry(int b, uint64_t* tab, uint64_t* ttab) {
  const int cl = jclass(b);
  uint64_t t = 0, u = 0;
  for (int st = 0; st < JS_N; ++st) t |= (uint64_t)jtrans(st, cl) << (7 * st);
  for (int ts = 0; ts < 16; ++ts) u |= (uint64_t)jtok_trans(ts, b) << (4 * ts);
  *tab = t;
  *ttab = u;
}

}  // namespace gf
