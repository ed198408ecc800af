// k_csv.hip -- GPU CSV/TSV ingest: Deserialization.CSVTSVToTSpatial.map
// (Deserialization.java:291-325) for a whole chunk of text lines at once, fused with
// HelperClass.assignGridCellID (Point.java:98).  Two kernels over HBM-resident text:
//
//   csv_nlindex the newline positions, in order, and their count: one read of the text (16-B
//               loads, SWAR byte compare, a decoupled look-back across 64 KB segments)
//   csv_parse   one lane per line: quotes dropped, fields split on the delimiter with the
//               surrounding whitespace (the reference's split("\\s*" + delim + "\\s*")),
//               the objID String as its key (canonical decimals directly, the rest queued for
//               the dictionary, k_objid.hip), Long.valueOf(time), Double.valueOf(x, y) correctly
//               rounded on the device (gf_decimal.hpp), cell (cx, cy), SoA stores.
#define GF_TU_NAME k_csv_hip
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include "gf_geojson.hpp"
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

__device__ __forceinline__ bool java_s(char c) {  // regex \s: [ \t\n\x0B\f\r]
  return c == ' ' || c == '\t' || c == '\n' || c == '\x0B' || c == '\f' || c == '\r';
}


// Field ranges of the wanted columns of line [b, e).  Returns the number of fields.
// A delimiter that is not whitespace (r05): the scan is branch-free -- every delimiter byte
// selects the wanted fields' raw ranges and advances the field count -- and only the (at most 4)
// wanted fields are trimmed afterwards, as close() below trims every field as it goes (64 lanes
// on 64 lines meet delimiters at different bytes: as a branch, close() ran at most steps).
template <class Src>
__device__ int split_line(const Src& s, int64_t b, int64_t e, char d, const int32_t* want, Field* got) {
  const bool wsd = java_s(d);
  if (!wsd) {
    int32_t wk[4];
    int64_t gb[4], ge[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      wk[k] = want[k];
      gb[k] = ge[k] = -1;
    }
    int32_t field = 0;
    int64_t fs = b;
    for (int64_t i = b; i < e; ++i) {
      const bool isd = s(i) == d;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool c = isd && wk[k] == field;
        gb[k] = c ? fs : gb[k];
        ge[k] = c ? i : ge[k];
      }
      field += (int32_t)isd;
      fs = isd ? i + 1 : fs;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // the last field [fs, e); then the wanted fields trimmed
      if (wk[k] == field) {
        gb[k] = fs;
        ge[k] = e;
      }
      if (gb[k] < 0) continue;
      int64_t x0 = gb[k], x1 = ge[k];
      if (wk[k] > 0)  // whitespace (and quotes) next to a delimiter belong to the delimiter
        while (x0 < x1 && (java_s(s(x0)) || s(x0) == '"')) ++x0;
      if (wk[k] != field)
        while (x1 > x0 && (java_s(s(x1 - 1)) || s(x1 - 1) == '"')) --x1;
      got[k] = Field{x0, x1};
    }
    return field + 1;
  }
  // a whitespace delimiter: a run of whitespace (quotes are transparent) holding it is one separator
  int field = 0;
  int64_t fs = b;
  auto close = [&](int64_t fe) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (want[k] == field) got[k] = Field{fs, fe};
    ++field;
  };
  {
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
          close(i);
          fs = j;
        }
        i = j;
      } else {
        ++i;
      }
    }
  }
  close(e);
  return field;
}

// One line, in the reference's order: strOId = get(objid) (any String: canonical decimals become
// their key here, the rest is queued for the dictionary), time = Long.valueOf(get(time)),
// x = Double.valueOf(get(x)), y = Double.valueOf(get(y)); the first missing field
// (IndexOutOfBounds) or malformed number (NumberFormatException) is the line's error.
template <class Src>
__device__ __forceinline__ int eval_csv_line(const CsvArgs& a, const Src& s, int64_t j, int64_t newlines, LineOut* o) {
  const int64_t b = j == 0 ? 0 : a.nl[j - 1] + 1;
  int64_t e = j < newlines ? a.nl[j] : a.len;
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

__device__ __forceinline__ void geo_tabs_fill(const CsvArgs& a, uint64_t* tab, uint64_t* ttab, char* keys) {
  for (int b = threadIdx.x; b < 256; b += blockDim.x) geo_tab_entry(b, tab + b, ttab + b);
  for (int i = threadIdx.x; i < kGeoKeys * kGeoPropMax; i += blockDim.x) {
    const int k = i / kGeoPropMax, c = i % kGeoPropMax;
    const char* names[5] = {"value", "geometry", "properties", "coordinates", "type"};
    const int nl[5] = {5, 8, 10, 11, 4};
    const int nk = k < 4 ? k : 4;
    char ch = 0;
    if (k == 4 || k == 5) ch = k == 4 ? a.prop_ts[c] : a.prop_obj[c];
    else ch = c < nl[nk] ? names[nk][c] : 0;
    keys[i] = ch;
  }
}

// line j's bytes [b, e) ('\r' dropped) and its first non-blank p; 0, or the error of a line that
// is not an object
template <class Src>
__device__ __forceinline__ int geojson_bounds(const CsvArgs& a, const Src& s, int64_t j, int64_t newlines, int64_t& p,
                                              int64_t& e) {
  const int64_t b = j == 0 ? 0 : a.nl[j - 1] + 1;
  e = j < newlines ? a.nl[j] : a.len;
  if (e > b && s(e - 1) == '\r') --e;
  if (e <= b) return kCsvEmptyLine;
  p = jskip(s, b, e);
  if (p >= e || s(p) != '{') return kCsvMissingField;  // not an object: malformed record
  return kCsvOk;
}
// FAST: try the one-pass locator first (the LDS-staged path); otherwise the walk
template <bool FAST, class Src>
__device__ __forceinline__ int eval_geojson_line(const CsvArgs& a, const Src& s, int64_t j, int64_t newlines, LineOut* o,
                                                 const GeoTabs& gt) {
  int64_t p = 0, e = 0;
  const int bs = geojson_bounds(a, s, j, newlines, p, e);
  if (bs) return bs;
  const GeoProps gp{gt.keys + 4 * kGeoPropMax, gt.keys + 5 * kGeoPropMax, a.len_ts, a.len_obj, a.date_fmt, a.tz_off_ms,
                    kPow5Dev};
  if constexpr (FAST) return geojson_line(gt, gp, s, p, e, a.value_lines, true, o);
  else return geojson_line(gt, gp, s, p, e, a.value_lines, o);
}

__device__ __forceinline__ bool store_line(const CsvArgs& a, int64_t j, int st, const LineOut& o, DictWork* w);
// parse + store line j; returns true when its objID needs the dictionary (*w filled)
template <int FMT, bool FAST, class Src>
__device__ __forceinline__ bool parse_line(const CsvArgs& a, const Src& s, int64_t j, int64_t newlines, DictWork* w,
                                           const GeoTabs& gt) {
  LineOut o{0, 0, 0.0, 0.0, false, {0, 0}};
  int st;
  if constexpr (FMT == 1) st = eval_geojson_line<FAST>(a, s, j, newlines, &o, gt);
  else st = eval_csv_line(a, s, j, newlines, &o);
  return store_line(a, j, st, o, w);
}
// line j's outputs (or its error); true when its objID needs the dictionary (*w filled)
__device__ __forceinline__ bool store_line(const CsvArgs& a, int64_t j, int st, const LineOut& o, DictWork* w) {
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
// The chunk's line counts from the device (csv_nlindex's total): false when the parse must not
// write -- the index was cut (more newlines than nl_cap: the host regrows and re-runs), more lines
// than the caller's capacity (GF_ERR_CAPACITY), or than the grid covers / 2^32 - 1
__device__ __forceinline__ bool csv_counts(const CsvArgs& a, int64_t& newlines, int64_t& lines) {
  newlines = (int64_t)*a.nl_total;
  lines = newlines + (a.text[a.len - 1] != '\n' ? 1 : 0);
  return newlines <= a.nl_cap && lines <= a.cap && lines <= a.grid_lines && lines <= (int64_t)UINT32_MAX;
}
// GeoJSON blocks hold 192 lines (GF_GEO_LINES), CSV blocks kBlock.  A block keeps its staged
// lines in LDS until its slowest lane is done, and LDS is what bounds the residency: a block of 256
// mean GeoJSON lines (~48 KB + 10 %, plus the locator's 4.5 KB of static tables) lets only two
// share a CU (8 waves); three 192-line blocks fit (9 waves).  r05 A/B, parse kernel per 1M lines
// (tools/gpu_r05_geo2.sh): 256 lines 3.05 ms, 192 lines 2.86, 128 lines 3.11 (four blocks, 8
// waves).  Handing a block's lines to lanes in length order (so that each wave's byte loop runs
// to a shorter longest line; the sum of the waves' longest lines drops 26 % on the bench lines)
// measured slower (3.18 / 2.90 ms): the block's LDS is held until its longest line is done
// either way, and the sort's ranks cost LDS.  So did lanes taking the block's next line from an
// LDS queue when theirs ends (3.08 vs 2.89 ms): with as many lines as lanes there is nothing left
// to take, and staging twice the lines per lane halves the resident waves instead (LDS).  The
// lanes idle for ~40 % of a block's life (mean line 189 B, the longest of 192 ~330 B).
#ifndef GF_GEO_LINES
#define GF_GEO_LINES 192
#endif
constexpr int kGeoLines = GF_GEO_LINES;
static_assert(kGeoLines % 64 == 0 && kGeoLines <= kBlock, "whole waves");
template <int FMT>
constexpr int parse_lines() { return FMT == 1 ? kGeoLines : kBlock; }
__device__ __forceinline__ void queue_dict(const CsvArgs& a, bool need, const DictWork& w);
template <int FMT>  // 0: CSV / TSV, 1: GeoJSON (a.format)
__global__ __launch_bounds__(parse_lines<FMT>()) void csv_parse_kernel(CsvArgs a) {
  constexpr int NB = parse_lines<FMT>();
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int64_t newlines, lines;
  const bool ok = csv_counts(a, newlines, lines);
  const int64_t L0 = (int64_t)blockIdx.x * NB;
  if (!ok || L0 >= lines) return;  // block-uniform
  const int64_t L1 = L0 + NB < lines ? L0 + NB : lines;  // exclusive
  const int64_t b0 = L0 == 0 ? 0 : a.nl[L0 - 1] + 1;
  const int64_t b1 = L1 - 1 < newlines ? a.nl[L1 - 1] : a.len;     // the last line's '\n' (or end)
  const int64_t a0 = b0 & ~(int64_t)15;
  const int64_t j = L0 + threadIdx.x;
  DictWork w{0, 0, 0};
  bool need = false;
  __shared__ uint64_t gtab[FMT == 1 ? 256 : 1], gttab[FMT == 1 ? 256 : 1];
  __shared__ char gkeys[FMT == 1 ? kGeoKeys * kGeoPropMax : 1];
  const GeoTabs gt{(GF_LDS_PTR(uint64_t))gtab, (GF_LDS_PTR(uint64_t))gttab, (GF_LDS_PTR(char))gkeys,
                   {5, 8, 10, 11, a.len_ts, a.len_obj, 4},
                   geo_pack16(a.prop_ts, a.len_ts <= 16 ? a.len_ts : 0),
                   geo_pack16(a.prop_obj, a.len_obj <= 16 ? a.len_obj : 0)};
  if (FMT == 1) {
    geo_tabs_fill(a, gtab, gttab, gkeys);
    __syncthreads();
  }
  if (b1 - a0 <= a.lds_cap) {  // block-uniform
    for (int64_t off = a0 + 16 * threadIdx.x; off < b1; off += 16 * NB) {
      if (off + 16 <= a.len) {
        *reinterpret_cast<uint4*>(lds + (off - a0)) = *reinterpret_cast<const uint4*>(a.text + off);
      } else {
        for (int k = 0; k < 16 && off + k < a.len; ++k) lds[off - a0 + k] = a.text[off + k];
      }
    }
    __syncthreads();
    if (j < L1) {
      if (a.geo_fast) need = parse_line<FMT, true>(a, LBytes{(GF_LDS_PTR(char))lds, a0}, j, newlines, &w, gt);
      else need = parse_line<FMT, false>(a, LBytes{(GF_LDS_PTR(char))lds, a0}, j, newlines, &w, gt);
    }
  } else if (j < L1) {
    need = parse_line<FMT, false>(a, GBytes{a.text}, j, newlines, &w, gt);
  }
  queue_dict(a, need, w);
}

// the wave's dictionary objIDs into the queue (one atomic per wave)
__device__ __forceinline__ void queue_dict(const CsvArgs& a, bool need, const DictWork& w) {
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

// ---------------------------------------------------------------------------------------
// r06: the wave-per-line structural scan (GeoJSON).  The lane locator above runs one line per
// lane, a dependent byte chain per lane with ~1,500 instructions per line (r05 PMC).  Here the
// whole wave reads ONE line, 64 bytes per step (one per lane, from the LDS-staged block), and
// derives the line's structure from ballots:
//   strings   a prefix XOR of the quote mask (a backslash anywhere sends the line to the walk, so
//             every quote toggles) with the carried in-string bit;
//   elements  brackets, ':' and ',' outside strings, opening quotes and token starts; the depth
//             before each byte from mbcnt of the open / close masks; each element's predecessor
//             (the highest element lane below it, or the last one of earlier steps);
//   containers per depth level present in the step: the kind (object / array) and role (Kafka
//             record, value, geometry, properties) of the innermost container from the last open
//             at that level below the lane (or the carried level state); a string is a key when
//             it follows '{' or ',' in an object;
//   grammar   each element against its predecessor and container (the JSON grammar as the lane
//             automaton's transitions state it, k_geojson.hpp jtrans);
//   tokens    numbers by local rules over (previous, byte, next) plus the token's earlier '.'/'e'
//             masks -- the lane automaton's number grammar -- literals by their first byte;
//   keys      a looked-up container's key: its bytes from LDS (<= 16) against the packed names;
//             the notes take the highest matching lane.
// It accepts a subset of the lines the lane locator accepts (a byte >= 0x80 goes to the walk
// too), with the same notes; GF_FLAG_GEOJSON_CHECK runs both and counts any difference
// (tests/test_gpu_geojson.py::test_wave_scan_matches_lane_locator).  The evaluation of the
// located members (geo_eval_body) stays one lane per line.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int32_t lanes_below(uint64_t m) {
  return (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ int top_lane(uint64_t m) { return 63 - __clzll((long long)m); }  // (m != 0)
__device__ __forceinline__ uint32_t lane_val(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint32_t from_lane(uint32_t v, int l) { return (uint32_t)__shfl((int)v, l, 64); }

// The line lp[0, len) (lp[0] == '{') by the whole wave (a wave-uniform call).  false: the line
// takes the walk; true: n[] = its notes (positions from lp, as geo_locate_notes).
__device__ __forceinline__ bool geo_wave_scan(GF_LDS_PTR(char) lp, int32_t len, GF_LDS_PTR(uint32_t) wtab,
                                              const GeoTabs& gt, int top_role, int32_t* n) {
  constexpr K16 kValue = geo_pack16("value", 5), kGeom = geo_pack16("geometry", 8);
  constexpr K16 kProps = geo_pack16("properties", 10), kCoord = geo_pack16("coordinates", 11);
  constexpr K16 kType = geo_pack16("type", 4);
  const int32_t lts = gt.klen[4], lobj = gt.klen[5];
  const int lane = (int)(threadIdx.x & 63u);
  const uint64_t below = (1ull << lane) - 1ull;
  // carried from step to step (wave-uniform)
  int32_t depth = 0, tok_start = 0, str_open = 0;
  uint32_t instr = 0, tok_open = 0, tok_dot = 0, tok_e = 0, str_key = 0, last = WT_NONE, pend = JK_NONE;
  uint32_t roles = 0;  // the open containers' roles at depths 1..3 (4 bits each)
  uint64_t kinds = 0;  // bit d: the open container at depth d is an object
  for (int k = 0; k < kGeoNotes; ++k) n[k] = -1;
  for (int32_t c0 = 0; c0 < len; c0 += 64) {
    const int32_t i = c0 + lane;
    const uint32_t b = i < len ? (uint32_t)(uint8_t)lp[i] : 32u;
    const uint32_t f = wtab[b];
    const uint64_t Qm = __ballot(f & WB_Q);
    uint64_t S = Qm;
    S ^= S << 1;
    S ^= S << 2;
    S ^= S << 4;
    S ^= S << 8;
    S ^= S << 16;
    S ^= S << 32;
    S = instr ? ~S : S;
    const uint64_t IN = (S << 1) | (uint64_t)instr;  // bit i: byte i is a string's content or closing quote
    instr = (uint32_t)(S >> 63);
    const bool in = (IN >> lane) & 1ull;
    if (__ballot(f & (WB_BAD | (in ? WB_WSC : WB_OTH)))) return false;
    const uint32_t fo = in ? 0u : f;  // the byte's classes outside strings (an opening quote included)
    const uint64_t OPm = __ballot(fo & (WB_OB | WB_OA)), CLm = __ballot(fo & (WB_CB | WB_CA));
    const uint64_t PUm = __ballot(fo & (WB_CO | WB_CM)), TKm = __ballot(fo & WB_TOK);
    const uint64_t OQ = Qm & ~IN, CQ = Qm & IN;
    const uint64_t TSm = TKm & ~((TKm << 1) | (uint64_t)tok_open);
    const uint64_t ELm = OPm | CLm | PUm | OQ | TSm;
    const bool el = (ELm >> lane) & 1ull, cq = (CQ >> lane) & 1ull;
    const uint32_t traw = el ? fo >> 24 : (uint32_t)WT_NONE;
    const bool isop = traw == WT_OB || traw == WT_OA;
    const int32_t dbef = depth + lanes_below(OPm) - lanes_below(CLm);  // the depth before the byte
    if (__ballot(((traw == WT_CB || traw == WT_CA || traw == WT_CM) && dbef <= 0) || (isop && dbef >= 63)))
      return false;
    const uint64_t pm = ELm & below;
    const int pl = pm ? top_lane(pm) : 0;
    const uint32_t praw0 = from_lane(traw, pl);
    const uint32_t praw = pm ? praw0 : last;  // the predecessor (a string: key-ness not needed here)
    // the depth levels the step's elements and closing quotes sit at, lowest first
    const bool ctx = el || cq;
    int32_t dl = depth, dh = depth;
    while (__ballot(ctx && dbef < dl)) --dl;
    while (__ballot(ctx && dbef > dh)) ++dh;
    const uint64_t qb = Qm & below;
    const int ql = qb ? top_lane(qb) : 0;  // a closing quote's opening quote (this step)
    uint32_t K = 0, crole = JR_NONE, orole = JR_NONE, iskey = 0, kkind = JK_NONE;
    for (int32_t D = dl; D <= dh + 1; ++D) {
      const uint64_t OD = __ballot(isop && dbef == D - 1), BD = __ballot(traw == WT_OB && dbef == D - 1);
      const bool at = ctx && dbef == D;
      const uint64_t om = OD & below;
      const int os = om ? top_lane(om) : 0;
      const uint32_t rin = from_lane(orole, os);
      const bool lowd = D >= 1 && D <= 3;
      if (at) {  // the innermost container: the last open to depth D below, or the carried one
        K = om ? (uint32_t)(BD >> os) & 1u : (uint32_t)(kinds >> (D & 63)) & 1u;
        crole = om ? rin : lowd ? (roles >> (4 * D)) & 15u : (uint32_t)JR_NONE;
        if (traw == WT_SV) iskey = praw == WT_OB || (praw == WT_CM && K);
      }
      const uint32_t kin = from_lane(iskey, ql);
      if (at && cq) iskey = qb ? kin : str_key;
      if (D <= 3) {  // (uniform) a looked-up container's keys; the roles of the containers opened here
        const bool kend = at && cq && iskey;
        const uint64_t KD = __ballot(kend);
        if (lowd && __ballot(kend && crole != JR_NONE)) {
          const int32_t kst = (qb ? c0 + ql : str_open) + 1, klen = i - kst;
          uint64_t hi = 0, lo = 0;
          if (kend && crole != JR_NONE && klen <= 16) {  // the key's last <= 16 bytes (16 independent reads)
            uint32_t kb[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              const int32_t x = i - 16 + q;
              kb[q] = x >= kst ? (uint32_t)(uint8_t)lp[x] : 0u;
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              hi = (hi << 8) | (lo >> 56);
              lo = (lo << 8) | kb[q];
            }
          }
          // (a key of <= 8 bytes leaves hi 0: the short names compare lo only)
          const bool e_type = klen == 4 && lo == kType.lo, e_value = klen == 5 && lo == kValue.lo;
          const bool e_geom = klen == 8 && lo == kGeom.lo;
          const bool e_props = klen == 10 && lo == kProps.lo && hi == kProps.hi;
          const bool e_coord = klen == 11 && lo == kCoord.lo && hi == kCoord.hi;
          const bool top = kend && crole == JR_TOP, val = kend && crole == JR_VAL;
          const bool geo = kend && crole == JR_GEO, prop = kend && crole == JR_PROP;
          const bool m_value = top && e_value, v_geom = val && e_geom, v_props = val && e_props;
          bool p_ts = prop && klen == lts && lts <= 16 && lo == gt.pts.lo && hi == gt.pts.hi;
          bool p_obj = prop && klen == lobj && lobj <= 16 && lo == gt.pobj.lo && hi == gt.pobj.hi;
          if ((lts > 16 || lobj > 16) && prop && klen > 16) {  // (rare: a property name longer than 16 bytes)
            const LBytes s{lp, 0};
            p_ts = jkey_eq(s, kst, klen, gt, 4);
            p_obj = jkey_eq(s, kst, klen, gt, 5);
          }
          kkind = kend ? (m_value ? JK_VALUE : v_geom ? JK_GEO : v_props ? JK_PROP : JK_NONE) : kkind;
          auto note = [&](int k, bool c) {
            const uint64_t M = __ballot(c);
            if (M) n[k] = c0 + top_lane(M);
          };
          note(GN_V, m_value);
          note(GN_TV, val && e_type);
          note(GN_CV, val && e_coord);
          note(GN_GV, v_geom);
          note(GN_PRV, v_props);
          note(GN_TG, geo && e_type);
          note(GN_CG, geo && e_coord);
          note(GN_TP, p_ts);
          note(GN_QP, p_obj);
        }
        if (D <= 2) {  // a container opened at depth D: its role from the key before it
          const uint64_t pk = KD & below;
          const uint32_t pin = from_lane(kkind, pk ? top_lane(pk) : 0);
          const uint32_t pe = pk ? pin : pend;
          if (at && isop)
            orole = traw == WT_OA ? (uint32_t)JR_NONE
                    : D == 0 ? (uint32_t)top_role
                    : crole == JR_TOP ? (0x0020u >> (4 * pe)) & 15u   // value -> V
                    : crole == JR_VAL ? (0x4300u >> (4 * pe)) & 15u   // geometry, properties
                    : (uint32_t)JR_NONE;
        }
      }
      if (OD) {  // the level's carried state: its last open of the step
        const int s = top_lane(OD);
        kinds = (kinds & ~(1ull << (D & 63))) | (((BD >> s) & 1ull) << (D & 63));
        if (lowd) roles = (roles & ~(15u << (4 * D))) | (lane_val(orole, s) << (4 * D));
      }
    }
    // the grammar: each element after its predecessor, in its container
    const uint32_t tr = traw == WT_SV && iskey ? (uint32_t)WT_SK : traw;
    const uint32_t pr0 = from_lane(tr, pl);
    const uint32_t pr = pm ? pr0 : last;
    const bool pve = (kWtValueEnd >> pr) & 1u;
    const bool ok = tr == WT_NONE || tr == WT_SK ? true
                    : tr == WT_CO ? pr == WT_SK
                    : tr == WT_CM ? pve
                    : tr == WT_CB ? K && (pr == WT_OB || pve)
                    : tr == WT_CA ? !K && (pr == WT_OA || pve)
                    : pr == WT_OA || pr == WT_CO || (pr == WT_CM && !K) || (pr == WT_NONE && tr == WT_OB);
    if (__ballot(!ok)) return false;
    // tokens: the number grammar by local rules, literals whole from their first byte
    if (TKm) {
      const uint64_t DOTm = __ballot(fo & WB_DOT), Em = __ballot(fo & WB_E);
      const bool tk = (TKm >> lane) & 1ull;
      const uint64_t tsb = TSm & (below | (1ull << lane));
      const int32_t ts = tsb ? c0 + top_lane(tsb) : tok_start;  // the token's first byte
      bool bad = false;
      if (tk) {
        const uint32_t fc = (uint8_t)lp[ts];
        const uint32_t prv = i > ts ? (uint32_t)(uint8_t)lp[i - 1] : 0u;
        const uint32_t nxt = i + 1 < len ? (uint32_t)(uint8_t)lp[i + 1] : 32u;
        const bool num = fc == '-' || fc - '0' < 10u;
        const bool ndig = nxt - '0' < 10u, pdig = prv - '0' < 10u, pexp = (prv | 0x20u) == 'e';
        if (!num) {
          if (i == ts) {  // true / false / null, and nothing else
            // the word's bytes after the first, and the byte after it (a blank past the line)
            uint32_t wb[5];
#pragma unroll
            for (int q = 0; q < 5; ++q) wb[q] = i + 1 + q < len ? (uint32_t)(uint8_t)lp[i + 1 + q] : 32u;
            const uint32_t w4 = wb[0] | wb[1] << 8 | wb[2] << 16, w5 = w4 | wb[3] << 24;  // little-endian
            const bool w = fc == 't' ? w4 == ('r' | 'u' << 8 | 'e' << 16) && !(wtab[wb[3]] & WB_TOK)
                         : fc == 'n' ? w4 == ('u' | 'l' << 8 | 'l' << 16) && !(wtab[wb[3]] & WB_TOK)
                         : fc == 'f' ? w5 == ('a' | 'l' << 8 | 's' << 16 | (uint32_t)'e' << 24) && !(wtab[wb[4]] & WB_TOK)
                         : false;
            bad = !w;
          }
        } else {  // -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]{1,2})?, shorter than 19 bytes
          const uint32_t sh = ts > c0 ? (uint32_t)(ts - c0) : 0u;
          const uint64_t rng = below & ~((1ull << sh) - 1ull);  // the token's bytes before this one (this step)
          const bool carried = ts < c0;
          if (b == '-') {
            bad = !((i == ts || pexp) && ndig);
          } else if (b == '+') {
            bad = !(pexp && ndig);
          } else if (b == '.') {
            bad = !(pdig && ndig) || ((DOTm | Em) & rng) != 0 || (carried && (tok_dot | tok_e));
          } else if ((b | 0x20u) == 'e') {
            const bool sg = nxt == '+' || nxt == '-';
            bad = !(pdig && (ndig || sg)) || (Em & rng) != 0 || (carried && tok_e);
            const int32_t x = i + (sg ? 2 : 1);  // the exponent's first digit: a third one is the walk's
            bad |= x + 2 < len && (uint32_t)(uint8_t)lp[x + 1] - '0' < 10u && (uint32_t)(uint8_t)lp[x + 2] - '0' < 10u;
          } else if (b - '0' >= 10u) {
            bad = true;  // a letter
          } else {
            bad = b == '0' && (i == ts || (i == ts + 1 && fc == '-')) && ndig;  // a leading zero
          }
          bad |= !(wtab[nxt] & WB_TOK) && i - ts + 1 >= 19;  // the token's last byte: its length
        }
      }
      if (__ballot(bad)) return false;
      const bool t63 = (TKm >> 63) & 1ull;
      if (t63) {  // a token runs into the next step
        const int32_t ts63 = (int32_t)lane_val((uint32_t)ts, 63);
        const uint32_t sh = ts63 > c0 ? (uint32_t)(ts63 - c0) : 0u;
        const uint64_t r = ~((1ull << sh) - 1ull);
        const bool car = ts63 < c0;
        tok_dot = (car && tok_dot) || (DOTm & r) != 0;
        tok_e = (car && tok_e) || (Em & r) != 0;
        tok_start = ts63;
      }
      tok_open = t63;
    } else {
      tok_open = 0;
    }
    if (ELm) last = lane_val(tr, top_lane(ELm));
    depth += __popcll(OPm) - __popcll(CLm);
    const uint64_t KCm = __ballot(cq && iskey);
    if (KCm) pend = lane_val(kkind, top_lane(KCm));
    if (instr && Qm) {  // a string runs into the next step
      const int s = top_lane(Qm);
      str_open = c0 + s;
      str_key = lane_val(iskey, s);
    }
  }
  return !instr && depth == 0 && last == WT_CB;
}

// GeoJSON blocks with the wave scan: the block's lines staged in LDS as csv_parse_kernel stages
// them; each wave scans its 64 lines one after the other (all lanes on each), the line's lane
// keeps the result, then every lane evaluates its own line from the notes (or walks it).
// CHECK: the lane locator runs too, and a.geo_check counts [both pass, same notes; the scan
// passes, the locator not; both pass, notes differ; the locator passes, the scan not].
template <bool CHECK>
__global__ __launch_bounds__(kGeoLines) void geojson_wave_kernel(CsvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int64_t newlines, lines;
  const bool ok = csv_counts(a, newlines, lines);
  const int64_t L0 = (int64_t)blockIdx.x * kGeoLines;
  if (!ok || L0 >= lines) return;  // block-uniform
  const int64_t L1 = L0 + kGeoLines < lines ? L0 + kGeoLines : lines;  // exclusive
  const int64_t b0 = L0 == 0 ? 0 : a.nl[L0 - 1] + 1;
  const int64_t b1 = L1 - 1 < newlines ? a.nl[L1 - 1] : a.len;
  const int64_t a0 = b0 & ~(int64_t)15;
  const int64_t j = L0 + threadIdx.x;
  DictWork w{0, 0, 0};
  bool need = false;
  __shared__ uint64_t gtab[256], gttab[256];
  __shared__ char gkeys[kGeoKeys * kGeoPropMax];
  __shared__ uint32_t wtab[256];
  const GeoTabs gt{(GF_LDS_PTR(uint64_t))gtab, (GF_LDS_PTR(uint64_t))gttab, (GF_LDS_PTR(char))gkeys,
                   {5, 8, 10, 11, a.len_ts, a.len_obj, 4},
                   geo_pack16(a.prop_ts, a.len_ts <= 16 ? a.len_ts : 0),
                   geo_pack16(a.prop_obj, a.len_obj <= 16 ? a.len_obj : 0)};
  geo_tabs_fill(a, gtab, gttab, gkeys);
  for (int c = threadIdx.x; c < 256; c += blockDim.x) wtab[c] = wave_class(c);
  const GeoProps gp{gt.keys + 4 * kGeoPropMax, gt.keys + 5 * kGeoPropMax, a.len_ts, a.len_obj, a.date_fmt,
                    a.tz_off_ms, kPow5Dev};
  if (b1 - a0 <= a.lds_cap) {  // block-uniform
    for (int64_t off = a0 + 16 * threadIdx.x; off < b1; off += 16 * kGeoLines) {
      if (off + 16 <= a.len) {
        *reinterpret_cast<uint4*>(lds + (off - a0)) = *reinterpret_cast<const uint4*>(a.text + off);
      } else {
        for (int k = 0; k < 16 && off + k < a.len; ++k) lds[off - a0 + k] = a.text[off + k];
      }
    }
    __syncthreads();
    const LBytes s{(GF_LDS_PTR(char))lds, a0};
    int64_t p = 0, e = 0;
    const int bs = j < L1 ? geojson_bounds(a, s, j, newlines, p, e) : (int)kCsvEmptyLine;
    const int32_t o0 = (int32_t)(p - a0), o1 = (int32_t)(e - a0);  // (staged: < 64 KB)
    const int top_role = a.value_lines ? JR_VAL : JR_TOP;
    const int lane = (int)(threadIdx.x & 63u);
    bool wok = false;
    int32_t wn[kGeoNotes];
    for (int k = 0; k < kGeoNotes; ++k) wn[k] = -1;
    for (uint64_t m = __ballot(j < L1 && bs == kCsvOk); m; m &= m - 1ull) {  // (wave-uniform)
      const int q = __builtin_ctzll(m);
      const int32_t q0 = __builtin_amdgcn_readlane(o0, q), q1 = __builtin_amdgcn_readlane(o1, q);
      int32_t nq[kGeoNotes];
      const bool okq = geo_wave_scan((GF_LDS_PTR(char))lds + q0, q1 - q0, (GF_LDS_PTR(uint32_t))wtab, gt, top_role, nq);
      if (lane == q) {
        wok = okq;
        for (int k = 0; k < kGeoNotes; ++k) wn[k] = nq[k];
      }
    }
    if (j < L1) {
      LineOut o{0, 0, 0.0, 0.0, false, {0, 0}};
      int st = bs;
      if (bs == kCsvOk) {
        if constexpr (CHECK) {
          int32_t ln[kGeoNotes];
          const bool lok = geo_locate_notes(s, p, e, gt, a.value_lines, ln);
          bool same = true;
          for (int k = 0; k < kGeoNotes; ++k) same = same && ln[k] == wn[k];
          const int c = wok && lok ? (same ? 0 : 2) : wok ? 1 : lok ? 3 : -1;
          if (c >= 0) atomicAdd(a.geo_check + c, 1ull);
        }
        if (wok) {
          GeoPos g;
          geo_notes_pos(s, p, e, a.value_lines, wn, &g);
          st = geo_eval_body(gp, s, e, g, &o);
        } else {
          LineOut wo{0, 0, 0.0, 0.0, false, {0, 0}};
          st = eval_geojson_walk(gp, s, p, e, a.value_lines, &wo);
          o = wo;
        }
      }
      need = store_line(a, j, st, o, &w);
    }
  } else if (j < L1) {
    need = parse_line<1, false>(a, GBytes{a.text}, j, newlines, &w, gt);
  }
  queue_dict(a, need, w);
}

// The call's last kernel: the error kind of the first bad line (re-derived by a one-lane pass over
// that line), then the head the host reads back in one copy (counts, error, dictionary work)
__global__ void csv_error_kernel(CsvArgs a) {
  int64_t newlines, lines;
  csv_counts(a, newlines, lines);
  const unsigned long long j = a.err->line;
  if (j != ~0ull) {  // block-uniform
    __shared__ uint64_t gtab[256], gttab[256];
    __shared__ char gkeys[kGeoKeys * kGeoPropMax];
    const GeoTabs gt{(GF_LDS_PTR(uint64_t))gtab, (GF_LDS_PTR(uint64_t))gttab, (GF_LDS_PTR(char))gkeys,
                     {5, 8, 10, 11, a.len_ts, a.len_obj, 4},
                     geo_pack16(a.prop_ts, a.len_ts <= 16 ? a.len_ts : 0),
                     geo_pack16(a.prop_obj, a.len_obj <= 16 ? a.len_obj : 0)};
    if (a.format == 1) geo_tabs_fill(a, gtab, gttab, gkeys);
    __syncthreads();
    if (threadIdx.x == 0) {
      LineOut o{0, 0, 0.0, 0.0, false, {0, 0}};
      const GBytes s{a.text};
      a.err->kind = a.format == 1 ? eval_geojson_line<false>(a, s, (int64_t)j, newlines, &o, gt)
                                  : eval_csv_line(a, s, (int64_t)j, newlines, &o);
    }
  }
  if (threadIdx.x == 0) {
    a.head->newlines = (unsigned long long)newlines;
    a.head->lines = (unsigned long long)lines;
    a.head->dict_n = *a.dict_n;
    a.head->dict_bytes = *a.dict_bytes;
    a.head->err = *a.err;
  }
}

// The newline index in ONE pass over the text (r05; the count + scan + index passes read the text
// twice: 2 x 190 MB per 1M GeoJSON lines, r04 PMC).  A block takes one 64 KB segment (logical id
// from a ticket taken at its start, so the look-back only waits on started blocks), keeps its 16
// chunk masks in registers, counts, publishes its count and looks back for its prefix (the
// decoupled look-back of expand_async_kernel, k_points.hip), then writes its newline positions in
// order from the masks.  nl holds nl_cap positions (the ones past it are counted, not stored:
// the host regrows and re-runs); the last logical block writes the total to *total.
constexpr int kNlIters = (int)(kCsvSeg / (16 * kBlock));
__global__ __launch_bounds__(kBlock) void csv_nlindex_kernel(const char* __restrict__ text, int64_t len,
                                                             int64_t* __restrict__ nl, int64_t nl_cap,
                                                             uint32_t* __restrict__ total, ExpandState st,
                                                             CsvErr* __restrict__ err,
                                                             unsigned long long* __restrict__ dict_counters) {
  __shared__ unsigned long long s_bid, s_prefix;
  __shared__ uint32_t ws[kBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_bid = atomicAdd(st.ticket, 1ull) - st.base;
  __syncthreads();
  const uint64_t bid = s_bid;
  if (bid == 0 && threadIdx.x == 0) {  // the parse's error slot and dictionary counters (no memset launches)
    *err = CsvErr{~0ull, -1, -1};
    dict_counters[0] = 0ull;
    dict_counters[1] = 0ull;
  }
  const int64_t s0 = (int64_t)bid * kCsvSeg;
  const int64_t s1 = s0 + kCsvSeg < len ? s0 + kCsvSeg : len;
  uint32_t m[kNlIters], c = 0;
#pragma unroll
  for (int it = 0; it < kNlIters; ++it) {
    const int64_t off = s0 + (int64_t)it * 16 * kBlock + 16 * threadIdx.x;
    m[it] = off < s1 ? chunk_mask(text, len, off) : 0u;
    c += (uint32_t)__popc(m[it]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) ws[w] = c;
  __syncthreads();
  uint32_t agg = 0;
#pragma unroll
  for (int v = 0; v < kBlock / 64; ++v) agg += ws[v];
  if (w == 0) {  // publish the aggregate, look back for the prefix (as scan1_kernel)
    unsigned long long* my = st.status + bid;
    const uint64_t ep = st.epoch & 0x3FFFFFFu;
    if (bid == 0) {
      if (lane == 0) {
        __hip_atomic_store(my, lb_pack(st.epoch, kLbInc, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_prefix = 0;
      }
    } else {
      if (lane == 0) __hip_atomic_store(my, lb_pack(st.epoch, kLbAgg, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint64_t prefix = 0;
      int64_t hi = (int64_t)bid - 1;
      for (;;) {
        const int64_t p = hi - lane;
        const uint64_t v = p >= 0 ? __hip_atomic_load(st.status + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const bool ready = p < 0 || ((v >> 38) == ep && ((v >> 36) & 3ull) != 0ull);
        if (__ballot(!ready)) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const bool incl = p >= 0 && ((v >> 36) & 3ull) == kLbInc;
        const uint64_t incm = __ballot(incl);
        const int stop = incm ? __ffsll((unsigned long long)incm) - 1 : 64;
        uint64_t add = lane <= stop ? (v & ((1ull << 36) - 1ull)) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) add += __shfl_xor(add, o, 64);
        prefix += add;
        if (incm || hi - 64 < 0) break;
        hi -= 64;
      }
      if (lane == 0) {
        __hip_atomic_store(my, lb_pack(st.epoch, kLbInc, prefix + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_prefix = prefix;
      }
    }
  }
  __syncthreads();
  uint64_t base = s_prefix;
  if (bid == gridDim.x - 1 && threadIdx.x == 0) *total = (uint32_t)(base + agg);
#pragma unroll
  for (int it = 0; it < kNlIters; ++it) {  // positions in order: chunk by chunk, threads in order
    const int64_t off = s0 + (int64_t)it * 16 * kBlock + 16 * threadIdx.x;
    const uint32_t cc = (uint32_t)__popc(m[it]);
    uint32_t inc = cc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    __syncthreads();  // (the previous iteration's reads of ws are done)
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int v = 0; v < kBlock / 64; ++v) {
      wbase += v < w ? ws[v] : 0u;
      tot += ws[v];
    }
    uint64_t pos = base + wbase + inc - cc;
    for (uint32_t mm = m[it]; mm; mm &= mm - 1, ++pos)
      if ((int64_t)pos < nl_cap) nl[pos] = off + __ffs(mm) - 1;
    base += tot;
  }
}

hipError_t launch_csv_nlindex(hipStream_t st, const char* text, int64_t len, int64_t nseg, int64_t* nl, int64_t nl_cap,
                              uint32_t* total, const ExpandState& es, CsvErr* err, unsigned long long* dict_counters) {
  hipLaunchKernelGGL(csv_nlindex_kernel, dim3((unsigned)nseg), dim3(kBlock), 0, st, text, len, nl, nl_cap, total, es,
                     err, dict_counters);
  return hipGetLastError();
}

// Staging size: a block's mean-length lines plus a tenth for the spread of a block's sum, in
// 1-KB steps between kCsvLds and kCsvLdsMax (CSV points ~55 B/line keep the 24 KB floor, so 6
// blocks share a CU; GeoJSON features, ~189 B/line: ~40 KB for 192 lines, 3 blocks per CU with
// the locator's tables).  A block whose lines exceed the staging area parses from global memory
// with the walk (same results, one dependent L2 read per byte).
hipError_t launch_csv_parse(gf_ctx* ctx, const CsvArgs& a0) {
  KTimer t(ctx, GF_K_CSV_PARSE);
  CsvArgs a = a0;
  const int64_t mean = a.mean_line;
  const int NB = a.format == 1 ? kGeoLines : kBlock;
  const int64_t need = mean * NB;
  int64_t cap = (need * 11 / 10 + 1023) & ~(int64_t)1023;
  a.lds_cap = (int32_t)(cap < kCsvLds ? kCsvLds : cap > kCsvLdsMax ? kCsvLdsMax : cap);
  if (a.grid_lines > 0) {  // (blocks past the chunk's lines return at once)
    const unsigned blocks = (unsigned)((a.grid_lines + NB - 1) / NB);
    if (a.format == 1 && a.geo_wave && a.geo_check)
      hipLaunchKernelGGL(geojson_wave_kernel<true>, dim3(blocks), dim3(NB), (size_t)a.lds_cap, ctx->stream, a);
    else if (a.format == 1 && a.geo_wave)
      hipLaunchKernelGGL(geojson_wave_kernel<false>, dim3(blocks), dim3(NB), (size_t)a.lds_cap, ctx->stream, a);
    else if (a.format == 1)
      hipLaunchKernelGGL(csv_parse_kernel<1>, dim3(blocks), dim3(NB), (size_t)a.lds_cap, ctx->stream, a);
    else
      hipLaunchKernelGGL(csv_parse_kernel<0>, dim3(blocks), dim3(kBlock), (size_t)a.lds_cap, ctx->stream, a);
  }
  hipLaunchKernelGGL(csv_error_kernel, dim3(1), dim3(64), 0, ctx->stream, a);
  return hipGetLastError();
}

}  // namespace gf
