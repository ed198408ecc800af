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

// parse + store line j; returns true when its objID needs the dictionary (*w filled)
template <int FMT, bool FAST, class Src>
__device__ __forceinline__ bool parse_line(const CsvArgs& a, const Src& s, int64_t j, int64_t newlines, DictWork* w,
                                           const GeoTabs& gt) {
  LineOut o{0, 0, 0.0, 0.0, false, {0, 0}};
  int st;
  if constexpr (FMT == 1) st = eval_geojson_line<FAST>(a, s, j, newlines, &o, gt);
  else st = eval_csv_line(a, s, j, newlines, &o);
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
    if (a.format == 1)
      hipLaunchKernelGGL(csv_parse_kernel<1>, dim3(blocks), dim3(NB), (size_t)a.lds_cap, ctx->stream, a);
    else
      hipLaunchKernelGGL(csv_parse_kernel<0>, dim3(blocks), dim3(kBlock), (size_t)a.lds_cap, ctx->stream, a);
  }
  hipLaunchKernelGGL(csv_error_kernel, dim3(1), dim3(64), 0, ctx->stream, a);
  return hipGetLastError();
}

}  // namespace gf
