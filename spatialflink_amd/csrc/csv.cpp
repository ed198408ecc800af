// csv.cpp -- host side of the GPU CSV/TSV ingest (k_csv.hip): Deserialization.CSVTSVToTSpatial
// (Deserialization.java:291-325) over a chunk of HBM-resident text.
//
//   newline positions and count in one pass (64 KB segments, decoupled look-back) -> one lane per
//   line parse + cell (the line count read on the device) -> the head (counts, first bad line,
//   dictionary work) written into mapped pinned memory -> the call's one sync -> objID Strings
//   that are not canonical decimals -> dictionary keys (objid.cpp)
#define GF_TU_NAME csv_cpp
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include <cstring>
#include <string>

#include "gf_internal.hpp"

using namespace gf;

// staging sizes of a context's first chunk (no mean line length yet): a GeoJSON Feature record
// (the bench's generated lines average 189 B; the reference's documented example line ~150 B) and
// a CSV point line (~55 B)
constexpr int64_t kGeoMeanLineDefault = 192, kCsvMeanLineDefault = 64;

extern "C" int gf_csv_parse(gf_ctx* ctx, const char* text, int64_t len, const gf_csv_schema* sc, const gf_grid* g,
                            double* x, double* y, int64_t* objID, int64_t* ts, int32_t* cx, int32_t* cy, int64_t cap,
                            int64_t* n_out, int64_t* bad_line, int32_t* bad_kind) {
  return gf_csv_parse_dict(ctx, nullptr, text, len, sc, g, x, y, objID, ts, cx, cy, cap, n_out, bad_line, bad_kind);
}

// The line pipeline shared by the CSV/TSV and GeoJSON ingest: `proto` carries the format's
// fields (delimiter + schema, or the GeoJSON properties); the rest is filled here.
static int parse_text_lines(gf_ctx* ctx, gf_objid_dict* dict, const char* text, int64_t len, const CsvArgs& proto,
                            const gf_grid* g, double* x, double* y, int64_t* objID, int64_t* ts, int32_t* cx,
                            int32_t* cy, int64_t cap, int64_t* n_out, int64_t* bad_line, int32_t* bad_kind) {
  if (!n_out || len < 0 || (len > 0 && !text) || !x || !y || !objID || !ts || (!cx) != (!cy) || (cx && !g))
    return set_err(ctx, GF_ERR_ARG, "gf_csv_parse: bad argument");
  if (g && !(g->n > 0 && g->cellLength > 0)) return set_err(ctx, GF_ERR_ARG, "gf_csv_parse: bad grid");
  if ((uintptr_t)text & 15) return set_err(ctx, GF_ERR_ALIGN, "gf_csv_parse: text must be 16-byte aligned");
  if (dict && dict->ctx != ctx) return set_err(ctx, GF_ERR_ARG, "gf_csv_parse: dictionary of another context");
  int st = bind(ctx);
  if (st) return st;
  if (!dict && (st = ctx_dict(ctx, &dict))) return st;
  *n_out = 0;
  if (bad_line) *bad_line = -1;
  if (bad_kind) *bad_kind = GF_CSV_OK;
  if (len == 0) return GF_OK;
  const int64_t nseg = (len + kCsvSeg - 1) / kCsvSeg;
  if (nseg >= (int64_t)INT32_MAX) return set_err(ctx, GF_ERR_ARG, "gf_csv_parse: text too large");
  // scratch: newline total | error | newline positions (sized for one line per 32 B; regrown and
  // the whole call re-run when the chunk holds more)
  const size_t o_tot = 0, o_err = 64, o_nl = 128;
  int64_t nl_cap = len / 32 + 2;
  // the head lands in mapped pinned memory, written by the call's last kernel: the sync is the
  // only host round trip (a 64-B device -> host copy was a ~20 us blit of its own)
  if (!ctx->csv_head && (st = gf_pinned_alloc(sizeof(CsvHead), &ctx->csv_head))) return set_err(ctx, st, "gf_csv_parse: pinned head");
  volatile CsvHead* const head = (volatile CsvHead*)ctx->csv_head;
  CsvHead h{};
  // One pass: index -> parse -> error/head kernels, then ONE sync.  The line count
  // stays on the device (CsvArgs.nl_total): the parse grid covers min(nl_cap + 1, cap) lines and
  // blocks past the chunk's lines return; when the count exceeds the index or the capacity the
  // parse writes nothing and the host re-runs (bigger index) or reports (GF_ERR_CAPACITY).  (r04:
  // a sync after the index for the count and another after the parse -- two host round trips and
  // four small copies per chunk.)
  for (int pass = 0; pass < 2; ++pass) {
    char* base = (char*)ctx_scratch(ctx, o_nl + sizeof(int64_t) * (size_t)nl_cap, &st);
    if (st) return st;
    const int64_t grid_lines = std::min<int64_t>(nl_cap + 1, cap);
    // the dictionary worklist: at most one String per line
    if (grid_lines > 0 && (st = dict_reserve_batch(dict, (uint64_t)grid_lines, (uint64_t)grid_lines))) return st;
    CsvErr* err = (CsvErr*)(base + o_err);
    ExpandState es;
    if ((st = lookback_state(ctx, nseg, &es))) return st;
    // (the index's first block also resets the error slot and the dictionary counters)
    GF_HIP_CHECK(ctx, launch_csv_nlindex(ctx->stream, text, len, nseg, (int64_t*)(base + o_nl), nl_cap,
                                         (uint32_t*)(base + o_tot), es, err, dict->counters + 2));
    ctx->expand_base += (unsigned long long)nseg;
    CsvArgs a = proto;
    a.text = text; a.len = len; a.nl = (int64_t*)(base + o_nl);
    a.nl_total = (const uint32_t*)(base + o_tot);
    a.nl_cap = nl_cap;
    a.cap = cap;
    a.grid_lines = grid_lines;
    // LDS staging per block from the mean line length: the last call's on this context, else a
    // per-format default (len / grid_lines undercounts it by the index's 1-line-per-32-B
    // sizing, so a cold context's first chunk had ~32 B "lines", a 24 KB staging area, and every
    // GeoJSON block fell back to the per-byte global-memory walk)
    const int64_t last_mean = ctx->csv_mean_line[proto.format == 1];
    a.mean_line = last_mean > 0 ? last_mean : (proto.format == 1 ? kGeoMeanLineDefault : kCsvMeanLineDefault);
    a.head = (CsvHead*)ctx->csv_head;
    a.x = x; a.y = y; a.objID = objID; a.ts = ts; a.cx = cx; a.cy = cy;
    if (g) { a.minX = g->minX; a.minY = g->minY; a.cl = g->cellLength; }
    a.err = err;
    a.dict_work = (DictWork*)dict->work[0];
    a.dict_n = (uint32_t*)(dict->counters + 2);
    a.dict_bytes = dict->counters + 3;
    GF_HIP_CHECK(ctx, launch_csv_parse(ctx, a));
    GF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    h.newlines = head->newlines;
    h.lines = head->lines;
    h.dict_n = head->dict_n;
    h.dict_bytes = head->dict_bytes;
    h.err.line = head->err.line;
    h.err.kind = head->err.kind;
    if ((int64_t)h.newlines <= nl_cap) break;
    nl_cap = (int64_t)h.newlines + 1;  // short lines: a larger index, the call again (nothing was written)
  }
  const int64_t lines = (int64_t)h.lines;
  *n_out = lines;
  if (lines > cap) return set_err(ctx, GF_ERR_CAPACITY, "gf_csv_parse: more lines than capacity");
  if (lines > (int64_t)UINT32_MAX) return set_err(ctx, GF_ERR_ARG, "gf_csv_parse: more than 2^32-1 lines");
  if (lines > 0) ctx->csv_mean_line[proto.format == 1] = (len + lines - 1) / lines;
  const CsvErr he = h.err;
  const unsigned long long dn[2] = {h.dict_n, h.dict_bytes};
  if (he.line != ~0ull) {
    if (bad_line) *bad_line = (int64_t)he.line;
    if (bad_kind) *bad_kind = he.kind;
    static const char* what[] = {"ok", "NumberFormatException", "unsupported literal (hexadecimal, > 19 significant "
                                 "digits at a rounding boundary, a JSON escape, a non-integer objID, a pre-1583 date)",
                                 "missing field (IndexOutOfBounds / no geometry coordinates / malformed JSON)",
                                 "empty line"};
    const int k = he.kind >= 0 && he.kind <= 4 ? he.kind : 1;
    return set_err(ctx, GF_ERR_ARG, std::string(proto.format == 1 ? "gf_geojson_parse" : "gf_csv_parse") + ": line " +
                                        std::to_string(he.line) + ": " + what[k]);
  }
  // objID Strings that are not canonical decimals: keys from the dictionary (ids in line order)
  const uint32_t nw = (uint32_t)dn[0];
  if (nw > 0) {
    if ((st = dict_reserve_table(dict, nw, dn[1]))) return st;
    if ((st = dict_run(dict, text, 1, nw, (uint64_t)lines, objID))) return st;
  }
  return GF_OK;
}

extern "C" int gf_csv_parse_dict(gf_ctx* ctx, gf_objid_dict* dict, const char* text, int64_t len,
                                 const gf_csv_schema* sc, const gf_grid* g, double* x, double* y, int64_t* objID,
                                 int64_t* ts, int32_t* cx, int32_t* cy, int64_t cap, int64_t* n_out, int64_t* bad_line,
                                 int32_t* bad_kind) {
  if (!ctx) return GF_ERR_ARG;
  if (!sc || sc->objid_field < 0 || sc->time_field < 0 || sc->x_field < 0 || sc->y_field < 0)
    return set_err(ctx, GF_ERR_ARG, "gf_csv_parse: bad schema");
  CsvArgs a{};
  a.format = 0;
  a.delim = sc->delimiter;
  a.want[0] = sc->objid_field; a.want[1] = sc->time_field; a.want[2] = sc->x_field; a.want[3] = sc->y_field;
  return parse_text_lines(ctx, dict, text, len, a, g, x, y, objID, ts, cx, cy, cap, n_out, bad_line, bad_kind);
}

// Deserialization.GeoJSONToTSpatial.map (Deserialization.java:149-211) -- k_csv.hip eval_geojson_line
extern "C" int gf_geojson_parse(gf_ctx* ctx, gf_objid_dict* dict, const char* text, int64_t len,
                                const gf_geojson_schema* sc, const gf_grid* g, double* x, double* y, int64_t* objID,
                                int64_t* ts, int32_t* cx, int32_t* cy, int64_t cap, int64_t* n_out, int64_t* bad_line,
                                int32_t* bad_kind) {
  if (!ctx) return GF_ERR_ARG;
  if (!sc || (sc->date_format != 0 && sc->date_format != 1) || (sc->value_lines != 0 && sc->value_lines != 1))
    return set_err(ctx, GF_ERR_ARG, "gf_geojson_parse: bad schema");
  CsvArgs a{};
  a.format = 1;
  a.len_obj = a.len_ts = -1;
  for (int k = 0; k < 2; ++k) {
    const char* name = k ? sc->time_property : sc->objid_property;
    if (!name) continue;
    const size_t n = std::strlen(name);
    if (n >= (size_t)kGeoPropMax) return set_err(ctx, GF_ERR_ARG, "gf_geojson_parse: property name longer than 63 bytes");
    std::memcpy(k ? a.prop_ts : a.prop_obj, name, n);
    (k ? a.len_ts : a.len_obj) = (int32_t)n;
  }
  a.date_fmt = sc->date_format;
  a.geo_fast = !ctx->geojson_walk;
  a.geo_wave = !ctx->geojson_walk && (ctx->geojson_wave || ctx->geojson_check);
  a.geo_check = ctx->geojson_check;
  a.value_lines = sc->value_lines;
  a.tz_off_ms = (int64_t)sc->tz_offset_minutes * 60000;
  return parse_text_lines(ctx, dict, text, len, a, g, x, y, objID, ts, cx, cy, cap, n_out, bad_line, bad_kind);
}
