// objid.cpp -- host side of the objID dictionary (k_objid.hip): String objIDs
// (Point.objID; Deserialization.java:317 keeps the CSV field as the String itself) <-> the
// int64 keys the SoA carries.  Canonical decimals are their own key; every other String is
// INT64_MIN + its id here.  One dictionary per stream of windows (the context's default one
// serves gf_csv_parse), so a String gets the same key in every window.
#define GF_TU_NAME objid_cpp
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include <algorithm>
#include <cstring>
#include <string>

#include "gf_decimal.hpp"
#include "gf_internal.hpp"

using namespace gf;

namespace {

int free_all(gf_objid_dict* d) {
  void* bufs[] = {d->slots, d->arena, d->counters, d->idmap, d->work[0], d->work[1], d->work[2],
                  d->slot_of, d->flag, d->rank, d->tmp, d->src};
  for (void* b : bufs)
    if (b) hipFree(b);
  return GF_OK;
}

DictDev dev_view(gf_objid_dict* d) {
  return DictDev{(DictSlot*)d->slots, d->cap - 1, d->arena, d->counters, d->idmap};
}

template <class T>
int grow(gf_ctx* ctx, T** p, uint64_t* cap, uint64_t need, uint64_t keep_bytes) {
  if (*cap >= need) return GF_OK;
  const uint64_t nc = std::max<uint64_t>(need, *cap * 2);
  T* np = nullptr;
  GF_HIP_CHECK(ctx, hipMalloc(&np, sizeof(T) * (size_t)nc));
  if (*p && keep_bytes) GF_HIP_CHECK(ctx, hipMemcpyAsync(np, *p, (size_t)keep_bytes, hipMemcpyDeviceToDevice, ctx->stream));
  if (*p) {
    GF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    GF_HIP_CHECK(ctx, hipFree(*p));
  }
  *p = np;
  *cap = nc;
  return GF_OK;
}

// table / arena / id capacity for `more` new Strings of at most `bytes` bytes in all
int reserve_table(gf_objid_dict* d, uint64_t more, uint64_t bytes) {
  gf_ctx* ctx = d->ctx;
  int st;
  unsigned long long used = 0;
  GF_HIP_CHECK(ctx, hipMemcpyAsync(&used, d->counters, sizeof used, hipMemcpyDeviceToHost, ctx->stream));
  GF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
  if ((st = grow(ctx, &d->arena, &d->arena_cap, used + bytes + 16, used))) return st;
  if ((st = grow(ctx, &d->idmap, &d->idmap_cap, (uint64_t)d->size + more + 1, sizeof(unsigned long long) * (uint64_t)d->size)))
    return st;
  uint64_t c = 1024;
  while (c < 2 * ((uint64_t)d->size + more)) c <<= 1;
  if (c > d->cap) {  // rehash every String into a larger table
    if (d->slots) GF_HIP_CHECK(ctx, hipFree(d->slots));
    d->slots = nullptr;
    GF_HIP_CHECK(ctx, hipMalloc(&d->slots, sizeof(DictSlot) * (size_t)c));
    GF_HIP_CHECK(ctx, hipMemsetAsync(d->slots, 0, sizeof(DictSlot) * (size_t)c, ctx->stream));
    d->cap = c;
    GF_HIP_CHECK(ctx, launch_dict_rehash(ctx->stream, dev_view(d), d->size));
  }
  return GF_OK;
}

// batch buffers: a worklist of `nwork` Strings over `lines` batch positions
int reserve_batch(gf_objid_dict* d, uint64_t nwork, uint64_t lines) {
  gf_ctx* ctx = d->ctx;
  if (d->work_cap < nwork) {
    GF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    for (void*& w : d->work) {
      if (w) GF_HIP_CHECK(ctx, hipFree(w));
      w = nullptr;
    }
    d->work_cap = std::max<uint64_t>(nwork, 1024);
    for (void*& w : d->work) GF_HIP_CHECK(ctx, hipMalloc(&w, sizeof(DictWork) * (size_t)d->work_cap));
  }
  if (d->line_cap < lines) {
    GF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    for (uint32_t** p : {&d->slot_of, &d->flag, &d->rank, &d->tmp}) {
      if (*p) GF_HIP_CHECK(ctx, hipFree(*p));
      *p = nullptr;
    }
    d->line_cap = std::max<uint64_t>(lines, 1024);
    GF_HIP_CHECK(ctx, hipMalloc(&d->slot_of, sizeof(uint32_t) * (size_t)d->line_cap));
    GF_HIP_CHECK(ctx, hipMalloc(&d->flag, sizeof(uint32_t) * (size_t)(d->line_cap + 1)));
    GF_HIP_CHECK(ctx, hipMalloc(&d->rank, sizeof(uint32_t) * (size_t)(d->line_cap + 1)));
    GF_HIP_CHECK(ctx, hipMalloc(&d->tmp, sizeof(uint32_t) * scan_tmp_elems((int64_t)d->line_cap)));
  }
  return GF_OK;
}

}  // namespace

namespace gf {

// Keys of the batch in d->work[0] (nwork Strings of src, positions < lines) -> keys[line].
// The caller reserved the batch buffers and table capacity for nwork new Strings.
int dict_run(gf_objid_dict* d, const char* src, int quotes, uint32_t nwork, uint64_t lines, int64_t* keys) {
  gf_ctx* ctx = d->ctx;
  if (nwork == 0) return GF_OK;
  hipStream_t s = ctx->stream;
  DictBatch B{};
  B.src = src;
  B.quotes = quotes;
  B.slot_of = d->slot_of;
  B.flag = d->flag;
  B.rank = d->rank;
  B.keys = keys;
  B.round0 = d->round;
  B.id_base = d->size;
  const DictDev dv = dev_view(d);
  uint32_t n = nwork;
  const DictWork* in = (const DictWork*)d->work[0];
  int out = 1;
  int st = GF_OK;
  uint32_t* pinned = (uint32_t*)ctx_pinned(ctx, 16, &st);
  if (st) return st;
  for (int rounds = 0; n > 0; ++rounds) {
    if (rounds > 64) return set_err(ctx, GF_ERR_HIP, "objID dictionary: probe did not converge");
    B.work = in;
    B.nwork = n;
    B.pend_out = (DictWork*)d->work[out];
    B.npend_out = (uint32_t*)(d->counters + 1);
    B.round = d->round++;
    GF_HIP_CHECK(ctx, hipMemsetAsync(d->counters + 1, 0, sizeof(unsigned long long), s));
    GF_HIP_CHECK(ctx, launch_dict(s, 0, dv, B));
    GF_HIP_CHECK(ctx, hipMemcpyAsync(pinned, d->counters + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    GF_HIP_CHECK(ctx, hipStreamSynchronize(s));
    n = pinned[0];
    in = (const DictWork*)d->work[out];
    out = out == 1 ? 2 : 1;
  }
  B.work = (const DictWork*)d->work[0];
  B.nwork = nwork;
  GF_HIP_CHECK(ctx, hipMemsetAsync(d->flag, 0, sizeof(uint32_t) * (size_t)(lines + 1), s));
  GF_HIP_CHECK(ctx, launch_dict(s, 1, dv, B));
  GF_HIP_CHECK(ctx, launch_exclusive_scan(s, d->flag, (int64_t)lines, d->rank, d->tmp));
  GF_HIP_CHECK(ctx, launch_dict(s, 2, dv, B));
  GF_HIP_CHECK(ctx, launch_dict(s, 3, dv, B));
  GF_HIP_CHECK(ctx, hipMemcpyAsync(pinned, d->rank + lines, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  GF_HIP_CHECK(ctx, hipStreamSynchronize(s));
  d->size += pinned[0];
  return GF_OK;
}

int dict_reserve_batch(gf_objid_dict* d, uint64_t nwork, uint64_t lines) { return reserve_batch(d, nwork, lines); }
int dict_reserve_table(gf_objid_dict* d, uint64_t more, uint64_t bytes) { return reserve_table(d, more, bytes); }

int ctx_dict(gf_ctx* ctx, gf_objid_dict** out) {
  if (!ctx->dict) {
    int st = gf_objid_dict_create(ctx, &ctx->dict);
    if (st) return st;
  }
  *out = ctx->dict;
  return GF_OK;
}

}  // namespace gf

extern "C" int gf_objid_dict_create(gf_ctx* ctx, gf_objid_dict** out) {
  if (!ctx || !out) return GF_ERR_ARG;
  *out = nullptr;
  int st = bind(ctx);
  if (st) return st;
  gf_objid_dict* d = new gf_objid_dict();
  d->ctx = ctx;
  auto fail = [&](int s) {
    free_all(d);
    delete d;
    return s;
  };
  if (hipMalloc(&d->counters, 4 * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(d->counters, 0, 4 * sizeof(unsigned long long)) != hipSuccess)
    return fail(set_err(ctx, GF_ERR_NOMEM, "gf_objid_dict_create: hipMalloc failed"));
  if ((st = reserve_table(d, 1024, 1 << 16)) || (st = reserve_batch(d, 1024, 1024))) return fail(st);
  *out = d;
  return GF_OK;
}

extern "C" void gf_objid_dict_destroy(gf_objid_dict* d) {
  if (!d) return;
  hipSetDevice(d->ctx->device);
  hipStreamSynchronize(d->ctx->stream);
  if (d->ctx->dict == d) d->ctx->dict = nullptr;
  free_all(d);
  delete d;
}

extern "C" int gf_ctx_objid_dict(gf_ctx* ctx, gf_objid_dict** out) {
  if (!ctx || !out) return GF_ERR_ARG;
  int st = bind(ctx);
  if (st) return st;
  return ctx_dict(ctx, out);
}

extern "C" int gf_objid_dict_size(const gf_objid_dict* d, int64_t* n) {
  if (!d || !n) return GF_ERR_ARG;
  *n = d->size;
  return GF_OK;
}

extern "C" int gf_objid_intern(gf_objid_dict* d, const char* bytes, const int64_t* offs, int64_t n, int64_t* keys) {
  if (!d || n < 0 || (n > 0 && (!offs || !keys))) return GF_ERR_ARG;
  gf_ctx* ctx = d->ctx;
  if (n > (int64_t)UINT32_MAX) return set_err(ctx, GF_ERR_ARG, "gf_objid_intern: batch too large");
  int st = bind(ctx);
  if (st) return st;
  if (n == 0) return GF_OK;
  // canonical decimals on the host; every other String goes through the device dictionary
  std::vector<DictWork> work;
  uint64_t total = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t b = offs[i], e = offs[i + 1];
    if (b < 0 || e < b || (e > b && !bytes)) return set_err(ctx, GF_ERR_ARG, "gf_objid_intern: bad offsets");
    if (e - b > (int64_t)kDictLenMask) return set_err(ctx, GF_ERR_ARG, "gf_objid_intern: objID longer than 1 MiB");
    int64_t v;
    auto src = [&](int64_t j) { return bytes[j]; };
    if (canonical_objid_key(src, Field{b, e}, &v) && std::memchr(bytes + b, '"', (size_t)(e - b)) == nullptr) {
      keys[i] = v;
    } else {
      work.push_back(DictWork{b - offs[0], (int32_t)(e - b), (uint32_t)i});
      total += (uint64_t)(e - b);
    }
  }
  if (work.empty()) return GF_OK;
  if ((st = reserve_batch(d, work.size(), (uint64_t)n)) || (st = reserve_table(d, work.size(), total))) return st;
  const int64_t span = offs[n] - offs[0];
  if ((st = grow(ctx, &d->src, &d->src_cap, (uint64_t)std::max<int64_t>(span, 1), 0))) return st;
  gf_ctx* c = ctx;
  if (span > 0) GF_HIP_CHECK(c, hipMemcpyAsync(d->src, bytes + offs[0], (size_t)span, hipMemcpyHostToDevice, c->stream));
  GF_HIP_CHECK(c, hipMemcpyAsync(d->work[0], work.data(), sizeof(DictWork) * work.size(), hipMemcpyHostToDevice, c->stream));
  int64_t* dkeys = nullptr;
  GF_HIP_CHECK(c, hipMalloc(&dkeys, sizeof(int64_t) * (size_t)n));
  st = dict_run(d, d->src, 0, (uint32_t)work.size(), (uint64_t)n, dkeys);
  if (!st) {
    std::vector<int64_t> hk((size_t)n);
    hipError_t e = hipMemcpy(hk.data(), dkeys, sizeof(int64_t) * (size_t)n, hipMemcpyDeviceToHost);
    if (e != hipSuccess) st = hip_err(c, e, "hipMemcpy(keys)");
    else
      for (const DictWork& w : work) keys[w.line] = hk[w.line];
  }
  hipFree(dkeys);
  return st;
}

extern "C" int gf_objid_decode(gf_objid_dict* d, const int64_t* keys, int64_t n, char* buf, int64_t cap, int64_t* offs) {
  if (!d || n < 0 || !offs || (n > 0 && !keys) || cap < 0) return GF_ERR_ARG;
  gf_ctx* ctx = d->ctx;
  int st = bind(ctx);
  if (st) return st;
  // extend the host mirror to every id assigned so far
  if ((int64_t)d->h_idmap.size() < d->size) {
    const size_t have = d->h_idmap.size();
    d->h_idmap.resize((size_t)d->size);
    GF_HIP_CHECK(ctx, hipMemcpyAsync(d->h_idmap.data() + have, d->idmap + have,
                                     sizeof(unsigned long long) * (d->h_idmap.size() - have), hipMemcpyDeviceToHost,
                                     ctx->stream));
    unsigned long long used = 0;
    GF_HIP_CHECK(ctx, hipMemcpyAsync(&used, d->counters, sizeof used, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    const size_t ha = d->h_arena.size();
    if (used > ha) {
      d->h_arena.resize((size_t)used);
      GF_HIP_CHECK(ctx, hipMemcpy(d->h_arena.data() + ha, d->arena + ha, (size_t)used - ha, hipMemcpyDeviceToHost));
    }
  }
  int64_t at = 0;
  char num[32];
  for (int64_t i = 0; i < n; ++i) {
    offs[i] = at;
    const int64_t k = keys[i];
    const char* p;
    size_t len;
    if (k < GF_OBJID_NUMERIC_MIN) {
      const uint64_t id = (uint64_t)k - (uint64_t)INT64_MIN;
      if (id >= d->h_idmap.size()) return set_err(ctx, GF_ERR_ARG, "gf_objid_decode: key not in this dictionary");
      const unsigned long long m = d->h_idmap[id];
      p = d->h_arena.data() + (m >> kDictLenBits);
      len = (size_t)(m & kDictLenMask);
    } else if (k == GF_OBJID_NULL) {  // a null objID decodes as the empty byte string
      p = num;
      len = 0;
    } else if (k >= GF_OBJID_NUMERIC_END) {
      return set_err(ctx, GF_ERR_ARG, "gf_objid_decode: not an objID key");
    } else {
      len = (size_t)snprintf(num, sizeof num, "%lld", (long long)k);  // Long.toString
      p = num;
    }
    if (at + (int64_t)len <= cap && buf) std::memcpy(buf + at, p, len);
    at += (int64_t)len;
  }
  offs[n] = at;
  return at > cap || (at > 0 && !buf) ? GF_ERR_CAPACITY : GF_OK;
}

// ---- kNN records with Strings (the cross-rank merge of dictionary objIDs) ----------------------
extern "C" size_t gf_knn_string_record_bytes(int32_t k, int64_t cap_bytes) {
  return k < 1 || cap_bytes < 0 ? 0 : str_record_bytes(k, cap_bytes);
}

extern "C" int gf_knn_attach_strings(gf_objid_dict* d, int32_t k, const void* records, int32_t nrec, int64_t cap_bytes,
                                     void* out) {
  if (!d || k < 1 || k > kMaxKLarge || nrec < 0 || cap_bytes < 0 || cap_bytes > (int64_t)UINT32_MAX ||
      (nrec > 0 && (!records || !out)))
    return d ? set_err(d->ctx, GF_ERR_ARG, "gf_knn_attach_strings: bad argument") : GF_ERR_ARG;
  gf_ctx* ctx = d->ctx;
  int st = bind(ctx);
  if (st || nrec == 0) return st;
  GF_HIP_CHECK(ctx, launch_knn_attach_strings(ctx, k, d->idmap, d->arena, d->size, records, nrec, cap_bytes, out));
  return GF_OK;
}

extern "C" int gf_knn_merge_dev_strings(gf_ctx* ctx, int32_t k, int64_t cap_bytes, const void* records, int32_t nrec,
                                        int32_t nwin, int32_t layout, void* results) {
  if (!ctx || k < 1 || k > kMaxKLarge || cap_bytes < 0 || cap_bytes > (int64_t)UINT32_MAX || nrec < 1 ||
      nrec > kMaxMergeRecs || nwin < 1 || nwin > 65535 || !records || !results ||
      (layout != GF_MERGE_SHARD_MAJOR && layout != GF_MERGE_WINDOW_MAJOR))
    return set_err(ctx, GF_ERR_ARG, "gf_knn_merge_dev_strings: bad argument");
  int st = bind(ctx);
  if (st) return st;
  const size_t sb = str_record_bytes(k, cap_bytes);
  const size_t rec_stride = layout == GF_MERGE_SHARD_MAJOR ? (size_t)nwin * sb : sb;
  const size_t win_stride = layout == GF_MERGE_SHARD_MAJOR ? sb : (size_t)nrec * sb;
  void* scratch = ctx_scratch(ctx, strmerge_bytes(nrec, k) * (size_t)nwin, &st);
  if (st) return st;
  GF_HIP_CHECK(ctx, launch_knn_merge_strings(ctx, k, cap_bytes, records, nrec, rec_stride, nwin, win_stride, results,
                                             scratch));
  return GF_OK;
}

extern "C" int gf_knn_string_record_decode(const void* rec, int32_t k, int64_t cap_bytes, int32_t* status,
                                           int64_t* objID, double* dist, int64_t* idx, char* buf, int64_t buf_cap,
                                           int64_t* offs, int32_t* n_out) {
  if (!rec || k < 1 || cap_bytes < 0 || !status || !n_out || !offs) return GF_ERR_ARG;
  const gf_knn_header* h = (const gf_knn_header*)rec;
  const double* d = (const double*)(h + 1);
  const int64_t* o = (const int64_t*)(d + k);
  const int64_t* i = o + k;
  const char* side = (const char*)rec + gf_knn_result_bytes(k);
  const int32_t side_status = *(const int32_t*)side;
  const uint32_t* off = (const uint32_t*)(side + 16);
  const char* bytes = (const char*)off + str_side_off(k);
  *status = h->status != 0 ? h->status : (side_status != 0 ? GF_KNN_STATUS_FOREIGN_KEYS : 0);
  *n_out = *status == 0 ? h->n : 0;
  int64_t at = 0;
  char num[32];
  for (int32_t j = 0; j < *n_out; ++j) {
    offs[j] = at;
    const int64_t key = o[j];
    const char* p = num;
    size_t len = 0;
    if (key < GF_OBJID_NUMERIC_MIN) {  // a dictionary String: from the record's own sidecar
      p = bytes + off[j];
      len = off[j + 1] - off[j];
    } else if (key != GF_OBJID_NULL) {
      len = (size_t)snprintf(num, sizeof num, "%lld", (long long)key);  // Long.toString
    }
    if (buf && at + (int64_t)len <= buf_cap) std::memcpy(buf + at, p, len);
    at += (int64_t)len;
    if (objID) objID[j] = key;
    if (dist) dist[j] = d[j];
    if (idx) idx[j] = i[j];
  }
  offs[*n_out] = at;
  return at > buf_cap || (at > 0 && !buf) ? GF_ERR_CAPACITY : GF_OK;
}
