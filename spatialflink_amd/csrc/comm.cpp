// comm.cpp -- RCCL behind the C ABI: the windowAll funnel across GPUs.
//
// The reference funnels every subtask's per-cell heaps through one parallelism-1 windowAll
// (PointPointKNNQuery.java:198-200) whose merge keeps the k smallest distinct objIDs
// (KNNQuery.java:213-272).  Sharded over the GPUs of a node (cell-column bands)
// that funnel is one all-gather of each GPU's top-k RECORDS over xGMI followed by the same
// deterministic top-k-distinct merge on every GPU (gf_knn_merge_dev_batch /
// gf_knn_merge_dev_strings), so every rank holds the window's result.
//
// RCCL is opened on first use (dlopen of librccl.so.1): processes that never build a
// communicator -- a one-GPU Flink job, the CPU test suite -- do not map the library, and a
// process that already holds RCCL (torch loads its own librccl.so.1) shares that copy.
// Communicators: ncclCommInitRank (one process per GPU, the id broadcast by the caller's own
// control plane -- torch.distributed, Flink's broadcast, a shared file) or ncclCommInitAll (one
// process driving every GPU).  Collectives are enqueued on the context's
// stream; nothing here synchronises the host.
#define GF_TU_NAME comm_cpp
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "gf_internal.hpp"

using namespace gf;

namespace {

struct Rccl {
  void* so = nullptr;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl& rccl_state() {
  static Rccl R;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names)
      if ((R.so = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
    if (!R.so) {
      const char* e = dlerror();
      R.err = std::string("dlopen(librccl.so.1): ") + (e ? e : "not found");
      return;
    }
    bool ok = true;
    auto sym = [&](auto& fp, const char* name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(R.so, name));
      if (!fp) { ok = false; R.err = std::string("librccl.so.1 lacks ") + name; }
    };
    sym(R.GetUniqueId, "ncclGetUniqueId");
    sym(R.CommInitRank, "ncclCommInitRank");
    sym(R.CommInitAll, "ncclCommInitAll");
    sym(R.CommDestroy, "ncclCommDestroy");
    sym(R.CommAbort, "ncclCommAbort");
    sym(R.CommGetAsyncError, "ncclCommGetAsyncError");
    sym(R.AllGather, "ncclAllGather");
    sym(R.GroupStart, "ncclGroupStart");
    sym(R.GroupEnd, "ncclGroupEnd");
    sym(R.GetErrorString, "ncclGetErrorString");
    if (!ok) { dlclose(R.so); R.so = nullptr; }
  });
  return R;
}

// the loaded library, or null (rccl_state().err says why)
Rccl* rccl() {
  Rccl& R = rccl_state();
  return R.so ? &R : nullptr;
}

// why this thread's last communicator-less call (unique id, create, create_all) failed
thread_local std::string t_comm_err;

int fail(const std::string& msg, int st = GF_ERR_COMM) {
  t_comm_err = msg;
  return st;
}

}  // namespace

struct gf_comm {
  ncclComm_t comm = nullptr;
  int32_t nranks = 0, rank = 0;
  int device = 0;
  // communicators created together by one gf_comm_create_all share a nonzero clique id (the
  // group exchange needs one whole clique); gf_comm_create's are 0.  aborted: an exchange failed
  // inside an RCCL group and the clique was aborted (every later call is refused)
  uint64_t clique = 0;
  bool aborted = false;
  std::string last_error;
  // device buffers of the exchange, grown on demand: the gathered records of every rank, and
  // this rank's string records (gf_knn_attach_strings' output) for the String exchange
  void* gather = nullptr;
  size_t gather_bytes = 0;
  void* strings = nullptr;
  size_t strings_bytes = 0;
};

static int comm_err(gf_comm* c, gf_ctx* ctx, const std::string& msg) {
  if (c) c->last_error = msg;
  if (ctx) ctx->last_error = msg;
  return GF_ERR_COMM;
}

static int nccl_check(gf_comm* c, gf_ctx* ctx, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return GF_OK;
  Rccl* R = rccl();
  return comm_err(c, ctx, std::string(what) + ": " + (R ? R->GetErrorString(r) : "RCCL unavailable"));
}

// a grow-only device buffer of the communicator; the work queued on `stream` (the only stream
// that uses the comm's buffers, see the header) is drained before the old one is freed
static int comm_buffer(gf_comm* c, gf_ctx* ctx, void** buf, size_t* have, size_t bytes) {
  if (bytes <= *have) return GF_OK;
  GF_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
  if (*buf) hipFree(*buf);
  *buf = nullptr;
  *have = 0;
  const size_t sz = std::max(bytes + bytes / 4, (size_t)1 << 16);
  hipError_t e = hipMalloc(buf, sz);
  if (e != hipSuccess) {
    int st = hip_err(ctx, e, "hipMalloc(comm buffer)");
    c->last_error = ctx->last_error;
    return st;
  }
  *have = sz;
  return GF_OK;
}

extern "C" int gf_comm_available(void) { return rccl() != nullptr; }

extern "C" int gf_comm_unique_id(uint8_t* id) {
  if (!id) return fail("gf_comm_unique_id: null id", GF_ERR_ARG);
  Rccl* R = rccl();
  if (!R) return fail(rccl_state().err);
  static_assert(sizeof(ncclUniqueId) == GF_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  const ncclResult_t r = R->GetUniqueId(&u);
  if (r != ncclSuccess) return fail(std::string("ncclGetUniqueId: ") + R->GetErrorString(r));
  std::memcpy(id, &u, sizeof u);
  return GF_OK;
}

extern "C" int gf_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int device, gf_comm** out) {
  if (!out) return GF_ERR_ARG;
  *out = nullptr;
  if (!id || nranks < 1 || nranks > kMaxMergeRecs || rank < 0 || rank >= nranks || device < 0)
    return fail("gf_comm_create: bad argument", GF_ERR_ARG);
  Rccl* R = rccl();
  if (!R) return fail(rccl_state().err);
  // ncclCommInitRank binds the communicator to the CURRENT device; the caller's is restored
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
    return fail("gf_comm_create: hipSetDevice failed", GF_ERR_HIP);
  gf_comm* c = new gf_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  const ncclResult_t r = R->CommInitRank(&c->comm, nranks, u, rank);
  hipSetDevice(prev);
  if (r != ncclSuccess) {
    delete c;
    return fail(std::string("ncclCommInitRank: ") + R->GetErrorString(r));
  }
  *out = c;
  return GF_OK;
}

extern "C" int gf_comm_create_all(int32_t ndev, const int* devices, gf_comm** out) {
  if (!out || ndev < 1 || ndev > kMaxMergeRecs || !devices) return fail("gf_comm_create_all: bad argument", GF_ERR_ARG);
  for (int32_t i = 0; i < ndev; ++i) out[i] = nullptr;
  Rccl* R = rccl();
  if (!R) return fail(rccl_state().err);
  std::vector<ncclComm_t> comms(ndev, nullptr);
  const ncclResult_t r = R->CommInitAll(comms.data(), ndev, devices);
  if (r != ncclSuccess) return fail(std::string("ncclCommInitAll: ") + R->GetErrorString(r));
  static std::atomic<uint64_t> next_clique{1};
  const uint64_t clique = next_clique.fetch_add(1);
  for (int32_t i = 0; i < ndev; ++i) {
    gf_comm* c = new gf_comm();
    c->comm = comms[i];
    c->nranks = ndev;
    c->rank = i;
    c->device = devices[i];
    c->clique = clique;
    out[i] = c;
  }
  return GF_OK;
}

extern "C" void gf_comm_destroy(gf_comm* c) {
  if (!c) return;
  hipSetDevice(c->device);
  hipDeviceSynchronize();  // exchanges still queued read the buffers
  if (c->comm && !c->aborted)
    if (Rccl* R = rccl()) R->CommDestroy(c->comm);
  if (c->gather) hipFree(c->gather);
  if (c->strings) hipFree(c->strings);
  delete c;
}

extern "C" int gf_comm_info(const gf_comm* c, int32_t* nranks, int32_t* rank, int* device) {
  if (!c) return GF_ERR_ARG;
  if (nranks) *nranks = c->nranks;
  if (rank) *rank = c->rank;
  if (device) *device = c->device;
  return GF_OK;
}

extern "C" const char* gf_comm_last_error(const gf_comm* c) {
  if (c) return c->last_error.c_str();
  // null: why this thread's last unique-id / create call failed, else why RCCL did not load
  return !t_comm_err.empty() ? t_comm_err.c_str() : rccl_state().err.c_str();
}

extern "C" int gf_comm_check(gf_comm* c) {
  if (!c) return GF_ERR_ARG;
  Rccl* R = rccl();
  ncclResult_t a = ncclSuccess;
  if (!R || R->CommGetAsyncError(c->comm, &a) != ncclSuccess) return comm_err(c, nullptr, "ncclCommGetAsyncError");
  return nccl_check(c, nullptr, a, "asynchronous RCCL error");
}

// ---- the kNN exchange --------------------------------------------------------------------------
static int exchange_args_ok(gf_comm* c, gf_ctx* ctx, int32_t k, const void* records, int32_t nwin, const void* merged,
                            const char* what) {
  if (!c || !ctx || k < 1 || k > kMaxKLarge || nwin < 1 || nwin > 65535 || !records || !merged)
    return set_err(ctx, GF_ERR_ARG, std::string(what) + ": bad argument");
  if (c->aborted) return comm_err(c, ctx, std::string(what) + ": the communicator was aborted after a failed group");
  if (ctx->device != c->device)
    return set_err(ctx, GF_ERR_ARG, std::string(what) + ": the context's device is not the communicator's");
  return bind(ctx);
}

// all-gather of nwin records of `rb` bytes per rank into c->gather (shard-major: rank s's window
// w at (s * nwin + w) * rb -- the layout GF_MERGE_SHARD_MAJOR reads)
static int gather_records(gf_comm* c, gf_ctx* ctx, const void* mine, size_t bytes) {
  int st = comm_buffer(c, ctx, &c->gather, &c->gather_bytes, bytes * (size_t)c->nranks);
  if (st) return st;
  return nccl_check(c, ctx, rccl()->AllGather(mine, c->gather, bytes, ncclUint8, c->comm, ctx->stream), "ncclAllGather");
}

static int32_t merge_layout(const gf_comm* c) {
  // a one-rank communicator's records are this context's own: its dictionary keys merge as is
  return GF_MERGE_SHARD_MAJOR | (c->nranks > 1 ? GF_MERGE_FOREIGN_KEYS : 0);
}

extern "C" int gf_knn_exchange_batch(gf_comm* c, gf_ctx* ctx, int32_t k, const void* records, int32_t nwin,
                                     void* merged) {
  int st = exchange_args_ok(c, ctx, k, records, nwin, merged, "gf_knn_exchange_batch");
  if (st) return st;
  if (!rccl()) return comm_err(c, ctx, "RCCL unavailable");
  const size_t rb = gf_knn_result_bytes(k);
  if ((st = gather_records(c, ctx, records, rb * (size_t)nwin))) return st;
  return gf_knn_merge_dev_batch(ctx, k, c->gather, c->nranks, nwin, merge_layout(c), merged);
}

extern "C" int gf_knn_exchange_strings_batch(gf_comm* c, gf_objid_dict* dict, int32_t k, int64_t cap_bytes,
                                             const void* records, int32_t nwin, void* merged) {
  gf_ctx* ctx = dict ? dict->ctx : nullptr;
  int st = exchange_args_ok(c, ctx, k, records, nwin, merged, "gf_knn_exchange_strings_batch");
  if (st) return st;
  if (cap_bytes < 0 || cap_bytes > (int64_t)UINT32_MAX)
    return set_err(ctx, GF_ERR_ARG, "gf_knn_exchange_strings_batch: bad cap_bytes");
  if (!rccl()) return comm_err(c, ctx, "RCCL unavailable");
  const size_t sb = gf_knn_string_record_bytes(k, cap_bytes);
  if ((st = comm_buffer(c, ctx, &c->strings, &c->strings_bytes, sb * (size_t)nwin))) return st;
  if ((st = gf_knn_attach_strings(dict, k, records, nwin, cap_bytes, c->strings))) return st;
  if ((st = gather_records(c, ctx, c->strings, sb * (size_t)nwin))) return st;
  return gf_knn_merge_dev_strings(ctx, k, cap_bytes, c->gather, c->nranks, nwin, GF_MERGE_SHARD_MAJOR, merged);
}

extern "C" int gf_knn_exchange_group(int32_t n, gf_comm* const* comms, gf_ctx* const* ctxs, int32_t k,
                                     const void* const* records, int32_t nwin, void* const* merged) {
  if (n < 1 || !comms || !ctxs || !records || !merged) return GF_ERR_ARG;
  const size_t rb = gf_knn_result_bytes(k);
  int st;
  // Everything that can fail is checked BEFORE ncclGroupStart: the group must hold
  // one all-gather for every rank of ONE clique -- issued for a subset, the launched kernels
  // would wait forever for peers that never join, and the next sync would hang the device.
  std::vector<uint8_t> seen((size_t)n, 0);
  for (int32_t i = 0; i < n; ++i) {
    if (!comms[i] || !ctxs[i]) return GF_ERR_ARG;
    if ((st = exchange_args_ok(comms[i], ctxs[i], k, records[i], nwin, merged[i], "gf_knn_exchange_group"))) return st;
    const gf_comm* c = comms[i];
    const bool whole = c->nranks == n && (n == 1 || (c->clique != 0 && c->clique == comms[0]->clique)) &&
                       c->rank >= 0 && c->rank < n && !seen[(size_t)c->rank];
    if (!whole)
      return set_err(ctxs[i], GF_ERR_ARG,
                     "gf_knn_exchange_group: the communicators must be one whole gf_comm_create_all clique, "
                     "each rank once");
    seen[(size_t)c->rank] = 1;
    if ((st = comm_buffer(comms[i], ctxs[i], &comms[i]->gather, &comms[i]->gather_bytes,
                          rb * (size_t)nwin * (size_t)comms[i]->nranks)))
      return st;
  }
  Rccl* R = rccl();
  if (!R) return comm_err(comms[0], ctxs[0], "RCCL unavailable");
  // one thread drives every communicator: the collectives form one group (RCCL launches them
  // together; issued one by one, the first would wait for peers that are never launched)
  if ((st = nccl_check(comms[0], ctxs[0], R->GroupStart(), "ncclGroupStart"))) return st;
  int first_err = GF_OK;
  for (int32_t i = 0; i < n && !first_err; ++i) {
    if (hipSetDevice(ctxs[i]->device) != hipSuccess) { first_err = hip_err(ctxs[i], hipErrorInvalidDevice, "hipSetDevice"); break; }
    first_err = nccl_check(comms[i], ctxs[i],
                           R->AllGather(records[i], comms[i]->gather, rb * (size_t)nwin, ncclUint8, comms[i]->comm,
                                        ctxs[i]->stream),
                           "ncclAllGather");
  }
  const int end_err = nccl_check(comms[0], ctxs[0], R->GroupEnd(), "ncclGroupEnd");
  if (first_err || end_err) {
    // a partial group may have launched some all-gathers whose peers never arrive: abort the
    // whole clique so its kernels are torn down instead of spinning (every later call refused)
    for (int32_t i = 0; i < n; ++i) {
      if (!comms[i]->aborted) R->CommAbort(comms[i]->comm);
      comms[i]->aborted = true;
    }
    return first_err ? first_err : end_err;
  }
  for (int32_t i = 0; i < n; ++i)
    if ((st = gf_knn_merge_dev_batch(ctxs[i], k, comms[i]->gather, comms[i]->nranks, nwin, merge_layout(comms[i]),
                                     merged[i])))
      return st;
  return GF_OK;
}
