// gf_internal.hpp -- context, plans and kernel launch interfaces of libgeoflink_hip.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/geoflink_hip.h"
#include "gf_text.hpp"
#include "gf_numerics.hpp"

// ---------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------
struct gf_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;
  std::string last_error;
  int timing = 0;  // bitmask of GF_K_* kernels to time
  int timing_period = 1;              // time every period-th launch of each kernel
  int64_t timing_seq[GF_K_COUNT] = {};
  struct Ev { hipEvent_t a, b; int kid; };
  std::vector<Ev> pending;
  std::vector<hipEvent_t> pool;
  double acc_ms[GF_K_COUNT] = {};
  int64_t acc_n[GF_K_COUNT] = {};
  // grow-only scratch (device) and pinned host staging
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  void* pinned = nullptr;
  size_t pinned_bytes = 0;
  int num_cus = 256;
  int join_legacy = 0;  // testing: force the original (unbucketed) join probe
  int join_coarse = 0;  // testing: the row path without sub-cells
  int join_stream = 0;  // experiment: the fine path's streaming probe (query side bucketed only)
  int geojson_walk = 0; // testing: every GeoJSON line takes the member-by-member walk
  int geojson_wave = 0; // GeoJSON: the wave-per-line scan instead of the lane locator (measured slower)
  unsigned long long* geojson_check = nullptr;  // GF_FLAG_GEOJSON_CHECK: the 4 counters (device; null: off)
  int64_t csv_mean_line[2] = {0, 0};  // per format (CSV, GeoJSON): the last call's mean line length (sizes the next one's LDS staging)
  int join_async_done = 0;  // gf_join_pp_async: the packing kernel wrote the count
  double join_ppp = 0.0;  // pairs per ordinary point of the last join (sizes the output chunks)
  hipStream_t aux = nullptr;   // kNN depth >= 3: the second stream of windows in flight (created on first use)
  hipStream_t aux2 = nullptr;  // kNN depth 4: the third
  gf_objid_dict* dict = nullptr;  // the context's default objID dictionary (created on first use)
  // gf_bitmap_to_indices_async: block tickets + look-back status (grown on demand)
  unsigned long long* expand_ticket = nullptr;
  unsigned long long expand_base = 0;
  unsigned long long* expand_status = nullptr;
  int64_t expand_status_cap = 0;
  uint32_t expand_epoch = 0;
  unsigned long long* join_gctr = nullptr;  // row-bucketed join: reserved output positions (zero between calls)
  unsigned long long* join_hint = nullptr;  // mapped pinned: the pair count of the last join (async too)
  void* csv_head = nullptr;                 // mapped pinned: the ingest head (CsvHead), written by csv_error_kernel
  uint64_t* join_hist = nullptr;            // band probe: the last join's pairs, points, slice start per block, did-not-fit ([3 * blocks + 1], zero: none)
  unsigned long long* join_ovf = nullptr;   // band probe: overflow counter (zero between calls)
  int64_t join_hint_no = 0;                 // ordinary points of that join
};

// objID dictionary (objid.cpp): device hash table + arena, batch buffers, host mirror for decode
struct gf_objid_dict {
  gf_ctx* ctx = nullptr;
  void* slots = nullptr;          // gf::DictSlot[cap]
  uint64_t cap = 0;               // power of two
  char* arena = nullptr;
  uint64_t arena_cap = 0;
  unsigned long long* counters = nullptr;  // [0] arena bytes used, [1] pending count, [2] csv count, [3] csv bytes
  unsigned long long* idmap = nullptr;
  uint64_t idmap_cap = 0;
  int64_t size = 0;               // ids assigned
  uint32_t round = 2;
  void* work[3] = {nullptr, nullptr, nullptr};  // gf::DictWork: the batch, two pending lists
  uint64_t work_cap = 0;
  uint32_t* slot_of = nullptr;
  uint32_t* flag = nullptr;
  uint32_t* rank = nullptr;
  uint32_t* tmp = nullptr;
  uint64_t line_cap = 0;
  char* src = nullptr;            // host intern: uploaded Strings
  uint64_t src_cap = 0;
  // host mirror of idmap / arena, extended on demand by gf_objid_decode
  std::vector<unsigned long long> h_idmap;
  std::vector<char> h_arena;
};

namespace gf {

int set_err(gf_ctx* ctx, int code, const std::string& msg);
int hip_err(gf_ctx* ctx, hipError_t e, const char* what);
void* ctx_scratch(gf_ctx* ctx, size_t bytes, int* status);
int sync_aux(gf_ctx* ctx);  // synchronize the kNN pipeline's extra streams (depth >= 3)
void* ctx_pinned(gf_ctx* ctx, size_t bytes, int* status);
int bind(gf_ctx* ctx);

#define GF_HIP_CHECK(ctx, call)                                   \
  do {                                                            \
    hipError_t _e = (call);                                       \
    if (_e != hipSuccess) return ::gf::hip_err((ctx), _e, #call); \
  } while (0)

// RAII event pair around one kernel launch when ctx->timing is on.
struct KTimer {
  gf_ctx* ctx;
  int kid;
  hipEvent_t a = nullptr, b = nullptr;
  KTimer(gf_ctx* c, int k);
  ~KTimer();
};

// ---------------------------------------------------------------------------------------
// kernel argument blocks
// ---------------------------------------------------------------------------------------
constexpr int kBlock = 256;         // streaming kernels: 4 waves
constexpr int kMaxK = 512;          // largest k of the one-block select (larger k: the sorted path)
constexpr int kFusedSelectMaxK = 256;  // largest k of the select fused into block 0 of a scan launch
constexpr int kSampleBlocks = 128;  // kNN sample: 128 blocks x 2048 points = 256K points
constexpr int kSamplePerBlock = 2048;
constexpr int64_t kSampleMinN = 1 << 20;

// A block barrier for LDS hand-offs only: waits for this wave's LDS operations (lgkmcnt(0)), not
// for its outstanding global loads -- __syncthreads() also drains vmcnt, which lands a tile loop's
// prefetched next-tile loads at the current tile's first barrier.  Global stores are not ordered
// by it either: use it only where the threads exchange data through LDS.
__device__ __forceinline__ void lds_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt(63) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Intra-wave LDS hand-off (r06): lanes of ONE wave write LDS slots (ballot
// compaction: a lane writes slot base + its rank among the writers) and lanes of the same wave
// then read slots OTHER lanes wrote.  The hardware runs a wave's LDS instructions in order, so no
// wait is needed -- but the compiler reasons per thread: a lane's write to slot p and its later
// read of slot q != p are independent to it, so without a wave-scope fence it may move the read
// above the write (or the write below the read) and the reading lane sees the slot's OLD contents.
// That is the cause of round 5's lost C3 hits: the in-stream test variant read the queued points'
// coordinates from a per-wave LDS ring, each point read by a group of 8 lanes that had not written
// it.  Every debug build that removed the cross-lane read lost nothing -- coordinates read from
// global memory (no LDS hand-off), a one-lane walk (each lane read the slot it had written itself:
// a same-thread dependency the compiler keeps) -- and accepting every candidate only hid the stale
// coordinates.  This marks every such hand-off: release + acquire at wavefront scope around a wave
// barrier; the fences emit no instruction (wavefront scope), the barrier appears in the ISA as
// "; wave barrier" (tests/test_isa_handoff.py checks the hand-offs carry it).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// single-query classification (exact, from host-side cell thresholds)
struct QueryRect {
  AxisIv cgx, cgy;   // valid cells within c layers
  AxisIv gx, gy;     // guaranteed rect (g > 0: valid cells within g; g == 0: the query cell)
  int g_any;         // g >= 0 and the guaranteed rect is non-empty
  double minX, minY; // NaN coordinates classify as cell 0 (Java (int)NaN == 0)
};

// device state of a kNN plan (zeroed at creation)
struct KnnState {
  uint32_t hist[kDistBins];
  uint32_t ticket;
  uint32_t pad;
  double T;          // distance threshold of the current window (<= r)
  double s_pre;      // prefilter bound on dx*dx+dy*dy for T
  unsigned long long count;  // candidates appended (may exceed capacity)
  double hint_T;     // next window's threshold guess (2 x this window's k-th distance); 0 = none
  unsigned long long tr[4];  // GF_TRACE builds only: sample start, scan first start / last end
  unsigned long long maybe;  // polygon queries: points past the cheap prefilter (refined next)
};

struct KnnScanArgs {
  const double* x;
  const double* y;
  const int64_t* objID;
  int64_t begin, end;   // [begin, end), begin even
  double qx, qy;
  QueryRect qr;
  double T, s_pre;      // used when !use_state
  int use_state;
  int metric;
  KnnState* st;
  double* cand_d;
  uint32_t* cand_i;
  int64_t* cand_o;
  unsigned long long cap;
};

struct KnnSampleArgs {
  const double* x;
  const double* y;
  int64_t n;
  double qx, qy;
  QueryRect qr;
  double r, s_r;
  int32_t k;
  int metric;
  int use_hint;         // take st->hint_T when set instead of sampling
  KnnState* st;
};

// one polygon set in device memory (CSR: polygon -> rings -> vertices; rings closed)
struct PolyView {
  const int32_t* ring_off;
  const int32_t* vert_off;
  const double* vx;
  const double* vy;
  const double* ring_env;  // [nrings*4] minx, maxx, miny, maxy
  int metric;
  const uint8_t* rect;     // [npoly] 1: one-ring axis-aligned rectangle (nullable)
};

// polygon-query kNN (PointPolygonKNNQuery): scan / sample arguments
struct KnnPolyArgs {
  const double* x;
  const double* y;
  const int64_t* objID;
  int64_t begin, end;   // points [begin, end)
  QueryRect qr;         // C u G of the polygon's bbox cells
  PolyView poly;        // the query polygon (index 0)
  double bbox[4];       // shell envelope x1, y1, x2, y2
  int approx;           // bbox distance (DistanceFunctions.java:150-200) instead of JTS
  double r;
  int32_t k;
  int use_state;        // scan: T = st->T (set by the sample); else T = r
  int use_hint;         // sample: take st->hint_T when set
  KnnState* st;
  double* cand_d;
  uint32_t* cand_i;
  int64_t* cand_o;
  unsigned long long cap;
  uint32_t* maybe_i;    // scan -> refine: indices past the prefilter (cap entries)
};

struct KnnSelectArgs {
  KnnState* st;
  const double* cand_d;
  const uint32_t* cand_i;
  const int64_t* cand_o;
  unsigned long long cap;
  int use_state;
  double T;             // when !use_state
  double r;
  int32_t k;
  int write_hint;       // store 2 x k-th distance as the next window's threshold guess
  int64_t idx_base;     // added to the window-local index in the record
  void* result;         // gf_knn_header + dist[k] + objID[k] + idx[k]
};

// partials: [kRangeMaxParts] (hits, multiset size) pairs, then the finalisation ticket
constexpr int kRangeMaxParts = 4096;
constexpr int kRangeTicketSlot = 2 * kRangeMaxParts;

// range: classification + tester
struct RangeArgs {
  const double* x;
  const double* y;
  int64_t n;
  uint64_t* bitmap;
  uint64_t* multi;           // nullable
  uint64_t* partials;        // [gridDim.x * 2]: hits, multiset size per block
  // nullable: the window's counts, summed by the last block of its last kernel.  Its ticket
  // sits right after the partials (kRangeTicketSlot) and the partial count follows from the
  // grid, so only this pointer is added to the arguments: every extra argument the scan keeps
  // live through its loop costs SGPRs (spilled into VGPR lanes, the 10M-point scan ran 2x slower
  // with the ticket and part count as arguments too)
  int64_t* counts;
  int32_t nq;                // multiplicity for approximate point-point
  // arithmetic classification (single query point)
  QueryRect qr;
  // table classification
  int32_t grid_n;
  double minX, minY, cl;
  const uint8_t* table;      // [n*n]: 0 none, 1 test, 2 accept, 3 inside (accept unless NaN)
  const uint32_t* rows;      // [n] first | last << 16 column of a non-none class per row
  const uint32_t* rowoff;    // [n] offset of each row's span in `spans`
  const uint8_t* spans;      // class table restricted to the row spans (concatenated)
  int32_t span_bytes;
  int32_t span_lds;          // spans small enough to stage in LDS
  const double* xt;          // [n+1] exact thresholds first_at_least(c) per axis (n <= 2048; else null)
  const double* yt;
  double x_lo, x_hi, y_lo, y_hi;  // xt[0], xt[n], yt[0], yt[n]
  double sx_lo, sx_hi;       // xt[first], xt[last + 1] over every row's span: x outside => no class
  double sy_lo, sy_hi;       // yt[first], yt[last + 1] over the rows holding a class
  int span_mode;             // deferred tests with the span prefilter (range_kernel DEFER 3)
  double inv_cl;
  const int32_t* extra;      // [n_extra*4]: x0, x1, y0, y1 (inclusive) accepted out-of-grid cells
  int32_t n_extra;
  const int32_t* cand_off;   // [n*n+1] objects to test per cell (CSR); null => test all
  const int32_t* cand_list;
  // tester
  int approx;
  int metric;
  double r, s_r;
  double thr;                // the point-point test's one bound: s_r (metric 0, on dx^2 + dy^2) or r (hypot)
  double qx0, qy0;           // the query point (ARITH mode)
  const double* qx;          // point-point queries (device)
  const double* qy;
  int32_t npoly;
  const int32_t* ring_off;   // polygons (device)
  const int32_t* vert_off;
  const double* vx;
  const double* vy;
  const double* bbox;        // [npoly*4] x1, y1, x2, y2 (shell envelope)
  const double* ring_env;    // [nrings*4] minx, maxx, miny, maxy
  // deferred candidate tests (table modes): scan appends, range_test_kernel drains
  uint32_t* queue;           // [blocks * seg_cap] point indices, a segment per scan block; null => inline
  uint32_t* queue_count;     // [blocks] entries per segment
  double* queue_xy;          // [2 * blocks * seg_cap] the queued points' coordinates
  int64_t seg_cap;           // points one scan block visits at most
  int32_t drain_lanes;       // testing (gf_range_plan_set_drain_lanes): the block-end drain runs on the first
                             // drain_lanes lanes of each wave only (0 = all) -- drain_own_queue takes any exec mask
  const uint8_t* rect;       // [npoly] axis-aligned rectangle shells without holes (nullable)
  // point-polygon join: bbox cells per polygon (x0, x1, y0, y1) and the layer counts
  const int32_t* brect;
  int32_t g_layers, c_layers;
};

// launchers (return hipError_t of the launch)
hipError_t launch_assign(gf_ctx* ctx, const gf_grid* g, const gf_points* p, int32_t* cx, int32_t* cy);
hipError_t launch_histogram(hipStream_t s, const uint32_t* keys, int64_t n, uint32_t* hist);
// K2: stable LSD radix bucketing (k_points.hip)
constexpr int kRadixMaxBits = 9;  // digit bits per pass (<=)
constexpr int kRadixMaxDigits = 1 << kRadixMaxBits;
constexpr int kRadixThreads = 1024;
constexpr int kRadixTile = 8192;  // points per scatter tile (16 waves x 512)
#ifndef GF_BUCKET_BITS
#define GF_BUCKET_BITS 9
#endif
constexpr int kBucketBits = GF_BUCKET_BITS;  // K2 (gf_bucket_by_cell): digit bits per pass, <= kRadixMaxBits
static_assert(kBucketBits >= 1 && kBucketBits <= kRadixMaxBits, "K2 digit bits");
struct RadixArgs {
  const double* x;          // pass 0 input (kin == null): keys from the cells of x, y
  const double* y;
  int64_t n;
  double minX, minY, cl;
  int32_t gn;
  const uint32_t* kin;      // later passes: keys, point indices
  const uint32_t* vin;
  uint32_t* kout;
  uint32_t* vout;
  int shift, bits;          // digit = (key >> shift) & ((1 << bits) - 1)
  int nblk;                 // blocks (chunks of whole tiles)
  uint32_t* M;              // stage 0: [digits][blocks]; stage 2: cell_start[0 .. gn*gn + 1] (output)
  const uint32_t* Ms;       // stage 1: the exclusive scan of M
  const uint32_t* n_dev;    // non-null: the item count is min(n, *n_dev), read on the device
  int32_t nbands;           // > 0: pass 0's key is the point's column band (gf_shard_by_columns), not its cell
  int32_t band_lo[64];      // the bands' first columns, ascending (band_lo[0] is taken as -inf)
  uint32_t bins;            // stage 2: cell_start entries - 1 (0: gn * gn + 1)
  int32_t tile;             // points per scatter tile (radix_tile()); chunks are whole tiles
  // row mode (gf_bucket_by_cell, gn + 1 <= 512 rows): pass A's key is row << 9 | column (row = cy,
  // gn for the out-of-grid bucket) sorted by row; pass B sorts every row's SEGMENTS by column
  int32_t rowmode;          // pass 0 keys are row keys
  int32_t seg;              // > 0: pass B -- blocks are row segments of <= seg points
  const uint32_t* MsA;      // pass B: pass A's scanned matrix (row r = [MsA[r nblkA], MsA[(r+1) nblkA]))
  int32_t nblkA;
  uint32_t* cstart;         // pass B: cell_start[0 .. gn*gn + 1], written by each row's first segment
  // row mode (r06): pass A's scatter writes each point's COLUMN as u16 (kout16; the row is its
  // position's row) and pass B reads those (kin16): 2 B instead of 4 per point written and read twice
  uint16_t* kout16;
  const uint16_t* kin16;
  int32_t self_count;       // pass B: a one-segment row's scatter block counts its columns (no histogram read)
  int32_t rowsort;          // pass B: one-segment rows sorted whole by radix_row_sort_kernel (the others by segments)
  // rowsort: a device word, zeroed by pass A's histogram, set by the row sort when some row has
  // several segments; pass B's segment kernels (and its scan) return at once while it is 0
  uint32_t* multiseg;
};
// scatter block size: 1024 threads (one 8192-point tile per block, one block per CU) or 512
// (4096-point tiles, two blocks per CU: one block's LDS phases overlap the other's memory);
// GF_RADIX_NT selects it (A/B), default below
int radix_threads();
inline int radix_tile() { return radix_threads() / 64 * 512; }
inline int radix_max_blocks(int num_cus) { return num_cus * (1024 / radix_threads()); }
int radix_row_sort_cap();  // k_points.hip: the largest row radix_row_sort_kernel sorts whole
constexpr int kMaxShardBands = 64;
size_t radix_scatter_lds_bytes();
hipError_t launch_gather_points(hipStream_t s, const gf_points& in, const uint32_t* perm, int64_t begin, int64_t m,
                                double* ox, double* oy, int64_t* oo, int64_t* ot);
// stage 0 histogram, 1 scatter, 2 cell_start from the sorted kout (every bucket's first position),
// 3 row-segment histogram (pass B of row mode; `blocks` = the segment bound)
hipError_t launch_radix(gf_ctx* ctx, int stage, const RadixArgs& a, int blocks);
// exclusive scan: out[0..L] (out[L] = total); tmp >= scan_tmp_elems(L) uint32
size_t scan_tmp_elems(int64_t L);
hipError_t launch_exclusive_scan(hipStream_t s, const uint32_t* in, int64_t L, uint32_t* out, uint32_t* tmp);
hipError_t launch_word_popcounts(hipStream_t s, const uint64_t* bitmap, int64_t words, uint32_t* pc);
hipError_t launch_expand_bitmap(hipStream_t s, const uint64_t* bitmap, int64_t words, int64_t n,
                                const uint32_t* off, uint32_t* idx, int64_t cap);
// single-pass compaction state (per context): block tickets and look-back status words
// decoupled look-back status words: epoch (26 bits) | flag (2) | value (36)
constexpr uint64_t kLbAgg = 1ull, kLbInc = 2ull;  // status flags: aggregate / inclusive prefix
__device__ __forceinline__ uint64_t lb_pack(uint32_t epoch, uint64_t flag, uint64_t v) {
  return ((uint64_t)(epoch & 0x3FFFFFFu) << 38) | (flag << 36) | v;  // v < 2^36
}
struct ExpandState {
  unsigned long long* ticket;  // grows across launches; this launch's blocks take [base, base + blocks)
  unsigned long long base;
  unsigned long long* status;  // [blocks] epoch-tagged aggregate / inclusive prefix
  uint32_t epoch;
};
constexpr int kExpandWords = 1024;  // bitmap words (= threads) per expand_async block
int64_t expand_blocks(int64_t words);
// single-pass exclusive scan (decoupled look-back on the same ticket / status words; see
// k_points.hip): out[L] = total, out2[0..n2) = a copy of out, in[0..nz) zeroed after reading.
// in / out / out2 16-byte aligned.
int64_t scan1_blocks(int64_t L);
hipError_t launch_scan1(hipStream_t s, uint32_t* in, int64_t L, uint32_t* out, uint32_t* out2, int64_t n2, int64_t nz,
                        const ExpandState& st, const uint32_t* skip_if_zero = nullptr);
hipError_t launch_expand_bitmap_async(hipStream_t s, const uint64_t* bitmap, int64_t words, int64_t n, uint32_t* idx,
                                      int64_t cap, int64_t* count, const ExpandState& st);
// a batch of windows (gf_range_run_batch): window w's expansion owns tickets [tile0[w], tile0[w+1])
constexpr int kRangeBatchMax = 16;
struct ExpandBatch {
  const uint64_t* bm[kRangeBatchMax];
  int64_t n[kRangeBatchMax];
  uint32_t* idx[kRangeBatchMax];
  int64_t cap[kRangeBatchMax];
  int64_t* count[kRangeBatchMax];
  int32_t tile0[kRangeBatchMax + 1];
  int32_t nwin;
};
hipError_t launch_expand_batch(hipStream_t s, const ExpandBatch& b, const ExpandState& st);

// objID dictionary (k_objid.hip, objid.cpp)
struct DictSlot {                 // 32 B
  unsigned long long tag;         // 0 = empty, else hash | 1
  unsigned long long meta;        // arena offset << kDictLenBits | length
  long long id;                   // -1 until the batch's id pass
  unsigned int first;             // smallest batch position mapping here (new slots)
  unsigned int round;             // probe round that created it (0 = being created)
};
struct DictWork {                 // one String of a batch: source bytes [b, b + n), '"' skipped if quotes
  int64_t b;
  int32_t n;
  uint32_t line;                  // batch position
};
struct DictDev {
  DictSlot* slots;
  uint64_t mask;
  char* arena;
  unsigned long long* arena_used;
  unsigned long long* idmap;      // [id] = meta
};
struct DictBatch {
  const char* src;
  int quotes;
  const DictWork* work;
  uint32_t nwork;
  DictWork* pend_out;
  uint32_t* npend_out;
  uint32_t* slot_of;              // [lines]
  uint32_t* flag;                 // [lines + 1]
  const uint32_t* rank;           // [lines + 1]
  uint32_t round, round0;
  int64_t id_base;
  int64_t* keys;                  // [lines]
};
hipError_t launch_dict(hipStream_t st, int stage, const DictDev& d, const DictBatch& B);
hipError_t launch_dict_rehash(hipStream_t st, const DictDev& d, int64_t n);
int dict_reserve_batch(gf_objid_dict* d, uint64_t nwork, uint64_t lines);
int dict_reserve_table(gf_objid_dict* d, uint64_t more, uint64_t bytes);
// keys of the batch in d->work[0] -> keys[line] (sync)
int dict_run(gf_objid_dict* d, const char* src, int quotes, uint32_t nwork, uint64_t lines, int64_t* keys);
int ctx_dict(gf_ctx* ctx, gf_objid_dict** out);  // the context's default dictionary

// CSV ingest (k_csv.hip)
constexpr int64_t kCsvSeg = 64 * 1024;  // text bytes per count / index block
constexpr int kCsvLds = 24 * 1024;      // parse: least LDS staging per block (256 lines staged when they fit)
constexpr int kCsvLdsMax = 64 * 1024;   // parse: most (sized from the mean line length, launch_csv_parse)
struct CsvErr {
  unsigned long long line;  // first bad line (~0 = none)
  int kind;
  int pad;
};
// What the host reads after an ingest call's one sync: written by csv_error_kernel, the call's
// last kernel, from the device-side counts into mapped pinned memory (gf_ctx.csv_head)
struct CsvHead {
  unsigned long long newlines;    // found by csv_nlindex (more than nl_cap: the index was cut)
  unsigned long long lines;       // newlines + (unterminated last line)
  unsigned long long dict_n;      // objIDs queued for the dictionary, and their bytes
  unsigned long long dict_bytes;
  CsvErr err;
};
struct CsvArgs {
  const char* text;
  int64_t len;
  const int64_t* nl;    // newline positions
  // the line count stays on the device between the index and the parse (no host round trip):
  // nl_total = csv_nlindex's count; the parse writes nothing unless newlines <= nl_cap,
  // lines <= cap and lines <= grid_lines (the host re-runs or reports after its one sync)
  const uint32_t* nl_total;
  int64_t nl_cap;
  int64_t cap;          // the caller's output capacity in lines
  int64_t grid_lines;   // lines the parse grid covers: min(nl_cap + 1, cap)
  int64_t mean_line;    // staging hint: the mean line length (the last call's, or len / grid_lines)
  CsvHead* head;
  char delim;
  int32_t want[4];      // field index of objID, time, x, y (csvTsvSchemaAttr)
  double* x;
  double* y;
  int64_t* objID;
  int64_t* ts;
  int32_t* cx;          // nullable: fused cell assignment
  int32_t* cy;
  double minX, minY, cl;
  CsvErr* err;
  // objID fields that are not canonical decimals (gf_decimal.hpp): queued for the dictionary
  DictWork* dict_work;           // [lines]
  uint32_t* dict_n;
  unsigned long long* dict_bytes;  // sum of their raw lengths (arena bound)
  // GeoJSON lines (gf_geojson_parse): format 1; the property names (propertyObjID,
  // propertyTimeStamp; length -1 = not requested) and the timestamp interpretation
  int32_t format;
  int32_t len_obj, len_ts;
  int32_t date_fmt;              // 0: Long.parseLong of a JSON integer; 1: "yyyy-MM-dd HH:mm:ss" text
  int64_t tz_off_ms;             // date_fmt 1: UTC offset of the JVM default time zone
  char prop_obj[kGeoPropMax];
  char prop_ts[kGeoPropMax];
  int32_t lds_cap;               // set by launch_csv_parse: the block's dynamic LDS staging bytes
  int32_t geo_fast;              // GeoJSON: 1 = one-pass member location first (k_csv.hip geo_locate)
  int32_t geo_wave;              // GeoJSON: 1 = the wave-per-line scan locates (k_csv.hip geo_wave_scan)
  unsigned long long* geo_check; // GeoJSON, geo_wave: non-null = run the lane locator too and count differences
  int32_t value_lines;           // GeoJSON: 1 = each line is the record's value (else the record)
};
hipError_t launch_csv_nlindex(hipStream_t st, const char* text, int64_t len, int64_t nseg, int64_t* nl, int64_t nl_cap,
                              uint32_t* total, const ExpandState& es, CsvErr* err, unsigned long long* dict_counters);
int lookback_state(gf_ctx* ctx, int64_t blocks, ExpandState* es);  // api.cpp
hipError_t launch_csv_parse(gf_ctx* ctx, const CsvArgs& a);

hipError_t launch_pane_bounds(hipStream_t s, const int64_t* ts, int64_t n, int64_t pane_ms, int64_t first_pane,
                              int32_t nb, int64_t* bounds);

hipError_t launch_knn_sample(gf_ctx* ctx, const KnnSampleArgs& a);
hipError_t launch_knn_scan(gf_ctx* ctx, const KnnScanArgs& a, int blocks, int unroll, int nt);
hipError_t launch_knn_select(gf_ctx* ctx, const KnnSelectArgs& a);
// k > kMaxK: candidate sorts (k_knn.hip), sized on the host by the window (m >= the candidate
// count) and bounded on the device by *cnt, so a window needs no host read.  op 0 iota perm,
// 1 key field -> keys, 2 the first entry of each objID appended to out (count cnt[1]), 4 the
// record, 5 start: cnt[0] = the lane's candidate count, cnt[1] = 0, lane counters reset
struct KnnLargeArgs {
  const double* cd;
  const int64_t* co;
  const uint32_t* ci;
  uint32_t* perm;
  int64_t m;
  int field;
  uint32_t* keys;
  uint32_t* out;
  uint32_t* cnt;                 // [2] candidates, survivors
  int pass;                      // ops 0 / 1: bounded by cnt[pass]
  unsigned long long* lane_count;
  unsigned long long* lane_maybe;
  int32_t k;
  double T;
  int64_t idx_base;
  void* result;
};
hipError_t launch_knn_large(gf_ctx* ctx, int op, const KnnLargeArgs& a);
constexpr int32_t kMaxKLarge = 1 << 24;  // largest k of the sorted (k > kMaxK) path
// the exact record (status 0) of one window through the sorted path, any k (api.cpp)
int knn_exact_record(gf_knn_plan* P, const gf_points* pts, void* result);

hipError_t launch_knn_poly_sample(gf_ctx* ctx, const KnnPolyArgs& a);
hipError_t launch_knn_poly_scan(gf_ctx* ctx, const KnnPolyArgs& a, int blocks);  // prefilter + refine
struct KnnSelectArgs;
struct KnnMergeArgs;
// depth 2: prefilter of this window + (block 0) the previous window's select / window merge, then refine
hipError_t launch_knn_poly_fused(gf_ctx* ctx, const KnnPolyArgs& a, const KnnSelectArgs& prev, int has_prev,
                                 int blocks, const KnnMergeArgs* merge);
// k > kMaxK: the merge ranks every entry by binary searches in the other (sorted) records and
// dedupes through a hash table, both in global scratch of merge_any_bytes(nrec, k) per window
// (`scratch` may be null for k <= kMaxK)
__host__ __device__ inline size_t merge_any_hash(int64_t e) {
  size_t h = 1024;
  while (h < 2 * (size_t)e) h <<= 1;
  return h;
}
__host__ __device__ inline size_t merge_any_bytes(int32_t nrec, int32_t k) {
  const int64_t e = (int64_t)nrec * k;
  return ((size_t)e * 24 + merge_any_hash(e) * 12 + 255) & ~(size_t)255;
}
hipError_t launch_knn_merge(gf_ctx* ctx, int32_t k, const void* records, int32_t nrec, size_t rec_stride,
                            int32_t nwin, size_t win_stride, void* result, size_t res_stride, int foreign,
                            void* scratch);
// String records (gf_knn_attach_strings / gf_knn_merge_dev_strings): a kNN record followed by
// the Strings of its dictionary objIDs -- {int32 status, int32 n, int64 nbytes, uint32 off[k+1],
// bytes[cap]}; entry i's String = bytes[off[i], off[i+1]) (empty for canonical decimal keys)
__host__ __device__ inline size_t str_side_off(int32_t k) { return ((size_t)4 * (k + 1) + 7) & ~(size_t)7; }
__host__ __device__ inline size_t str_record_bytes(int32_t k, int64_t cap) {
  return 32 + (size_t)24 * k + 16 + str_side_off(k) + (((size_t)cap + 7) & ~(size_t)7);
}
__host__ __device__ inline size_t strmerge_pow2(int64_t e) {
  size_t p = 2;
  while (p < (size_t)e) p <<= 1;
  return p;
}
__host__ __device__ inline size_t strmerge_bytes(int32_t nrec, int32_t k) {
  const int64_t e = (int64_t)nrec * k;
  return ((size_t)e * 40 + strmerge_pow2(e) * 4 + strmerge_pow2(2 * e) * 8 + (size_t)k * 16 + 1024) & ~(size_t)255;
}
hipError_t launch_knn_attach_strings(gf_ctx* ctx, int32_t k, const unsigned long long* idmap, const char* arena,
                                     int64_t dict_size, const void* records, int32_t nrec, int64_t cap, void* out);
hipError_t launch_knn_merge_strings(gf_ctx* ctx, int32_t k, int64_t cap, const void* records, int32_t nrec,
                                    size_t rec_stride, int32_t nwin, size_t win_stride, void* results, void* scratch);
// records of one merge given as a pointer list (kernel argument; the panes of a sliding window)
constexpr int kMaxMergeRecs = 64;
struct KnnRecList {
  const char* rec[kMaxMergeRecs];
};
hipError_t launch_knn_merge_list(gf_ctx* ctx, int32_t k, const KnnRecList& list, int32_t nrec, void* result,
                                 void* scratch);
// a window merge folded into block 0 of the next fused launch (after the select it waits for)
constexpr int kFusedMergeMaxK = 128;
struct KnnMergeArgs {
  int32_t nrec;   // 0 = none
  void* result;
  KnnRecList list;
};
hipError_t launch_knn_fused(gf_ctx* ctx, const KnnScanArgs& a, const KnnSelectArgs& prev, int has_prev,
                            int scan_blocks, int nt, const KnnMergeArgs* merge);
// gf_knn_enqueue with an optional window merge for the fused launch; *merged = 1 if it was
// folded in (depth 2, a pending select, k <= kFusedMergeMaxK), else the caller launches it
int knn_enqueue_merge(gf_knn_plan* P, const gf_points* pts, void* result, const KnnMergeArgs* merge, int* merged);

hipError_t launch_range(gf_ctx* ctx, const RangeArgs& a, int table_mode, int poly, int blocks);
// a batch of windows of one plan in one launch (blockIdx.y = window; inline tests, DEFER 0)
struct RangeWin {
  const double* x;
  const double* y;
  int64_t n;
  uint64_t* bitmap;
  uint64_t* multi;
  uint64_t* partials;  // the window's own partials + ticket
  int64_t* counts;
};
struct RangeBatch {
  RangeWin w[kRangeBatchMax];
};
hipError_t launch_range_batch(gf_ctx* ctx, const RangeArgs& a, const RangeBatch& b, int nwin, int table_mode, int poly,
                              int blocks);
// sliding range (sliding.cpp): a closed window's emitted indices = its non-empty panes' index
// lists concatenated, each shifted by the pane's first position in the window (k_points.hip)
struct RangeGatherArgs {
  const uint32_t* list[kMaxMergeRecs];  // pane-local ascending indices (gf_bitmap_to_indices_async)
  const int64_t* cnt[kMaxMergeRecs];    // their device counts
  int64_t base[kMaxMergeRecs];          // the pane's first position in the window
  int32_t npanes;
  int64_t total;                        // points in the window (an upper bound of the hits)
  uint32_t* out;
  int64_t* count;
};
hipError_t launch_range_window_gather(hipStream_t s, const RangeGatherArgs& a);
hipError_t launch_join_ppoly(gf_ctx* ctx, const RangeArgs& a, int blocks, int jblocks, uint32_t* ecnt, uint32_t* ecand,
                             uint32_t* btot, unsigned long long* total, uint32_t* pairs, int64_t cap, int aligned);

struct JoinArgs {
  const double* ox;
  const double* oy;
  int64_t no;
  double u_minX, u_minY, u_cl;   // ugrid (ordinary points)
  int32_t qn;                    // qgrid n (validKey of replicated cells)
  int64_t c;                     // candidate layers; < 0 => r == 0 (all valid cells)
  const uint32_t* q_off;         // [(qn+2)^2 + 1] clamped-cell bucket offsets
  const double* sqx;
  const double* sqy;
  const int32_t* sqcx;
  const int32_t* sqcy;
  const uint32_t* sqidx;
  int approx;
  int metric;
  double r;
  uint32_t* counts;              // count pass: per-block pair counts
  const uint32_t* offsets;       // write pass: per-block output offsets
  uint32_t* pairs;               // write pass
};
hipError_t launch_join_qkeys(hipStream_t s, const double* qx, const double* qy, int64_t nq, double minX,
                             double minY, double cl, int32_t qn, uint32_t* keys, int32_t* qcx, int32_t* qcy);
hipError_t launch_join_qscatter(hipStream_t s, const double* qx, const double* qy, const int32_t* qcx,
                                const int32_t* qcy, const uint32_t* keys, int64_t nq, uint32_t* cursor,
                                double* sqx, double* sqy, int32_t* sqcx, int32_t* sqcy, uint32_t* sqidx);
hipError_t launch_join_probe(gf_ctx* ctx, const JoinArgs& a, int write_pass, int blocks);

// row-bucketed join (c >= 0): see k_join.hip
constexpr int kJoinTask = 8192;      // ordinary points per probe task (part of one row)
constexpr int kJoinThreads = 1024;   // two probe blocks per CU when the staged rows fit 80 KB
constexpr int kJoinMaxRows = 16;     // staged query rows (2c+1) per task
// Join output (k_join.hip).  Pairs go straight to the caller's buffer: every wave of the
// (persistent) probe owns one chunk of `chunk` positions at a time, reserved with one atomic on
// gctr; its last chunk stays partly filled, so the reserved space [0, G) holds one hole per wave
// and T = G - (the holes) pairs.  The fix-up moves the pairs stored at positions >= T into the
// holes below T: dense [0, T), in an unspecified order.  Positions >= cap live in `spill`
// (sized for every wave's hole), so a window whose T fits cap is complete.
struct JoinOut {
  uint32_t* pairs;           // caller's [2 * cap]
  uint64_t cap;
  int aligned;               // 8-byte aligned: one 8-byte store per pair
  uint32_t chunk;            // positions per chunk
  uint2* spill;              // [spill_cap]: positions cap, cap + 1, ...
  uint64_t spill_cap;
  unsigned long long* gctr;  // reserved positions (0 between calls: the fix-up resets it)
  uint64_t* tail_base;       // [nwaves] base of each wave's last chunk (~0: none)
  uint32_t* tail_fill;       // [nwaves]
  uint32_t nwaves;           // tail entries: the probe's waves (regions: its blocks)
  // Band probe REGIONS (k_join.hip): block b owns a region of positions (derived by every block
  // alike from hist) and fills it through an LDS cursor (no global atomic); pairs beyond its
  // region go to the dense overflow area after the regions (one atomic per overflowing flush).
  // Regions come from the last call's pairs per point of every block (hist), scaled down to e_lim
  // when they would exceed it; the fix-up moves the pairs above T into the regions' unused tails.
  int regions;
  uint64_t* bcount;          // [G] this call's pairs per block
  uint64_t* bslice;          // [G] this call's ordinary points per block
  uint64_t* hist;            // [3G + 1] persistent: the last call's pairs | points | slice start per block, did-not-fit (zero: none)
  unsigned long long* ovf;   // persistent overflow counter (the fix-up resets it)
  uint64_t e_lim;            // the regions' total never exceeds it (cap + spill covers it)
  double ppp;                // pairs per point when there is no history
};
// The join's fix-up (k_join.hip): the pairs stored at positions >= T moved into the holes < T.
struct JoinFixup {
  JoinOut o;
  unsigned long long* total;  // the pair count T (device or mapped pinned memory)
  unsigned long long* hint;   // mapped pinned: T again, the next call's chunk-size hint
  uint64_t* hole_start;       // [nwaves] holes below T, by position
  uint64_t* hole_pref;        // [nwaves + 1] their exclusive prefix of lengths
  uint64_t* seg_start;        // [nwaves + 1] stored runs in [T, G), by position
  uint64_t* seg_pref;         // [nwaves + 2]
  uint32_t* counts;           // [2] holes below T, runs above T
};
struct JoinRowArgs {
  const double* ox;
  const double* oy;
  int64_t no;
  double u_minX, u_minY, u_cl;
  int32_t qn;
  int64_t c;
  const uint32_t* q_off;
  const double* sqx;
  const double* sqy;
  const int32_t* sqcx;
  const int32_t* sqcy;
  const uint32_t* sqidx;
  int approx, metric;
  double r, s_r;            // s_r = smax(r): exact squared-distance bound for metric 0
  int32_t nblk;             // ordinary-side bucketing blocks
  int32_t nrows;            // ordinary-side rows: qn cell rows, or f*qn sub-rows on the fine path
  uint32_t* row_mat;        // [nrows * nblk] per-block row histograms (row-major)
  const uint32_t* row_mat_scan;  // its exclusive scan (+ mat_base): run start per (row, block)
  uint32_t mat_base;        // the matrix scan's offset (it follows the query histogram's)
  uint32_t* row_off_w;      // [nrows+1] row starts (written by the finish kernel)
  const uint32_t* row_off;  // same buffer, read by the probe
  uint32_t* task_off_w;     // [nrows+1] first task of each row (finish kernel)
  const uint32_t* task_off; // same buffer, read by the probe
  double* soxy;             // [2*no] row-bucketed ordinary xy
  uint32_t* soidx;          // [no]
  JoinOut out;              // pairs straight to the caller's buffer in per-wave chunks
  int lds_budget;
  // fine sub-cells (k_join.hip, "fine path"): f > 1 splits every cell into f x f sub-cells of
  // side cl / f > r, the query side is sorted by sub-cell and q_off indexes sub-cells
  // ((f*(qn+2))^2 + 1 entries); f == 1: q_off indexes cells as before
  int32_t f;
  double fs;                // f / cl
  // band probe: its last block (ticket) computes the regions' fix-up (join_region_prep) --
  // no separate launch; the copy kernel follows
  JoinFixup fx;
  unsigned long long* ticket;  // zero between calls (the last block resets it)
};
__device__ __forceinline__ void join_store(uint32_t* pairs, int aligned, uint64_t pos, uint2 v) {
  if (aligned) {
    reinterpret_cast<uint2*>(pairs)[pos] = v;
  } else {
    pairs[2 * pos] = v.x;
    pairs[2 * pos + 1] = v.y;
  }
}
__device__ __forceinline__ uint2 join_load(const uint32_t* pairs, int aligned, uint64_t pos) {
  if (aligned) return reinterpret_cast<const uint2*>(pairs)[pos];
  return make_uint2(pairs[2 * pos], pairs[2 * pos + 1]);
}
hipError_t launch_join_fixup(gf_ctx* ctx, const JoinFixup& f);
hipError_t launch_join_stream(gf_ctx* ctx, const JoinRowArgs& a);
hipError_t launch_join_band(gf_ctx* ctx, const JoinRowArgs& a, int blocks);  // fine path
constexpr int kJoinReg = 3;  // pairs per ordinary point kept in registers by the probe
// LDS bytes of one staged query row with m points: u16 bucket offsets, xy
__host__ __device__ inline size_t join_row_lds_bytes(int64_t W, uint32_t m) {
  return ((size_t)(W + 1) * 2 + 15) / 16 * 16 + (size_t)m * 16;
}
// LDS budget of the probe's staged query rows for nq query points on a qn x qn grid, 2c+1 rows
int join_probe_budget(int64_t nq, int32_t qn, int64_t c, int32_t f);
// sub-cells per cell and axis for the fine path (1: the cell path) -- see k_join.hip
int32_t join_fine_factor(double cl, double r, int32_t qn, double maxabs);
// row path, query side: cell-sorted query arrays + q_off without global atomics
struct JoinQueryArgs {
  const double* qx;
  const double* qy;
  int64_t nq;
  double minX, minY, cl;
  int32_t qn;
  int32_t nblk;            // query blocks at the front of the histogram / scatter launches
  uint32_t* qmat;          // [(qn+2) * nblk] per-block clamped-row histograms (row-major)
  const uint32_t* qmat_scan;  // its exclusive scan (the front of the joint scan)
  double* txy;             // [2*nq] row-bucketed xy
  uint32_t* tidx;          // [nq] their input indices
  uint32_t* q_off;         // [(f(qn+2))^2 + 1] first point of each sub-cell (cell when f == 1)
  double* sqx;
  double* sqy;
  int32_t* sqcx;
  int32_t* sqcy;
  uint32_t* sqidx;
  int32_t f;               // sub-cells per cell and axis (1: cells)
  double fs;               // f / cl
};
// launches of the row path (k_join.hip): 0 histograms, 1 scatter, 2 row / task offsets, 3 probe
hipError_t launch_join_rows(gf_ctx* ctx, const JoinRowArgs& a, const JoinQueryArgs& q, int stage);
size_t join_scatter_lds_bytes(int32_t nrows, int tile);


}  // namespace gf

// plans ---------------------------------------------------------------------------------
struct gf_range_plan {
  gf_ctx* ctx = nullptr;
  gf_grid grid{};
  double r = 0;
  int approx = 0, metric = 0, poly = 0, table_mode = 0;
  int32_t nq = 0, g_layers = 0, c_layers = 0;
  gf::QueryRect qr{};
  double qx0 = 0, qy0 = 0;
  // device buffers (owned)
  uint8_t* table = nullptr;
  uint32_t* rows = nullptr;
  uint32_t* rowoff = nullptr;
  uint8_t* spans = nullptr;
  int64_t span_bytes = 0;
  double* xt = nullptr;            // exact cell thresholds (table modes, n <= 2048)
  double* yt = nullptr;
  double x_lo = 0, x_hi = 0, y_lo = 0, y_hi = 0;
  double sx_lo = 0, sx_hi = 0;
  double sy_lo = 0, sy_hi = 0;
  double span_frac = 1.0;  // share of the grid's cells inside the x / y spans
  int32_t* extra = nullptr;
  int32_t n_extra = 0;
  int32_t* cand_off = nullptr;
  int32_t* cand_list = nullptr;
  double* qx = nullptr;
  double* qy = nullptr;
  int32_t npoly = 0;
  int32_t* ring_off = nullptr;
  int32_t* vert_off = nullptr;
  double* vx = nullptr;
  double* vy = nullptr;
  double* bbox = nullptr;
  double* ring_env = nullptr;
  uint64_t* partials = nullptr;
  uint64_t* batch_partials = nullptr;  // gf_range_run_batch: kRangeBatchMax x (partials + ticket)
  int blocks = 0;
  uint32_t* queue = nullptr;       // deferred candidate tests (grown to blocks x seg_cap)
  double* queue_xy = nullptr;
  int64_t queue_cap = 0;
  uint32_t* queue_count = nullptr; // [num_cus * 8] per-segment counts
  int64_t cls_cells[4] = {0, 0, 0, 0};  // in-grid cells per class (diagnostics)
  int32_t scan_blocks = 0;         // tuning: 0 = auto
  int32_t defer_mode = 0;          // tuning: 0 auto, 1 test inline, 2 defer
  int32_t drain_lanes = 0;         // testing: lanes per wave running the block-end drain (0 = all)
  // point-polygon join plans (gf_join_ppoly_plan_create)
  int join = 0;
  int32_t* brect = nullptr;        // [npoly * 4] bbox cells x0, x1, y0, y1
  uint8_t* rect = nullptr;         // [npoly] 1: axis-aligned rectangle shell, no holes
  uint32_t* jecnt = nullptr;       // [queue_cap] pairs per queued point
  uint32_t* jecand = nullptr;      // [queue_cap * 4] their first polygon indices (kJoinKeep)
  uint32_t* jbtot = nullptr;       // [num_cus * 8] pairs per join block
  unsigned long long* jtotal = nullptr;
};

struct gf_knn_plan {
  gf_ctx* ctx = nullptr;
  gf_grid grid{};
  double qx = 0, qy = 0, r = 0;
  int32_t k = 0;
  int metric = 0;
  gf::QueryRect qr{};
  // a lane = device state + candidate buffers of one in-flight window.  Lane 1 exists only
  // at pipeline depth 2 (gf_knn_plan_set_pipeline): window i uses lane i % 2, and its select
  // runs inside window i+1's fused scan kernel (or at gf_knn_plan_flush).
  struct Lane {
    gf::KnnState* st = nullptr;
    double* cand_d = nullptr;
    uint32_t* cand_i = nullptr;
    int64_t* cand_o = nullptr;
  } lane[6];  // depth d >= 3 uses 2 (d - 1): two per stream
  int64_t cap = 0;
  int pipeline = 1;               // 1: sample -> scan -> select per window; 2: fused
  uint64_t seq = 0;
  int pend_lane = -1;             // depth 2: the window whose select has not run yet
  int lane_warm[6] = {0, 0, 0, 0, 0, 0};  // depth >= 2: the lane has a hint from an earlier window
  void* pend_result = nullptr;
  int64_t pend_idx_base = 0;      // depth 2: idx_base of the pending window (set at its enqueue)
  // depth 3: windows whose select has not run yet (seq k-1, k-2), oldest first
  struct Pend {
    int lane;
    void* result;
    int64_t idx_base;
    uint64_t seq;
  };
  Pend pq[3];
  int npq = 0;
  int use_hint = 1;             // reuse the previous window's k-th distance as the threshold guess
  int64_t idx_base = 0;
  void* tmp_result = nullptr;   // device record used by gf_knn_run / fallback
  void* host_result = nullptr;  // pinned
  int scan_blocks = 0;   // tuning: 0 = auto (4 blocks per CU)
  int scan_unroll = 1;   // point pairs per lane per iteration (tools/tune_knn.py sweep)
  int scan_nt = 1;       // nontemporal loads
  int large = 0;         // k > kMaxK: every candidate within r, sorted (knn_large)
  // polygon query (gf_knn_ppoly_plan_create): device copy of the polygon, depth 1 only
  int poly = 0, approx = 0;
  int32_t* ring_off = nullptr;
  int32_t* vert_off = nullptr;
  double* vx = nullptr;
  double* vy = nullptr;
  double* ring_env = nullptr;
  double bbox[4] = {0, 0, 0, 0};
  uint32_t* maybe_i[3] = {nullptr, nullptr, nullptr};  // per stream, cap entries
  int64_t maybe_cap = 0;
};

struct gf_window {
  gf_ctx* ctx = nullptr;
  int64_t capacity = 0, n = 0;
  double* x = nullptr;
  double* y = nullptr;
  int64_t* objID = nullptr;
  int64_t* ts = nullptr;
  bool has_objid = false, has_ts = false;  // columns of the last upload
  const int64_t* objid_mapped = nullptr;   // gf_window_upload_mapped: the caller's pinned objID column
  // uploads run on the window's own copy stream: they wait for the work already enqueued on
  // the context's streams (which may still read the previous contents), and gf_window_points
  // makes the context's streams wait for the copy -- so upload(i+1) overlaps evaluate(i)
  hipStream_t copy = nullptr;
  hipEvent_t ready = nullptr, fence_main = nullptr, fence_aux = nullptr, fence_aux2 = nullptr;
  bool pending = false;
};
