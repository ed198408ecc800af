// k_join.hip -- grid-partitioned point-point join of one window:
//   JoinQuery.getReplicatedPointQueryStream (JoinQuery.java:73-90): each query point q is
//   replicated to every valid cell within c = ceil(r/l) layers of its cell (all cells if r==0)
//   PointPointJoinQuery.windowBased (:148-182): equi-join on the cell, then d(p, q) <= r.
// Instead of replicating q (2c+1)^2 times, the query side is bucketed once by its (clamped)
// cell -- counting sort: histogram, exclusive scan, scatter -- and each ordinary point probes
// the (2c+1) bucket rows around its cell.  A pair (p, q) qualifies iff p's cell is a valid
// query-grid cell within Chebyshev distance c of q's cell, exactly the replicated-key match.
// Output: two passes over the ordinary side (count, then write at per-block scanned
// offsets), so no global atomics and pairs come out grouped by ordinary point.
#define GF_TU_NAME k_join_hip
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include <type_traits>

#include "gf_internal.hpp"

namespace gf {

__global__ __launch_bounds__(kBlock) void join_qkeys_kernel(const double* __restrict__ qx,
                                                            const double* __restrict__ qy, int64_t nq,
                                                            double minX, double minY, double cl, int32_t qn,
                                                            uint32_t* __restrict__ keys, int32_t* __restrict__ qcx,
                                                            int32_t* __restrict__ qcy) {
  const int64_t W = (int64_t)qn + 2;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nq; i += (int64_t)gridDim.x * kBlock) {
    const int32_t cx = cell_index(qx[i], minX, cl);
    const int32_t cy = cell_index(qy[i], minY, cl);
    qcx[i] = cx;
    qcy[i] = cy;
    const int64_t kx = (cx < -1 ? -1 : (cx > qn ? qn : cx)) + 1;
    const int64_t ky = (cy < -1 ? -1 : (cy > qn ? qn : cy)) + 1;
    keys[i] = (uint32_t)(ky * W + kx);
  }
}

hipError_t launch_join_qkeys(hipStream_t s, const double* qx, const double* qy, int64_t nq, double minX,
                             double minY, double cl, int32_t qn, uint32_t* keys, int32_t* qcx, int32_t* qcy) {
  if (nq <= 0) return hipSuccess;
  int64_t blocks = (nq + kBlock - 1) / kBlock;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(join_qkeys_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, qx, qy, nq, minX, minY, cl, qn,
                     keys, qcx, qcy);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void join_qscatter_kernel(
    const double* __restrict__ qx, const double* __restrict__ qy, const int32_t* __restrict__ qcx,
    const int32_t* __restrict__ qcy, const uint32_t* __restrict__ keys, int64_t nq, uint32_t* __restrict__ cursor,
    double* __restrict__ sqx, double* __restrict__ sqy, int32_t* __restrict__ sqcx, int32_t* __restrict__ sqcy,
    uint32_t* __restrict__ sqidx) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nq; i += (int64_t)gridDim.x * kBlock) {
    const uint32_t pos = atomicAdd(&cursor[keys[i]], 1u);
    sqx[pos] = qx[i];
    sqy[pos] = qy[i];
    sqcx[pos] = qcx[i];
    sqcy[pos] = qcy[i];
    sqidx[pos] = (uint32_t)i;
  }
}

hipError_t launch_join_qscatter(hipStream_t s, const double* qx, const double* qy, const int32_t* qcx,
                                const int32_t* qcy, const uint32_t* keys, int64_t nq, uint32_t* cursor,
                                double* sqx, double* sqy, int32_t* sqcx, int32_t* sqcy, uint32_t* sqidx) {
  if (nq <= 0) return hipSuccess;
  int64_t blocks = (nq + kBlock - 1) / kBlock;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(join_qscatter_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, qx, qy, qcx, qcy, keys, nq,
                     cursor, sqx, sqy, sqcx, sqcy, sqidx);
  return hipGetLastError();
}

// Probe one ordinary point; EMIT writes its pairs from `pos`, else only counts.
template <bool EMIT>
__device__ uint32_t join_probe_point(const JoinArgs& a, int64_t p, uint64_t pos) {
  const double px = a.ox[p], py = a.oy[p];
  const int32_t cx = cell_index(px, a.u_minX, a.u_cl);
  const int32_t cy = cell_index(py, a.u_minY, a.u_cl);
  if (!(cx >= 0 && cy >= 0 && cx < a.qn && cy < a.qn)) return 0;  // p.gridID must be a replicated key
  const int64_t W = (int64_t)a.qn + 2, qn = a.qn, c = a.c;
  int64_t x0, x1, y0, y1;
  if (c < 0) {
    x0 = -1; x1 = qn; y0 = -1; y1 = qn;
  } else {
    x0 = cx - c < -1 ? -1 : cx - c; x1 = cx + c > qn ? qn : cx + c;
    y0 = cy - c < -1 ? -1 : cy - c; y1 = cy + c > qn ? qn : cy + c;
  }
  uint32_t cnt = 0;
  for (int64_t ry = y0; ry <= y1; ++ry) {
    const int64_t row = (ry + 1) * W;
    const uint32_t b = a.q_off[row + x0 + 1], e = a.q_off[row + x1 + 2];
    for (uint32_t t = b; t < e; ++t) {
      if (c >= 0) {
        const int64_t ddx = (int64_t)a.sqcx[t] - cx, ddy = (int64_t)a.sqcy[t] - cy;
        if (ddx > c || ddx < -c || ddy > c || ddy < -c) continue;
      }
      if (!a.approx && !(distance(px, py, a.sqx[t], a.sqy[t], a.metric) <= a.r)) continue;
      if (EMIT) {
        a.pairs[2 * (pos + cnt)] = (uint32_t)p;
        a.pairs[2 * (pos + cnt) + 1] = a.sqidx[t];
      }
      ++cnt;
    }
  }
  return cnt;
}

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[kBlock / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  uint32_t before = 0, tot = 0;
  for (int w = 0; w < kBlock / 64; ++w) {
    if (w < wid) before += wsum[w];
    tot += wsum[w];
  }
  *total = tot;
  __syncthreads();
  return before + inc - v;
}

// each block owns a contiguous chunk of ordinary points
template <int WRITE>
__global__ __launch_bounds__(kBlock) void join_probe_kernel(JoinArgs a) {
  const int64_t chunk = (a.no + gridDim.x - 1) / gridDim.x;
  const int64_t beg = (int64_t)blockIdx.x * chunk;
  const int64_t end = beg + chunk < a.no ? beg + chunk : a.no;
  uint64_t run = WRITE ? a.offsets[blockIdx.x] : 0;
  uint32_t total_cnt = 0;
  for (int64_t s = beg; s < end; s += kBlock) {
    const int64_t p = s + threadIdx.x;
    uint32_t c = p < end ? join_probe_point<false>(a, p, 0) : 0u;
    if (!WRITE) {
      total_cnt += c;
      continue;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan256(c, &tot);
    if (p < end && c) join_probe_point<true>(a, p, run + ex);
    run += tot;
  }
  if (!WRITE) {
    uint32_t tot;
    block_excl_scan256(total_cnt, &tot);
    if (threadIdx.x == 0) a.counts[blockIdx.x] = tot;
  }
}

hipError_t launch_join_probe(gf_ctx* ctx, const JoinArgs& a, int write_pass, int blocks) {
  KTimer t(ctx, GF_K_JOIN_PROBE);
  if (write_pass)
    hipLaunchKernelGGL(join_probe_kernel<1>, dim3(blocks), dim3(kBlock), 0, ctx->stream, a);
  else
    hipLaunchKernelGGL(join_probe_kernel<0>, dim3(blocks), dim3(kBlock), 0, ctx->stream, a);
  return hipGetLastError();
}

// =======================================================================================
// Row-bucketed join (the default path when c >= 0).  The ordinary points are bucketed by
// their cell row (block-local LDS histograms -> one scan -> write-combined scatter), then
// processed as tasks of <= kJoinTask points of one row: a task stages the query buckets of rows
// cy-c .. cy+c (u16 bucket offsets + xy) in LDS and tests each ordinary point against the
// (2c+1) bucket runs around its cell -- all LDS.  A task whose rows do not fit the LDS budget
// probes the same runs from global memory.  The query side is sorted by (sub-)cell with a
// global histogram.  One window = 6 launches: histograms (both sides) -> one scan of both ->
// scatter (both sides) -> row / task offsets -> probe (its last block scans the task counts)
// -> packing.
// =======================================================================================
constexpr int kRowMax = 8192;  // rows staged as LDS histograms by the bucketing kernels

// Bucketing: block b owns the contiguous input chunk b; its row histogram goes to column b of
// the row-major matrix M[row][block] (plain stores).  The exclusive scan of M (flattened) is
// then, for every (row, block), the start of that block's run of the row -- no contended
// atomics, and the order inside a row is the block order.
__device__ __forceinline__ void chunk_of(int64_t no, int64_t bid, int64_t nblk, int64_t& beg, int64_t& end) {
  const int64_t chunk = (no + nblk - 1) / nblk;
  beg = bid * chunk;
  end = beg + chunk < no ? beg + chunk : no;
  if (beg > no) beg = no;
}

// kBucketU points per thread are loaded before any is used (the loop is latency-bound
// otherwise: one HBM round trip per point per wave)
#ifndef GF_JOIN_BUCKET_U
#define GF_JOIN_BUCKET_U 8
#endif
constexpr int kBucketU = GF_JOIN_BUCKET_U;

constexpr int kScatThreads = 1024;
constexpr int kHistSplit = 2;  // histogram chunks per scatter block
// points per write-combining tile: 6144 where the row arrays leave room in LDS (6-point row
// runs at C4's 1000 rows: scatter 121 -> 110 us), else 4096
constexpr int kScatTileBig = 7168, kScatTileSmall = 4096;

__device__ __forceinline__ int32_t clamp_key(int32_t c, int32_t qn) { return (c < -1 ? -1 : (c > qn ? qn : c)) + 1; }

// Sub-cell of coordinate v inside its in-grid cell c (0 .. f-1): any function that is monotone
// in v, identical for both sides and gives every sub-cell a width > r serves (see the fine path
// below); this one is within a few ulps of the cell split into f equal parts.
__device__ __forceinline__ int32_t join_sub(double v, double mn, double cl, int32_t c, double fs, int32_t f) {
  // == clamp(jint(s), 0, f - 1): s < 1 (NaN included) -> 0, s >= f - 1 (+inf included) -> f - 1,
  // else the truncation (in range) -- compares and one conversion, no saturation cases
  const double s = (v - (mn + (double)c * cl)) * fs;
  return !(s >= 1.0) ? 0 : (s >= (double)(f - 1) ? f - 1 : (int32_t)s);
}

// q_off index of a query point: its sub-cell (f sub-rows x f sub-columns per clamped cell) in
// row-major order over f(qn+2) sub-columns; f == 1: the clamped cell.  A point outside the grid
// goes to the sub-cell of its clamped cell ADJACENT to the grid (sub f-1 below the grid, 0
// above): it can pair only with an ordinary point within r < cl/f of the grid's edge, i.e. in
// the outermost sub-cell, whose 3 x 3 neighbourhood then holds it -- so edge lanes need no
// true-cell check either (a clamped point farther than one cell out fails d <= r).
__device__ __forceinline__ int32_t join_sub_clamped(double v, double mn, double cl, int32_t c, double fs, int32_t f,
                                                    int32_t qn) {
  return c < 0 ? f - 1 : (c >= qn ? 0 : join_sub(v, mn, cl, c, fs, f));
}
__device__ __forceinline__ uint32_t join_fine_key(const JoinQueryArgs& q, double x, double y, int32_t& cx,
                                                  int32_t& cy) {
  cx = cell_index(x, q.minX, q.cl);
  cy = cell_index(y, q.minY, q.cl);
  const int64_t fW = (int64_t)q.f * (q.qn + 2);
  int32_t jx = 0, jy = 0;
  if (q.f > 1) {
    jx = join_sub_clamped(x, q.minX, q.cl, cx, q.fs, q.f, q.qn);
    jy = join_sub_clamped(y, q.minY, q.cl, cy, q.fs, q.f, q.qn);
  }
  return (uint32_t)(((int64_t)q.f * clamp_key(cy, q.qn) + jy) * fW + (int64_t)q.f * clamp_key(cx, q.qn) + jx);
}

// Row of an ordinary point: its cell row, -1 when the row is outside the grid; a point whose
// COLUMN is outside the grid is bucketed too and dropped by the probe's sort (no replicated key
// can match it), so the histogram pass reads y alone.  Row of a query point: its clamped cell
// row (0 .. qn+1).
__device__ __forceinline__ int32_t join_orow(const JoinRowArgs& a, double, double y) {
  const int32_t cy = cell_index(y, a.u_minY, a.u_cl);
  return cy >= 0 && cy < a.qn ? cy : -1;
}
__device__ __forceinline__ int32_t join_qrow(const JoinQueryArgs& q, double, double y) {
  return clamp_key(cell_index(y, q.minY, q.cl), q.qn);
}

// Block `bid` of `nblk` counts its chunk of (X, Y) per row in LDS and stores the counts as
// column bid of the row-major matrix M[row][block] (plain stores, no global atomics).
template <class RowF>
__device__ __forceinline__ void lds_row_hist(const double* X, const double* Y, int64_t n, int64_t bid, int64_t nblk,
                                             int32_t nrows, uint32_t* M, RowF rowf) {
  __shared__ uint32_t h[kRowMax];
  int64_t beg, end;
  chunk_of(n, bid, nblk, beg, end);
  for (int j = threadIdx.x; j < nrows; j += kScatThreads) h[j] = 0u;
  __syncthreads();
  for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += kScatThreads * kBucketU) {
    double x[kBucketU], y[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int64_t i = i0 + u * kScatThreads;
      x[u] = i < end ? __builtin_nontemporal_load(X + i) : 0.0;
      y[u] = i < end ? __builtin_nontemporal_load(Y + i) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      if (i0 + u * kScatThreads >= end) continue;
      const int32_t row = rowf(x[u], y[u]);
      if (row >= 0) atomicAdd(&h[row], 1u);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nrows; j += kScatThreads) M[(size_t)j * nblk + bid] = h[j];
}

// Launch 1: blocks [0, kHistSplit * q.nblk) histogram the query side by clamped row (matrix
// q.qmat), the rest the ordinary side by row (a.row_mat); one scan of [q.qmat | a.row_mat]
// follows.  Each side is cut into kHistSplit chunks per scatter block (two histogram blocks per
// CU keep more loads in flight; scatter block b takes chunks kHistSplit*b ..).
__global__ __launch_bounds__(kScatThreads) void join_hist_kernel(JoinRowArgs a, JoinQueryArgs q) {
  if ((int)blockIdx.x < kHistSplit * q.nblk)
    lds_row_hist(q.qx, q.qy, q.nq, blockIdx.x, kHistSplit * q.nblk, q.qn + 2, q.qmat,
                 [&](double x, double y) { return join_qrow(q, x, y); });
  else
    lds_row_hist(a.ox, a.oy, a.no, (int64_t)blockIdx.x - kHistSplit * q.nblk, kHistSplit * a.nblk, a.nrows,
                 a.row_mat, [&](double x, double y) { return join_orow(a, x, y); });
}

// Launch 3: write-combining row scatter of both sides (query blocks first).  Stores straight
// from the registers would put every lane of a wave into a different row: 64 separate 16 B +
// 4 B writes per store instruction, each a partial line that reaches HBM on its own (rocprofv3
// r02: WRITE_SIZE 2.5x the bytes, 208 us).  Here a block takes its chunk in tiles of kScatTile
// points: rows -> LDS row histogram -> scan -> the tile's points placed row-contiguously in LDS
// (with their destination) -> written out in that order, so consecutive lanes write
// consecutive slots of one row (runs of ~tile/rows points) and successive tiles extend the
// same runs.  Destinations: the block's run start of each row (the matrix scan, minus `base`)
// advanced tile by tile.
size_t join_scatter_lds_bytes(int32_t nrows, int tile) {
  return (size_t)tile * (16 + 2 + 2) + 2 * 4 * (size_t)nrows + 4 * (kScatThreads / 64);
}
int join_scatter_tile(int32_t nrows) {
  return join_scatter_lds_bytes(nrows, kScatTileBig) <= 160 * 1024 ? kScatTileBig : kScatTileSmall;
}

template <int kScatTile, class RowF>
__device__ __forceinline__ void wc_row_scatter(const double* X, const double* Y, int64_t n, int64_t bid, int64_t nblk,
                                               int32_t nrows, const uint32_t* Ms, uint32_t base, double2* oxy,
                                               uint32_t* oidx, RowF rowf) {
  constexpr int kScatPer = kScatTile / kScatThreads;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  // per slot (r06: 20 B, was 24): the point, its tile-local input position, its row -- the
  // destination is gd[row] + slot at write-out -- so a tile holds 7168 points instead of 6144
  // (longer row runs: fewer partial lines per point written)
  double2* const sxy = reinterpret_cast<double2*>(sm);
  uint16_t* const sloc = reinterpret_cast<uint16_t*>(sxy + kScatTile);
  uint16_t* const srow = sloc + kScatTile;
  uint32_t* const th = reinterpret_cast<uint32_t*>(srow + kScatTile);  // [nrows] tile counts -> starts -> ends
  uint32_t* const gd = th + nrows;        // [nrows] next global slot of the row (tile-local: minus start)
  uint32_t* const wsum = gd + nrows;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t beg, end, b2, e2;
  chunk_of(n, kHistSplit * bid, kHistSplit * nblk, beg, end);  // the block's histogram chunks
  chunk_of(n, kHistSplit * bid + kHistSplit - 1, kHistSplit * nblk, b2, e2);
  end = e2 > end ? e2 : end;
  for (int r = threadIdx.x; r < nrows; r += kScatThreads) {
    gd[r] = Ms[(size_t)r * kHistSplit * nblk + kHistSplit * bid] - base;
    th[r] = 0u;
  }
  lds_barrier();
  const int per = (nrows + kScatThreads - 1) / kScatThreads, r0 = threadIdx.x * per;
  // the next tile's coordinates are loaded while this tile goes through its LDS phases
  double xn[kScatPer], yn[kScatPer];
  auto load_tile = [&](int64_t t0) {
#pragma unroll
    for (int u = 0; u < kScatPer; ++u) {
      const int64_t i = t0 + threadIdx.x + u * kScatThreads;
      xn[u] = i < end ? __builtin_nontemporal_load(X + i) : 0.0;
      yn[u] = i < end ? __builtin_nontemporal_load(Y + i) : 0.0;
    }
  };
  load_tile(beg);
  for (int64_t t0 = beg; t0 < end; t0 += kScatTile) {
    double x[kScatPer], y[kScatPer];
    int32_t row[kScatPer];
#pragma unroll
    for (int u = 0; u < kScatPer; ++u) {
      x[u] = xn[u];
      y[u] = yn[u];
    }
    if (t0 + kScatTile < end) load_tile(t0 + kScatTile);
#pragma unroll
    for (int u = 0; u < kScatPer; ++u) {
      const int64_t i = t0 + threadIdx.x + u * kScatThreads;
      row[u] = i < end ? rowf(x[u], y[u]) : -1;
      if (row[u] >= 0) atomicAdd(&th[row[u]], 1u);
    }
    lds_barrier();
    // exclusive scan of the tile counts (a contiguous run of rows per thread); gd becomes
    // (next global slot - tile start) so that slot + gd is the destination
    uint32_t run = 0;
    for (int r = r0; r < r0 + per && r < nrows; ++r) run += th[r];
    uint32_t inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[wid] = inc;
    lds_barrier();
    uint32_t before = inc - run;
    for (int w = 0; w < wid; ++w) before += wsum[w];
    uint32_t kept = 0;
    for (int w = 0; w < kScatThreads / 64; ++w) kept += wsum[w];
    for (int r = r0; r < r0 + per && r < nrows; ++r) {
      const uint32_t v = th[r];
      th[r] = before;
      gd[r] -= before;
      before += v;
    }
    lds_barrier();
#pragma unroll
    for (int u = 0; u < kScatPer; ++u) {
      if (row[u] < 0) continue;
      const uint32_t slot = atomicAdd(&th[row[u]], 1u);
      sxy[slot] = make_double2(x[u], y[u]);
      sloc[slot] = (uint16_t)(threadIdx.x + u * kScatThreads);
      srow[slot] = (uint16_t)row[u];
    }
    lds_barrier();
#ifndef GF_SCAT_EXP_NOSTORE  // experiment build: the tile is placed in LDS but not written out
    for (uint32_t k = threadIdx.x; k < kept; k += kScatThreads) {
      const uint32_t d = gd[srow[k]] + k;
      oxy[d] = sxy[k];
      oidx[d] = (uint32_t)t0 + sloc[k];
    }
#endif
    lds_barrier();  // (the write-out read gd of any row)
    for (int r = r0; r < r0 + per && r < nrows; ++r) {  // th[r] = tile end of the row
      gd[r] += th[r];
      th[r] = 0u;
    }
    lds_barrier();
  }
}

template <int TILE>
__global__ __launch_bounds__(kScatThreads) void join_scatter_kernel(JoinRowArgs a, JoinQueryArgs q) {
  if ((int)blockIdx.x < q.nblk)
    wc_row_scatter<TILE>(q.qx, q.qy, q.nq, blockIdx.x, q.nblk, q.qn + 2, q.qmat_scan, 0u,
                         reinterpret_cast<double2*>(q.txy), q.tidx, [&](double x, double y) { return join_qrow(q, x, y); });
  else
    wc_row_scatter<TILE>(a.ox, a.oy, a.no, (int64_t)blockIdx.x - q.nblk, a.nblk, a.nrows, a.row_mat_scan, a.mat_base,
                         reinterpret_cast<double2*>(a.soxy), a.soidx,
                         [&](double x, double y) { return join_orow(a, x, y); });
}

// block-wide exclusive scan of one value per thread (NT threads); *total = the block's sum
template <int NT>
__device__ __forceinline__ uint32_t join_block_scan(uint32_t v, uint32_t* total, uint32_t* ws) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    before += w < wid ? ws[w] : 0u;
    tot += ws[w];
  }
  *total = tot;
  __syncthreads();
  return before + inc - v;
}

// Launch 4.  Blocks [0, qn+2): query row ky sorted by sub-cell -- (sub-row, sub-column) keys
// (join_fine_key; f == 1: the clamped column) counted in LDS, scanned, the row's q_off entries
// written (coalesced), the points placed (with their true cells and input index).  Block qn+2:
// the ordinary side's row starts (row_off[j] = M_scan[j][0], row_off[rows] = the total), tasks
// per row (ceil(row / kJoinTask)) and their exclusive scan task_off[0..rows]; it also zeroes
// the overflow count the probe accumulates.
// 256-thread blocks: ~1000 query points per row, and all qn + 3 blocks resident at once
// (five per CU by the LDS histogram) -- with 1024-thread blocks two rounds of latency-bound
// blocks took 34 us for 1M points
constexpr int kSortThreads = 256;
// A row of <= kSortStage points is placed in LDS in its sorted order and written out coalesced
// (its scattered 8-B / 4-B stores cost ~9 of the kernel's 30 us at C4); larger rows scatter
// straight to global memory.
constexpr int kSortStage = 1536;
size_t join_sort_lds_bytes(int32_t f, int32_t qn) {
  return ((size_t)f * f * (qn + 2) * 4 + 15) / 16 * 16 + (size_t)kSortStage * 20;
}
__global__ __launch_bounds__(kSortThreads) void join_sort_finish_kernel(JoinRowArgs a, JoinQueryArgs q) {
  extern __shared__ __attribute__((aligned(16))) char sort_lds[];
  uint32_t* const h = reinterpret_cast<uint32_t*>(sort_lds);  // [H] key histogram -> cursors
  __shared__ uint32_t ws[kSortThreads / 64];
  const int32_t W = q.qn + 2;
  if ((int)blockIdx.x == W) {
    const int nr = a.nrows, per = (nr + kSortThreads - 1) / kSortThreads, j0 = threadIdx.x * per;
    const uint32_t* Ms = a.row_mat_scan;
    const size_t nc = (size_t)kHistSplit * a.nblk, tot_idx = (size_t)nr * nc;
    auto rows_at = [&](int j, uint32_t& b, uint32_t& e) {
      b = Ms[(size_t)j * nc] - a.mat_base;
      e = Ms[j + 1 < nr ? (size_t)(j + 1) * nc : tot_idx] - a.mat_base;
    };
    uint32_t run = 0;
    for (int j = j0; j < j0 + per && j < nr; ++j) {
      uint32_t b, e;
      rows_at(j, b, e);
      a.row_off_w[j] = b;
      run += (e - b + kJoinTask - 1) / kJoinTask;
    }
    uint32_t total;
    uint32_t before = join_block_scan<kSortThreads>(run, &total, ws);
    for (int j = j0; j < j0 + per && j < nr; ++j) {
      uint32_t b, e;
      rows_at(j, b, e);
      a.task_off_w[j] = before;
      before += (e - b + kJoinTask - 1) / kJoinTask;
    }
    if (threadIdx.x == 0) {
      a.row_off_w[nr] = Ms[tot_idx] - a.mat_base;
      a.task_off_w[nr] = total;
    }
    return;
  }
  const int32_t ky = blockIdx.x, H = q.f * q.f * W;  // H <= kRowMax (host)
  const uint32_t* Ms = q.qmat_scan;
  const size_t nc = (size_t)kHistSplit * q.nblk;
  const uint32_t rb = Ms[(size_t)ky * nc], re = Ms[ky + 1 < W ? (size_t)(ky + 1) * nc : (size_t)W * nc];
  const double2* txy = reinterpret_cast<const double2*>(q.txy);
  const uint32_t fH = (uint32_t)((int64_t)q.f * W);  // sub-columns per sub-row
  auto key_of = [&](double2 v, int32_t& cx, int32_t& cy) {
    const uint32_t k = join_fine_key(q, v.x, v.y, cx, cy);
    return k - (uint32_t)ky * (uint32_t)q.f * fH;  // relative to the row's first sub-row
  };
  for (int j = threadIdx.x; j < H; j += kSortThreads) h[j] = 0u;
  __syncthreads();
  for (uint32_t i0 = rb + threadIdx.x; i0 < re; i0 += kSortThreads * 4) {
    double2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = txy[i0 + u * kSortThreads < re ? i0 + u * kSortThreads : rb];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i0 + u * kSortThreads >= re) continue;
      int32_t cx, cy;
      atomicAdd(&h[key_of(v[u], cx, cy)], 1u);
    }
  }
  __syncthreads();
  {  // exclusive scan of h[0..H) in place, as cursors (absolute positions): wave w owns the
     // quarter [w Q, (w + 1) Q), walked in 64-key chunks (lane = key: no bank conflicts -- a
     // contiguous span per thread put 16 lanes on one bank), its total first, then the chunks
     // scanned with the running offset
    constexpr int NW = kSortThreads / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, Q = (H + NW - 1) / NW;
    const int q0 = wid * Q, q1 = q0 + Q < H ? q0 + Q : H;
    uint32_t sum = 0;
    for (int j = q0 + lane; j < q1; j += 64) sum += h[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) ws[wid] = sum;
    __syncthreads();
    uint32_t run = rb;
    for (int w = 0; w < wid; ++w) run += ws[w];
    for (int j0 = q0; j0 < q1; j0 += 64) {  // wave-uniform
      const uint32_t v = j0 + lane < q1 ? h[j0 + lane] : 0u;
      uint32_t inc = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (j0 + lane < q1) h[j0 + lane] = run + inc - v;
      run += (uint32_t)__shfl(inc, 63, 64);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < H; j += kSortThreads) q.q_off[(size_t)ky * H + j] = h[j];
  if (ky == W - 1 && threadIdx.x == 0) q.q_off[(size_t)W * H] = re;
  __syncthreads();
  const bool staged = re - rb <= (uint32_t)kSortStage;  // block-uniform
  double2* const sxy = reinterpret_cast<double2*>(sort_lds + ((size_t)H * 4 + 15) / 16 * 16);
  uint32_t* const sidx = reinterpret_cast<uint32_t*>(sxy + kSortStage);
  for (uint32_t i0 = rb + threadIdx.x; i0 < re; i0 += kSortThreads * 4) {
    double2 v[4];
    uint32_t ix[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t i = i0 + u * kSortThreads < re ? i0 + u * kSortThreads : rb;
      v[u] = txy[i];
      ix[u] = q.tidx[i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i0 + u * kSortThreads >= re) continue;
      int32_t cx, cy;
      const uint32_t pos = atomicAdd(&h[key_of(v[u], cx, cy)], 1u);
      if (staged && q.f > 1) {
        sxy[pos - rb] = v[u];
        sidx[pos - rb] = ix[u];
        continue;
      }
      q.sqx[pos] = v[u].x;
      q.sqy[pos] = v[u].y;
      if (q.f == 1) {  // true cells: only the cell path's clamped-bucket check reads them
        q.sqcx[pos] = cx;
        q.sqcy[pos] = cy;
      }
      q.sqidx[pos] = ix[u];
    }
  }
  if (staged && q.f > 1) {  // the sorted row, coalesced
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < re - rb; t += kSortThreads) {
      const double2 v = sxy[t];
      q.sqx[rb + t] = v.x;
      q.sqy[rb + t] = v.y;
      q.sqidx[rb + t] = sidx[t];
    }
  }
}

// View of one staged query row: bucket kx (0..W-1) holds points [off(kx), off(kx+1)).
// LDS mode: u16 bucket offsets relative to gbase at byte offset loff of the dynamic LDS, the
// row's xy pairs at byte offset lxy (offsets, not pointers, so the loads stay ds_read).
struct QRow {
  int32_t ry;      // clamped row index in [-1, qn]
  uint32_t gbase;  // global index of the row's first point (sorted query arrays)
  uint32_t loff;   // 0xffffffff: the row is read from global memory
  uint32_t lxy;
};

struct JoinProbeHdr {
  int32_t row, fit;
  uint32_t need;     // staged bytes of the task's query rows
  uint32_t beg, end;
  uint32_t wsum[kJoinThreads / 64];
  QRow rows[kJoinMaxRows];
  uint32_t g0;       // fine path: sorted index of the first staged query point
  uint32_t gm;       // fine path: staged query points (0: none; their indices are in LDS)
  uint32_t lqidx;    // fine path: LDS byte offset of the staged query indices
  uint32_t kept;     // the task's points inside the grid (sorted; the rest dropped)
};
constexpr int kJoinHdrBytes = (int)((sizeof(JoinProbeHdr) + 15) / 16 * 16);
// pairs a wave collects in LDS: a wave-step's pairs (64 points) normally fit, so the walk's
// inner loop has no global memory operation (the buffer is written out after the step, or when a
// round could overflow it -- outside the round loop, join_*_walk)
constexpr int kJoinWaveBuf = 384;
constexpr int kJoinRound = 4;  // candidates per lane per walk round (their loads in flight together)
static_assert(kJoinTask <= 8192, "local index packed in 13 bits");
// Dynamic LDS of the probe: header | staged rows (budget) | sorted (column << 13 | local index)
// u32 per point | union { task prologue: u16 column keys + column histogram [columns + 1]
// (columns = qn, or f(qn+2) sub-columns on the fine path); walk: the wave pair buffers }
static size_t join_probe_union_bytes(int32_t qn, int32_t f) {
  const size_t cols = f > 1 ? (size_t)f * ((size_t)qn + 2) : (size_t)qn;
  const size_t pro = 2 * (size_t)kJoinTask + 4 * (cols + 1), wb = (size_t)kJoinWaveBuf * 8 * (kJoinThreads / 64);
  return ((pro > wb ? pro : wb) + 15) / 16 * 16;
}
static size_t join_probe_lds_fixed(int32_t qn, int32_t f) {
  return kJoinHdrBytes + 4 * (size_t)kJoinTask + join_probe_union_bytes(qn, f);
}
static size_t join_probe_lds_bytes(int lds_budget, int32_t qn, int32_t f) {
  return join_probe_lds_fixed(qn, f) + (size_t)lds_budget;
}

// The staged query rows get what the fixed layout leaves of the 160 KB (one block per CU).  A
// task whose rows exceed the budget reads them from global memory (same results, slower).
int join_probe_budget(int64_t nq, int32_t qn, int64_t c, int32_t f) {
  const int64_t W = (int64_t)qn + 2;
  const double mean = (double)nq / (double)(qn > 0 ? qn : 1);
  size_t need;
  if (f > 1) {  // 3 sub-rows
    const double m = mean * 3.0 / (double)f;
    need = 3 * join_row_lds_bytes((int64_t)f * W, 0) + (size_t)(m + 4.0 * std::sqrt(m) + 16.0) * 20;
  } else {
    need = (size_t)(2 * c + 1) * join_row_lds_bytes(W, (uint32_t)(mean + 4.0 * std::sqrt(mean) + 16.0));
  }
  // one block per CU (the probe's registers: > 64 VGPRs), so the staged rows get the rest
  (void)need;
  const size_t fixed = join_probe_lds_fixed(qn, f), full = 160 * 1024;
  return fixed < full ? (int)(full - fixed) : 0;
}

// Fine path factor: the largest f <= 4 whose sub-cells are wider than r with a margin far
// above the rounding of the sub-cell bounds (cl/f against r: relative 1e-9, plus 64 ulps of the
// largest grid coordinate), and whose per-row sort keys fit the LDS histogram.
int32_t join_fine_factor(double cl, double r, int32_t qn, double maxabs) {
  const double slack = 1e-9 * cl + 64.0 * std::ldexp(1.0, std::ilogb(maxabs > 1.0 ? maxabs : 1.0) - 52);
  for (int32_t f = 4; f >= 2; --f) {
    if ((int64_t)f * f * ((int64_t)qn + 2) > kRowMax || (int64_t)f * ((int64_t)qn + 2) >= (1 << 13)) continue;
    if (cl / f - slack > r * (1.0 + 1e-12)) return f;
  }
  return 1;
}

// Wave-uniform value (the compiler cannot prove it): one readfirstlane, so the loops that use
// it run on scalar registers.
__device__ __forceinline__ uint32_t join_uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int32_t join_uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

struct JoinLane {  // this lane's ordinary point
  double px, py;
  int32_t cx, cy;
  uint32_t pidx;
};

__device__ __forceinline__ uint64_t join_uni64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}

// A wave's output chunk (wave-uniform): positions [base, base + chunk) of the reserved space,
// `fill` of them used (fill == chunk: take a new one at the next store).
struct JoinWaveOut {
  uint64_t base;
  uint32_t fill;
};
__device__ __forceinline__ void join_vstore(const JoinOut& o, uint64_t pos, uint2 v) {
  if (pos < o.cap) join_store(o.pairs, o.aligned, pos, v);
  else if (pos - o.cap < o.spill_cap) o.spill[pos - o.cap] = v;
}
// The wave stores entries get(0 .. cnt) (cnt wave-uniform) at its chunk's next positions,
// taking new chunks (one device atomic each) as they fill: consecutive lanes, consecutive slots.
template <class Get>
__device__ __forceinline__ void join_emit(const JoinOut& o, JoinWaveOut& w, uint32_t cnt, Get get) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t done = 0;
  while (done < cnt) {  // wave-uniform
    if (w.fill >= o.chunk) {
      unsigned long long b = 0;
      if (lane == 0) b = atomicAdd(o.gctr, (unsigned long long)o.chunk);
      w.base = join_uni64(b);
      w.fill = 0;
    }
    const uint32_t take = cnt - done < o.chunk - w.fill ? cnt - done : o.chunk - w.fill;
    for (uint32_t i = lane; i < take; i += 64) join_vstore(o, w.base + w.fill + i, get(done + i));
    w.fill += take;
    done += take;
  }
}
// the wave's last chunk, for the fix-up (hole = [base + fill, base + chunk))
__device__ __forceinline__ void join_emit_close(const JoinOut& o, const JoinWaveOut& w, uint32_t wslot) {
  if ((threadIdx.x & 63) == 0) {
    o.tail_base[wslot] = w.fill <= o.chunk && w.base != ~0ull ? w.base : ~0ull;
    o.tail_fill[wslot] = w.fill;
  }
}

// The wave's pair buffer in LDS: hits are appended in ballot order (one mbcnt per hit round,
// the count stays in a scalar register); past kJoinWaveBuf - 64 the wave writes the buffer out
// (join_emit: coalesced stores into its output chunk) with each query slot mapped to its query
// index (from LDS when the fine path staged it, else an L2 gather of the sorted query side).
struct JoinWaveBuf {
  uint2* buf;
  uint32_t cnt;
  __device__ __forceinline__ void flush(const JoinRowArgs& a, JoinProbeHdr& hd, JoinWaveOut& wo) {
    const uint32_t g0 = hd.g0, gm = join_uni(hd.gm);
    const uint32_t* lq = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(&hd) + hd.lqidx);
    const uint2* b = buf;
    wave_lds_sync();  // the entries other lanes of this wave pushed (intra-wave LDS hand-off)
    auto get = [&](uint32_t i) {
      const uint2 v = b[i];
      const uint32_t qi = v.y & 0x80000000u ? v.y & 0x7fffffffu : (v.y - g0 < gm ? lq[v.y - g0] : a.sqidx[v.y]);
      return make_uint2(v.x, qi);
    };
    join_emit(a.out, wo, cnt, get);
    cnt = 0;
  }
  // one round's hits: hit i of this lane (candidate q[i]) goes after all hits of rounds < i.
  // The caller guarantees room for a full round (room()).
  template <int R>
  __device__ __forceinline__ void push(const bool (&hit)[R], uint32_t p, const uint32_t (&q)[R]) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const uint64_t m = __ballot(hit[i]);
      if (hit[i])
        buf[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
            make_uint2(p, q[i]);
      cnt += (uint32_t)__popcll(m);
    }
  }
  __device__ __forceinline__ bool room() const { return cnt <= (uint32_t)(kJoinWaveBuf - 64 * kJoinRound); }
};

// One lane's candidates [tb, te) of one query row (relative to the row's first point gb): the
// lanes walk their own runs together, two candidates per round, until every run is done (the
// exit is a ballot, so the loop and the pair count stay wave-uniform).  Column-sorted lanes
// share columns, so most lanes of a round read the same few LDS addresses.  SLOW: the run
// touches a clamped bucket or row, so each candidate's true cell is checked (Chebyshev <= c).
template <int MODE, bool LDS, bool SLOW>
__device__ __forceinline__ void join_lane_run(const JoinRowArgs& a, const double2* lxy, uint32_t gb, uint32_t tb,
                                              uint32_t te, const JoinLane& ln, JoinWaveBuf& wbuf, JoinProbeHdr& hd,
                                              JoinWaveOut& wo) {
  const uint32_t len = te - tb;
  auto test = [&](bool act, uint32_t t, double2 q) {
    bool in = act;
    if constexpr (SLOW) {
      if (act) {
        const int64_t ddx = (int64_t)a.sqcx[gb + t] - ln.cx, ddy = (int64_t)a.sqcy[gb + t] - ln.cy;
        in = ddx <= a.c && ddx >= -a.c && ddy <= a.c && ddy >= -a.c;
      }
    }
    const double dx = ln.px - q.x, dy = ln.py - q.y;
    bool ok;
    if constexpr (MODE == 0) ok = dx * dx + dy * dy <= a.s_r;  // s <= smax(r) <=> sqrt(s) <= r
    else ok = a.approx || (a.metric == 0 ? dx * dx + dy * dy <= a.s_r : fdlibm_hypot(dx, dy) <= a.r);
    return in && ok;
  };
  constexpr int R = kJoinRound;
  uint32_t k = 0;
  for (;;) {  // the round loop stops only to write a full buffer out (outside it: no VMEM inside)
    bool full = false;
    for (; __ballot(k < len) != 0; k += R) {
      if (!wbuf.room()) {
        full = true;
        break;
      }
      bool act[R], hit[R];
      uint32_t t[R], q[R];
      double2 v[R];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        act[i] = k + i < len;
        t[i] = tb + (act[i] ? k + i : 0u);
        q[i] = gb + t[i];
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        if constexpr (LDS) {  // a stale slot for a finished lane reads in-bounds LDS, masked below
          v[i] = lxy[t[i]];
        } else {
          v[i] = make_double2(0.0, 0.0);
          if (act[i]) v[i] = make_double2(a.sqx[q[i]], a.sqy[q[i]]);
        }
      }
#pragma unroll
      for (int i = 0; i < R; ++i) hit[i] = test(act[i], t[i], v[i]);
      wbuf.push<R>(hit, ln.pidx, q);
    }
    if (!full) break;
    wbuf.flush(a, hd, wo);
  }
}

// Fine path: one lane's candidates are three runs [b_s, e_s) of the sorted query side (the
// sub-columns SC-1 .. SC+1 of the sub-rows SR-1 .. SR+1 around its sub-cell), walked as ONE
// concatenated sequence, R candidates per round until every lane is done (ballot exit).  Indices
// are relative to the first staged point g0; LDS: the staged xy at those indices.
template <int MODE, bool LDS, int R>
__device__ __forceinline__ void join_fine_walk(const JoinRowArgs& a, const double2* lxy, uint32_t g0,
                                               const uint32_t (&b)[3], const uint32_t (&e)[3], const JoinLane& ln,
                                               JoinWaveBuf& wbuf, JoinProbeHdr& hd, JoinWaveOut& wo) {
  const uint32_t L0 = e[0] - b[0], L1 = L0 + (e[1] - b[1]), L2 = L1 + (e[2] - b[2]);
  const uint32_t d0 = b[0], d1 = b[1] - L0, d2 = b[2] - L1;  // run s: index = k + d_s (mod 2^32)
  uint32_t k = 0;
  for (;;) {  // as join_lane_run: the buffer is written out only outside the round loop
    bool full = false;
    for (; __ballot(k < L2) != 0; k += R) {
      if (!wbuf.room()) {
        full = true;
        break;
      }
      bool hit[R];
      uint32_t t[R], q[R];
      double2 v[R];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const uint32_t kk = k + i;
        t[i] = kk < L2 ? kk + (kk < L0 ? d0 : (kk < L1 ? d1 : d2)) : 0u;
        q[i] = g0 + t[i];
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        if constexpr (LDS) {  // a finished lane reads staged slot 0 (some lane has a candidate)
          v[i] = lxy[t[i]];
        } else {
          v[i] = make_double2(0.0, 0.0);
          if (k + i < L2) v[i] = make_double2(a.sqx[q[i]], a.sqy[q[i]]);
        }
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double dx = ln.px - v[i].x, dy = ln.py - v[i].y;
        bool ok;
        if constexpr (MODE == 0) ok = dx * dx + dy * dy <= a.s_r;
        else ok = a.metric == 0 ? dx * dx + dy * dy <= a.s_r : fdlibm_hypot(dx, dy) <= a.r;
        hit[i] = k + i < L2 && ok;
      }
      wbuf.push<R>(hit, ln.pidx, q);
    }
    if (!full) break;
    wbuf.flush(a, hd, wo);
  }
}


// One block per task = <= kJoinTask ordinary points of one cell row.  The 2c+1 query rows
// around it are staged in LDS (u16 bucket offsets per column + xy), then the task's points are
// counting-sorted by column in LDS.  A wave takes 64 consecutive points of that order and, per
// staged row, each lane walks its own candidate run (the buckets cx-c .. cx+c of that row = the
// replicated-key match, true cell within Chebyshev c) with the exact distance test.  Sorting
// makes the lanes' runs overlap, so the per-round LDS reads hit few distinct addresses, and
// the rounds per row are the longest run among ~8 columns instead of the union of all of them.
// Pairs go through the wave's LDS buffer into its output chunk in coalesced runs (join_emit);
// join_fixup_* makes the output dense.
//
// FINE (the fine path, f > 1: c == 1, exact distances, one grid for both sides, cl/f > r): a
// pair needs d <= r, so its points lie in sub-cells at most one apart on each axis (sub-cells are
// wider than r and the sub-cell index is monotone), and then their cells are at most one apart --
// the key match is implied.  Every lane therefore tests only the 3 x 3 sub-cells around its own:
// runs of the f + 2 sub-rows the task stages (cl^2 (3/f)^2 of candidates instead of 9 cl^2).
// Query points outside the grid sit in the sub-cell adjacent to it (join_fine_key), so lanes in
// the grid's edge cells need no true-cell check.  (A first version sent every wave holding an
// edge lane through the cell path over global memory: ~2 such waves per task, each a chain of
// dependent global round trips the whole task waited for: probe 282 -> 225 us without it.)
template <int MODE, int FINE>  // MODE 0: exact, metric 0 (squared-distance bound); 1: approximate or hypot
__device__ __forceinline__ void join_probe_task(const JoinRowArgs& a, uint32_t task, char* const lds_base,
                                                JoinWaveOut& wo) {
  JoinProbeHdr& hd = *reinterpret_cast<JoinProbeHdr*>(lds_base);
  char* const lds = lds_base + kJoinHdrBytes;
  QRow* const rows = hd.rows;
  const int64_t W = (int64_t)a.qn + 2, c = a.c, qn = a.qn;
  const int32_t f = FINE ? a.f : 1;
  const int64_t fW = (int64_t)f * W;  // sub-columns (FINE) per sub-row
  // the task's row: the one j with task_off[j] <= task < task_off[j+1] (a parallel search --
  // one round of loads, where a serial binary search costs ~10 dependent ones)
  if (threadIdx.x == 0) {
    hd.need = 0u;
    hd.fit = 1;
    hd.gm = 0u;
    hd.g0 = 0u;
    hd.lqidx = 0u;
  }
  for (int j = threadIdx.x; j < a.nrows; j += kJoinThreads)
    if (a.task_off[j] <= task && task < a.task_off[j + 1]) hd.row = j;
  __syncthreads();
  const int32_t orow = hd.row, cy = orow;  // the task's cell row
  const int64_t r0 = cy - c < -1 ? -1 : cy - c, r1 = cy + c > qn ? qn : cy + c;
  const int nrows = (int)(r1 - r0 + 1);
  const size_t fine_rb = join_row_lds_bytes(fW, 0);          // one staged sub-row's u16 offsets
  if (threadIdx.x == 0) {
    // the row's tasks split it evenly (10000 points: 2 x 5000, not 8192 + 1808)
    const uint32_t k = task - a.task_off[orow], nt = a.task_off[orow + 1] - a.task_off[orow];
    const uint32_t rb = a.row_off[orow], re = a.row_off[orow + 1], size = (re - rb + nt - 1) / nt;
    hd.beg = rb + k * size;
    hd.end = rb + (k + 1) * size < re ? rb + (k + 1) * size : re;
    if (FINE) {  // sub-rows f(cy+1)-1 .. f(cy+1)+f: consecutive in the sorted query side
      {
        const int64_t fy0 = (int64_t)f * (cy + 1) - 1;
        const uint32_t g0 = a.q_off[fy0 * fW], g1 = a.q_off[(fy0 + f + 2) * fW], m = g1 - g0;
        hd.g0 = g0;
        hd.need = (uint32_t)((size_t)(f + 2) * fine_rb + (size_t)m * 20);
        hd.fit = m < 65536u && hd.need <= (uint32_t)a.lds_budget;
        if (hd.fit) {
          hd.gm = m;
          hd.lqidx = (uint32_t)(kJoinHdrBytes + (size_t)(f + 2) * fine_rb + (size_t)m * 16);
        }
      }
    }
  }
  if (!FINE && (int)threadIdx.x < nrows && nrows <= kJoinMaxRows) {  // staged bytes of every query row
    const uint32_t* qo = a.q_off + (r0 + threadIdx.x + 1) * W;
    const uint32_t m = qo[W] - qo[0];
    if (m >= 65536u) hd.fit = 0;
    atomicAdd(&hd.need, (uint32_t)join_row_lds_bytes(W, m < 65536u ? m : 65536u));
  }
  __syncthreads();
  const bool fit = FINE ? hd.fit != 0 : (hd.fit && nrows <= kJoinMaxRows && hd.need <= (uint32_t)a.lds_budget);
  const uint32_t g0 = FINE ? hd.g0 : 0u;
  if (FINE) {
    if (fit) {  // u16 offsets (relative to g0) of every sub-column of the f + 2 sub-rows, then xy, indices
      const int64_t fy0 = (int64_t)f * (cy + 1) - 1;
      for (int sr = 0; sr < f + 2; ++sr) {
        uint16_t* lo16 = reinterpret_cast<uint16_t*>(lds + sr * fine_rb);
        const uint32_t* qo = a.q_off + (fy0 + sr) * fW;
        for (int64_t t = threadIdx.x; t <= fW; t += kJoinThreads) lo16[t] = (uint16_t)(qo[t] - g0);
      }
      double2* lxy = reinterpret_cast<double2*>(lds + (f + 2) * fine_rb);
      const uint32_t m = hd.gm;
      uint32_t* lq = reinterpret_cast<uint32_t*>(lxy + m);
      for (uint32_t t = threadIdx.x; t < m; t += kJoinThreads) {
        lxy[t] = make_double2(a.sqx[g0 + t], a.sqy[g0 + t]);
        lq[t] = a.sqidx[g0 + t];
      }
    }
  } else {
    // stage (or describe) the query rows
    size_t off = 0;
    for (int j = 0; j < nrows; ++j) {
      const int64_t ry = r0 + j;
      const uint32_t* qo = a.q_off + (ry + 1) * W;
      const uint32_t b = qo[0], e = qo[W];
      if (fit) {
        const uint32_t o16 = (uint32_t)off;
        uint16_t* lo16 = reinterpret_cast<uint16_t*>(lds + off);
        off += ((size_t)(W + 1) * 2 + 15) / 16 * 16;
        const uint32_t oxy = (uint32_t)off;
        double2* lxy = reinterpret_cast<double2*>(lds + off);
        off += (size_t)(e - b) * 16;
        for (int64_t t = threadIdx.x; t <= W; t += kJoinThreads) lo16[t] = (uint16_t)(qo[t] - b);
        for (uint32_t t = threadIdx.x; t < e - b; t += kJoinThreads) lxy[t] = make_double2(a.sqx[b + t], a.sqy[b + t]);
        if (threadIdx.x == 0) rows[j] = QRow{(int32_t)ry, b, o16, oxy};
      } else if (threadIdx.x == 0) {
        rows[j] = QRow{(int32_t)ry, b, 0xffffffffu, 0u};
      }
    }
  }
  // the task's points, counting-sorted by column: column per point (u16; FINE: sub-column |
  // sub-row << 13), column histogram -> exclusive scan (cursors) -> sorted (column << 13 |
  // local index; FINE: sub-column << 15 | sub-row << 13 | local index)
  const int32_t ncol = FINE ? (int32_t)fW : a.qn;
  uint32_t* const lsort = reinterpret_cast<uint32_t*>(lds + a.lds_budget);
  uint16_t* const lcx = reinterpret_cast<uint16_t*>(lsort + kJoinTask);
  uint32_t* const hist = reinterpret_cast<uint32_t*>(lcx + kJoinTask);  // [ncol + 1] (kJoinTask even: 4-B aligned)
  const uint32_t beg = hd.beg, cnt = hd.end - hd.beg;
  for (int j = threadIdx.x; j <= ncol; j += kJoinThreads) hist[j] = 0u;
  __syncthreads();
  {
    constexpr int PER = kJoinTask / kJoinThreads;  // all loads in flight before the first use
    double xs[PER], ys[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const uint32_t i = threadIdx.x + u * kJoinThreads;
      if (FINE) {
        const double2 v = i < cnt ? reinterpret_cast<const double2*>(a.soxy)[beg + i] : make_double2(0.0, 0.0);
        xs[u] = v.x;
        ys[u] = v.y;
      } else {
        xs[u] = i < cnt ? a.soxy[2 * (size_t)(beg + i)] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const uint32_t i = threadIdx.x + u * kJoinThreads;
      if (i < cnt) {
        const int32_t cx = cell_index(xs[u], a.u_minX, a.u_cl);  // the row is in the grid, the column maybe not
        if (cx < 0 || cx >= qn) {
          lcx[i] = 0xFFFFu;  // outside the grid: no key matches (never a valid key: < 4 << 13)
          continue;
        }
        int32_t col = cx, key = cx;
        if (FINE) {
          col = f * (cx + 1) + join_sub(xs[u], a.u_minX, a.u_cl, cx, a.fs, f);
          key = join_sub(ys[u], a.u_minY, a.u_cl, cy, a.fs, f) << 13 | col;
        }
        lcx[i] = (uint16_t)key;
        atomicAdd(&hist[col], 1u);
      }
    }
  }
  __syncthreads();
  {  // exclusive scan of hist[0 .. ncol) in place (each thread a contiguous run of columns)
    uint32_t* const wsum = hd.wsum;
    const int per = (ncol + kJoinThreads - 1) / kJoinThreads, j0 = threadIdx.x * per;
    uint32_t run = 0;
    for (int j = j0; j < j0 + per && j < ncol; ++j) run += hist[j];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t before = inc - run;
    for (int w = 0; w < wid; ++w) before += wsum[w];
    for (int j = j0; j < j0 + per && j < ncol; ++j) {
      const uint32_t v = hist[j];
      hist[j] = before;
      before += v;
    }
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int w = 0; w < kJoinThreads / 64; ++w) t += wsum[w];
      hd.kept = t;
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < cnt; i += kJoinThreads) {
    const uint32_t key = lcx[i];
    if (key == 0xFFFFu) continue;
    if (FINE) lsort[atomicAdd(&hist[key & 8191u], 1u)] = (key & 8191u) << 15 | (key >> 13) << 13 | i;
    else lsort[atomicAdd(&hist[key], 1u)] = key << 13 | i;
  }
  __syncthreads();  // lcx is dead from here: its space holds the wave buffers

  const uint32_t lane = threadIdx.x & 63;
  const int32_t qnn = a.qn, cc = (int32_t)c;
  JoinWaveBuf wbuf{reinterpret_cast<uint2*>(lcx) + (threadIdx.x >> 6) * kJoinWaveBuf, 0u};
  // the next wave-step's points are fetched before this step's candidates are walked;
  // branch-free (a lane past the end re-reads entry 0): a load under a branch is waited on at the
  // branch's join
  struct Pt {
    double2 v;
    uint32_t idx, e;
  };
  const uint32_t kept = hd.kept;
  auto fetch = [&](uint32_t s) {  // past the end: entry 0 of the task's points (always present)
    Pt p;
    p.e = s + lane < kept ? lsort[s + lane] : 0u;
    p.v = reinterpret_cast<const double2*>(a.soxy)[beg + (p.e & 8191u)];
    p.idx = a.soidx[beg + (p.e & 8191u)];
    return p;
  };
  // per wave-step: the next step's points are fetched, this step's candidates walked (LDS only,
  // pairs into the wave buffer), then -- the fetch has landed during the walk -- the wait is
  // taken BEFORE the step's stores go out: a wait after them would be vmcnt(0) (the compiler
  // cannot count a data-dependent number of stores) and every step would pay the store latency
  Pt cur = fetch((threadIdx.x >> 6) * 64);
  for (uint32_t s = (threadIdx.x >> 6) * 64; s < kept; s += kJoinThreads) {  // wave-uniform
    const bool valid = s + lane < kept;
    const Pt nxt = fetch(s + kJoinThreads);
    auto step_end = [&]() {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nxt is in registers
      if (!wbuf.room()) wbuf.flush(a, hd, wo);  // the next step starts with room for a round
      cur = nxt;
    };
    if (FINE) {
      const int32_t col = (int32_t)(cur.e >> 15), sub = (int32_t)((cur.e >> 13) & 3u);
      const int32_t cx = col / f - 1;
      {
        const JoinLane ln{cur.v.x, cur.v.y, cx, cy, cur.idx};
        uint32_t b[3], e[3];
        if (fit) {
          const uint16_t* lo = reinterpret_cast<const uint16_t*>(lds);
          const uint32_t rs = (uint32_t)(fine_rb / 2);
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            b[k] = valid ? lo[(sub + k) * rs + col - 1] : 0u;
            e[k] = valid ? lo[(sub + k) * rs + col + 2] : 0u;
          }
          const double2* lxy = reinterpret_cast<const double2*>(lds + (f + 2) * fine_rb);
          join_fine_walk<MODE, true, kJoinRound>(a, lxy, g0, b, e, ln, wbuf, hd, wo);
        } else {
          const int64_t fy0 = (int64_t)f * (cy + 1) - 1;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const uint32_t* qo = a.q_off + (fy0 + sub + k) * fW;
            b[k] = valid ? qo[col - 1] - g0 : 0u;
            e[k] = valid ? qo[col + 2] - g0 : 0u;
          }
          join_fine_walk<MODE, false, kJoinRound>(a, nullptr, g0, b, e, ln, wbuf, hd, wo);
        }
      }
      step_end();
      continue;
    }
    const JoinLane ln{cur.v.x, cur.v.y, valid ? (int32_t)(cur.e >> 13) : 0, cy, cur.idx};
    const int32_t kb = (ln.cx - cc < -1 ? -1 : ln.cx - cc) + 1, ke = (ln.cx + cc > qnn ? qnn : ln.cx + cc) + 2;
    for (int j = 0; j < nrows; ++j) {
      const QRow R = rows[j];
      const int32_t ry = join_uni(R.ry);
      const uint32_t gb = join_uni(R.gbase);
      const bool brow = ry < 0 || ry >= qnn;  // clamped row: the true cells differ
      if (join_uni(R.loff) != 0xffffffffu) {
        const uint16_t* lo16 = reinterpret_cast<const uint16_t*>(lds + join_uni(R.loff));
        const double2* lxy = reinterpret_cast<const double2*>(lds + join_uni(R.lxy));
        const uint32_t tb = valid ? lo16[kb] : 0u, te = valid ? lo16[ke] : 0u;
        // clamped buckets 0 (column -1) and W-1 (column qn): [0, lo16[1]) and [lo16[W-1], ...)
        const bool slow = te > tb && (brow || kb == 0 || ke == (int32_t)W);
        if (__ballot(slow) != 0) join_lane_run<MODE, true, true>(a, lxy, gb, tb, te, ln, wbuf, hd, wo);
        else join_lane_run<MODE, true, false>(a, lxy, gb, tb, te, ln, wbuf, hd, wo);
      } else {
        const uint32_t* qo = a.q_off + (size_t)(ry + 1) * W;
        const uint32_t tb = valid ? qo[kb] - gb : 0u, te = valid ? qo[ke] - gb : 0u;
        const bool slow = te > tb && (brow || kb == 0 || ke == (int32_t)W);
        if (__ballot(slow) != 0) join_lane_run<MODE, false, true>(a, nullptr, gb, tb, te, ln, wbuf, hd, wo);
        else join_lane_run<MODE, false, false>(a, nullptr, gb, tb, te, ln, wbuf, hd, wo);
      }
    }
    step_end();
  }
  if (wbuf.cnt > 0) wbuf.flush(a, hd, wo);
  __syncthreads();  // the task's LDS is reused by the next one
}

// Persistent: gridDim blocks (one per CU, the staged rows fill its LDS) take the tasks in an
// XCD-aware order -- workgroups go round-robin to the 8 XCDs, so XCD x gets the consecutive
// tasks [x * per, (x + 1) * per): neighbouring row tasks stage the same query rows, and they meet
// in the same L2.  Each wave keeps one output chunk across its tasks (join_emit), closed at exit.
template <int MODE, int FINE>
__global__ __launch_bounds__(kJoinThreads) void join_row_probe_kernel(JoinRowArgs a) {
  // every LDS variable lives in the dynamic region, header first (a static __shared__ block in
  // front would shift the dynamic base off 16 B: misaligned ds_read_b128 of the staged xy)
  extern __shared__ __attribute__((aligned(16))) char lds_base[];
  const uint32_t ntask = a.task_off[a.nrows];
  const uint32_t per = (ntask + 7) / 8, xcd = blockIdx.x & 7u, nb = (gridDim.x + 7 - xcd) / 8;
  JoinWaveOut wo{~0ull, a.out.chunk};
  for (uint32_t k = blockIdx.x >> 3; k < per; k += nb) {  // block-uniform
    const uint32_t task = xcd * per + k;
    if (task < ntask) join_probe_task<MODE, FINE>(a, task, lds_base, wo);
  }
  join_emit_close(a.out, wo, blockIdx.x * (kJoinThreads / 64) + (threadIdx.x >> 6));
}

// ---- streaming probe (experiment, GF_FLAG_JOIN_STREAM) --------------------------------------
// Only the query side is bucketed (sorted by sub-cell, q_off); the ordinary points are read once
// in input order, one lane each, and every lane walks its 3 x 3 sub-cell neighbourhood straight
// from the sorted query arrays in global memory (L2 / Infinity Cache gathers: the lanes of a wave
// hold unrelated points).  The alternative the row-bucketed path is measured against (VERDICT r02
// "bucket only the query side; stream the ordinary points").  Fine path only (f > 1).
template <int MODE>
__global__ __launch_bounds__(kBlock) void join_stream_kernel(JoinRowArgs a) {
  __shared__ uint2 wbuf[kBlock / 64][kJoinWaveBuf];
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint2* const buf = wbuf[wid];
  uint32_t cnt = 0;
  JoinWaveOut wo{~0ull, a.out.chunk};
  const int32_t f = a.f, qn = a.qn;
  const int64_t fW = (int64_t)f * (qn + 2);
  auto flush = [&]() {
    wave_lds_sync();  // the entries other lanes of this wave pushed (intra-wave LDS hand-off)
    join_emit(a.out, wo, cnt, [&](uint32_t i) {
      const uint2 v = buf[i];
      return make_uint2(v.x, a.sqidx[v.y]);
    });
    cnt = 0;
  };
  const int64_t nwave = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t s0 = ((int64_t)blockIdx.x * (kBlock / 64) + wid) * 64; s0 < a.no; s0 += nwave * 64) {  // wave-uniform
    const int64_t p = s0 + lane;
    const bool valid = p < a.no;
    const double px = valid ? a.ox[p] : 0.0, py = valid ? a.oy[p] : 0.0;
    const int32_t cx = cell_index(px, a.u_minX, a.u_cl), cy = cell_index(py, a.u_minY, a.u_cl);
    const bool in = valid && cx >= 0 && cy >= 0 && cx < qn && cy < qn;
    uint32_t b[3] = {0u, 0u, 0u}, e[3] = {0u, 0u, 0u};
    if (in) {
      const int32_t col = f * (cx + 1) + join_sub(px, a.u_minX, a.u_cl, cx, a.fs, f);
      const int32_t srow = f * (cy + 1) + join_sub(py, a.u_minY, a.u_cl, cy, a.fs, f);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const uint32_t* qo = a.q_off + (int64_t)(srow - 1 + k) * fW;
        b[k] = qo[col - 1];
        e[k] = qo[col + 2];
      }
    }
    const uint32_t L0 = e[0] - b[0], L1 = L0 + (e[1] - b[1]), L2 = L1 + (e[2] - b[2]);
    const uint32_t d0 = b[0], d1 = b[1] - L0, d2 = b[2] - L1;
    constexpr int R = 4;
    for (uint32_t k = 0; __ballot(k < L2) != 0; k += R) {
      bool hit[R];
      uint32_t q[R];
      double2 v[R];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const uint32_t kk = k + i;
        q[i] = kk < L2 ? kk + (kk < L0 ? d0 : (kk < L1 ? d1 : d2)) : 0u;
        v[i] = kk < L2 ? make_double2(a.sqx[q[i]], a.sqy[q[i]]) : make_double2(0.0, 0.0);
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double dx = px - v[i].x, dy = py - v[i].y;
        const bool ok = MODE == 0 ? dx * dx + dy * dy <= a.s_r : fdlibm_hypot(dx, dy) <= a.r;
        hit[i] = k + i < L2 && ok;
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const uint64_t m = __ballot(hit[i]);
        if (m == 0) continue;
        if (hit[i])
          buf[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
              make_uint2((uint32_t)p, q[i]);
        cnt += (uint32_t)__popcll(m);
        if (cnt > kJoinWaveBuf - 64) flush();
      }
    }
  }
  if (cnt > 0) flush();
  join_emit_close(a.out, wo, blockIdx.x * (kBlock / 64) + wid);
}

hipError_t launch_join_stream(gf_ctx* ctx, const JoinRowArgs& a) {
  KTimer t(ctx, GF_K_JOIN_PROBE);
  const dim3 g(a.out.nwaves / (kBlock / 64));
  if (!a.approx && a.metric == 0) hipLaunchKernelGGL(join_stream_kernel<0>, g, dim3(kBlock), 0, ctx->stream, a);
  else hipLaunchKernelGGL(join_stream_kernel<1>, g, dim3(kBlock), 0, ctx->stream, a);
  return hipGetLastError();
}

// ---- band probe (the fine path's default) ---------------------------------------------------
// Block b takes an equal slice of the row-bucketed ordinary points (slices of one XCD are
// consecutive: neighbouring rows share query sub-rows in its L2).  A slice crosses ~2-3 rows;
// per row segment the block stages the row's query BAND -- the f + 2 sub-rows around the row:
// u16 sub-column offsets (absolute staged slots), xy and query indices -- in LDS, then streams
// the segment's points in bucket order: coalesced 16-B + 4-B loads, two points per lane per
// wave-step with the next step in flight, no per-task sort (the row probe's sorted lanes gathered
// their points from global memory one wave-step at a time and paid a histogram / scan / scatter
// per 8192-point task).  Each lane tests the 3 x 3 sub-cells around its own (see the fine path
// above) out of LDS.  A band larger than the staging budget (clustered input) is staged in
// sub-column WINDOWS [c0, c1) -- the query points of sub-columns [c0 - 1, c1 + 1) of every band
// sub-row -- and the segment is streamed once per window, each lane working only in the window of
// its sub-column; a window that cannot hold even one sub-column reads that sub-column's
// candidates from global memory.
// Pairs: the wave's LDS buffer (ordinary index, staged slot | global index), written out between
// wave-steps into the block's REGION of the output (JoinOut.regions): one LDS atomic per flush,
// no device atomic unless the region is full (then the dense overflow area).  Per-wave output
// chunks cost one device atomic each on ONE counter: ~20K of them serialised at the memory side
// (the row probe: 240 us with block chunks, 361 us with wave chunks).
#ifndef GF_BAND_THREADS  // experiment builds: a smaller block (with GF_BAND_LDS_KB / GF_BAND_MINBLK)
#define GF_BAND_THREADS 1024
#endif
constexpr int kBandThreads = GF_BAND_THREADS, kBandWaves = kBandThreads / 64;
static_assert(kBandThreads % 64 == 0 && kBandThreads <= 1024, "whole waves");
typedef const uint32_t __attribute__((address_space(3)))* lds_u32;
#ifndef GF_BAND_BUF
#define GF_BAND_BUF 512
#endif
constexpr int kBandBuf = GF_BAND_BUF;        // pairs per wave buffer (written out before a round could overflow it)
#ifndef GF_BAND_R
#define GF_BAND_R 4
#endif
constexpr int kBandRound = GF_BAND_R;  // candidates per lane per walk round
#ifndef GF_BAND_R1
#define GF_BAND_R1 2
#endif
constexpr int kBandRound1 = GF_BAND_R1;  // the same for MODE 1 (hypot: at 4 its walk spills to scratch in the loops)
#ifndef GF_BAND_PAIR
#define GF_BAND_PAIR 1
#endif
#ifndef GF_BAND_FLATSEL
#define GF_BAND_FLATSEL 1
#endif
constexpr bool kBandPair = GF_BAND_PAIR != 0;  // sparse whole-band windows: a lane's two points in one walk
constexpr int kBandMaxSub = 6;       // staged sub-rows f + 2 (f <= 4)
constexpr uint32_t kBandGlobal = 0x80000000u;  // buffer entry: a global sorted query index
struct BandHdr {
  int32_t row;
  uint32_t c1;           // the window's end (wave 0)
  uint32_t m;            // staged query points
  uint32_t gstart[kBandMaxSub], lstart[kBandMaxSub + 1];  // per band sub-row: first global / staged point
  unsigned long long fill;  // the block's pairs so far: its region cursor
  uint64_t roff, rlen, E;   // the block's region, the regions' end (overflow area start)
  uint64_t wsum[kBandWaves];
  uint32_t p0, p1;          // the block's slice of the bucketed points (band_regions)
  int32_t nopart, unbal;    // band_regions: the history's slices not a partition / not balanced
  int32_t last;             // this block took the last ticket
};
constexpr int kBandHdrBytes = (int)((sizeof(BandHdr) + 15) / 16 * 16);
#ifndef GF_BAND_LDS_KB  // experiment builds: a smaller block (GF_BAND_MINBLK blocks per CU)
#define GF_BAND_LDS_KB 160
#endif
#ifndef GF_BAND_MINBLK
#define GF_BAND_MINBLK 1
#endif
#ifndef GF_BAND_QUEUE
#define GF_BAND_QUEUE 128
#endif
constexpr size_t kBandLds = GF_BAND_LDS_KB * 1024;
constexpr int kBandQueue = GF_BAND_QUEUE;  // windowed bands: queued point positions per wave
constexpr size_t kBandPerWave = (size_t)kBandBuf * 8 + kBandQueue * 4;
constexpr size_t kBandStage = kBandLds - kBandHdrBytes - (size_t)kBandWaves * kBandPerWave;
static_assert(kBandStage >= 5 * 8 * 1024 / GF_BAND_MINBLK, "band_regions' scratch (5 G u64, G <= 1024 / MINBLK) in the staging area");
// staged offset entries per band sub-row for window [c0, c1): sub-columns c0 - 1 .. c1 + 1
__device__ __forceinline__ uint32_t band_ncol(uint32_t c0, uint32_t c1) { return (c1 - c0 + 3 + 7) & ~7u; }
__device__ __forceinline__ uint32_t band_off_bytes(int32_t f, uint32_t c0, uint32_t c1) {
  return (uint32_t)(f + 2) * band_ncol(c0, c1) * 2u;
}
// the slice of the bucketed points block `blk` of G takes (G % 8 == 0, host): XCD x = blk % 8
// holds the consecutive slices [x G/8, (x + 1) G/8)
__device__ __forceinline__ void band_slice(uint32_t N, uint32_t G, uint32_t blk, uint32_t& p0, uint32_t& p1) {
  const uint32_t s = (blk & 7u) * (G >> 3) + (blk >> 3);
  p0 = (uint32_t)((uint64_t)N * s / G);
  p1 = (uint32_t)((uint64_t)N * (s + 1) / G);
}
// block-wide exclusive scan of one u64 per thread (kBandThreads), *total = the sum
__device__ __forceinline__ uint64_t band_scan(uint64_t v, uint64_t* total, uint64_t* ws) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += t;
  }
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  uint64_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBandWaves; ++w) {
    before += w < (int)wid ? ws[w] : 0ull;
    tot += ws[w];
  }
  *total = tot;
  __syncthreads();
  return before + inc - v;
}
#ifndef GF_BAND_BALANCED
#define GF_BAND_BALANCED 1.125
#endif
constexpr double kBandBalanced = GF_BAND_BALANCED;  // the last call's slices are kept below this max / mean work
// the block that took slice s (the inverse of band_slice's mapping)
__device__ __forceinline__ uint32_t band_block_of(uint32_t G, uint32_t s) {
  return (s % (G >> 3)) * 8u + s / (G >> 3);
}
// Every block derives all G slices and regions the same way (so no launch is needed for them).
// History (hist, per block of the last call): its pairs, its slice's length and start, and
// whether the call fit its output.  Slices: without a history, equal point slices.  With one,
// the last call's slices (scaled to this call's N) when their WORK (pairs + points) was within
// 1/8 of balanced or when the last call did not fit (a capacity retry: the same slices, so the
// regions come from exact counts); else the bucketed points are cut at equal quantiles of the
// last call's work, spread evenly over each of its slices (clustered input: equal point slices
// left the busiest block ~1.8x the mean work).  Regions: the slice's pairs (by the same
// interpolation; no history: the host's pairs per point x the slice), + 1/32 + 256; scaled
// down so that the total stays <= e_lim.  scr: LDS scratch for 5 G u64 (the band staging area,
// not yet in use); my_p0: block t's slice start for thread t (the history, join_region_prep).
__device__ __forceinline__ void band_regions(const JoinOut& o, uint32_t N, BandHdr& hd, uint64_t* scr,
                                             uint64_t& my_off, uint64_t& my_len, uint32_t& my_p0) {
  const uint32_t G = gridDim.x, t = threadIdx.x;
  uint64_t hp = 0, hn = 0, hs = 0;
  if (t < G) {  // thread t: slice t's history
    const uint32_t b = band_block_of(G, t);
    hp = o.hist[b];
    hn = o.hist[G + b];
    hs = o.hist[2 * G + b];
  }
  if (t == 0) {  // (seen by all after band_scan's barriers; __syncthreads_or would add static LDS
    hd.nopart = 0;  // to the kernel's full 160 KB: an invalid dispatch)
    hd.unbal = 0;
  }
  uint64_t HP, HN;
  const uint64_t pc = band_scan(hp, &HP, hd.wsum), op = band_scan(hn, &HN, hd.wsum);
  uint64_t* const sW = scr;            // work before slice s
  uint64_t* const sOP = scr + G;       // points before slice s (last call)
  uint64_t* const sPC = scr + 2 * G;   // pairs before slice s
  uint64_t* const sHN = scr + 3 * G;
  uint64_t* const sHP = scr + 4 * G;
  if (t < G) {
    sW[t] = pc + op;
    sOP[t] = op;
    sPC[t] = pc;
    sHN[t] = hn;
    sHP[t] = hp;
  }
  const uint64_t Wtot = HP + HN;
  // the last call's slices a partition of [0, HN) in slice order (as a history from this probe
  // always is), and every slice's work within 1/8 of the mean
  if (t < G && hs != op) hd.nopart = 1;
  if (t < G && (double)(hp + hn) * G > kBandBalanced * (double)Wtot) hd.unbal = 1;
  __syncthreads();
  const bool reuse = HN > 0 && !hd.nopart && (!hd.unbal || o.hist[3 * G] != 0);
  const double scale = HN > 0 ? (double)N / (double)HN : 0.0;
  // position (this call) and pairs before (last call) of the k-th of G work quantiles.  Integer
  // positions, so the slices partition [0, N) exactly: within a slice floor(fr * HN) < HN for
  // q before the next slice's work (fr < 1 in double at these magnitudes), and the next slice
  // starts at sOP + HN -- monotone in k, and every block computes the same boundaries.
  auto quantile = [&](uint32_t k, uint32_t& pos, double& pairs) {
    if (k == 0) { pos = 0; pairs = 0.0; return; }
    if (k >= G) { pos = N; pairs = (double)HP; return; }
    const uint64_t q = (uint64_t)k * Wtot / G;  // (k < G <= 1024, Wtot < 2^53)
    uint32_t lo = 0, hi = G;  // the last slice whose work starts at or before q
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (sW[mid] <= q) lo = mid;
      else hi = mid;
    }
    const uint64_t w = sHN[lo] + sHP[lo];
    const double fr = w > 0 ? (double)(q - sW[lo]) / (double)w : 0.0;
    const uint64_t old = sOP[lo] + (uint64_t)(fr * (double)sHN[lo]);  // <= HN
    pos = (uint32_t)(old * (uint64_t)N / HN);
    pairs = (double)sPC[lo] + fr * (double)sHP[lo];
  };
  uint64_t est = 0;
  if (t < G) {  // block t's slice and region
    const uint32_t s = (t & 7u) * (G >> 3) + (t >> 3);
    uint32_t p0, p1;
    if (reuse) {  // (floor(x * N / HN) of a partition of [0, HN): a partition of [0, N))
      p0 = (uint32_t)(sOP[s] * (uint64_t)N / HN);
      p1 = (uint32_t)((sOP[s] + sHN[s]) * (uint64_t)N / HN);
      est = (uint64_t)ceil((double)sHP[s] * scale * 1.03125) + 256;
    } else if (HN > 0) {
      double a0, a1;
      quantile(s, p0, a0);
      quantile(s + 1, p1, a1);
      est = (uint64_t)ceil((a1 - a0) * scale * 1.03125) + 256;
    } else {
      band_slice(N, G, t, p0, p1);
      est = (uint64_t)ceil(o.ppp * (double)(p1 - p0) * 1.03125) + 256;
    }
    if (t == blockIdx.x) {
      hd.p0 = p0;
      hd.p1 = p1;
    }
    my_p0 = p0;
  }
  uint64_t E;
  uint64_t off = band_scan(est, &E, hd.wsum);
  if (E > o.e_lim) {  // floor(est * s) with s < e_lim / E: the sum stays <= e_lim
    const double sc = (double)(o.e_lim > (uint64_t)G + 1 ? o.e_lim - G - 1 : 0) / (double)E;
    est = t < G ? (uint64_t)((double)est * sc) : 0;
    off = band_scan(est, &E, hd.wsum);
  }
  if (t == blockIdx.x) {
    hd.roff = off;
    hd.rlen = est;
  }
  if (t == 0) {
    hd.E = E;
    hd.fill = 0ull;
  }
  my_off = off;  // thread t keeps region t (the last block's fix-up reads them from registers)
  my_len = est;
  __syncthreads();
}
// The wave's cnt pairs get(0 .. cnt) at the block's next region positions; those past the region
// go to the overflow area (one device atomic for the wave's excess).
template <class Get>
__device__ __forceinline__ void band_emit(const JoinOut& o, BandHdr& hd, uint32_t cnt, Get get) {
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long off = 0;
  if (lane == 0) off = atomicAdd(&hd.fill, (unsigned long long)cnt);
  off = join_uni64(off);
  const uint64_t R = hd.rlen, O = hd.roff, split = off > R ? off : R;
  uint64_t ob = 0;
  if (off + cnt > R) {  // wave-uniform
    unsigned long long b = 0;
    if (lane == 0) b = atomicAdd(o.ovf, (unsigned long long)(off + cnt - split));
    ob = hd.E + join_uni64(b);
  }
  for (uint32_t i = lane; i < cnt; i += 64) {
    const uint64_t p = off + i;
    join_vstore(o, p < R ? O + p : ob + (p - split), get(i));
  }
}

// The regions' fix-up (one block, G <= 1023 regions): T = the pairs; region t keeps
// [off_t, off_t + min(n_t, len_t)), its unused tail is a hole, and the overflow area
// [E, E + ovf) is the last run; holes below T and stored runs at or above T (both already in
// position order -- no sort) with their exclusive prefixes for join_fixup_copy_kernel.  Also:
// the history (pairs, points per block) for the next call's regions, and the overflow reset.
// A pair stored past cap + spill_cap was dropped: when T <= cap that is reported as T = cap + 1
// (GF_ERR_CAPACITY; the caller's retry gets regions sized from this call's exact counts).
// O, R: region t of thread t (every block derived all of them, band_regions), E their end.  The
// other blocks' counts were stored write-through and drained before their tickets, so they are
// read with agent-scope loads -- no __threadfence (an L2 write-back per block).  This is the
// write-through hand-off of cdna_hip_programming.md Guideline 16 (R1): sc1 stores of the payload,
// s_waitcnt vmcnt(0) by the storing lane, an atomic counter, sc1 loads in the last arriver (which
// bypass its CU's L1, so no acquire is needed); tests/test_isa_handoff.py checks it in the ISA.
__device__ __forceinline__ void join_region_prep(const JoinFixup& f, uint64_t* ws, uint64_t O, uint64_t R, uint64_t E,
                                                 uint32_t P0) {
  const JoinOut& o = f.o;
  const uint32_t G = o.nwaves, t = threadIdx.x;
  uint64_t n = 0, sl0 = 0;
  if (t < G) {
    n = __hip_atomic_load(o.bcount + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sl0 = __hip_atomic_load(o.bslice + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const uint64_t u = n < R ? n : R;
  uint64_t T;
  band_scan(n, &T, ws);
  const uint64_t ov = __hip_atomic_load(o.ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // lost = some pair was STORED past cap + spill_cap: region t holds [O, O + u), the overflow
  // area [E, E + ov) (a region's unused tail past the limit loses nothing, so a count-only call,
  // cap = spill_cap = 0, with no pairs reports 0, not cap + 1)
  const uint64_t lim = o.cap + o.spill_cap;
  uint64_t past = 0;
  if (t < G) past = O + u > lim ? O + u - (O > lim ? O : lim) : 0;
  else if (t == G) past = E + ov > lim ? E + ov - (E > lim ? E : lim) : 0;
  uint64_t PAST;
  band_scan(past, &PAST, ws);
  const bool lost = PAST > 0;
  const bool fits = T <= o.cap && !lost;
  uint64_t hl = 0, hs = 0, sl = 0, ss = 0;
  if (t < G) {
    hs = O + u;
    hl = hs < T ? (O + R < T ? O + R : T) - hs : 0;
    ss = O > T ? O : T;
    sl = O + u > ss ? O + u - ss : 0;
  } else if (t == G) {
    ss = E > T ? E : T;
    sl = E + ov > ss ? E + ov - ss : 0;
  }
  uint64_t H, S;
  const uint64_t hp = band_scan(hl, &H, ws), sp = band_scan(sl, &S, ws);
  if (t < G) {
    f.hole_start[t] = hs;
    f.hole_pref[t] = hp;
    o.hist[t] = n;
    o.hist[G + t] = sl0;
    o.hist[2 * G + t] = P0;
  }
  if (t <= G) {
    f.seg_start[t] = ss;
    f.seg_pref[t] = sp;
  }
  if (t == 0) {
    f.hole_pref[G] = H;
    f.seg_pref[G + 1] = S;
    f.counts[0] = fits ? G : 0u;
    f.counts[1] = fits ? G + 1 : 0u;
    *f.total = T <= o.cap && lost ? o.cap + 1 : T;
    o.hist[3 * G] = fits ? 0ull : 1ull;  // did not fit: the retry keeps these slices
    if (f.hint) *f.hint = T;
    *o.ovf = 0ull;
  }
}

template <int MODE>
__global__ __launch_bounds__(kBandThreads, (kBandWaves * GF_BAND_MINBLK + 3) / 4) void join_band_probe_kernel(JoinRowArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds_base[];
  BandHdr& hd = *reinterpret_cast<BandHdr*>(lds_base);
  constexpr int kR = MODE == 0 ? kBandRound : kBandRound1;  // candidates per lane per walk round
  char* const stg = lds_base + kBandHdrBytes + (size_t)kBandWaves * kBandPerWave;
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  char* const wbase = lds_base + kBandHdrBytes + (size_t)wid * kBandPerWave;
  uint2* const buf = reinterpret_cast<uint2*>(wbase);
  uint32_t* const wq = reinterpret_cast<uint32_t*>(wbase + kBandBuf * 8);
  uint32_t cnt = 0;  // wave-uniform
  uint32_t sink = 0;  // experiment builds (GF_BAND_EXP_*) only
  const int32_t f = a.f, qn = a.qn;
  const int64_t fW = (int64_t)f * (qn + 2);
  const uint32_t cbeg = (uint32_t)f, cend = (uint32_t)f * (uint32_t)(qn + 1);  // in-grid sub-columns
  const uint32_t N = a.row_off[qn];
  uint64_t my_off, my_len;
  uint32_t my_p0 = 0;
  band_regions(a.out, N, hd, reinterpret_cast<uint64_t*>(stg), my_off, my_len, my_p0);
  uint32_t pos = hd.p0;
  const uint32_t P0 = pos, P1 = hd.p1;
  while (pos < P1) {  // block-uniform: one row segment
    for (int j = threadIdx.x; j < qn; j += kBandThreads)
      if (a.row_off[j] <= pos && pos < a.row_off[j + 1]) hd.row = j;
    __syncthreads();
    const int32_t cy = hd.row;
    const uint32_t sb = pos, se = a.row_off[cy + 1] < P1 ? a.row_off[cy + 1] : P1;
    const int64_t fy0 = (int64_t)f * (cy + 1) - 1;  // the band's first sub-row
    for (uint32_t c0 = cbeg; c0 < cend;) {          // block-uniform: one window
      if (wid == 0) {
        // the window's end: the largest c1 <= cend whose staged bytes fit (64-way search)
        auto cost = [&](uint32_t c1) {
          uint32_t m = 0;
          for (int s = 0; s < f + 2; ++s) {
            const uint32_t* qo = a.q_off + (fy0 + s) * fW;
            m += qo[c1 + 1] - qo[c0 - 1];
          }
          return (uint64_t)band_off_bytes(f, c0, c1) + 20ull * m;
        };
        uint32_t lo = c0, hi = cend;
        if (cost(cend) <= kBandStage) {
          lo = cend;
        } else {
          while (hi - lo > 1) {  // cost(lo) fits (lo == c0: nothing), cost(hi) does not
            const uint32_t step = (hi - lo + 63) / 64, c = lo + (lane + 1) * step;
            const uint64_t ok = __ballot(c < hi && cost(c) <= kBandStage);
            if (ok == 0) {
              hi = lo + step < hi ? lo + step : hi;
            } else {
              const uint32_t L = 63u - (uint32_t)__builtin_clzll(ok), lo2 = lo + (L + 1) * step;
              hi = lo + (L + 2) * step < hi ? lo + (L + 2) * step : hi;
              lo = lo2;
            }
          }
        }
        if (lane == 0) {
          hd.c1 = lo;  // == c0: not even one sub-column fits -- [c0, c0 + 1) from global memory
          uint32_t m = 0;
          if (lo > c0) {
            for (int s = 0; s < f + 2; ++s) {
              const uint32_t* qo = a.q_off + (fy0 + s) * fW;
              hd.gstart[s] = qo[c0 - 1];
              hd.lstart[s] = m;
              m += qo[lo + 1] - qo[c0 - 1];
            }
          }
          hd.lstart[f + 2] = m;
          hd.m = m;
        }
      }
      __syncthreads();
      const bool lds = hd.c1 > c0;
      const uint32_t c1 = lds ? hd.c1 : c0 + 1, m = hd.m, ncol = band_ncol(c0, c1);
      uint16_t* const lo16 = reinterpret_cast<uint16_t*>(stg);
      double2* const lxy = reinterpret_cast<double2*>(stg + ((band_off_bytes(f, c0, c1) + 15u) & ~15u));
      uint32_t* const lq = reinterpret_cast<uint32_t*>(lxy + m);
#ifdef GF_BAND_EXP_NOSTAGE  // experiment build (with NOWALK only): the band is not staged
      if (false) {
#else
      if (lds) {  // stage: offsets (absolute staged slots), xy, query indices -- loads batched
#endif
        const uint32_t nent = (uint32_t)(f + 2) * ncol, span = c1 - c0 + 3;
        for (uint32_t t0 = threadIdx.x; t0 < nent; t0 += 8 * kBandThreads) {
          uint32_t v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const uint32_t t = t0 + u * kBandThreads, s = t / ncol, j = t - s * ncol;
            v[u] = t < nent && j < span ? a.q_off[(fy0 + s) * fW + c0 - 1 + j] - hd.gstart[s] + hd.lstart[s] : 0u;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (t0 + u * kBandThreads < nent) lo16[t0 + u * kBandThreads] = (uint16_t)v[u];
        }
        for (uint32_t t0 = threadIdx.x; t0 < m; t0 += 4 * kBandThreads) {
          double x[4], y[4];
          uint32_t qi[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t t = t0 + u * kBandThreads < m ? t0 + u * kBandThreads : t0;
            int s = 0;
            while (t >= hd.lstart[s + 1]) ++s;
            const uint32_t g = hd.gstart[s] + (t - hd.lstart[s]);
            x[u] = a.sqx[g];
            y[u] = a.sqy[g];
            qi[u] = a.sqidx[g];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t t = t0 + u * kBandThreads;
            if (t < m) {
              lxy[t] = make_double2(x[u], y[u]);
              lq[t] = qi[u];
            }
          }
        }
      }
      __syncthreads();
      // Pairs out.  With the band staged (lds: block-uniform) every buffered entry is a staged slot
      // and the flush reads LDS only; the global form (a sub-column read from global memory) is a
      // separate COMPILE-TIME path (st: std::true_type = staged): the staged streaming loops
      // contain no global load but the prefetch.  r05: with both forms behind one runtime branch
      // in the same loop, the global form's load and the walk's hit-mask register were the same
      // VGPR, and the compiler's wait for that write-after-write (vmcnt(0), in the FIRST walk
      // round of every wave-step) drained the prefetched next points: their latency was exposed
      // once per 128 points.  (r04 fixed the same hazard between the two flush forms.)
      // st: std::true_type / std::false_type -- staged or not, fixed at compile time
      auto staged = [](auto st) constexpr -> bool { return decltype(st)::value; };
      auto flush_as = [&](auto st) {
#ifdef GF_BAND_EXP_NOEMIT  // experiment build: the buffered pairs are dropped (no band_emit)
        sink ^= cnt;
        cnt = 0;
        return;
#endif
        wave_lds_sync();  // the entries other lanes of this wave pushed (intra-wave LDS hand-off)
        if (staged(st)) {
          band_emit(a.out, hd, cnt, [&](uint32_t i) {
            const uint2 v = buf[i];
            return make_uint2(v.x, ((lds_u32)lq)[v.y]);
          });
        } else {
          band_emit(a.out, hd, cnt, [&](uint32_t i) {
            const uint2 v = buf[i];
            return make_uint2(v.x, a.sqidx[v.y & ~kBandGlobal]);
          });
        }
        cnt = 0;
      };
      // DENSE window (clustered input: ~> 12 candidates per point): each wave-step's 64 points are
      // sorted by (sub-column, sub-row) across the wave first (bitonic over 64 lanes in
      // registers), so neighbouring lanes share most candidates -- LDS broadcast reads, and
      // similar run lengths (the rounds are the longest run of the wave).  Not worth its ~300
      // instructions at ~3 candidates per point.
      const bool dense = lds && (uint64_t)m * 9u > 12ull * (uint64_t)(f + 2) * (c1 - c0 + 2);
      // one point: its 3 x 3 sub-cell neighbourhood, kBandRound candidates per round
      auto probe = [&](auto st, double px, double py, uint32_t pidx, bool valid) {
        const bool S = staged(st);  // staged band (lds)
        int32_t cx = cell_index(px, a.u_minX, a.u_cl);
        bool in = valid && cx >= 0 && cx < qn;  // outside the grid's columns: no key matches
        int32_t col = in ? f * (cx + 1) + join_sub(px, a.u_minX, a.u_cl, cx, a.fs, f) : 0;
        int32_t sub = join_sub(py, a.u_minY, a.u_cl, cy, a.fs, f);
        in = in && (uint32_t)col >= c0 && (uint32_t)col < c1;
        if (S && dense) {  // wave-uniform (dense implies staged)
          uint32_t key = in ? (uint32_t)(col - (int32_t)c0) << 3 | (uint32_t)sub : 0xFFFFFFFFu, src = lane;
#pragma unroll
          for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
              const uint32_t ko = __shfl_xor(key, stride, 64), so = __shfl_xor(src, stride, 64);
              const bool asc = (lane & (uint32_t)size) == 0 || size == 64, lower = (lane & (uint32_t)stride) == 0;
              const bool less = ko < key || (ko == key && so < src);
              if (lower == asc ? less : !less && !(ko == key && so == src)) {
                key = ko;
                src = so;
              }
            }
          px = __shfl(px, (int)src, 64);
          py = __shfl(py, (int)src, 64);
          pidx = __shfl(pidx, (int)src, 64);
          col = __shfl(col, (int)src, 64);
          sub = __shfl(sub, (int)src, 64);
          in = key != 0xFFFFFFFFu;
        }
        uint32_t b[3], e[3];
        if (S) {  // (a lane outside the window reads in-bounds entries, masked)
          const uint16_t* lo = lo16 + (in ? sub * ncol + (col - (int32_t)c0) : 0);
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            b[k] = in ? lo[k * ncol] : 0u;
            e[k] = in ? lo[k * ncol + 3] : 0u;
          }
        } else {
          const uint32_t* qo = a.q_off + (in ? (fy0 + sub) * fW + col : fy0 * fW + c0);
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            b[k] = in ? qo[k * fW - 1] : 0u;
            e[k] = in ? qo[k * fW + 2] : 0u;
          }
        }
#ifdef GF_BAND_EXP_NOWALK  // experiment build: setup and streaming only (no pairs)
        sink += e[0] ^ e[1] ^ e[2] ^ b[0] ^ b[1] ^ b[2];
        return;
#endif
        const uint32_t L0 = e[0] - b[0], L1 = L0 + (e[1] - b[1]), L2 = L1 + (e[2] - b[2]);
        const uint32_t d0 = b[0], d1 = b[1] - L0, d2 = b[2] - L1;
        // the three runs walked as one sequence by each lane, kBandRound candidates per round
        // (ballot exit); the buffer is written out before a round whose hits might not fit.
        // (Measured, r03, probe us: a PACKED walk -- the wave's candidates laid out densely in LDS
        // and tested 64 per round through lane permutes -- 184.8 vs 183.0: the walk is not bound
        // by its idle lanes; R = 2: 182.6, R = 8: 211; buffers of 384 / 768 pairs: +4 / +81 (the
        // band then needs windows); flushing at the step's start instead of its end: no change.)
        for (uint32_t k = 0; __ballot(k < L2) != 0; k += kR) {
          if (cnt > (uint32_t)(kBandBuf - 64 * kR)) flush_as(st);
          {
            uint32_t t[kR];
            double2 v[kR];
#pragma unroll
            for (int i = 0; i < kR; ++i) {
              const uint32_t kk = k + i;
#if GF_BAND_FLATSEL
              uint32_t d = kk < L1 ? d1 : d2;
              d = kk < L0 ? d0 : d;
              t[i] = kk < L2 ? kk + d : (S ? 0u : b[0]);
#else
              t[i] = kk < L2 ? kk + (kk < L0 ? d0 : (kk < L1 ? d1 : d2)) : (S ? 0u : b[0]);
#endif
            }
#pragma unroll
            for (int i = 0; i < kR; ++i) {
              if (S) {
                v[i] = lxy[t[i]];  // a finished lane reads slot 0 (staged: m > 0 when any lane runs)
              } else {
                v[i] = make_double2(0.0, 0.0);
                if (k + i < L2) v[i] = make_double2(a.sqx[t[i]], a.sqy[t[i]]);
              }
            }
#pragma unroll
            for (int i = 0; i < kR; ++i) {
              const double dx = px - v[i].x, dy = py - v[i].y;
              bool ok;
              if constexpr (MODE == 0) ok = dx * dx + dy * dy <= a.s_r;
              else ok = a.metric == 0 ? dx * dx + dy * dy <= a.s_r : fdlibm_hypot(dx, dy) <= a.r;
              const bool hit = k + i < L2 && ok;
              const uint64_t hm = __ballot(hit);
#ifdef GF_BAND_EXP_NOPUSH  // experiment build: hits ballotted, never stored
              sink ^= (uint32_t)hm;
              continue;
#endif
              if (hit)
                buf[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u))] =
                    make_uint2(pidx, S ? t[i] : (t[i] | kBandGlobal));
              cnt += (uint32_t)__popcll(hm);
            }
          }
        }
      };
      // TWO points per lane walked as one sequence of six runs (sparse whole-band windows): the
      // rounds of a wave are set by its longest lane, and the sum of two points' candidate counts
      // varies less than one point's, so fewer slots idle (~3.2 candidates per point at C4)
      auto probe2 = [&](double pxa, double pya, uint32_t ia, bool va, double pxb, double pyb, uint32_t ib,
                        bool vb) {
        uint32_t b[6], e[6];
        auto runs = [&](double px, double py, bool valid, uint32_t (&bb)[3], uint32_t (&ee)[3]) {
          const int32_t cx = cell_index(px, a.u_minX, a.u_cl);
          bool in = valid && cx >= 0 && cx < qn;
          const int32_t col = in ? f * (cx + 1) + join_sub(px, a.u_minX, a.u_cl, cx, a.fs, f) : 0;
          const int32_t sub = join_sub(py, a.u_minY, a.u_cl, cy, a.fs, f);
          in = in && (uint32_t)col >= c0 && (uint32_t)col < c1;
          const uint16_t* lo = lo16 + (in ? sub * ncol + (col - (int32_t)c0) : 0);
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            bb[k] = in ? lo[k * ncol] : 0u;
            ee[k] = in ? lo[k * ncol + 3] : 0u;
          }
        };
        {
          uint32_t b0[3], e0[3], b1[3], e1[3];
          runs(pxa, pya, va, b0, e0);
          runs(pxb, pyb, vb, b1, e1);
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            b[k] = b0[k]; e[k] = e0[k];
            b[k + 3] = b1[k]; e[k + 3] = e1[k];
          }
        }
        uint32_t L[6], dd[6], acc = 0;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          dd[k] = b[k] - acc;  // slot kk of run k is kk + dd[k] (mod 2^32)
          acc += e[k] - b[k];
          L[k] = acc;
        }
        const uint32_t LA = L[2], LT = L[5];
#if defined(GF_BAND_EXP_NOSTAGE) && !defined(GF_BAND_EXP_NOWALK)
#error "GF_BAND_EXP_NOSTAGE needs GF_BAND_EXP_NOWALK (unstaged offsets must not be walked)"
#endif
#ifdef GF_BAND_EXP_NOWALK  // experiment build: setup and streaming only (no pairs)
        sink += LT ^ dd[0] ^ dd[3];
        return;
#endif
        for (uint32_t k = 0; __ballot(k < LT) != 0; k += kR) {
          if (cnt > (uint32_t)(kBandBuf - 64 * kR)) flush_as(std::true_type{});
          uint32_t t[kR];
          double2 v[kR];
#pragma unroll
          for (int i = 0; i < kR; ++i) {
            const uint32_t kk = k + i;
#if GF_BAND_FLATSEL  // a flat select chain (the nested ?: compiles to exec-masked branches per level)
            uint32_t d = dd[5];
#pragma unroll
            for (int j = 4; j >= 0; --j) d = kk < L[j] ? dd[j] : d;
#else
            const uint32_t d = kk < L[0] ? dd[0] : kk < L[1] ? dd[1] : kk < L[2] ? dd[2]
                             : kk < L[3] ? dd[3] : kk < L[4] ? dd[4] : dd[5];
#endif
            t[i] = kk < LT ? kk + d : 0u;
          }
#pragma unroll
          for (int i = 0; i < kR; ++i) v[i] = lxy[t[i]];  // a finished lane reads slot 0
#pragma unroll
          for (int i = 0; i < kR; ++i) {
            const bool second = k + i >= LA;
            const double dx = (second ? pxb : pxa) - v[i].x, dy = (second ? pyb : pya) - v[i].y;
            bool ok;
            if constexpr (MODE == 0) ok = dx * dx + dy * dy <= a.s_r;
            else ok = a.metric == 0 ? dx * dx + dy * dy <= a.s_r : fdlibm_hypot(dx, dy) <= a.r;
            const bool hit = k + i < LT && ok;
            const uint64_t hm = __ballot(hit);
#ifdef GF_BAND_EXP_NOPUSH  // experiment build: hits ballotted, never stored
            sink ^= (uint32_t)hm;
            continue;
#endif
            if (hit)
              buf[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u))] =
                  make_uint2(second ? ib : ia, t[i]);
            cnt += (uint32_t)__popcll(hm);
          }
        }
      };
      // the segment, 128 consecutive points per wave-step (two per lane); past the end a lane
      // re-reads the segment's first point (always present) and is masked
      struct Pt {
        double2 v[2];
        uint32_t idx[2];
      };
      auto fetch = [&](uint32_t s0) {
        Pt p;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint32_t i = s0 + u * 64 + lane, k = i < se ? i : sb;
          p.v[u] = reinterpret_cast<const double2*>(a.soxy)[k];
          p.idx[u] = a.soidx[k];
        }
        return p;
      };
      // the whole band in one window: every point streams through
      auto stream_band = [&](auto st) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing of another path pending in the loop
        Pt cur = fetch(sb + wid * 128);
        for (uint32_t s0 = sb + wid * 128; s0 < se; s0 += kBandWaves * 128) {  // wave-uniform
          const Pt nxt = fetch(s0 + kBandWaves * 128);
          bool two = false;
          if (staged(st)) {
            if (kBandPair && !dense) {  // wave-uniform
              probe2(cur.v[0].x, cur.v[0].y, cur.idx[0], s0 + lane < se, cur.v[1].x, cur.v[1].y, cur.idx[1],
                     s0 + 64 + lane < se);
              two = true;
            }
          }
          if (!two) {
            probe(st, cur.v[0].x, cur.v[0].y, cur.idx[0], s0 + lane < se);
            probe(st, cur.v[1].x, cur.v[1].y, cur.idx[1], s0 + 64 + lane < se);
          }
          __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nxt is in registers (before any store)
          if (cnt > (uint32_t)(kBandBuf - 64 * kR)) flush_as(st);
          cur = nxt;
        }
        if (cnt > 0) flush_as(st);  // staged slots change with the next window
      };
      // windowed band: the wave queues the positions of its points inside the window (LDS) and
      // probes them 64 at a time, so the lanes of other windows do not ride along
      auto window_band = [&](auto st) {
        __builtin_amdgcn_s_waitcnt(0x0F70);
        uint32_t qc = 0;  // wave-uniform
        for (uint32_t s0 = sb + wid * 64; s0 < se; s0 += kBandWaves * 64) {
          const uint32_t i = s0 + lane;
          const bool valid = i < se;
          const double px = a.soxy[2 * (size_t)(valid ? i : sb)];
          const int32_t cx = cell_index(px, a.u_minX, a.u_cl);
          bool act = valid && cx >= 0 && cx < qn;
          const int32_t col = act ? f * (cx + 1) + join_sub(px, a.u_minX, a.u_cl, cx, a.fs, f) : 0;
          act = act && (uint32_t)col >= c0 && (uint32_t)col < c1;
          const uint64_t am = __ballot(act);
          if (act) wq[qc + __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u))] = i;
          qc += (uint32_t)__popcll(am);
          if (qc >= 64) {
            wave_lds_sync();  // positions other lanes queued (intra-wave LDS hand-off)
            const uint32_t k = wq[lane], rest = qc - 64;
            const uint32_t mv = lane < rest ? wq[64 + lane] : 0u;
            wave_lds_sync();  // every lane read its slot before the tail moves to the front
            if (lane < rest) wq[lane] = mv;
            qc = rest;
            const double2 v = reinterpret_cast<const double2*>(a.soxy)[k];
            probe(st, v.x, v.y, a.soidx[k], true);
            if (cnt > (uint32_t)(kBandBuf - 64 * kR)) flush_as(st);
          }
        }
        if (qc > 0) {
          wave_lds_sync();
          const uint32_t k = wq[lane < qc ? lane : 0];
          const double2 v = reinterpret_cast<const double2*>(a.soxy)[k];
          probe(st, v.x, v.y, a.soidx[k], lane < qc);
        }
        if (cnt > 0) flush_as(st);  // staged slots change with the next window
      };
      if (c0 == cbeg && c1 == cend) {
        if (lds) stream_band(std::true_type{});
        else stream_band(std::false_type{});
      } else {
        if (lds) window_band(std::true_type{});
        else window_band(std::false_type{});
      }
      __syncthreads();
      c0 = c1;
    }
    pos = se;
  }
  __syncthreads();  // every wave's pairs are counted
  if (sink == 0xdeadbeefu) a.out.bslice[blockIdx.x] = sink;  // keeps experiment builds' work alive
  if (threadIdx.x == 0) {  // write-through, drained before the ticket (see join_region_prep)
    __hip_atomic_store(a.out.bcount + blockIdx.x, (uint64_t)hd.fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.out.bslice + blockIdx.x, (uint64_t)(P1 - P0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    hd.last = atomicAdd(a.ticket, 1ull) == (unsigned long long)gridDim.x - 1;
  }
  __syncthreads();
  if (hd.last) {  // block-uniform: every other block's counts are in
    join_region_prep(a.fx, hd.wsum, my_off, my_len, hd.E, my_p0);
    if (threadIdx.x == 0) __hip_atomic_store(a.ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

hipError_t launch_join_band(gf_ctx* ctx, const JoinRowArgs& a, int blocks) {
  KTimer t(ctx, GF_K_JOIN_PROBE);
  if (!a.approx && a.metric == 0)
    hipLaunchKernelGGL(join_band_probe_kernel<0>, dim3(blocks), dim3(kBandThreads), kBandLds, ctx->stream, a);
  else
    hipLaunchKernelGGL(join_band_probe_kernel<1>, dim3(blocks), dim3(kBandThreads), kBandLds, ctx->stream, a);
  return hipGetLastError();
}


// ---- the output fix-up ------------------------------------------------------------------------
// (1) one block: the waves' last chunks sorted by position; their holes; T = G - the holes = the
// pair count (written to *total; gctr reset to 0 for the next call); the holes below T and the
// stored runs in [T, G) with their exclusive prefixes.  (2) a grid: stored position k of the runs
// goes to hole position k (both lists in position order; dst < T <= src, no overlap).
constexpr int kFixupMax = 8192;  // waves of the probe grid
__global__ __launch_bounds__(1024) void join_fixup_prep_kernel(JoinFixup f) {
  __shared__ uint64_t key[kFixupMax];  // chunk index << 20 | hole length (~0: no chunk)
  __shared__ uint64_t wsum[16];
  __shared__ unsigned long long s_T;
  const uint32_t n = f.o.nwaves, C = f.o.chunk, tid = threadIdx.x;
  uint32_t np = 1;
  while (np < n) np <<= 1;
  for (uint32_t i = tid; i < np; i += 1024) {
    uint64_t k = ~0ull;
    if (i < n) {
      const uint64_t b = f.o.tail_base[i];
      const uint32_t fill = f.o.tail_fill[i];
      if (b != ~0ull && fill < C) k = (b / C) << 20 | (uint64_t)(C - fill);
    }
    key[i] = k;
  }
  __syncthreads();
  for (uint32_t kk = 2; kk <= np; kk <<= 1)  // bitonic sort, ascending
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      for (uint32_t i = tid; i < np; i += 1024) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const uint64_t x = key[i], y = key[l];
          if ((x > y) == ((i & kk) == 0)) { key[i] = y; key[l] = x; }
        }
      }
      __syncthreads();
    }
  // hole i: [start_i, start_i + len_i), start_i = (chunk + 1) * C - len_i; total H
  auto hstart = [&](uint64_t k) { return ((k >> 20) + 1) * (uint64_t)C - (k & 0xFFFFF); };
  uint64_t h = 0;
  for (uint32_t i = tid; i < np; i += 1024) h += key[i] == ~0ull ? 0 : (key[i] & 0xFFFFF);
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
  if ((tid & 63) == 0) wsum[tid >> 6] = h;
  __syncthreads();
  if (tid == 0) {
    uint64_t H = 0;
    for (int w = 0; w < 16; ++w) H += wsum[w];
    const unsigned long long G = *f.o.gctr;
    s_T = G - H;
    *f.total = G - H;
    if (f.hint) *f.hint = G - H;
    *f.o.gctr = 0ull;
  }
  __syncthreads();
  const uint64_t T = s_T, G = T + [&] { uint64_t H = 0; for (int w = 0; w < 16; ++w) H += wsum[w]; return H; }();
  // the holes (sorted by position; those below T are a prefix: clipped to [0, T)) and the runs
  // of [T, G) before each hole (empty ones kept: join_bsearch takes the last equal prefix), plus
  // the run after the last hole; exclusive prefixes by a block scan over per-thread spans
  const bool fits = T <= f.o.cap;
  const uint32_t per = np / 1024 > 0 ? np / 1024 : 1, i0 = tid * per;
  auto ent = [&](uint32_t i, uint64_t& st, uint64_t& en) {  // hole i, or [G, G) past the last
    if (i < np && key[i] != ~0ull) { st = hstart(key[i]); en = st + (key[i] & 0xFFFFF); }
    else { st = G; en = G; }
  };
  uint64_t hl = 0, rl = 0;  // this thread's hole / run lengths
  for (uint32_t i = i0; i < i0 + per && i < np; ++i) {
    uint64_t st, en, ps, pe;
    ent(i, st, en);
    if (i == 0) pe = T; else { ent(i - 1, ps, pe); pe = pe > T ? pe : T; }
    hl += st < T ? (en < T ? en : T) - st : 0;
    rl += st > pe ? st - pe : 0;
  }
  // block exclusive scans of (hl, rl)
  __shared__ uint64_t sh[1024], sr[1024];
  sh[tid] = hl; sr[tid] = rl;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    const uint64_t a1 = tid >= o ? sh[tid - o] : 0, b1 = tid >= o ? sr[tid - o] : 0;
    __syncthreads();
    sh[tid] += a1; sr[tid] += b1;
    __syncthreads();
  }
  uint64_t hp = sh[tid] - hl, rp = sr[tid] - rl;
  // holes with a chunk (nk) and those of them starting below T (nh: a prefix of the sorted list)
  uint64_t cnt2 = 0;  // nk << 32 | nh
  for (uint32_t i = tid; i < np; i += 1024)
    if (key[i] != ~0ull) cnt2 += (1ull << 32) | (hstart(key[i]) < T ? 1ull : 0ull);
  for (int o = 32; o > 0; o >>= 1) cnt2 += __shfl_xor(cnt2, o, 64);
  __syncthreads();
  if ((tid & 63) == 0) wsum[tid >> 6] = cnt2;
  __syncthreads();
  uint64_t c2 = 0;
  for (int w = 0; w < 16; ++w) c2 += wsum[w];
  const uint32_t nk = (uint32_t)(c2 >> 32), nh = (uint32_t)c2;
  for (uint32_t i = i0; i < i0 + per && i < np; ++i) {
    uint64_t st, en, ps, pe;
    ent(i, st, en);
    if (i == 0) pe = T; else { ent(i - 1, ps, pe); pe = pe > T ? pe : T; }
    if (i < nk && st < T) { f.hole_start[i] = st; f.hole_pref[i] = hp; hp += (en < T ? en : T) - st; }
    if (i <= nk) { f.seg_start[i] = pe; f.seg_pref[i] = rp; rp += st > pe ? st - pe : 0; }
  }
  if (tid == 1023) {
    f.hole_pref[nh] = sh[1023];
    f.seg_pref[nk + 1] = sr[1023];
    f.counts[0] = fits ? nh : 0;
    f.counts[1] = fits ? nk + 1 : 0;
  }
}

__device__ __forceinline__ uint2 join_vload(const JoinOut& o, uint64_t pos) {
  return pos < o.cap ? join_load(o.pairs, o.aligned, pos) : o.spill[pos - o.cap];
}
// the last index i < n with pref[i] <= k
__device__ __forceinline__ uint32_t join_bsearch(const uint64_t* pref, uint32_t n, uint64_t k) {
  uint32_t lo = 0, hi = n;  // pref[lo] <= k < pref[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pref[mid] <= k) lo = mid;
    else hi = mid;
  }
  return lo;
}
// kFixupParts blocks per hole (blocks past the holes exit), block p of a hole taking its pieces
// p, p + kFixupParts, .. of kBlock pairs: each piece's first source run by one binary search,
// then each thread walks forward from it (a piece crosses few runs).  A grid-stride loop with two
// binary searches per pair was latency-bound (17 us for ~1M pairs).
constexpr int kFixupParts = 8;
__global__ __launch_bounds__(kBlock) void join_fixup_copy_kernel(JoinFixup f) {
  const uint32_t nh = f.counts[0], ns = f.counts[1];
  if (nh == 0 || ns == 0) return;
  __shared__ uint32_t s_sg;
  const uint32_t part = blockIdx.x % kFixupParts;
  for (uint32_t h = blockIdx.x / kFixupParts; h < nh; h += gridDim.x / kFixupParts) {  // block-uniform
    const uint64_t hk0 = f.hole_pref[h], k1 = f.hole_pref[h + 1], d0 = f.hole_start[h];
    for (uint64_t k0 = hk0 + (uint64_t)part * kBlock; k0 < k1; k0 += (uint64_t)kFixupParts * kBlock) {
      if (threadIdx.x == 0) s_sg = join_bsearch(f.seg_pref, ns, k0);
      __syncthreads();
      const uint64_t k = k0 + threadIdx.x;
      if (k < k1) {
        uint32_t sg = s_sg;
        int steps = 0;
        while (sg + 1 < ns && f.seg_pref[sg + 1] <= k && steps < 8) {
          ++sg;
          ++steps;
        }
        if (steps == 8) sg = join_bsearch(f.seg_pref, ns, k);
        const uint64_t src = f.seg_start[sg] + (k - f.seg_pref[sg]);
        join_store(f.o.pairs, f.o.aligned, d0 + (k - hk0), join_vload(f.o, src));
      }
      __syncthreads();
    }
  }
}

hipError_t launch_join_fixup(gf_ctx* ctx, const JoinFixup& f) {
  KTimer t(ctx, GF_K_JOIN_COMPACT);
  if (!f.o.regions)  // regions: the band probe's last block prepared the fix-up
    hipLaunchKernelGGL(join_fixup_prep_kernel, dim3(1), dim3(1024), 0, ctx->stream, f);
  hipLaunchKernelGGL(join_fixup_copy_kernel, dim3(f.o.nwaves * kFixupParts), dim3(kBlock), 0, ctx->stream, f);
  return hipGetLastError();
}

hipError_t launch_join_rows(gf_ctx* ctx, const JoinRowArgs& a, const JoinQueryArgs& q, int stage) {
  hipStream_t s = ctx->stream;
  const dim3 grid((unsigned)(q.nblk + a.nblk));
  switch (stage) {
    case 0: {
      KTimer t(ctx, GF_K_JOIN_BUCKET);
      hipLaunchKernelGGL(join_hist_kernel, dim3((unsigned)(kHistSplit * (q.nblk + a.nblk))), dim3(kScatThreads), 0, s,
                         a, q);
      break;
    }
    case 1: {
      KTimer t(ctx, GF_K_JOIN_BUCKET);
      const int32_t nr = a.nrows > q.qn + 2 ? a.nrows : q.qn + 2;
      if (join_scatter_tile(nr) == kScatTileBig)
        hipLaunchKernelGGL(join_scatter_kernel<kScatTileBig>, grid, dim3(kScatThreads),
                           join_scatter_lds_bytes(nr, kScatTileBig), s, a, q);
      else
        hipLaunchKernelGGL(join_scatter_kernel<kScatTileSmall>, grid, dim3(kScatThreads),
                           join_scatter_lds_bytes(nr, kScatTileSmall), s, a, q);
      break;
    }
    case 2:
      hipLaunchKernelGGL(join_sort_finish_kernel, dim3((unsigned)(q.qn + 3)), dim3(kSortThreads),
                         join_sort_lds_bytes(q.f, q.qn), s, a, q);
      break;
    case 3: {
      KTimer t(ctx, GF_K_JOIN_PROBE);
      const size_t lds = join_probe_lds_bytes(a.lds_budget, a.qn, a.f);
      const dim3 pg(a.out.nwaves / (kJoinThreads / 64));
      const bool m0 = !a.approx && a.metric == 0;
      if (a.f > 1) {  // host: the fine path is exact (never approximate)
        if (m0) hipLaunchKernelGGL((join_row_probe_kernel<0, 1>), pg, dim3(kJoinThreads), lds, s, a);
        else hipLaunchKernelGGL((join_row_probe_kernel<1, 1>), pg, dim3(kJoinThreads), lds, s, a);
      } else if (m0) {
        hipLaunchKernelGGL((join_row_probe_kernel<0, 0>), pg, dim3(kJoinThreads), lds, s, a);
      } else {
        hipLaunchKernelGGL((join_row_probe_kernel<1, 0>), pg, dim3(kJoinThreads), lds, s, a);
      }
      break;
    }
  }
  return hipGetLastError();
}

}  // namespace gf
