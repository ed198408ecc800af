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
// their cell row (counting sort over qn rows, block-local LDS histograms, one global atomic
// per block and row to reserve a run), then processed as tasks of <= kJoinTask points of one
// row: a task stages the query buckets of rows cy-c .. cy+c (u16 bucket offsets + xy) in LDS
// and tests each ordinary point against the (2c+1) bucket runs around its cell -- all LDS.
// A task whose rows do not fit the LDS budget probes the same runs from global memory.
// Counts pass -> scan over tasks -> write pass; pair order inside a task is unspecified.
// =======================================================================================
constexpr int kRowMax = 8192;  // rows staged as LDS histograms by the bucketing kernels
#ifndef GF_JOIN_BATCH
#define GF_JOIN_BATCH 4
#endif
constexpr int kJoinBatch = GF_JOIN_BATCH;
  // candidates of one row loaded together in the probe

// Bucketing: block b owns the contiguous input chunk b; its row histogram goes to column b of
// the row-major matrix M[row][block] (plain stores).  The exclusive scan of M (flattened) is
// then, for every (row, block), the start of that block's run of the row -- no contended
// atomics, and the order inside a row is the block order.
__device__ __forceinline__ void chunk_of(int64_t no, int64_t& beg, int64_t& end) {
  const int64_t chunk = (no + gridDim.x - 1) / gridDim.x;
  beg = (int64_t)blockIdx.x * chunk;
  end = beg + chunk < no ? beg + chunk : no;
  if (beg > no) beg = no;
}

// kBucketU points per thread are loaded before any is used (the loop is latency-bound
// otherwise: one HBM round trip per point per wave)
constexpr int kBucketU = 8;

__global__ __launch_bounds__(kBlock) void join_orow_hist_kernel(JoinRowArgs a, uint32_t* __restrict__ M) {
  __shared__ uint32_t h[kRowMax];
  int64_t beg, end;
  chunk_of(a.no, beg, end);
  for (int j = threadIdx.x; j < a.qn; j += kBlock) h[j] = 0u;
  __syncthreads();
  for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += kBlock * kBucketU) {
    double x[kBucketU], y[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int64_t i = i0 + u * kBlock;
      x[u] = i < end ? __builtin_nontemporal_load(a.ox + i) : NAN;
      y[u] = i < end ? __builtin_nontemporal_load(a.oy + i) : NAN;
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      if (!(x[u] == x[u])) {  // NaN (or past the end): cell 0 per Java, but i may be past the end
        if (i0 + u * kBlock >= end) continue;
      }
      const int32_t cx = cell_index(x[u], a.u_minX, a.u_cl);
      const int32_t cy = cell_index(y[u], a.u_minY, a.u_cl);
      if (cx >= 0 && cy >= 0 && cx < a.qn && cy < a.qn) atomicAdd(&h[cy], 1u);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < a.qn; j += kBlock) M[(size_t)j * gridDim.x + blockIdx.x] = h[j];
}

__global__ __launch_bounds__(kBlock) void join_orow_scatter_kernel(JoinRowArgs a, const uint32_t* __restrict__ Ms) {
  __shared__ uint32_t h[kRowMax];
  int64_t beg, end;
  chunk_of(a.no, beg, end);
  for (int j = threadIdx.x; j < a.qn; j += kBlock) h[j] = Ms[(size_t)j * gridDim.x + blockIdx.x];
  __syncthreads();
  for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += kBlock * kBucketU) {
    double x[kBucketU], y[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int64_t i = i0 + u * kBlock;
      x[u] = i < end ? __builtin_nontemporal_load(a.ox + i) : 0.0;
      y[u] = i < end ? __builtin_nontemporal_load(a.oy + i) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int64_t i = i0 + u * kBlock;
      if (i >= end) continue;
      const int32_t cx = cell_index(x[u], a.u_minX, a.u_cl);
      const int32_t cy = cell_index(y[u], a.u_minY, a.u_cl);
      if (cx >= 0 && cy >= 0 && cx < a.qn && cy < a.qn) {
        const uint32_t pos = atomicAdd(&h[cy], 1u);
        reinterpret_cast<double2*>(a.soxy)[pos] = make_double2(x[u], y[u]);
        a.soidx[pos] = (uint32_t)i;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Query side of the row path: the same cell order as the histogram + scan + atomic scatter
// of the legacy path (q_off[(ky)*W + kx] = first point of clamped cell (kx, ky)), built
// without global atomics: row histograms in LDS -> one scan -> row scatter -> one block per
// row counting-sorts its points by clamped column in LDS and writes that row of q_off.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int32_t clamp_key(int32_t c, int32_t qn) { return (c < -1 ? -1 : (c > qn ? qn : c)) + 1; }

__global__ __launch_bounds__(kBlock) void join_qrow_hist_kernel(JoinQueryArgs a, uint32_t* __restrict__ M) {
  __shared__ uint32_t h[kRowMax];
  int64_t beg, end;
  chunk_of(a.nq, beg, end);
  const int32_t W = a.qn + 2;
  for (int j = threadIdx.x; j < W; j += kBlock) h[j] = 0u;
  __syncthreads();
  for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += kBlock * kBucketU) {
    double y[kBucketU];  // all loads in flight before the first use
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) y[u] = i0 + u * kBlock < end ? a.qy[i0 + u * kBlock] : 0.0;
#pragma unroll
    for (int u = 0; u < kBucketU; ++u)
      if (i0 + u * kBlock < end) atomicAdd(&h[clamp_key(cell_index(y[u], a.minY, a.cl), a.qn)], 1u);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < W; j += kBlock) M[(size_t)j * gridDim.x + blockIdx.x] = h[j];
}

__global__ __launch_bounds__(kBlock) void join_qrow_scatter_kernel(JoinQueryArgs a, const uint32_t* __restrict__ Ms) {
  __shared__ uint32_t h[kRowMax];
  int64_t beg, end;
  chunk_of(a.nq, beg, end);
  const int32_t W = a.qn + 2;
  for (int j = threadIdx.x; j < W; j += kBlock) h[j] = Ms[(size_t)j * gridDim.x + blockIdx.x];
  __syncthreads();
  for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += kBlock * kBucketU) {
    double x[kBucketU], y[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int64_t i = i0 + u * kBlock;
      x[u] = i < end ? a.qx[i] : 0.0;
      y[u] = i < end ? a.qy[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int64_t i = i0 + u * kBlock;
      if (i >= end) continue;
      const int32_t cx = cell_index(x[u], a.minX, a.cl), cy = cell_index(y[u], a.minY, a.cl);
      const uint32_t pos = atomicAdd(&h[clamp_key(cy, a.qn)], 1u);
      reinterpret_cast<double2*>(a.txy)[pos] = make_double2(x[u], y[u]);
      reinterpret_cast<int2*>(a.tc)[pos] = make_int2(cx, cy);
      a.tidx[pos] = (uint32_t)i;
    }
  }
}

// one block per clamped row ky: column histogram + scan in LDS, q_off row, scatter in the row
__global__ __launch_bounds__(kBlock) void join_qrow_sort_kernel(JoinQueryArgs a, const uint32_t* __restrict__ Ms,
                                                                uint32_t total_idx) {
  __shared__ uint32_t h[kRowMax];
  __shared__ uint32_t wsum[kBlock / 64];
  const int32_t W = a.qn + 2, ky = blockIdx.x;
  const uint32_t rb = Ms[(size_t)ky * a.nblk], re = ky + 1 < W ? Ms[(size_t)(ky + 1) * a.nblk] : Ms[total_idx];
  for (int j = threadIdx.x; j < W; j += kBlock) h[j] = 0u;
  __syncthreads();
  for (uint32_t i0 = rb + threadIdx.x; i0 < re; i0 += kBlock * 4) {
    int32_t cx[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) cx[u] = i0 + u * kBlock < re ? a.tc[2 * (i0 + u * kBlock)] : 0;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * kBlock < re) atomicAdd(&h[clamp_key(cx[u], a.qn)], 1u);
  }
  __syncthreads();
  // exclusive scan of h[0..W) in place: each thread owns a contiguous span of columns
  const int per = (W + kBlock - 1) / kBlock, j0 = threadIdx.x * per;
  uint32_t run = 0;
  for (int j = j0; j < j0 + per && j < W; ++j) run += h[j];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = run;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  uint32_t before = inc - run;
  for (int w = 0; w < wid; ++w) before += wsum[w];
  for (int j = j0; j < j0 + per && j < W; ++j) {
    const uint32_t c = h[j];
    h[j] = rb + before;  // now the cell's cursor (absolute position)
    a.q_off[(size_t)ky * W + j] = rb + before;
    before += c;
  }
  if (ky == W - 1 && threadIdx.x == 0) a.q_off[(size_t)W * W] = re;
  __syncthreads();
  for (uint32_t i0 = rb + threadIdx.x; i0 < re; i0 += kBlock * 4) {
    int2 cc[4];
    double2 v[4];
    uint32_t ix[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t i = i0 + u * kBlock < re ? i0 + u * kBlock : rb;
      cc[u] = reinterpret_cast<const int2*>(a.tc)[i];
      v[u] = reinterpret_cast<const double2*>(a.txy)[i];
      ix[u] = a.tidx[i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i0 + u * kBlock >= re) continue;
      const uint32_t pos = atomicAdd(&h[clamp_key(cc[u].x, a.qn)], 1u);
      a.sqx[pos] = v[u].x;
      a.sqy[pos] = v[u].y;
      a.sqcx[pos] = cc[u].x;
      a.sqcy[pos] = cc[u].y;
      a.sqidx[pos] = ix[u];
    }
  }
}

hipError_t launch_join_qrows(gf_ctx* ctx, const JoinQueryArgs& a, int stage) {
  hipStream_t s = ctx->stream;
  KTimer t(ctx, GF_K_JOIN_BUCKET);
  if (stage == 0)
    hipLaunchKernelGGL(join_qrow_hist_kernel, dim3(a.nblk), dim3(kBlock), 0, s, a, a.qmat);
  else if (stage == 1)
    hipLaunchKernelGGL(join_qrow_scatter_kernel, dim3(a.nblk), dim3(kBlock), 0, s, a, a.qmat_scan);
  else
    hipLaunchKernelGGL(join_qrow_sort_kernel, dim3(a.qn + 2), dim3(kBlock), 0, s, a, a.qmat_scan,
                       (uint32_t)((size_t)(a.qn + 2) * a.nblk));
  return hipGetLastError();
}

// row_off[j] = Ms[j][0] (row starts), row_off[qn] = total; tasks per row
__global__ __launch_bounds__(kBlock) void join_rows_finish_kernel(const uint32_t* __restrict__ Ms, int32_t qn,
                                                                  int32_t nblk, uint32_t total_idx,
                                                                  uint32_t* __restrict__ row_off,
                                                                  uint32_t* __restrict__ row_tasks) {
  for (int j = blockIdx.x * kBlock + threadIdx.x; j <= qn; j += gridDim.x * kBlock) {
    const uint32_t b = Ms[j < qn ? (size_t)j * nblk : total_idx];
    row_off[j] = b;
    if (j < qn) {
      const uint32_t e = Ms[j + 1 < qn ? (size_t)(j + 1) * nblk : total_idx];
      row_tasks[j] = (e - b + kJoinTask - 1) / kJoinTask;
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

// Candidates of ordinary point (px, py) in cell (cx, cy) among the staged rows: calls
// hit(slot) for every pair, in a fixed order, where slot = the query point's position in the
// cell-sorted query arrays; returns the number of pairs.  The slot -> query index lookup
// (sqidx) is left to join_compact_kernel, where the gathers are independent of each other
// (inside the probe loop each one stalls the candidate walk that follows it).
// EXACT0: the plan is exact with metric 0 (squared-distance prefilter only, no hypot code).
template <bool EXACT0, class Hit>
__device__ __forceinline__ uint32_t join_row_point(const JoinRowArgs& a, const char* lds, const QRow* rows, int nrows,
                                                   double px, double py, int32_t cx, int32_t cy, Hit&& hit) {
  const int32_t W = a.qn + 2, c = (int32_t)a.c, qn = a.qn;
  const int32_t kb = (cx - c < -1 ? -1 : cx - c) + 1, ke = (cx + c > qn ? qn : cx + c) + 2;
  const bool fast_ok = EXACT0;
  uint32_t cnt = 0;
  for (int j = 0; j < nrows; ++j) {
    const QRow R = rows[j];
    const bool in_lds = R.loff != 0xffffffffu;
    uint32_t tb, te, t_lo, t_hi;  // candidate run; [t_lo, t_hi) holds the interior buckets
    if (in_lds) {
      const uint16_t* lo16 = reinterpret_cast<const uint16_t*>(lds + R.loff);
      tb = lo16[kb]; te = lo16[ke]; t_lo = lo16[1]; t_hi = lo16[W - 1];
    } else {
      const uint32_t* qo = a.q_off + (size_t)(R.ry + 1) * W;
      tb = qo[kb] - R.gbase; te = qo[ke] - R.gbase; t_lo = qo[1] - R.gbase; t_hi = qo[W - 1] - R.gbase;
    }
    const bool brow = R.ry < 0 || R.ry >= qn;  // clamped row: true cells differ
    uint32_t t = tb;
    if (fast_ok && in_lds && !brow && te > tb && tb >= t_lo && te <= t_hi) {
      // interior LDS run: kJoinBatch candidates loaded together (independent ds_read_b128)
      const double2* lxy = reinterpret_cast<const double2*>(lds + R.lxy);
      for (; t < te; t += kJoinBatch) {
        double2 q[kJoinBatch];
#pragma unroll
        for (int k = 0; k < kJoinBatch; ++k) q[k] = lxy[t + k < te ? t + k : t];
#pragma unroll
        for (int k = 0; k < kJoinBatch; ++k) {
          const double dx = px - q[k].x, dy = py - q[k].y;
          if (t + k < te && dx * dx + dy * dy <= a.s_r) {  // s <= smax(r) <=> sqrt(s) <= r
            hit(R.gbase + t + k);
            ++cnt;
          }
        }
      }
      continue;
    }
    for (; t < te; ++t) {
      const uint32_t gi = R.gbase + t;
      if (brow || t < t_lo || t >= t_hi) {  // clamped bucket: Chebyshev test on the true cell
        const int64_t ddx = (int64_t)a.sqcx[gi] - cx, ddy = (int64_t)a.sqcy[gi] - cy;
        if (ddx > c || ddx < -c || ddy > c || ddy < -c) continue;
      }
      if (EXACT0 || !a.approx) {
        double qx, qy;
        if (in_lds) {
          const double2 q = reinterpret_cast<const double2*>(lds + R.lxy)[t];
          qx = q.x; qy = q.y;
        } else {
          qx = a.sqx[gi]; qy = a.sqy[gi];
        }
        const double dx = px - qx, dy = py - qy;
        if (EXACT0 || a.metric == 0 ? !(dx * dx + dy * dy <= a.s_r) : !(fdlibm_hypot(dx, dy) <= a.r)) continue;
      }
      hit(gi);
      ++cnt;
    }
  }
  return cnt;
}

// Output sinks of the probe: a task's private region (capacity checked by the caller), and
// the overflow, stored from the END of the caller's buffer (dropped past cap; still counted).
struct RegionSink {
  uint2* out;
  __device__ void operator()(uint64_t pos, uint32_t p, uint32_t q) const { out[pos] = make_uint2(p, q); }
};
struct OverflowSink {
  uint32_t* pairs;
  uint64_t cap;
  int aligned;
  __device__ void operator()(uint64_t pos, uint32_t p, uint32_t q) const {
    if (pos < cap) join_store(pairs, aligned, cap - 1 - pos, make_uint2(p, q));
  }
};

struct JoinProbeHdr {
  int32_t row, fit;
  uint32_t beg, end;
  uint32_t used;     // pairs placed in the task's region so far (wave reservations)
  uint32_t fit_end;  // end of the last reservation that fit the region
  QRow rows[kJoinMaxRows];
};
constexpr int kJoinHdrBytes = (int)((sizeof(JoinProbeHdr) + 15) / 16 * 16);

// One pass per task: a round = kJoinThreads ordinary points.  Each thread probes its point
// keeping the first kJoinReg query slots in registers; each wave reserves its pairs' run in the
// task's private output region with one LDS atomic -- no block barrier and no global atomic in
// the loop.  A point with more than kJoinReg pairs
// is probed again for the rest (rare; same probe order both times).  A round that no longer
// fits the region goes to the overflow region.  join_compact_kernel packs the regions.
template <bool EXACT0>
__global__ __launch_bounds__(kJoinThreads) __attribute__((amdgpu_waves_per_eu(8)))  // 2 blocks per CU
void join_row_probe_kernel(JoinRowArgs a) {
  // every LDS variable lives in the dynamic region, header first: static __shared__ would sit
  // in front of it and shift its base off 16 B, and each misaligned ds_read_b128 of the staged
  // rows is then replayed (measured: the probe ran 4x slower with a 408-byte static block)
  extern __shared__ __attribute__((aligned(16))) char lds_base[];
  JoinProbeHdr& hd = *reinterpret_cast<JoinProbeHdr*>(lds_base);
  char* const lds = lds_base + kJoinHdrBytes;
  int32_t& s_row = hd.row;
  int32_t& s_fit = hd.fit;
  uint32_t& s_beg = hd.beg;
  uint32_t& s_end = hd.end;
  QRow* const rows = hd.rows;
  const uint32_t ntask = a.task_off[a.qn];
  const uint32_t task = blockIdx.x;
  if (task >= ntask) {
    if (threadIdx.x == 0) a.task_cnt[task] = 0u;
    return;
  }
  const int64_t W = (int64_t)a.qn + 2, c = a.c, qn = a.qn;
  if (threadIdx.x == 0) {
    hd.used = 0u;
    hd.fit_end = 0u;
    int lo = 0, hi = a.qn;  // row = last j with task_off[j] <= task
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (a.task_off[mid] <= task) lo = mid; else hi = mid;
    }
    const uint32_t k = task - a.task_off[lo];
    const uint32_t rb = a.row_off[lo], re = a.row_off[lo + 1];
    s_row = lo;
    s_beg = rb + k * kJoinTask;
    s_end = rb + (k + 1) * kJoinTask < re ? rb + (k + 1) * kJoinTask : re;
    // staged rows and their LDS footprint
    const int64_t r0 = lo - c < -1 ? -1 : lo - c, r1 = lo + c > qn ? qn : lo + c;
    size_t need = 0;
    bool fit = (r1 - r0 + 1) <= kJoinMaxRows;
    for (int64_t ry = r0; fit && ry <= r1; ++ry) {
      const uint32_t b = a.q_off[(ry + 1) * W], e = a.q_off[(ry + 1) * W + W];
      fit = (e - b) < 65536u;
      need += join_row_lds_bytes(W, e - b);
    }
    s_fit = fit && need <= (size_t)a.lds_budget;
  }
  __syncthreads();
  const int32_t cy = s_row;
  const int64_t r0 = cy - c < -1 ? -1 : cy - c, r1 = cy + c > qn ? qn : cy + c;
  const int nrows = (int)(r1 - r0 + 1);
  // stage (or describe) the rows
  size_t off = 0;
  for (int j = 0; j < nrows && j < kJoinMaxRows; ++j) {
    const int64_t ry = r0 + j;
    const uint32_t* qo = a.q_off + (ry + 1) * W;
    const uint32_t b = qo[0], e = qo[W];
    if (s_fit) {
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
  __syncthreads();
  const uint32_t beg = s_beg, end = s_end;
  struct Pt {
    double x, y;
    uint32_t idx;
    bool valid;
  };
  auto load = [&](uint32_t i, Pt& p) {
    p.valid = i < end;
    p.x = p.y = 0.0;
    p.idx = 0u;
    if (p.valid) {
      const double2 v = reinterpret_cast<const double2*>(a.soxy)[i];
      p.x = v.x;
      p.y = v.y;
      p.idx = a.soidx[i];
    }
  };
  struct Hits {
    uint32_t n = 0, h0 = 0, h1 = 0, h2 = 0;  // kJoinReg = 3 (no dynamic register indexing)
  };
  auto probe = [&](const Pt& p, Hits& H) {
    if (!p.valid) return;
    const int32_t cx = cell_index(p.x, a.u_minX, a.u_cl);
    join_row_point<EXACT0>(a, lds, rows, nrows, p.x, p.y, cx, cy, [&](uint32_t q) {
      const uint32_t n = H.n;  // selects, not an indexed array (which would live in scratch)
      H.h0 = n == 0 ? q : H.h0;
      H.h1 = n == 1 ? q : H.h1;
      H.h2 = n == 2 ? q : H.h2;
      H.n = n + 1;
    });
  };
  auto emit = [&](const Pt& p, const Hits& H, const auto& put, uint64_t pos) {
    if (H.n > 0) put(pos, p.idx, H.h0);
    if (H.n > 1) put(pos + 1, p.idx, H.h1);
    if (H.n > 2) put(pos + 2, p.idx, H.h2);
    if (H.n > kJoinReg) {  // the rest: probe again, skipping the first kJoinReg pairs
      uint32_t m = 0;
      const int32_t cx = cell_index(p.x, a.u_minX, a.u_cl);
      join_row_point<EXACT0>(a, lds, rows, nrows, p.x, p.y, cx, cy, [&](uint32_t q) {
        if (m >= kJoinReg) put(pos + m, p.idx, q);
        ++m;
      });
    }
  };
  uint2* const region = a.tpairs + (size_t)task * a.task_cap;
  const uint32_t lane = threadIdx.x & 63;
  Pt A;
  load(beg + threadIdx.x, A);
  for (uint32_t s = beg; s < end; s += kJoinThreads) {
    Pt B;  // the next round's point in flight while this round is probed
    load(s + kJoinThreads + threadIdx.x, B);
    Hits H;
    probe(A, H);
    // wave-level placement, no block barrier in the loop: a wave prefix sum, then one LDS
    // atomic per wave reserves its run in the task's region (pair order is unspecified)
    uint32_t inc = H.n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += t;
    }
    const uint32_t wt = __shfl(inc, 63, 64), ex = inc - H.n;
    if (wt) {
      uint32_t wb = 0;
      if (lane == 0) wb = atomicAdd(&hd.used, wt);
      wb = __shfl(wb, 0, 64);
      if (wb + wt <= a.task_cap) {
        if (lane == 0) atomicMax(&hd.fit_end, wb + wt);
        emit(A, H, RegionSink{region}, wb + ex);
      } else {  // overflow (dense spots): one device atomic per wave
        unsigned long long ob = 0;
        if (lane == 0) ob = atomicAdd(a.ovf_count, (unsigned long long)wt);
        ob = ((unsigned long long)__shfl((uint32_t)(ob >> 32), 0, 64) << 32) | __shfl((uint32_t)ob, 0, 64);
        emit(A, H, OverflowSink{a.pairs, a.cap, a.pairs_aligned}, ob + ex);
      }
    }
    A = B;
  }
  __syncthreads();
  if (threadIdx.x == 0) a.task_cnt[task] = hd.fit_end;
}

// Block t < ntask: its output offset = sum of task_cnt[0..t) (a block reduction over <= a few
// thousand L2-resident counts -- no separate scan launches), then a coalesced copy of the
// region to [off, off + n) with each pair's query slot mapped to the query index.  Blocks >=
// ntask handle the overflow, which sits at [cap - n_ovf, cap): its pair i goes to T + i (T =
// sum of all regions); where [T, T + n_ovf) overlaps the source the pairs are mapped in place,
// the rest of the target takes the source's remainder (every position read and written by one
// thread; disjoint from [0, T) whenever T + n_ovf <= cap -- otherwise the call fails anyway).
__global__ __launch_bounds__(kBlock) void join_compact_kernel(JoinCompactArgs a) {
  __shared__ unsigned long long part[kBlock / 64];
  const uint32_t t = blockIdx.x < a.ntask ? blockIdx.x : a.ntask;
  unsigned long long sum = 0;
  for (uint32_t i = threadIdx.x; i < t; i += kBlock) sum += a.task_cnt[i];
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_down(sum, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
  __syncthreads();
  unsigned long long off = 0;
  for (int w = 0; w < kBlock / 64; ++w) off += part[w];
  if (blockIdx.x < a.ntask) {
    const uint32_t n0 = a.task_cnt[blockIdx.x];
    const uint32_t n = off >= a.cap ? 0u : (uint32_t)(off + n0 > a.cap ? a.cap - off : n0);  // capacity clip
    const uint2* src = a.tpairs + (size_t)blockIdx.x * a.task_cap;
    // kCompactU pairs per thread in flight: the region loads, then the slot -> index gathers,
    // then the stores (one at a time, each gather stalled the loop on its L2 round trip: 87 -> 67 us
    // per 10M x 1M window)
    constexpr int kCompactU = 4;
    for (uint32_t i0 = threadIdx.x; i0 < n; i0 += kBlock * kCompactU) {
      uint2 v[kCompactU];
      uint32_t q[kCompactU];
#pragma unroll
      for (int u = 0; u < kCompactU; ++u) {
        const uint32_t i = i0 + u * kBlock;
        v[u] = src[i < n ? i : i0];
      }
#pragma unroll
      for (int u = 0; u < kCompactU; ++u) q[u] = a.sqidx[v[u].y];
#pragma unroll
      for (int u = 0; u < kCompactU; ++u) {
        const uint32_t i = i0 + u * kBlock;
        if (i < n) join_store(a.pairs, a.pairs_aligned, off + i, make_uint2(v[u].x, q[u]));
      }
    }
    return;
  }
  const unsigned long long nov = *a.ovf_count, T = off;
  if (blockIdx.x == a.ntask && threadIdx.x == 0) *a.total = T + nov;
  if (nov == 0 || T + nov > a.cap) return;
  const uint64_t lo = a.cap - nov;  // overflow source [lo, cap), target [T, T + nov)
  const bool apart = lo >= T + nov;
  for (uint64_t i = (uint64_t)(blockIdx.x - a.ntask) * kBlock + threadIdx.x; i < nov;
       i += (uint64_t)(gridDim.x - a.ntask) * kBlock) {
    const uint64_t dst = T + i;
    const uint64_t src = apart ? lo + i : (dst < lo ? T + nov + i : dst);
    const uint2 v = join_load(a.pairs, a.pairs_aligned, src);
    join_store(a.pairs, a.pairs_aligned, dst, make_uint2(v.x, a.sqidx[v.y]));
  }
}

hipError_t launch_join_compact(gf_ctx* ctx, const JoinCompactArgs& a) {
  KTimer t(ctx, GF_K_JOIN_COMPACT);
  hipLaunchKernelGGL(join_compact_kernel, dim3(a.ntask + 64), dim3(kBlock), 0, ctx->stream, a);
  return hipGetLastError();
}

hipError_t launch_join_rows(gf_ctx* ctx, const JoinRowArgs& a, int stage, int blocks) {
  hipStream_t s = ctx->stream;
  switch (stage) {
    case 0: {
      KTimer t(ctx, GF_K_JOIN_BUCKET);
      hipLaunchKernelGGL(join_orow_hist_kernel, dim3(blocks), dim3(kBlock), 0, s, a, a.row_mat);
      break;
    }
    case 1: {
      KTimer t(ctx, GF_K_JOIN_BUCKET);
      hipLaunchKernelGGL(join_orow_scatter_kernel, dim3(blocks), dim3(kBlock), 0, s, a, a.row_mat_scan);
      break;
    }
    case 2:  // blocks = the bucketing grid size
      hipLaunchKernelGGL(join_rows_finish_kernel, dim3((a.qn + 1 + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                         a.row_mat_scan, a.qn, blocks, (uint32_t)((size_t)a.qn * blocks), a.row_off_w, a.row_tasks);
      break;
    case 3: {
      KTimer t(ctx, GF_K_JOIN_PROBE);
      if (!a.approx && a.metric == 0)
        hipLaunchKernelGGL(join_row_probe_kernel<true>, dim3(blocks), dim3(kJoinThreads), a.lds_budget + kJoinHdrBytes,
                           s, a);
      else
        hipLaunchKernelGGL(join_row_probe_kernel<false>, dim3(blocks), dim3(kJoinThreads), a.lds_budget + kJoinHdrBytes,
                           s, a);
      break;
    }
  }
  return hipGetLastError();
}

}  // namespace gf
