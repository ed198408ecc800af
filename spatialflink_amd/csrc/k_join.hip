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

}  // namespace gf
