// k_points.hip -- per-point kernels: K1 cell assignment, K2 bucketing by cell (histogram,
// exclusive scan, scatter), and selection-bitmap -> index expansion.  gfx950, wave64.
#include "gf_internal.hpp"

namespace gf {

// ---------------------------------------------------------------------------------------
// K1: HelperClass.assignGridCellID per point (HelperClass.java:104-116, Point.java:98).
// Two points per lane: 16-B loads of x and y, 16-B stores of (cx, cy) pairs as int2.
// HBM-bound: 16 B in + 8 B out per point.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void assign_kernel(const double* __restrict__ x,
                                                        const double* __restrict__ y, int64_t n,
                                                        double minX, double minY, double cl,
                                                        int32_t* __restrict__ cx,
                                                        int32_t* __restrict__ cy) {
  const int64_t npairs = (n + 1) >> 1;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < npairs;
       p += (int64_t)gridDim.x * kBlock) {
    const int64_t i = 2 * p;
    if (i + 1 < n) {
      const double2 xv = *reinterpret_cast<const double2*>(x + i);
      const double2 yv = *reinterpret_cast<const double2*>(y + i);
      int2 a, b;
      a.x = cell_index(xv.x, minX, cl);
      a.y = cell_index(xv.y, minX, cl);
      b.x = cell_index(yv.x, minY, cl);
      b.y = cell_index(yv.y, minY, cl);
      *reinterpret_cast<int2*>(cx + i) = a;
      *reinterpret_cast<int2*>(cy + i) = b;
    } else {
      cx[i] = cell_index(x[i], minX, cl);
      cy[i] = cell_index(y[i], minY, cl);
    }
  }
}

static int stream_blocks(int64_t work_items, int per_block) {
  int64_t b = (work_items + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (int)b;
}

hipError_t launch_assign(gf_ctx* ctx, const gf_grid* g, const gf_points* p, int32_t* cx, int32_t* cy) {
  if (p->n <= 0) return hipSuccess;
  KTimer t(ctx, GF_K_ASSIGN);
  const int blocks = stream_blocks((p->n + 1) / 2, kBlock);
  hipLaunchKernelGGL(assign_kernel, dim3(blocks), dim3(kBlock), 0, ctx->stream, p->x, p->y, p->n,
                     g->minX, g->minY, g->cellLength, cx, cy);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Pane boundaries of a time-ordered batch (the sliding-window assembler): bounds[j] = first i
// with ts[i] >= (first_pane + j) * pane_ms, i.e. floor(ts / pane_ms) >= first_pane + j.  One
// lane per boundary, binary search over the (non-decreasing) timestamps.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void pane_bounds_kernel(const int64_t* __restrict__ ts, int64_t n, int64_t pane_ms,
                                                         int64_t first_pane, int32_t nb, int64_t* __restrict__ bounds) {
  const int32_t j = blockIdx.x * 64 + threadIdx.x;
  if (j >= nb) return;
  const int64_t target = (first_pane + j) * pane_ms;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (ts[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  bounds[j] = lo;
}

hipError_t launch_pane_bounds(hipStream_t s, const int64_t* ts, int64_t n, int64_t pane_ms, int64_t first_pane,
                              int32_t nb, int64_t* bounds) {
  hipLaunchKernelGGL(pane_bounds_kernel, dim3((nb + 63) / 64), dim3(64), 0, s, ts, n, pane_ms, first_pane, nb,
                     bounds);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// K2 building blocks.  Bucket key of a point:
//   clamp_pad == 0: valid cell -> cy*n + cx, out-of-grid -> n*n            (gf_bucket_by_cell)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void cell_keys_kernel(const double* __restrict__ x,
                                                           const double* __restrict__ y, int64_t n,
                                                           double minX, double minY, double cl,
                                                           int32_t gn, uint32_t* __restrict__ keys) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const int32_t cx = cell_index(x[i], minX, cl);
    const int32_t cy = cell_index(y[i], minY, cl);
    const bool valid = cx >= 0 && cy >= 0 && cx < gn && cy < gn;
    keys[i] = valid ? (uint32_t)cy * (uint32_t)gn + (uint32_t)cx : (uint32_t)gn * (uint32_t)gn;
  }
}

hipError_t launch_cell_keys(hipStream_t s, const gf_grid* g, const double* x, const double* y, int64_t n,
                            int /*clamp_pad*/, uint32_t* keys) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(cell_keys_kernel, dim3(stream_blocks(n, kBlock)), dim3(kBlock), 0, s, x, y, n,
                     g->minX, g->minY, g->cellLength, g->n, keys);
  return hipGetLastError();
}

// Global-atomic histogram (bins up to n*n+1 do not fit LDS for the large grids).
__global__ __launch_bounds__(kBlock) void histogram_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                           uint32_t* __restrict__ hist) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    atomicAdd(&hist[keys[i]], 1u);
}

hipError_t launch_histogram(hipStream_t s, const uint32_t* keys, int64_t n, uint32_t* hist) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(histogram_kernel, dim3(stream_blocks(n, kBlock)), dim3(kBlock), 0, s, keys, n, hist);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void scatter_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                         uint32_t* __restrict__ cursor,
                                                         uint32_t* __restrict__ perm) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const uint32_t pos = atomicAdd(&cursor[keys[i]], 1u);
    perm[pos] = (uint32_t)i;
  }
}

hipError_t launch_scatter(hipStream_t s, const uint32_t* keys, int64_t n, uint32_t* cursor, uint32_t* perm) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_kernel, dim3(stream_blocks(n, kBlock)), dim3(kBlock), 0, s, keys, n, cursor, perm);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Exclusive scan of uint32 (reduce-then-scan, 3 launches).  Tile = 1024 threads x 4 items.
// Wave-level inclusive scans with __shfl_up (64 lanes), wave totals through LDS.
// ---------------------------------------------------------------------------------------
constexpr int kScanThreads = 1024;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(v, off, 64);
    if (lane >= off) v += t;
  }
  return v;
}

// block exclusive scan of one value per thread; returns exclusive prefix, *total = block sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[kScanThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  const uint32_t inc = wave_incl_scan(v);
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  if (wid == 0) {
    uint32_t w = lane < nw ? wsum[lane] : 0u;
    w = wave_incl_scan(w);
    if (lane < nw) wsum[lane] = w;
  }
  __syncthreads();
  const uint32_t before = wid > 0 ? wsum[wid - 1] : 0u;
  *total = wsum[nw - 1];
  __syncthreads();
  return before + inc - v;
}

__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(const uint32_t* __restrict__ in,
                                                                   int64_t L, uint32_t* __restrict__ sums) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j)
    if (base + j < L) s += in[base + j];
  uint32_t total;
  block_excl_scan(s, &total);
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// single block: exclusive scan of the tile sums in place (any count, sequential tiles)
__global__ __launch_bounds__(kScanThreads) void scan_sums_kernel(uint32_t* __restrict__ sums, int64_t nt) {
  uint32_t carry = 0;
  for (int64_t base = 0; base < nt; base += kScanThreads) {
    const int64_t i = base + threadIdx.x;
    const uint32_t v = i < nt ? sums[i] : 0u;
    uint32_t total;
    const uint32_t ex = block_excl_scan(v, &total);
    if (i < nt) sums[i] = carry + ex;
    carry += total;
  }
}

__global__ __launch_bounds__(kScanThreads) void scan_apply_kernel(const uint32_t* __restrict__ in, int64_t L,
                                                                  const uint32_t* __restrict__ sums,
                                                                  uint32_t* __restrict__ out) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = base + j < L ? in[base + j] : 0u;
    s += v[j];
  }
  uint32_t total;
  uint32_t run = sums[blockIdx.x] + block_excl_scan(s, &total);
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    if (base + j < L) out[base + j] = run;
    run += v[j];
  }
}

__global__ void scan_total_kernel(const uint32_t* __restrict__ in, int64_t L, uint32_t* __restrict__ out) {
  // out[L] = out[L-1] + in[L-1]
  if (L > 0) out[L] = out[L - 1] + in[L - 1];
  else out[0] = 0u;
}

size_t scan_tmp_elems(int64_t L) { return (size_t)((L + kScanTile - 1) / kScanTile + 1); }

hipError_t launch_exclusive_scan(hipStream_t s, const uint32_t* in, int64_t L, uint32_t* out, uint32_t* tmp) {
  const int64_t nt = (L + kScanTile - 1) / kScanTile;
  if (nt > 0) {
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nt), dim3(kScanThreads), 0, s, in, L, tmp);
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanThreads), 0, s, tmp, nt);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nt), dim3(kScanThreads), 0, s, in, L, tmp, out);
  }
  hipLaunchKernelGGL(scan_total_kernel, dim3(1), dim3(1), 0, s, in, L, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// selection bitmap -> ascending indices
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void word_popc_kernel(const uint64_t* __restrict__ bm, int64_t words,
                                                           uint32_t* __restrict__ pc) {
  for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < words; w += (int64_t)gridDim.x * kBlock)
    pc[w] = (uint32_t)__popcll(bm[w]);
}

hipError_t launch_word_popcounts(hipStream_t s, const uint64_t* bitmap, int64_t words, uint32_t* pc) {
  if (words <= 0) return hipSuccess;
  hipLaunchKernelGGL(word_popc_kernel, dim3(stream_blocks(words, kBlock)), dim3(kBlock), 0, s, bitmap, words, pc);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void expand_kernel(const uint64_t* __restrict__ bm, int64_t words, int64_t n,
                                                        const uint32_t* __restrict__ off,
                                                        uint32_t* __restrict__ idx, int64_t cap) {
  for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < words; w += (int64_t)gridDim.x * kBlock) {
    uint64_t m = bm[w];
    int64_t pos = off[w];
    while (m) {
      const int b = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      const int64_t i = w * 64 + b;
      if (i < n && pos < cap) idx[pos] = (uint32_t)i;
      ++pos;
    }
  }
}

hipError_t launch_expand_bitmap(hipStream_t s, const uint64_t* bitmap, int64_t words, int64_t n,
                                const uint32_t* off, uint32_t* idx, int64_t cap) {
  if (words <= 0) return hipSuccess;
  hipLaunchKernelGGL(expand_kernel, dim3(stream_blocks(words, kBlock)), dim3(kBlock), 0, s, bitmap, words, n, off,
                     idx, cap);
  return hipGetLastError();
}

}  // namespace gf
