// k_points.hip -- per-point kernels: K1 cell assignment, K2 bucketing by cell (stable LSD
// radix sort: per-wave LDS histograms, wave-ballot ranking), exclusive scan, and selection-
// bitmap -> index expansion.  gfx950, wave64.
#define GF_TU_NAME k_points_hip
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include <cstdlib>

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

// ---------------------------------------------------------------------------------------
// Sliding range: a closed window's index list.  The window's virtual position space is its
// panes concatenated (pane j at base[j], n_j points); block b owns positions [b*span, (b+1)*span)
// and copies the ones that are list entries (position - base[j] < cnt[j]) to their place in the
// window's list (the prefix of the earlier panes' counts + the entry's rank).  Every block
// prefix-sums the <= 64 counts itself (one wave), so there is no inter-block step; block 0
// writes the window's count.  O(window points / span) blocks, O(hits) bytes moved.
// ---------------------------------------------------------------------------------------
constexpr int kGatherThreads = 256;
constexpr int64_t kGatherSpan = 8192;

__global__ __launch_bounds__(kGatherThreads) void range_window_gather_kernel(RangeGatherArgs a) {
  __shared__ int64_t s_pre[kMaxMergeRecs + 1];
  __shared__ int64_t s_base[kMaxMergeRecs + 1];
  const int t = threadIdx.x;
  if (t < 64) {
    int64_t c = t < a.npanes ? *a.cnt[t] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t v = __shfl_up(c, o, 64);
      if (t >= o) c += v;
    }
    s_pre[t + 1] = c;
    s_base[t] = t < a.npanes ? a.base[t] : INT64_MAX;
    if (t == 0) {
      s_pre[0] = 0;
      s_base[64] = INT64_MAX;
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && t == 0) *a.count = s_pre[a.npanes];
  const int64_t v0 = (int64_t)blockIdx.x * kGatherSpan;
  const int64_t v1 = v0 + kGatherSpan < a.total ? v0 + kGatherSpan : a.total;
  // the pane holding v0 (largest j with base[j] <= v0), then walk forward with v
  int j = 0;
  while (j + 1 < a.npanes && s_base[j + 1] <= v0) ++j;
  for (int64_t v = v0 + t; v < v1; v += kGatherThreads) {
    int p = j;
    while (p + 1 < a.npanes && s_base[p + 1] <= v) ++p;
    const int64_t e = v - s_base[p];
    if (e < s_pre[p + 1] - s_pre[p]) a.out[s_pre[p] + e] = (uint32_t)(s_base[p] + a.list[p][e]);
  }
}

hipError_t launch_range_window_gather(hipStream_t s, const RangeGatherArgs& a) {
  const int64_t blocks = a.total > 0 ? (a.total + kGatherSpan - 1) / kGatherSpan : 1;
  hipLaunchKernelGGL(range_window_gather_kernel, dim3((unsigned)blocks), dim3(kGatherThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_pane_bounds(hipStream_t s, const int64_t* ts, int64_t n, int64_t pane_ms, int64_t first_pane,
                              int32_t nb, int64_t* bounds) {
  hipLaunchKernelGGL(pane_bounds_kernel, dim3((nb + 63) / 64), dim3(64), 0, s, ts, n, pane_ms, first_pane, nb,
                     bounds);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// K2: bucketing by cell -- the keyBy(gridID) shuffle (PointPointRangeQuery.java:144-148): a
// stable LSD radix sort of the points' bucket keys (valid cell -> cy*n + cx, out-of-grid ->
// n*n), <= 9 bits per pass, so every bucket lists its points in input (arrival) order -- the
// order Flink's per-key window buffer iterates -- and the result never depends on scheduling.
//   radix_hist     block b's digit histogram of its chunk in LDS -> column b of M[digit][block]
//   (scan)         of M, digit-major (one look-back launch): every block's first output slot
//                  per digit
//   radix_scatter  block b walks its chunk in tiles of kRadixTile points.  A tile's element e
//                  belongs to wave e / 512; a wave ranks its elements stably (lanes sharing a
//                  digit found with `bits` ballots, rank = popcount below + the wave's running
//                  count of that digit in LDS), a digit-major scan over (digit, wave) of the
//                  waves' counts gives every element its slot in the tile, the tile is placed
//                  in LDS in that order and written out in it -- consecutive lanes write
//                  consecutive slots of one digit's run (r02's per-wave scatter wrote 4 B per
//                  lane to up to 64 digits per store: 201 us per pass on 10M points).
// Pass 0's histogram reads x, y (16 B/point) and stores the keys; every scatter reads (key,
// index) -- pass 0's index is the position itself.
// Afterwards: bucket sizes from the sorted keys' run boundaries -> exclusive scan = cell_start.
// ---------------------------------------------------------------------------------------
#ifndef GF_RADIX_EXP
#define GF_RADIX_EXP 0  // experiment builds only (tools/build_exp.sh): 1 no stores, 2 fake ranks, 3 no LDS permutation (scatter); 4 no histogram atomics, 5 no key stores (pass-0 histogram)
#endif
__device__ __forceinline__ uint32_t bucket_key(double x, double y, const RadixArgs& a) {
  const int32_t cx = cell_index(x, a.minX, a.cl), cy = cell_index(y, a.minY, a.cl);
  const bool valid = cx >= 0 && cy >= 0 && cx < a.gn && cy < a.gn;
  return valid ? (uint32_t)cy * (uint32_t)a.gn + (uint32_t)cx : (uint32_t)a.gn * (uint32_t)a.gn;
}

// gf_shard_by_columns: the band of a point's cell column (Java (int) of the floored x, NaN -> 0);
// columns left of band 1 -- out-of-grid ones included -- belong to band 0, right of the last
// band's start to the last band (sharding.shard_of_columns)
__device__ __forceinline__ uint32_t band_key(double x, const RadixArgs& a) {
  const int32_t cx = cell_index(x, a.minX, a.cl);
  uint32_t b = 0;
  for (int j = 1; j < a.nbands; ++j) b += cx >= a.band_lo[j] ? 1u : 0u;
  return b;
}
// row mode: row << 9 | column; the out-of-grid bucket is row gn, column 0 (so the row-major
// order of (row, column) is the order of the cell keys cy * gn + cx, gn * gn last)
__device__ __forceinline__ uint32_t row_key(double x, double y, const RadixArgs& a) {
  const int32_t cx = cell_index(x, a.minX, a.cl), cy = cell_index(y, a.minY, a.cl);
  const bool valid = cx >= 0 && cy >= 0 && cx < a.gn && cy < a.gn;
  return valid ? (uint32_t)cy << kRadixMaxBits | (uint32_t)cx : (uint32_t)a.gn << kRadixMaxBits;
}
__device__ __forceinline__ uint32_t pass0_key(double x, double y, const RadixArgs& a) {
  return a.nbands > 0 ? band_key(x, a) : (a.rowmode ? row_key(x, y, a) : bucket_key(x, y, a));
}

// Row mode, pass B: block b is segment j of row r -- rows have max(1, ceil(size / seg)) segments
// (an empty row keeps one, which writes its cells' starts), numbered row by row.  Every block
// derives the numbering from pass A's row totals (one scan over <= 512 rows, blockDim >= 512).
struct RowSeg {
  uint32_t r, j, nseg, base;  // row, segment in it, the row's segments, segments before the row
  int64_t beg, end;           // positions [beg, end) of the sorted-by-row arrays
  uint32_t total;             // segments of all rows (blocks >= total: none)
  uint32_t wsum[16];
};
__device__ __forceinline__ void row_segment(const RadixArgs& a, RowSeg& rs, uint32_t b) {
  // rows t * RPT .. t * RPT + RPT - 1 per thread (RPT = 2 for 256-thread blocks, else 1)
  const uint32_t t = threadIdx.x, lane = t & 63, wid = t >> 6, R = (uint32_t)a.gn + 1u;
  const uint32_t RPT = blockDim.x >= 512 ? 1u : 2u, nw = blockDim.x / 64;
  int64_t lo[2] = {0, 0}, hi[2] = {0, 0};
  uint32_t ns[2] = {0u, 0u}, sum = 0;
#pragma unroll
  for (uint32_t q = 0; q < 2; ++q) {
    const uint32_t r = t * RPT + q;
    if (q < RPT && r < R) {
      lo[q] = a.MsA[(size_t)r * a.nblkA];
      hi[q] = a.MsA[(size_t)(r + 1) * a.nblkA];  // r + 1 <= 512 digits: entry mat is the total
      ns[q] = hi[q] > lo[q] ? (uint32_t)((hi[q] - lo[q] + a.seg - 1) / a.seg) : 1u;
    }
    sum += ns[q];
  }
  uint32_t inc = sum;  // block exclusive scan of the threads' sums
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += v;
  }
  if (lane == 63 && wid < 16) rs.wsum[wid] = inc;
  if (t == 0) rs.r = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t before = inc - sum, tot = 0;
  for (uint32_t w = 0; w < nw && w < 16; ++w) {
    before += w < wid ? rs.wsum[w] : 0u;
    tot += rs.wsum[w];
  }
#pragma unroll
  for (uint32_t q = 0; q < 2; ++q) {
    const uint32_t r = t * RPT + q;
    if (q < RPT && r < R && b >= before && b < before + ns[q]) {
      rs.r = r;
      rs.j = b - before;
      rs.nseg = ns[q];
      rs.base = before;
      rs.beg = lo[q] + (int64_t)(b - before) * a.seg;
      rs.end = rs.beg + a.seg < hi[q] ? rs.beg + a.seg : hi[q];
      if (rs.beg > hi[q]) rs.beg = hi[q];
    }
    before += ns[q];
  }
  if (t == 0) rs.total = tot;
  __syncthreads();
}

// pass B histogram: column counts of segment j of row r into M[(base * D) + d * nseg + j] -- for
// every row the (column, segment) entries are consecutive and column-major, rows in order, so
// ONE exclusive scan of M gives every (row, column, segment) its first output position.  Blocks
// past the segments zero their D entries (the scan covers the launch's bound).
// (rowsort: launched inside radix_row_sort_kernel's grid -- blocks past the rows -- for the
// multi-segment rows only; their scatter blocks scan their own row's entries, no global scan)
__device__ __forceinline__ void seg_hist_block(const RadixArgs& a, uint32_t bid) {
  __shared__ uint32_t h[kRadixMaxDigits];
  __shared__ RowSeg rs;
  const uint32_t D = 1u << a.bits, mask = D - 1u;
  for (uint32_t j = threadIdx.x; j < D; j += kRadixThreads) h[j] = 0u;
  row_segment(a, rs, bid);
  if (rs.r == 0xFFFFFFFFu) {  // block-uniform
    if (!a.rowsort)
      for (uint32_t d = threadIdx.x; d < D; d += kRadixThreads) a.M[(size_t)bid * D + d] = 0u;
    return;
  }
  if (rs.nseg == 1 && a.rowsort) return;  // sorted whole by radix_row_sort_kernel
  if (rs.nseg == 1 && a.self_count) {
    // r06: a one-segment row (every row of a uniform 10M-point window on 500 x 500) is sorted by
    // its own scatter block, which counts its columns itself (radix_scatter_kernel): no histogram
    // read here.  Its entries only carry the row's total (column 0) so that the ONE scan of M still
    // gives the later rows' segments their absolute slots.
    for (uint32_t d = threadIdx.x; d < D; d += kRadixThreads)
      a.M[(size_t)rs.base * D + d] = d == 0 ? (uint32_t)(rs.end - rs.beg) : 0u;
    return;
  }
  constexpr int U = 8;
  for (int64_t i0 = rs.beg + threadIdx.x; i0 < rs.end; i0 += (int64_t)kRadixThreads * U) {
    uint32_t k[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // clamped addresses (i0 < end): the U loads fly together
      const int64_t i = i0 + (int64_t)u * kRadixThreads;
      k[u] = a.kin16[i < rs.end ? i : rs.end - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + (int64_t)u * kRadixThreads < rs.end) atomicAdd(&h[k[u] & mask], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < D; d += kRadixThreads)
    a.M[(size_t)rs.base * D + (size_t)d * rs.nseg + rs.j] = h[d];
}
__global__ __launch_bounds__(kRadixThreads) void radix_seg_hist_kernel(RadixArgs a) { seg_hist_block(a, blockIdx.x); }

// block b's chunk [beg, end) of the a.nblk chunks (whole tiles except the last)
__device__ __forceinline__ void radix_chunk(const RadixArgs& a, int64_t& beg, int64_t& end) {
  int64_t n = a.n;
  if (a.n_dev && (int64_t)*a.n_dev < n) n = (int64_t)*a.n_dev;
  const int64_t T = a.tile, tiles = (n + T - 1) / T;
  const int64_t per = (tiles + a.nblk - 1) / a.nblk;
  beg = (int64_t)blockIdx.x * per * T;
  end = beg + per * T < n ? beg + per * T : n;
  if (beg > n) beg = n;
}

template <bool FIRST>
__global__ __launch_bounds__(kRadixThreads) void radix_hist_kernel(RadixArgs a) {
  __shared__ uint32_t h[kRadixMaxDigits];
  const uint32_t D = 1u << a.bits, mask = D - 1u;
  for (uint32_t j = threadIdx.x; j < D; j += kRadixThreads) h[j] = 0u;
  __syncthreads();
  int64_t beg, end;
  radix_chunk(a, beg, end);
  if (FIRST && a.multiseg && blockIdx.x == 0 && threadIdx.x == 0) *a.multiseg = 0u;  // (pass B's row sort sets it)
  if (FIRST) {
    // pass 0: two points per lane (16-B loads of x and y; chunks start at whole tiles, so pairs
    // are 16-B aligned), keys stored as uint2
    constexpr int U = 4;  // pairs in flight together
    // Full steps first: every lane's U pairs exist, so the loads are unconditional and all in
    // flight together (a load under a per-pair branch was waited on inside its branch: the U
    // round trips ran one after another); the chunk's remainder goes point by point.
    constexpr int64_t kStep = (int64_t)kRadixThreads * 2 * U;
    const int64_t full = beg + (end - beg) / kStep * kStep;  // block-uniform
    typedef double v2d __attribute__((ext_vector_type(2)));
    for (int64_t i0 = beg + 2 * (int64_t)threadIdx.x; i0 < full; i0 += kStep) {
      v2d xv[U], yv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + (int64_t)u * kRadixThreads * 2;
        xv[u] = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(a.x + i));
        yv[u] = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(a.y + i));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + (int64_t)u * kRadixThreads * 2;
        const uint32_t k0 = pass0_key(xv[u].x, yv[u].x, a), k1 = pass0_key(xv[u].y, yv[u].y, a);
#if GF_RADIX_EXP != 4  // experiment build 4: no LDS histogram atomics
        atomicAdd(&h[(k0 >> a.shift) & mask], 1u);
        atomicAdd(&h[(k1 >> a.shift) & mask], 1u);
#endif
#if GF_RADIX_EXP != 5  // experiment build 5: no key stores
        *reinterpret_cast<uint2*>(a.kout + i) = make_uint2(k0, k1);  // pass 0's scatter reads the keys
#endif
      }
    }
    // (r04: software-pipelining the steps -- the next step's loads before this step's keys, two
    // pairs per step to keep two blocks per CU -- measured 41.9 vs 40.9 us: no gain)
    for (int64_t i = full + threadIdx.x; i < end; i += kRadixThreads) {
      const uint32_t k0 = pass0_key(a.x[i], a.y[i], a);
      atomicAdd(&h[(k0 >> a.shift) & mask], 1u);
      a.kout[i] = k0;
    }
  } else {
    constexpr int U = 8;  // loads in flight together
    for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += (int64_t)kRadixThreads * U) {
      uint32_t k[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // clamped (always valid) addresses: the U loads fly together
        const int64_t i = i0 + (int64_t)u * kRadixThreads;
        k[u] = a.kin[i < end ? i : end - 1];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (i0 + (int64_t)u * kRadixThreads < end) atomicAdd(&h[(k[u] >> a.shift) & mask], 1u);
    }
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < D; j += kRadixThreads) a.M[(size_t)j * a.nblk + blockIdx.x] = h[j];
}

int radix_threads() {
  static const int nt = [] {
    const char* e = std::getenv("GF_RADIX_NT");
    return e && std::atoi(e) == 1024 ? 1024 : 512;  // r04 A/B on K2: 512 (3 blocks per CU) 68 vs 77 us per pass
  }();
  return nt;
}
size_t radix_scatter_lds_bytes() {
  return (size_t)radix_tile() * 8 + (size_t)(radix_threads() / 64) * kRadixMaxDigits * 4 +
         2 * (size_t)(kRadixMaxDigits + 1) * 4;
}

template <int NT, int MINW>
__global__ __launch_bounds__(NT, MINW) void radix_scatter_kernel(RadixArgs a) {
  extern __shared__ uint32_t rsm[];
  constexpr int kTile = NT / 64 * 512;
  constexpr int W = NT / 64, EPW = kTile / W, U = EPW / 64;  // elements per wave, steps
  uint32_t* const lk = rsm;                           // [kTile] the tile's keys in sorted order
  uint32_t* const lv = lk + kTile;               // [kTile] their values
  uint32_t* const wc = lv + kTile;               // [W][kRadixMaxDigits] wave counts -> slots
  uint32_t* const tb = wc + W * kRadixMaxDigits;      // [D + 1] tile start per digit
  uint32_t* const gc = tb + kRadixMaxDigits + 1;      // [D] next global slot per digit
  __shared__ uint32_t ws[NT / 64];
  const uint32_t D = 1u << a.bits, mask = D - 1u;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  int64_t beg, end;
  if (a.seg > 0) {  // row mode pass B: a row segment; its columns' first slots; cells' starts
    if (a.multiseg && *a.multiseg == 0u) return;  // grid-uniform: every row was sorted whole
    __shared__ RowSeg rs;
    row_segment(a, rs, blockIdx.x);
    if (rs.r == 0xFFFFFFFFu) return;  // block-uniform
    if (rs.nseg == 1 && a.rowsort) return;  // sorted whole by radix_row_sort_kernel
    beg = rs.beg;
    end = rs.end;
    const size_t m0 = (size_t)rs.base * D;
    if (rs.nseg == 1 && a.self_count) {  // (GF_K2_SELFCOUNT=1 A/B; rowsort off)
      // r06: a one-segment row counts its own columns (the histogram kernel skipped it): an LDS
      // histogram of the row's u16 columns, a block scan -> each column's first slot
      for (uint32_t d = threadIdx.x; d < D; d += NT) gc[d] = 0u;
      lds_barrier();
      constexpr int HU = 8;
      for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += (int64_t)NT * HU) {
        uint32_t c[HU];
#pragma unroll
        for (int u = 0; u < HU; ++u) {  // clamped addresses: the loads fly together
          const int64_t i = i0 + (int64_t)u * NT;
          c[u] = a.kin16[i < end ? i : end - 1];
        }
#pragma unroll
        for (int u = 0; u < HU; ++u)
          if (i0 + (int64_t)u * NT < end) atomicAdd(&gc[c[u] & mask], 1u);
      }
      lds_barrier();
      // exclusive scan of gc[0 .. D) (D <= 512 <= NT: one entry per thread), plus the row's start
      const uint32_t v = threadIdx.x < D ? gc[threadIdx.x] : 0u;
      uint32_t inc = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (lane == 63) ws[w] = inc;
      lds_barrier();
      uint32_t before = inc - v + (uint32_t)beg;
      for (int q = 0; q < w; ++q) before += ws[q];
      if (threadIdx.x < D) gc[threadIdx.x] = before;
      lds_barrier();
      if (rs.r < (uint32_t)a.gn) {  // the row's cells start at their columns' first slots
        for (int32_t c = threadIdx.x; c < a.gn; c += NT) a.cstart[(size_t)rs.r * a.gn + c] = gc[c];
      } else if (threadIdx.x == 0) {
        a.cstart[(size_t)a.gn * a.gn] = (uint32_t)beg;
        a.cstart[(size_t)a.gn * a.gn + 1] = (uint32_t)a.n;
      }
    } else if (a.rowsort) {
      // r06: the row's own (column, segment) counts scanned by this block (column-major, as the
      // global scan would order them; the row starts at pass A's row total): every segment block of
      // the row reads the row's D x nseg entries, so no scan launch sits between the histograms and
      // this scatter
      const uint32_t E = D * rs.nseg, per = (E + NT - 1) / NT, e0 = threadIdx.x * per;
      const uint32_t* Mr = a.M + m0;
      uint32_t run = 0;
      for (uint32_t e = e0; e < e0 + per && e < E; ++e) run += Mr[e];
      uint32_t inc = run;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (lane == 63) ws[w] = inc;
      lds_barrier();
      uint32_t before = a.MsA[(size_t)rs.r * a.nblkA] + inc - run;
      for (int q = 0; q < w; ++q) before += ws[q];
      for (uint32_t e = e0; e < e0 + per && e < E; ++e) {
        const uint32_t d = e / rs.nseg, s = e - d * rs.nseg;
        if (s == rs.j) gc[d] = before;
        if (rs.j == 0 && s == 0) {  // the row's cells start at their columns' first slots
          if (rs.r < (uint32_t)a.gn) {
            if (d < (uint32_t)a.gn) a.cstart[(size_t)rs.r * a.gn + d] = before;
          } else if (d == 0) {
            a.cstart[(size_t)a.gn * a.gn] = before;
            a.cstart[(size_t)a.gn * a.gn + 1] = (uint32_t)a.n;
          }
        }
        before += Mr[e];
      }
      lds_barrier();
    } else {
      for (uint32_t d = threadIdx.x; d < D; d += NT) gc[d] = a.Ms[m0 + (size_t)d * rs.nseg + rs.j];
      if (rs.j == 0) {  // the row's cells start at their columns' first slots
        if (rs.r < (uint32_t)a.gn) {
          for (int32_t c = threadIdx.x; c < a.gn; c += NT)
            a.cstart[(size_t)rs.r * a.gn + c] = a.Ms[m0 + (size_t)c * rs.nseg];
        } else if (threadIdx.x == 0) {
          a.cstart[(size_t)a.gn * a.gn] = a.Ms[m0];
          a.cstart[(size_t)a.gn * a.gn + 1] = (uint32_t)a.n;
        }
      }
    }
  } else {
    radix_chunk(a, beg, end);
    for (uint32_t d = threadIdx.x; d < D; d += NT) gc[d] = a.Ms[(size_t)d * a.nblk + blockIdx.x];
  }
  // The next tile's keys / values are loaded into the same registers as soon as this tile sits in
  // LDS (after its placement), so their latency overlaps the write-out and the barriers.  (r04: a
  // prefetch into SEPARATE registers at the top pushed the 1024-thread kernel to 128 VGPRs + 80 B
  // of scratch per lane and cost 76 -> 88 us per pass.)
  uint32_t k[U], v[U], r[U];
  // (clamped addresses, masked after: a load under a per-element branch is waited on inside it,
  // which ran the U loads one round trip after another)
  auto load_tile = [&](int64_t t) {
    const uint32_t c = (uint32_t)(end - t < kTile ? end - t : kTile);
    int64_t idx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t e = w * EPW + u * 64 + lane;
      idx[u] = t + (e < c ? e : c - 1);
      k[u] = a.kin16 ? (uint32_t)a.kin16[idx[u]] : a.kin[idx[u]];
    }
    if (a.vin) {  // kernel-uniform
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = a.vin[idx[u]];
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = (uint32_t)(t + w * EPW + u * 64 + lane);
    }
  };
  if (beg < end) load_tile(beg);
  for (int64_t t0 = beg; t0 < end; t0 += kTile) {  // block-uniform
    const uint32_t cnt = (uint32_t)(end - t0 < kTile ? end - t0 : kTile);
    for (uint32_t d = lane; d < D; d += 64) wc[w * kRadixMaxDigits + d] = 0u;  // this wave's row
#pragma unroll
    for (int u = 0; u < U; ++u) {  // stable ranks within the wave
      const uint32_t e = w * EPW + u * 64 + lane;
      const bool valid = e < cnt;
      const uint32_t d = (k[u] >> a.shift) & mask;
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < a.bits; ++b) {
        const uint64_t bal = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bal : ~bal;
      }
#if GF_RADIX_EXP == 2  // experiment build: counts only, fake ranks (output wrong, accesses in bounds)
      if (valid) atomicAdd(&wc[w * kRadixMaxDigits + d], 1u);
      r[u] = (uint32_t)(u * 64 + lane) + (uint32_t)(peers & 1u);
      continue;
#endif
      uint32_t base = 0;
      if (valid && (peers & below) == 0) base = atomicAdd(&wc[w * kRadixMaxDigits + d], (uint32_t)__popcll(peers));
      const int leader = valid ? __ffsll((unsigned long long)peers) - 1 : lane;
      base = __shfl(base, leader, 64);
      r[u] = base + (uint32_t)__popcll(peers & below);
    }
    lds_barrier();
    {  // exclusive scan of the counts in (digit, wave) order: entry j = d * W + w
      constexpr int PT = W * kRadixMaxDigits / NT;  // entries per thread
      const uint32_t j0 = threadIdx.x * PT;
      uint32_t run = 0;  // (the counts are read twice: keeping them costs PT registers)
#pragma unroll
      for (int q = 0; q < PT; ++q) {
        const uint32_t j = j0 + q, d = j / W, ww = j % W;
        run += d < D ? wc[ww * kRadixMaxDigits + d] : 0u;
      }
      uint32_t inc = run;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (lane == 63) ws[w] = inc;
      lds_barrier();
      uint32_t before = inc - run;
      for (int q = 0; q < w; ++q) before += ws[q];
#pragma unroll
      for (int q = 0; q < PT; ++q) {
        const uint32_t j = j0 + q, d = j / W, ww = j % W;
        if (d < D) {
          const uint32_t c = wc[ww * kRadixMaxDigits + d];
          wc[ww * kRadixMaxDigits + d] = before;
          if (ww == 0) tb[d] = before;
          before += c;
        }
      }
      if (threadIdx.x == 0) tb[D] = cnt;
    }
    lds_barrier();
#pragma unroll
    for (int u = 0; u < U; ++u) {  // the tile in (digit, input) order
      const uint32_t e = w * EPW + u * 64 + lane;
      if (e < cnt) {
#if GF_RADIX_EXP == 3  // experiment build: no permutation in LDS
        const uint32_t p = e + (wc[w * kRadixMaxDigits + ((k[u] >> a.shift) & mask)] + r[u] == 0xFFFFFFFFu ? 1u : 0u);
#elif GF_RADIX_EXP == 2
        const uint32_t p = (wc[w * kRadixMaxDigits + ((k[u] >> a.shift) & mask)] + r[u]) & (uint32_t)(kTile - 1);
#else
        const uint32_t p = wc[w * kRadixMaxDigits + ((k[u] >> a.shift) & mask)] + r[u];
#endif
        lk[p] = k[u];
        lv[p] = v[u];
      }
    }
    lds_barrier();
    if (t0 + kTile < end) load_tile(t0 + kTile);  // block-uniform: in flight during the write-out
#pragma unroll
    for (int q = 0; q < kTile / NT; ++q) {  // runs of one digit: consecutive slots
      const uint32_t p = threadIdx.x + q * NT;
      if (p >= cnt) break;
      const uint32_t kk = lk[p], d = (kk >> a.shift) & mask;
      const uint32_t o = gc[d] + (p - tb[d]);
#if GF_RADIX_EXP == 1  // experiment build: no global stores
      if (o == 0xFFFFFFFFu) a.vout[0] = kk ^ lv[p];
      continue;
#elif GF_RADIX_EXP >= 2
      if (o >= (uint32_t)a.n) continue;
#endif
      if (a.kout16) a.kout16[o] = (uint16_t)(kk & (uint32_t)(kRadixMaxDigits - 1));  // row mode pass A: the column
      else if (a.kout) a.kout[o] = kk;  // (pass B of row mode keeps only the permutation)
      a.vout[o] = lv[p];
    }
    lds_barrier();
    for (uint32_t d = threadIdx.x; d < D; d += NT) gc[d] += tb[d + 1] - tb[d];
    lds_barrier();
  }
}

// ---- row mode pass B, one-segment rows (r06) ---------------------------------------------------
// A row of <= a.seg points (<= kRowSortCap; the rows of the K2 bench window -- 10M points over
// the 357 occupied rows of the 500 x 500 grid -- hold ~28K) is sorted by column inside ONE
// 1024-thread block, the row's output staged whole in LDS.  Wave w takes the w-th contiguous part
// of the row (<= 32 elements per lane, every load in flight at once) and ranks its elements stably
// per 64-element step (9 ballots; the step's leader of each column advances the wave's u16 count
// of it); one block scan in (column, wave) order gives every (column, wave) its first row-local
// slot -- and the row's cell starts; each element lands in the LDS copy of the row's permutation
// at slot + its rank, and the row is written out contiguously.  The tile scatter
// (radix_scatter_kernel) wrote ~8-point column runs per 4096-point tile (partial lines, written
// by blocks of every XCD) and scanned 4096 counts per tile.  r06 A/B (profiles/r06_k2c_ab.jsonl):
// the window 0.189 vs 0.196-0.202 ms (0.170-0.172 once pass B's empty launches went: the
// multiseg flag, the segment histograms as extra blocks of this launch).  Measured and not kept: the permutation stored straight from
// the registers into the row's range (no staging: 24 KB of LDS, two 768-thread blocks per CU,
// every row in one round) 120 vs 61 us -- the scattered 4-B stores cost more than the second
// round of blocks; the steps' counts taken with LDS atomics, broadcast after the last step (no
// wait per step) 63 vs 61 us.
constexpr int kRowSortNT = 1024, kRowSortW = kRowSortNT / 64, kRowSortU = 32;
constexpr int kRowSortCap = kRowSortNT * kRowSortU;  // >= api.cpp kRowSeg (checked there)
size_t radix_row_sort_lds_bytes() { return (size_t)kRowSortCap * 4 + (size_t)kRowSortW * kRadixMaxDigits * 2; }
int radix_row_sort_cap() { return kRowSortCap; }

__global__ __launch_bounds__(kRowSortNT, 4) void radix_row_sort_kernel(RadixArgs a) {
  extern __shared__ uint32_t rsm[];
  uint32_t* const out = rsm;                                              // [cap] the row's permutation
  uint16_t* const wc = reinterpret_cast<uint16_t*>(out + kRowSortCap);     // [W][512] counts -> slots
  __shared__ uint32_t ws[kRowSortW];
  const uint32_t r = blockIdx.x;
  if (r > (uint32_t)a.gn) {  // block-uniform: the multi-segment rows' column histograms
    seg_hist_block(a, r - (uint32_t)a.gn - 1u);
    return;
  }
  const uint32_t lo = a.MsA[(size_t)r * a.nblkA], hi = a.MsA[(size_t)(r + 1) * a.nblkA];
  const uint32_t nr = hi - lo;
  if (nr > (uint32_t)a.seg) {  // a multi-segment row: radix_seg_hist / radix_scatter sort it
    if (threadIdx.x == 0 && a.multiseg) atomicOr(a.multiseg, 1u);
    return;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  const uint32_t per = (nr + kRowSortW - 1) / kRowSortW;  // <= 64 * kRowSortU
  const uint32_t wb = w * per < nr ? w * per : nr, we = wb + per < nr ? wb + per : nr;
  for (uint32_t d = lane; d < (uint32_t)kRadixMaxDigits; d += 64) wc[w * kRadixMaxDigits + d] = 0;
  uint32_t cr[kRowSortU];  // column | rank within the wave's column << 16
  uint32_t v[kRowSortU];
  if (we > wb) {  // wave-uniform: the part's columns, clamped addresses (all loads in flight)
#pragma unroll
    for (int u = 0; u < kRowSortU; ++u) {
      const uint32_t j = wb + u * 64 + lane;
      cr[u] = a.kin16[lo + (j < we ? j : we - 1)];
    }
  }
  wave_lds_sync();
#pragma unroll
  for (int u = 0; u < kRowSortU; ++u) {  // stable ranks per 64-element step
    if (wb + u * 64 >= we) break;  // wave-uniform
    const bool valid = wb + u * 64 + lane < we;
    const uint32_t d = cr[u] & (uint32_t)(kRadixMaxDigits - 1);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < kRadixMaxBits; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const bool lead = valid && (peers & below) == 0;
    uint32_t base = 0;
    if (lead) {
      base = wc[w * kRadixMaxDigits + d];
      wc[w * kRadixMaxDigits + d] = (uint16_t)(base + (uint32_t)__popcll(peers));
    }
    base = __shfl(base, valid ? __ffsll((unsigned long long)peers) - 1 : lane, 64);
    cr[u] = d | (base + (uint32_t)__popcll(peers & below)) << 16;
    wave_lds_sync();  // the next step's leaders read the counts other lanes wrote
  }
  if (we > wb) {  // the permutation entries (in flight during the scan)
#pragma unroll
    for (int u = 0; u < kRowSortU; ++u) {
      const uint32_t j = wb + u * 64 + lane;
      v[u] = a.vin[lo + (j < we ? j : we - 1)];
    }
  }
  __syncthreads();
  {  // exclusive scan of the counts in (column, wave) order: thread t owns column t / 2, waves
     // 8 (t % 2) .. + 8
    constexpr int PT = kRowSortW * kRadixMaxDigits / kRowSortNT;  // 8
    const uint32_t d = threadIdx.x / 2, w0 = (threadIdx.x % 2) * PT;
    uint32_t cnt[PT], run = 0;
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      cnt[q] = wc[(w0 + q) * kRadixMaxDigits + d];
      run += cnt[q];
    }
    uint32_t inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    uint32_t before = inc - run;
    for (int q = 0; q < w; ++q) before += ws[q];
    if (w0 == 0) {  // the row's cells start at their columns' first slots
      if (r < (uint32_t)a.gn) {
        if (d < (uint32_t)a.gn) a.cstart[(size_t)r * a.gn + d] = lo + before;
      } else if (d == 0) {
        a.cstart[(size_t)a.gn * a.gn] = lo;
        a.cstart[(size_t)a.gn * a.gn + 1] = (uint32_t)a.n;
      }
    }
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      wc[(w0 + q) * kRadixMaxDigits + d] = (uint16_t)before;
      before += cnt[q];
    }
  }
  __syncthreads();
  if (we > wb) {
#pragma unroll
    for (int u = 0; u < kRowSortU; ++u) {  // each element at its (column, wave) slot + rank
      if (wb + u * 64 + lane < we) {
        const uint32_t d = cr[u] & 0xFFFFu;
        out[wc[w * kRadixMaxDigits + d] + (cr[u] >> 16)] = v[u];
      }
    }
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < nr; p += kRowSortNT) a.vout[lo + p] = out[p];  // contiguous
}

// cell_start straight from the sorted keys (no histogram, no scan): cell_start[b] = the first
// position whose key is >= b, so position i (key[-1] = -1, key[n] = bins as sentinels) starts
// every bucket b in (key[i-1], key[i]].  One wave per 1024 consecutive positions (16 per lane,
// four 16-B loads in flight).  A lane writes the range of each of its boundaries itself when it is
// short (< kBoundsShort buckets: uniform input, one store per boundary, all lanes' stores in one
// instruction); long ranges (clustered input, the out-of-grid bucket) are written by the whole
// wave, one range at a time.  Every entry of cell_start[0 .. bins] is written exactly once.
// (r04: the wave-at-a-time walk over EVERY boundary -- three lane shuffles and a store loop per
// boundary, ~25 per wave on uniform input -- took 42-53 us for 10M points.)
constexpr int kBoundsPer = 16, kBoundsShort = 8;
__global__ __launch_bounds__(kBlock) void radix_bounds_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                              uint32_t bins, uint32_t* __restrict__ cell_start) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * (64 * kBoundsPer);
  if (w0 > n) return;  // wave-uniform
  const int64_t p0 = w0 + (int64_t)lane * kBoundsPer;
  uint32_t k[kBoundsPer];
  if (w0 + 64 * kBoundsPer <= n) {  // keys (scratch) are 16-B aligned and w0 % 1024 == 0
#pragma unroll
    for (int q = 0; q < kBoundsPer / 4; ++q) {
      const uint4 v = *reinterpret_cast<const uint4*>(keys + p0 + 4 * q);
      k[4 * q] = v.x; k[4 * q + 1] = v.y; k[4 * q + 2] = v.z; k[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kBoundsPer; ++j) {
      const int64_t p = p0 + j;
      k[j] = p < n ? keys[p] : bins;  // the sentinel key[n] = bins (positions past n are masked)
    }
  }
  uint32_t prev = __shfl_up(k[kBoundsPer - 1], 1, 64);
  if (lane == 0) prev = w0 == 0 ? 0u : keys[w0 - 1];
  const bool first = lane == 0 && w0 == 0;  // key[-1] = -1: position 0 starts buckets [0, key[0]]
#pragma unroll
  for (int j = 0; j < kBoundsPer; ++j) {
    const int64_t p = p0 + j;
    const uint32_t cur = k[j], pv = j == 0 ? prev : k[j - 1];
    const bool start = j == 0 && first;
    const bool bd = p <= n && (cur != pv || start);
    const int64_t lo = start ? 0 : (int64_t)pv + 1, hi = cur;
    const bool lng = bd && hi - lo >= kBoundsShort;
    if (bd && !lng)
      for (int64_t b = lo; b <= hi; ++b) cell_start[b] = (uint32_t)p;
    uint64_t m = __ballot(lng);
    while (m) {  // wave-uniform: the long ranges, one at a time
      const int src = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      const int64_t l0 = __shfl(lo, src, 64), h0 = __shfl(hi, src, 64);
      const uint32_t val = (uint32_t)(w0 + (int64_t)src * kBoundsPer + j);
      for (int64_t b = l0 + lane; b <= h0; b += 64) cell_start[b] = val;
    }
  }
}

hipError_t launch_radix(gf_ctx* ctx, int stage, const RadixArgs& a, int blocks) {
  hipStream_t s = ctx->stream;
  KTimer t(ctx, GF_K_BUCKET);
  switch (stage) {
    case 0:  // kin == null: pass 0, keys from x, y stored to kout
      if (!a.kin) hipLaunchKernelGGL(radix_hist_kernel<true>, dim3(blocks), dim3(kRadixThreads), 0, s, a);
      else hipLaunchKernelGGL(radix_hist_kernel<false>, dim3(blocks), dim3(kRadixThreads), 0, s, a);
      break;
    case 1:
      // (r04: row mode pass B with 256-thread blocks -- 2048-point tiles, four blocks per CU --
      // measured 104 vs 58 us per pass: the 512-thread tiles stay)
      if (radix_threads() == 1024)
        hipLaunchKernelGGL((radix_scatter_kernel<1024, 1>), dim3(blocks), dim3(1024), radix_scatter_lds_bytes(), s, a);
      else
        hipLaunchKernelGGL((radix_scatter_kernel<512, 1>), dim3(blocks), dim3(512), radix_scatter_lds_bytes(), s, a);
      break;
    case 3:
      hipLaunchKernelGGL(radix_seg_hist_kernel, dim3(blocks), dim3(kRadixThreads), 0, s, a);
      break;
    case 4:  // blocks = rows (gn + 1)
      hipLaunchKernelGGL(radix_row_sort_kernel, dim3(blocks), dim3(kRowSortNT), radix_row_sort_lds_bytes(), s, a);
      break;
    default: {  // cell_start[0 .. gn*gn + 1] of the sorted kout into a.M: one wave per 256 positions
      const int64_t waves = (a.n + 1 + 64 * kBoundsPer - 1) / (64 * kBoundsPer);
      const int64_t nb = (waves + kBlock / 64 - 1) / (kBlock / 64);
      hipLaunchKernelGGL(radix_bounds_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, a.kout, a.n,
                         a.bins ? a.bins : (uint32_t)a.gn * (uint32_t)a.gn + 1u, a.M);
      break;
    }
  }
  return hipGetLastError();
}

// gf_gather_points: out[i] = in[perm[begin + i]] for the columns given (a shard's SoA slice)
__global__ __launch_bounds__(kBlock) void gather_points_kernel(gf_points in, const uint32_t* __restrict__ perm,
                                                               int64_t begin, int64_t m, double* ox, double* oy,
                                                               int64_t* oo, int64_t* ot) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < m; i += (int64_t)gridDim.x * kBlock) {
    const uint32_t p = perm[begin + i];
    if (ox) ox[i] = in.x[p];
    if (oy) oy[i] = in.y[p];
    if (oo) oo[i] = in.objID[p];
    if (ot) ot[i] = in.ts[p];
  }
}
hipError_t launch_gather_points(hipStream_t s, const gf_points& in, const uint32_t* perm, int64_t begin, int64_t m,
                                double* ox, double* oy, int64_t* oo, int64_t* ot) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_points_kernel, dim3(stream_blocks(m, kBlock)), dim3(kBlock), 0, s, in, perm, begin, m, ox,
                     oy, oo, ot);
  return hipGetLastError();
}

// Global-atomic histogram / scatter (the legacy join path's query side)
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

// ---------------------------------------------------------------------------------------
// Exclusive scan of uint32 with the total at out[L] (reduce-then-scan, 3 launches; one
// single-block launch up to 8 tiles).  Tile = 1024 threads x 4 items.
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
    if (base + j == L - 1) out[L] = run;  // the total
  }
}

// single block, any L: the tiles in sequence with a carried prefix, the total at out[L] -- one
// launch where the 3-kernel scan is launch-bound (row / task counts of a few thousand)
__global__ __launch_bounds__(kScanThreads) void scan_small_kernel(const uint32_t* __restrict__ in, int64_t L,
                                                                  uint32_t* __restrict__ out) {
  uint32_t carry = 0;
  for (int64_t b = 0; b < L; b += kScanTile) {
    const int64_t base = b + (int64_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      v[j] = base + j < L ? in[base + j] : 0u;
      s += v[j];
    }
    uint32_t total;
    uint32_t run = carry + block_excl_scan(s, &total);
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      if (base + j < L) out[base + j] = run;
      run += v[j];
    }
    carry += total;
  }
  if (threadIdx.x == 0) out[L] = carry;
}

size_t scan_tmp_elems(int64_t L) { return (size_t)((L + kScanTile - 1) / kScanTile + 1); }

hipError_t launch_exclusive_scan(hipStream_t s, const uint32_t* in, int64_t L, uint32_t* out, uint32_t* tmp) {
  const int64_t nt = (L + kScanTile - 1) / kScanTile;
  if (nt <= 8) {
    hipLaunchKernelGGL(scan_small_kernel, dim3(1), dim3(kScanThreads), 0, s, in, L, out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nt), dim3(kScanThreads), 0, s, in, L, tmp);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanThreads), 0, s, tmp, nt);
  hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nt), dim3(kScanThreads), 0, s, in, L, tmp, out);
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

// One-launch expansion (gf_bitmap_to_indices_async): a single-pass stream compaction with a
// decoupled look-back.  A block takes kExpandWords consecutive words (one per thread, 64K
// points); its LOGICAL index comes from a ticket taken at its start, so every logical
// predecessor has already started and the look-back never waits on a block that is not running.
// Each block publishes its aggregate, then its inclusive prefix (64-bit status words tagged with
// the launch's epoch, so nothing is reset between launches).  Wave 0 looks back 64 predecessors
// a round.  The block's indices are expanded into LDS in order, as 16-bit offsets from the
// block's first point (128 KB), and copied out with coalesced stores.  The last logical block
// writes the count.
// Measured (10M points, 1% / 22% set): 256-thread blocks 14.2 / 18.0 us, 1024-thread blocks
// 6.4 / 9.4 us.  The ticket atomics serialise on one address and every poll is a round of
// uncached status loads, so fewer, larger blocks win; reading 4 or 8 predecessors per lane a
// round (fewer rounds, more polling traffic) measured slower (7.9 / 9.7 us).
constexpr int kLbPerLane = 1;  // (kLbAgg / kLbInc / lb_pack: gf_internal.hpp)

// One window's expansion by the block with global ticket `bid`: its tiles are the global ids
// [lo, last]; the look-back stops at lo (a batch of windows shares one ticket sequence, each
// window a contiguous range of it, so every logical predecessor within the window has started).
__device__ __forceinline__ void expand_window(const uint64_t* __restrict__ bm, int64_t words, int64_t n,
                                              uint32_t* __restrict__ idx, int64_t cap, int64_t* __restrict__ count,
                                              const ExpandState& st, uint64_t bid, uint64_t lo, uint64_t last,
                                              uint16_t* lidx, uint32_t* wsum, unsigned long long& s_prefix) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t tile = bid - lo;
  const int64_t w = (int64_t)tile * kExpandWords + threadIdx.x;
  uint64_t m = w < words ? bm[w] : 0ull;
  if (w == words - 1 && (n & 63)) m &= (1ull << (n & 63)) - 1ull;
  const uint32_t c = (uint32_t)__popcll(m);
  uint32_t inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (int v = 0; v < kExpandWords / 64; ++v) {
    before += v < wid ? wsum[v] : 0u;
    total += wsum[v];
  }
  if (wid == 0) {  // publish the aggregate; wave 0 looks back 64 x kLbPerLane predecessors a round
    unsigned long long* my = st.status + bid;
    const uint64_t ep = st.epoch & 0x3FFFFFFu;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(my, lb_pack(st.epoch, kLbInc, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0) s_prefix = 0;
    } else {
      if (lane == 0) __hip_atomic_store(my, lb_pack(st.epoch, kLbAgg, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint64_t prefix = 0;
      int64_t hi = (int64_t)bid - 1;  // lane l reads predecessors hi - l*kLbPerLane - j (nearest first)
      const int64_t l0 = (int64_t)lo;
      for (;;) {
        uint64_t v[kLbPerLane];
        bool ready = true;
#pragma unroll
        for (int j = 0; j < kLbPerLane; ++j) {
          const int64_t p = hi - lane * kLbPerLane - j;
          v[j] = p >= l0 ? __hip_atomic_load(st.status + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
          ready = ready && (p < l0 || ((v[j] >> 38) == ep && ((v[j] >> 36) & 3ull) != 0ull));
        }
        if (__ballot(!ready)) {  // some predecessor has not published: poll the window again
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        uint64_t sum = 0;  // this lane's values up to and including its nearest inclusive
        bool incl = false;
#pragma unroll
        for (int j = 0; j < kLbPerLane; ++j) {
          if (!incl) {
            sum += v[j] & ((1ull << 36) - 1ull);
            incl = ((v[j] >> 36) & 3ull) == kLbInc;
          }
        }
        const uint64_t incm = __ballot(incl);
        const int stop = incm ? __ffsll((unsigned long long)incm) - 1 : 64;  // nearest inclusive
        uint64_t add = lane <= stop ? sum : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) add += __shfl_xor(add, o, 64);
        prefix += add;
        if (incm || hi - 64 * kLbPerLane < l0) break;
        hi -= 64 * kLbPerLane;
      }
      if (lane == 0) {
        __hip_atomic_store(my, lb_pack(st.epoch, kLbInc, prefix + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_prefix = prefix;
      }
    }
  }
  // this thread's indices into LDS, in order
  uint32_t pos = before + inc - c;
  const uint32_t lw = (uint32_t)threadIdx.x * 64u;
  while (m) {
    const int bit = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    lidx[pos++] = lw + bit;
  }
  __syncthreads();
  const uint64_t base = s_prefix;
  const uint32_t first = (uint32_t)((int64_t)tile * kExpandWords * 64);
  for (uint32_t j = threadIdx.x; j < total; j += kExpandWords)  // coalesced copy out
    if ((int64_t)(base + j) < cap) idx[base + j] = first + lidx[j];
  if (bid == last && threadIdx.x == 0) *count = (int64_t)(base + total);
}

__global__ __launch_bounds__(kExpandWords) void expand_async_kernel(const uint64_t* __restrict__ bm, int64_t words, int64_t n,
                                                              uint32_t* __restrict__ idx, int64_t cap,
                                                              int64_t* __restrict__ count, ExpandState st) {
  extern __shared__ uint16_t lidx[];  // [kExpandWords * 64] this block's indices - its first point
  __shared__ uint32_t wsum[kExpandWords / 64];
  __shared__ unsigned long long s_bid, s_prefix;
  if (threadIdx.x == 0) s_bid = atomicAdd(st.ticket, 1ull) - st.base;
  __syncthreads();
  expand_window(bm, words, n, idx, cap, count, st, s_bid, 0, gridDim.x - 1, lidx, wsum, s_prefix);
}

// A batch of windows' expansions in one launch: window w owns the tickets [tile0[w], tile0[w+1]).
__global__ __launch_bounds__(kExpandWords) void expand_batch_kernel(ExpandBatch b, ExpandState st) {
  extern __shared__ uint16_t lidx[];
  __shared__ uint32_t wsum[kExpandWords / 64];
  __shared__ unsigned long long s_bid, s_prefix;
  if (threadIdx.x == 0) s_bid = atomicAdd(st.ticket, 1ull) - st.base;
  __syncthreads();
  const uint64_t bid = s_bid;
  int w = 0;
  while (w + 1 < b.nwin && (uint64_t)b.tile0[w + 1] <= bid) ++w;
  expand_window(b.bm[w], (b.n[w] + 63) / 64, b.n[w], b.idx[w], b.cap[w], b.count[w], st, bid, (uint64_t)b.tile0[w],
                (uint64_t)b.tile0[w + 1] - 1, lidx, wsum, s_prefix);
}

// Single-pass exclusive scan (one launch): tiles of 1024 threads x 16 items, each tile's
// prefix by the same decoupled look-back as expand_async (ticket-ordered tile ids, epoch-tagged
// status words).  out[L] = total; out2[i] = out[i] for i < n2 (a cursor copy); in[i] = 0 for
// i < nz after it is read (a histogram that must be zero for the next call).
constexpr int kScan1Items = 16;
constexpr int kScan1Tile = kScanThreads * kScan1Items;
int64_t scan1_blocks(int64_t L) { return (L + kScan1Tile - 1) / kScan1Tile; }

__global__ __launch_bounds__(kScanThreads) void scan1_kernel(uint32_t* __restrict__ in, int64_t L,
                                                             uint32_t* __restrict__ out, uint32_t* __restrict__ out2,
                                                             int64_t n2, int64_t nz, ExpandState st,
                                                             const uint32_t* __restrict__ skip_if_zero) {
  __shared__ unsigned long long s_bid, s_prefix;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_bid = atomicAdd(st.ticket, 1ull) - st.base;  // (every block takes its ticket)
  __syncthreads();
  if (skip_if_zero && *skip_if_zero == 0u) return;  // grid-uniform: nothing to scan (K2 pass B, no multi-segment row)
  const uint64_t bid = s_bid;
  const int64_t base = (int64_t)bid * kScan1Tile + (int64_t)threadIdx.x * kScan1Items;
  uint32_t v[kScan1Items];
  uint32_t s = 0;
  if (base + kScan1Items <= L) {  // 16-byte aligned (host): four uint4 loads
#pragma unroll
    for (int j = 0; j < kScan1Items / 4; ++j) {
      const uint4 u = reinterpret_cast<const uint4*>(in + base)[j];
      v[4 * j] = u.x; v[4 * j + 1] = u.y; v[4 * j + 2] = u.z; v[4 * j + 3] = u.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kScan1Items; ++j) v[j] = base + j < L ? in[base + j] : 0u;
  }
#pragma unroll
  for (int j = 0; j < kScan1Items; ++j) s += v[j];
  if (base < nz) {
    if (base + kScan1Items <= nz) {
#pragma unroll
      for (int j = 0; j < kScan1Items / 4; ++j) reinterpret_cast<uint4*>(in + base)[j] = make_uint4(0u, 0u, 0u, 0u);
    } else {
      for (int j = 0; j < kScan1Items; ++j) if (base + j < nz) in[base + j] = 0u;
    }
  }
  uint32_t total;
  const uint32_t ex = block_excl_scan(s, &total);
  if (wid == 0) {  // publish the aggregate, then look back (as expand_async_kernel)
    unsigned long long* my = st.status + bid;
    const uint64_t ep = st.epoch & 0x3FFFFFFu;
    if (bid == 0) {
      if (lane == 0) __hip_atomic_store(my, lb_pack(st.epoch, kLbInc, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0) s_prefix = 0;
    } else {
      if (lane == 0) __hip_atomic_store(my, lb_pack(st.epoch, kLbAgg, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint64_t prefix = 0;
      int64_t hi = (int64_t)bid - 1;
      for (;;) {
        const int64_t p = hi - lane;
        const uint64_t w = p >= 0 ? __hip_atomic_load(st.status + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const bool ready = p < 0 || ((w >> 38) == ep && ((w >> 36) & 3ull) != 0ull);
        if (__ballot(!ready)) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const bool incl = p >= 0 && ((w >> 36) & 3ull) == kLbInc;
        const uint64_t incm = __ballot(incl);
        const int stop = incm ? __ffsll((unsigned long long)incm) - 1 : 64;
        uint64_t add = lane <= stop ? (w & ((1ull << 36) - 1ull)) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) add += __shfl_xor(add, o, 64);
        prefix += add;
        if (incm || hi - 64 < 0) break;
        hi -= 64;
      }
      if (lane == 0) {
        __hip_atomic_store(my, lb_pack(st.epoch, kLbInc, prefix + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_prefix = prefix;
      }
    }
  }
  __syncthreads();
  uint32_t run = (uint32_t)s_prefix + ex;
  uint32_t o[kScan1Items];
#pragma unroll
  for (int j = 0; j < kScan1Items; ++j) {
    o[j] = run;
    run += v[j];
    if (base + j == L - 1) out[L] = run;  // the total
  }
  if (base + kScan1Items <= L) {
#pragma unroll
    for (int j = 0; j < kScan1Items / 4; ++j)
      reinterpret_cast<uint4*>(out + base)[j] = make_uint4(o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]);
  } else {
    for (int j = 0; j < kScan1Items; ++j) if (base + j < L) out[base + j] = o[j];
  }
  if (base < n2) {
    if (base + kScan1Items <= n2) {
#pragma unroll
      for (int j = 0; j < kScan1Items / 4; ++j)
        reinterpret_cast<uint4*>(out2 + base)[j] = make_uint4(o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]);
    } else {
      for (int j = 0; j < kScan1Items; ++j) if (base + j < n2) out2[base + j] = o[j];
    }
  }
}

hipError_t launch_scan1(hipStream_t s, uint32_t* in, int64_t L, uint32_t* out, uint32_t* out2, int64_t n2, int64_t nz,
                        const ExpandState& st, const uint32_t* skip_if_zero) {
  if (L <= 0) return hipMemsetAsync(out, 0, sizeof(uint32_t), s);
  hipLaunchKernelGGL(scan1_kernel, dim3((unsigned)scan1_blocks(L)), dim3(kScanThreads), 0, s, in, L, out, out2, n2, nz,
                     st, skip_if_zero);
  return hipGetLastError();
}

int64_t expand_blocks(int64_t words) { return (words + kExpandWords - 1) / kExpandWords; }

hipError_t launch_expand_bitmap_async(hipStream_t s, const uint64_t* bitmap, int64_t words, int64_t n, uint32_t* idx,
                                      int64_t cap, int64_t* count, const ExpandState& st) {
  if (words <= 0) return hipMemsetAsync(count, 0, sizeof(int64_t), s);
  hipLaunchKernelGGL(expand_async_kernel, dim3((unsigned)expand_blocks(words)), dim3(kExpandWords),
                     sizeof(uint16_t) * 64 * kExpandWords, s, bitmap, words, n, idx, cap, count, st);
  return hipGetLastError();
}

hipError_t launch_expand_batch(hipStream_t s, const ExpandBatch& b, const ExpandState& st) {
  const int32_t blocks = b.tile0[b.nwin];
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(expand_batch_kernel, dim3((unsigned)blocks), dim3(kExpandWords),
                     sizeof(uint16_t) * 64 * kExpandWords, s, b, st);
  return hipGetLastError();
}

hipError_t launch_expand_bitmap(hipStream_t s, const uint64_t* bitmap, int64_t words, int64_t n,
                                const uint32_t* off, uint32_t* idx, int64_t cap) {
  if (words <= 0) return hipSuccess;
  hipLaunchKernelGGL(expand_kernel, dim3(stream_blocks(words, kBlock)), dim3(kBlock), 0, s, bitmap, words, n, off,
                     idx, cap);
  return hipGetLastError();
}

}  // namespace gf
