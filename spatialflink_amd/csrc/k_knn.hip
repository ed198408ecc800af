// k_knn.hip -- per-query kNN over one window (PointPointKNNQuery.java:132-201 per-cell heaps +
// KNNQuery.java:213-272 windowAll merge), restated as a three-kernel pipeline for gfx950:
//
//   knn_sample  picks the window's distance threshold T.  Continuous queries: T = the previous
//               window's hint (2 x its k-th distance) and the kernel exits at once.  Otherwise
//               128 blocks read a strided 256K-point sample, histogram candidate distances in
//               LDS (4096 log-spaced bins), flush to a global histogram, and the last block
//               (atomic ticket) takes the upper edge of the bin holding the sample's k-th
//               candidate (>= the window's k-th distance: the sample is a subset).
//   knn_scan    the HBM-bound pass: 16 B/point (x, y), one compare per point against the exact
//               prefilter s = dx*dx+dy*dy <= smax(T); survivors get the exact cell test (C u G)
//               and are appended (d, idx, objID) with one atomic per wave.
//   knn_select  one 1024-thread block: candidates loaded at once, LDS histogram -> bins up to
//               the k-th -> sort (in one wave's registers when <= 64, else LDS bitonic) ->
//               objID dedupe -> first k; stores the next window's hint.
//
// Exactness never depends on T: the record is final only if at least k distinct objIDs lie
// below T (or T == r); otherwise it is flagged and gf_knn_decode re-evaluates the window
// (sample path, then exhaustive T = r partitions).  Output: (d, objID) ascending, the
// minimum-(d, idx) occurrence per objID.
#define GF_TU_NAME k_knn_hip
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include <type_traits>

#include "gf_geom.hpp"
#include "gf_internal.hpp"

namespace gf {

__device__ __forceinline__ bool classify_cg(const QueryRect& q, double px, double py) {
  const double xs = (px == px) ? px : q.minX;  // Java (int)NaN == 0 -> cell 0
  const double ys = (py == py) ? py : q.minY;
  const bool inG = q.g_any && in_iv(q.gx, xs) && in_iv(q.gy, ys);
  return inG || (in_iv(q.cgx, xs) && in_iv(q.cgy, ys));
}

// kNN candidate: cell in C u G (PointPointKNNQuery.java:145-150) and d <= T (<= r, :170-177).
// The hot test keeps no distance live; the rare append recomputes it from x, y.
template <int METRIC>
__device__ __forceinline__ bool knn_pass(double qx, double qy, const QueryRect& qr, double px, double py,
                                         double sp, double T) {
  const double dx = qx - px, dy = qy - py;
  const double s = dx * dx + dy * dy;
  if (!(s <= sp)) return false;
  if (!classify_cg(qr, px, py)) return false;
  return METRIC == 0 ? true : fdlibm_hypot(dx, dy) <= T;  // metric 0: s <= smax(T) <=> sqrt(s) <= T
}
template <int METRIC>
__device__ __forceinline__ double knn_dist(double qx, double qy, double px, double py) {
  const double dx = qx - px, dy = qy - py;
  return METRIC == 0 ? sqrt(dx * dx + dy * dy) : fdlibm_hypot(dx, dy);
}

__device__ __forceinline__ uint64_t okey(int64_t o) { return (uint64_t)o ^ 0x8000000000000000ull; }
__device__ __forceinline__ int64_t from_okey(uint64_t k) { return (int64_t)(k ^ 0x8000000000000000ull); }

struct RecView {
  gf_knn_header* h;
  double* d;
  int64_t* o;
  int64_t* i;
};
__host__ __device__ inline RecView rec_view(void* base, int k) {
  RecView v;
  v.h = (gf_knn_header*)base;
  v.d = (double*)(v.h + 1);
  v.o = (int64_t*)(v.d + k);
  v.i = v.o + k;
  return v;
}

// ---------------------------------------------------------------------------------------
// sample
// ---------------------------------------------------------------------------------------
// The sample kernels' common end: flush the block's LDS histogram, and the last-arriving block
// (atomic ticket) sets T = the upper edge of the bin holding the sample's k-th candidate.
__device__ void sample_finish(KnnState* st, uint32_t* lh, int32_t k, double r, int metric, int64_t bbase) {
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ int s_last, s_bin;
  __syncthreads();
  for (int j = threadIdx.x; j < kDistBins; j += kBlock)
    if (lh[j]) atomicAdd(&st->hist[j], lh[j]);
  // last-arriving block picks the threshold (ticket).  No fences (Guideline 16, R1): the
  // histogram adds are agent-scope atomics (performed at the memory side), every wave drains
  // them before the barrier, the last block reads the bins with agent-scope (sc1) loads.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = atomicAdd(&st->ticket, 1u);
    s_last = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last) return;
  constexpr int kPer = kDistBins / kBlock;  // 16 bins per thread
  uint32_t v[kPer];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    v[j] = __hip_atomic_load(&st->hist[threadIdx.x * kPer + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s += v[j];
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) wsum[wid] = inc;
  if (threadIdx.x == 0) s_bin = -1;
  __syncthreads();
  uint32_t before = 0;
  for (int w = 0; w < wid; ++w) before += wsum[w];
  const uint32_t excl = before + inc - s;
  const uint32_t kk = (uint32_t)k;
  if (excl < kk && kk <= excl + s) {
    uint32_t run = excl;
    for (int j = 0; j < kPer; ++j) {
      run += v[j];
      if (run >= kk) { s_bin = threadIdx.x * kPer + j; break; }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double T = r;
    if (s_bin >= 0) {
      const double up = dist_bin_upper(s_bin, bbase);
      T = up < r ? up : r;
    }
    st->T = T;
    st->s_pre = s_prefilter(T, metric);
    __hip_atomic_store(&st->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int j = threadIdx.x; j < kDistBins; j += kBlock) st->hist[j] = 0u;
}

template <int METRIC>
__global__ __launch_bounds__(kBlock) void knn_sample_kernel(KnnSampleArgs a) {
  __shared__ uint32_t lh[kDistBins];
#ifdef GF_TRACE
  if (blockIdx.x == 0 && threadIdx.x == 0) a.st->tr[0] = wall_clock64();
#endif
  if (a.use_hint) {
    const double h = a.st->hint_T;
    if (h > 0.0) {  // continuous query: the previous window's guess; nothing to sample
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        const double T = h < a.r ? h : a.r;
        a.st->T = T;
        a.st->s_pre = s_prefilter(T, a.metric);
      }
      return;
    }
  }
  constexpr int kPairs = kSamplePerBlock / 2 / kBlock;  // pairs per thread
  for (int j = threadIdx.x; j < kDistBins; j += kBlock) lh[j] = 0u;
  const int64_t npairs = a.n >> 1;
  const int64_t stride = npairs / gridDim.x;  // >= kSamplePerBlock/2 since n >= kSampleMinN
  const int64_t p0 = (int64_t)blockIdx.x * stride;
  const int64_t bbase = dist_bin_base(a.r);
  double2 xv[kPairs], yv[kPairs];
#pragma unroll
  for (int u = 0; u < kPairs; ++u) {
    const int64_t i = 2 * (p0 + u * kBlock + threadIdx.x);
    xv[u] = *reinterpret_cast<const double2*>(a.x + i);
    yv[u] = *reinterpret_cast<const double2*>(a.y + i);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kPairs; ++u) {
    if (knn_pass<METRIC>(a.qx, a.qy, a.qr, xv[u].x, yv[u].x, a.s_r, a.r))
      atomicAdd(&lh[dist_bin(knn_dist<METRIC>(a.qx, a.qy, xv[u].x, yv[u].x), bbase)], 1u);
    if (knn_pass<METRIC>(a.qx, a.qy, a.qr, xv[u].y, yv[u].y, a.s_r, a.r))
      atomicAdd(&lh[dist_bin(knn_dist<METRIC>(a.qx, a.qy, xv[u].y, yv[u].y), bbase)], 1u);
  }
  sample_finish(a.st, lh, a.k, a.r, a.metric, bbase);
}

hipError_t launch_knn_sample(gf_ctx* ctx, const KnnSampleArgs& a) {
  KTimer t(ctx, GF_K_KNN_SAMPLE);
  if (a.metric == 0)
    hipLaunchKernelGGL(knn_sample_kernel<0>, dim3(kSampleBlocks), dim3(kBlock), 0, ctx->stream, a);
  else
    hipLaunchKernelGGL(knn_sample_kernel<1>, dim3(kSampleBlocks), dim3(kBlock), 0, ctx->stream, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// scan
// ---------------------------------------------------------------------------------------
typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int NT>
__device__ __forceinline__ dbl2 ld2(const dbl2* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}

__device__ __forceinline__ void wave_append(bool c, double d, uint32_t idx, const KnnScanArgs& a) {
  const uint64_t m = __ballot(c);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(&a.st->count, (unsigned long long)__popcll(m));
  base = __shfl(base, leader, 64);
  if (c) {
    const unsigned long long pos = base + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
    if (pos < a.cap) {
      a.cand_d[pos] = d;
      a.cand_i[pos] = idx;
      a.cand_o[pos] = a.objID[idx];
    }
  }
}

// Per-iteration body shared by the unchecked main loop and the checked tail.
template <int METRIC, int U>
__device__ __forceinline__ void knn_scan_tile(const KnnScanArgs& a, const dbl2 (&xv)[U], const dbl2 (&yv)[U],
                                              int64_t p0, int64_t wstride, double sp, double T) {
  uint32_t cm = 0;  // candidate bits, 2 per pair
#pragma unroll
  for (int u = 0; u < U; ++u) {
    cm |= (uint32_t)knn_pass<METRIC>(a.qx, a.qy, a.qr, xv[u].x, yv[u].x, sp, T) << (2 * u);
    cm |= (uint32_t)knn_pass<METRIC>(a.qx, a.qy, a.qr, xv[u].y, yv[u].y, sp, T) << (2 * u + 1);
  }
  if (__ballot(cm != 0)) {  // wave-uniform, rare once T is tight
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i0 = (uint32_t)(2 * (p0 + u * wstride));
      const bool c0 = (cm >> (2 * u)) & 1u, c1 = (cm >> (2 * u + 1)) & 1u;
      wave_append(c0, c0 ? knn_dist<METRIC>(a.qx, a.qy, xv[u].x, yv[u].x) : 0.0, i0, a);
      wave_append(c1, c1 ? knn_dist<METRIC>(a.qx, a.qy, xv[u].y, yv[u].y) : 0.0, i0 + 1, a);
    }
  }
}

// Main loop: every wave runs the same number of full U-pair tiles with no bounds checks (loads
// issued back to back from bumped pointers, counted waits); the remainder goes through a
// checked one-pair-per-lane tail.  `bid` / `nblk`: this block's index among the scanning blocks.
template <int METRIC, int U, int NT>
__device__ __forceinline__ void knn_scan_body(const KnnScanArgs& a, double sp, double T, int64_t bid, int64_t nblk) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = nblk * kBlock;
  const int64_t pbeg = a.begin >> 1;
  const int64_t npf = (a.end - a.begin) >> 1;  // complete pairs
  const int64_t iters = npf / (U * wstride);    // full tiles for every wave
  const int64_t off = bid * kBlock + (threadIdx.x & ~63) + lane;
  const dbl2* px = reinterpret_cast<const dbl2*>(a.x) + pbeg + off;
  const dbl2* py = reinterpret_cast<const dbl2*>(a.y) + pbeg + off;
#ifdef GF_TRACE
  if (threadIdx.x == 0) atomicMin(&a.st->tr[1], (unsigned long long)wall_clock64());
#endif
  for (int64_t it = 0; it < iters; ++it) {
    dbl2 xv[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xv[u] = ld2<NT>(px + u * wstride);
      yv[u] = ld2<NT>(py + u * wstride);
    }
    knn_scan_tile<METRIC, U>(a, xv, yv, pbeg + off + it * U * wstride, wstride, sp, T);
    px += U * wstride;
    py += U * wstride;
  }
  const int64_t pend = (a.end + 1) >> 1;
  for (int64_t p = pbeg + iters * U * wstride + off; p - lane < pend; p += wstride) {
    const int64_t i = 2 * p;
    dbl2 xv[1], yv[1];
    if (i + 1 < a.end) {
      xv[0] = *reinterpret_cast<const dbl2*>(a.x + i);
      yv[0] = *reinterpret_cast<const dbl2*>(a.y + i);
    } else {
      xv[0].x = i < a.end ? a.x[i] : NAN; yv[0].x = i < a.end ? a.y[i] : NAN;
      xv[0].y = NAN; yv[0].y = NAN;  // NaN never passes the prefilter
    }
    knn_scan_tile<METRIC, 1>(a, xv, yv, p, wstride, sp, T);
  }
#ifdef GF_TRACE
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&a.st->tr[2], (unsigned long long)wall_clock64());
#endif
}

template <int METRIC, int U, int NT>
__global__ __launch_bounds__(kBlock) void knn_scan_kernel(KnnScanArgs a) {
  const double sp = a.use_state ? a.st->s_pre : a.s_pre;
  const double T = a.use_state ? a.st->T : a.T;
  knn_scan_body<METRIC, U, NT>(a, sp, T, blockIdx.x, gridDim.x);
}

template <int METRIC>
static void launch_scan_u(gf_ctx* ctx, const KnnScanArgs& a, int blocks, int unroll, int nt) {
  const dim3 g(blocks), b(kBlock);
#define GF_SCAN(U, N) hipLaunchKernelGGL((knn_scan_kernel<METRIC, U, N>), g, b, 0, ctx->stream, a)
  if (nt) {
    if (unroll <= 1) GF_SCAN(1, 1); else if (unroll == 2) GF_SCAN(2, 1); else if (unroll <= 4) GF_SCAN(4, 1); else GF_SCAN(8, 1);
  } else {
    if (unroll <= 1) GF_SCAN(1, 0); else if (unroll == 2) GF_SCAN(2, 0); else if (unroll <= 4) GF_SCAN(4, 0); else GF_SCAN(8, 0);
  }
#undef GF_SCAN
}

hipError_t launch_knn_scan(gf_ctx* ctx, const KnnScanArgs& a, int blocks, int unroll, int nt) {
  KTimer t(ctx, GF_K_KNN_SCAN);
  if (a.metric == 0) launch_scan_u<0>(ctx, a, blocks, unroll, nt);
  else launch_scan_u<1>(ctx, a, blocks, unroll, nt);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// select / merge: one 256-thread block (4 waves).  Keys (d bits, objID key, idx): d >= 0 so
// its IEEE bits order like the values; idx is unique, so keys never tie.
// Two LDS layouts share the code: SelFull (standalone select / merge kernels: 1024-key sort
// area, chunked general path) and SelLite (28 KB, block 0 of the fused scan kernel, which
// must leave room for 4 scanning blocks per CU).  The histogram is dead once the survivors
// are compacted, so it shares storage with the merge runs and the dedupe hash table.
// ---------------------------------------------------------------------------------------
constexpr int kSelT = 256;
static_assert(kSelT == kBlock, "the fused kernel's select block is a scan-sized block");

struct SelFull {
  static constexpr int kCap = 1024, kHBits = 11, kK = kMaxK;
  uint64_t sd[kCap], so[kCap];
  int64_t si[kCap];
  uint64_t rd[kK], ro[kK];  // running / final top-k-distinct list
  int64_t ri[kK];
  union {
    uint32_t hist[kDistBins];
    struct {
      uint64_t rund[kSelT], runo[kSelT];
      int64_t runi[kSelT];
      uint64_t hkey[1 << kHBits];
      uint32_t hpos[1 << kHBits];
    };
  };
  uint32_t wsum[kSelT / 64];
  int s_cnt, s_bin, s_maxpos;
  uint32_t s_S, s_below;
  unsigned long long s_rng[4];  // the k-th bin's key range (tie refinement): d min / max, objID min / max
};
struct SelLite {
  static constexpr int kCap = 256, kHBits = 9, kK = 256;
  uint64_t sd[kCap], so[kCap];
  int64_t si[kCap];
  uint64_t rd[kK], ro[kK];
  int64_t ri[kK];
  union {
    uint32_t hist[kDistBins];
    struct {
      uint64_t rund[kSelT], runo[kSelT];
      int64_t runi[kSelT];
      uint64_t hkey[1 << kHBits];
      uint32_t hpos[1 << kHBits];
    };
  };
  uint32_t wsum[kSelT / 64];
  int s_cnt, s_bin, s_maxpos;
  uint32_t s_S, s_below;
  unsigned long long s_rng[4];  // the k-th bin's key range (tie refinement): d min / max, objID min / max
};
static_assert(SelFull::kCap > kMaxK, "the general path needs room for the running list plus a chunk");
static_assert(sizeof(SelLite) <= 29 * 1024, "fused kernel: 5 blocks per CU must fit the LDS");

__device__ __forceinline__ bool kless(uint64_t ad, uint64_t ao, int64_t ai, uint64_t bd, uint64_t bo, int64_t bi) {
  if (ad != bd) return ad < bd;
  if (ao != bo) return ao < bo;
  return ai < bi;
}

// bitonic network over one wave's registers (64 keys, ascending by lane)
__device__ __forceinline__ void wave_bitonic(uint64_t& d, uint64_t& o, int64_t& i) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint64_t pd = __shfl_xor(d, stride, 64), po = __shfl_xor(o, stride, 64);
      const int64_t pi = __shfl_xor(i, stride, 64);
      const bool up = (lane & size) == 0;
      const bool lower = (lane & stride) == 0;
      const bool plt = kless(pd, po, pi, d, o, i);
      if ((lower == up) ? plt : !plt) { d = pd; o = po; i = pi; }
    }
  }
}

// <= kSelT keys, one per thread (padding: i == INT64_MAX, the largest key) -> L.sd/so/si
// ascending.  Each wave sorts its 64 in registers; a key's final rank is its lane plus, for
// every other wave's run, the number of keys below it (binary search in LDS).
template <class LDS>
__device__ void sort_regs(LDS& L, uint64_t d, uint64_t o, int64_t i) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  wave_bitonic(d, o, i);
  L.rund[tid] = d; L.runo[tid] = o; L.runi[tid] = i;
  __syncthreads();
  if (i != INT64_MAX) {
    int rank = lane;
#pragma unroll
    for (int v = 0; v < kSelT / 64; ++v) {
      if (v == w) continue;
      int lo = 0;  // keys of run v below (d, o, i): 6 halving steps reach 63, one more check 64
#pragma unroll
      for (int step = 32; step > 0; step >>= 1) {
        const int m = 64 * v + lo + step - 1;
        if (kless(L.rund[m], L.runo[m], L.runi[m], d, o, i)) lo += step;
      }
      if (lo == 63 && kless(L.rund[64 * v + 63], L.runo[64 * v + 63], L.runi[64 * v + 63], d, o, i)) lo = 64;
      rank += lo;
    }
    L.sd[rank] = d; L.so[rank] = o; L.si[rank] = i;
  }
  __syncthreads();
}

template <class LDS>
__device__ void bitonic_lds(LDS& L, int P) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < (P >> 1); t += kSelT) {
        const int i = 2 * stride * (t / stride) + (t & (stride - 1));
        const int j = i + stride;
        const bool up = (i & size) == 0;
        if (kless(L.sd[j], L.so[j], L.si[j], L.sd[i], L.so[i], L.si[i]) == up) {
          uint64_t td = L.sd[i]; L.sd[i] = L.sd[j]; L.sd[j] = td;
          uint64_t to = L.so[i]; L.so[i] = L.so[j]; L.so[j] = to;
          int64_t ti = L.si[i]; L.si[i] = L.si[j]; L.si[j] = ti;
        }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ int pow2ceil(int v) {
  int p = 2;
  while (p < v) p <<= 1;
  return p;
}

// sort L.sd/so/si[0, cnt) ascending in place (cnt <= LDS::kCap)
template <class LDS>
__device__ void sort_lds(LDS& L, int cnt) {
  if (cnt <= kSelT) {
    const int tid = threadIdx.x;
    const bool in = tid < cnt;
    const uint64_t d = in ? L.sd[tid] : ~0ull, o = in ? L.so[tid] : ~0ull;
    const int64_t i = in ? L.si[tid] : INT64_MAX;
    __syncthreads();  // sort_regs reuses storage the loads above may share
    sort_regs(L, d, o, i);
  } else {
    const int P = pow2ceil(cnt);
    for (int t = cnt + threadIdx.x; t < P; t += kSelT) { L.sd[t] = ~0ull; L.so[t] = ~0ull; L.si[t] = INT64_MAX; }
    __syncthreads();
    bitonic_lds(L, P);
  }
}

// Keep the first (lowest-rank) entry of every objID among the ascending L.sd/so/si[0, cnt):
// an LDS hash table maps objID -> lowest rank (CAS insert, atomicMin), a block prefix over
// the keep flags places the first k kept entries into L.rd/ro/ri.  Returns their number.
template <class LDS>
__device__ int dedupe_topk(LDS& L, int cnt, int k) {
  constexpr int kH = 1 << LDS::kHBits;
  constexpr int kR = LDS::kCap / kSelT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int s = tid; s < kH; s += kSelT) { L.hkey[s] = ~0ull; L.hpos[s] = 0xFFFFFFFFu; }
  if (tid == 0) L.s_maxpos = 0x7FFFFFFF;
  __syncthreads();
  uint32_t slot[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int p = r * kSelT + tid;
    slot[r] = 0;
    if (p < cnt) {
      const uint64_t o = L.so[p];
      if (o == ~0ull) {  // the table's empty marker is a real objID key (INT64_MAX): own slot
        atomicMin(&L.s_maxpos, p);
        slot[r] = kH;
      } else {
        uint32_t h = (uint32_t)((o * 0x9E3779B97F4A7C15ull) >> (64 - LDS::kHBits));
        for (;;) {  // load factor <= 1/2: terminates
          const unsigned long long prev = atomicCAS((unsigned long long*)&L.hkey[h], ~0ull, o);
          if (prev == ~0ull || prev == o) break;
          h = (h + 1) & (kH - 1);
        }
        atomicMin(&L.hpos[h], (uint32_t)p);
        slot[r] = h;
      }
    }
  }
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    if (r * kSelT < cnt && base < k) {  // block-uniform
      const int p = r * kSelT + tid;
      bool keep = false;
      if (p < cnt) keep = (slot[r] == (uint32_t)kH) ? (L.s_maxpos == p) : (L.hpos[slot[r]] == (uint32_t)p);
      const uint64_t m = __ballot(keep);
      if (lane == 0) L.wsum[w] = (uint32_t)__popcll(m);
      __syncthreads();
      int before = base;
      for (int v = 0; v < w; ++v) before += (int)L.wsum[v];
      const int total = (int)(L.wsum[0] + L.wsum[1] + L.wsum[2] + L.wsum[3]);
      const int pos = before + __popcll(m & ((1ull << lane) - 1ull));
      if (keep && pos < k) { L.rd[pos] = L.sd[p]; L.ro[pos] = L.so[p]; L.ri[pos] = L.si[p]; }
      base += total;
      __syncthreads();
    }
  }
  return base < k ? base : k;
}

// wave-aggregated append into the LDS sort area
template <class LDS>
__device__ __forceinline__ void lds_push(LDS& L, bool c, uint64_t d, uint64_t o, int64_t i) {
  const uint64_t m = __ballot(c);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(&L.s_cnt, __popcll(m));
  base = __shfl(base, leader, 64);
  if (c) {
    const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
    L.sd[pos] = d; L.so[pos] = o; L.si[pos] = i;
  }
}

// The bin of L.hist holding the target-th entry (1-based): L.s_bin, L.s_S = base + entries in
// bins <= it, L.s_below = base + entries below it (bin kDistBins - 1 with everything when the
// histogram holds fewer).  16 bins per thread, block scan over 4 waves.
template <class LDS>
__device__ void kth_bin(LDS& L, uint32_t target, uint32_t base) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int kB = kDistBins / kSelT;
  uint32_t v[kB], s = 0;
#pragma unroll
  for (int j = 0; j < kB; ++j) { v[j] = L.hist[kB * tid + j]; s += v[j]; }
  uint32_t inc = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) L.wsum[wid] = inc;
  __syncthreads();
  const uint32_t total = L.wsum[0] + L.wsum[1] + L.wsum[2] + L.wsum[3];
  uint32_t before = 0;
  for (int w = 0; w < wid; ++w) before += L.wsum[w];
  const uint32_t excl = before + inc - s;
  if (target > total) {
    if (tid == kSelT - 1) { L.s_bin = kDistBins - 1; L.s_S = base + total; L.s_below = base + total - v[kB - 1]; }
  } else if (excl < target && target <= excl + s) {
    uint32_t run = excl;
    for (int j = 0; j < kB; ++j) {
      run += v[j];
      if (run >= target) { L.s_bin = kB * tid + j; L.s_S = base + run; L.s_below = base + run - v[j]; break; }
    }
  }
  __syncthreads();
}

#ifdef GF_TRACE  // phase timestamps (100 MHz wall clock) after the record, tools/trace_select.py
#define GF_TR(j) do { if (threadIdx.x == 0) tr[j] = wall_clock64(); } while (0)
#else
#define GF_TR(j) do { } while (0)
#endif

// Select body.  The count and the first LDS::kCap candidates are loaded at once (one memory
// latency).
//   M <= 256        sort all of them (register sorts + rank merge), dedupe, done.
//   otherwise       LDS histogram of log-spaced distance bins -> bin of the k-th -> survivors
//                   (bins <= it) sorted and deduped.
//   GENERAL         if that leaves < k distinct (or the survivors overflow the sort area):
//                   every candidate, chunk by chunk, against a running top-k-distinct list.
//                   Without it (fused lite select) such a window is flagged for re-evaluation.
// Next window's threshold guess (write_hint): 2 x the k-th distance; r if fewer than k exist
// within r; after an overflow the threshold shrunk to fill half the candidate buffer; after
// too few below T, 2T.  A flagged window is re-evaluated exactly by gf_knn_decode.
template <class LDS, bool GENERAL>
__device__ void knn_select_body(const KnnSelectArgs& a, LDS& L) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int k = a.k;
  constexpr int kPer = LDS::kCap / kSelT;
#ifdef GF_TRACE
  uint64_t* tr = (uint64_t*)((char*)a.result + sizeof(gf_knn_header) + 24 * (size_t)k);
#endif
  GF_TR(0);
  const unsigned long long count = a.st->count;
  const double T = a.use_state ? a.st->T : a.T;
  double dv[kPer];
  uint32_t iv[kPer];
  int64_t ov[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = tid + (int64_t)j * kSelT;
    const bool in = (unsigned long long)i < a.cap;
    dv[j] = in ? a.cand_d[i] : 0.0;
    iv[j] = in ? a.cand_i[i] : 0u;
    ov[j] = in ? a.cand_o[i] : 0;
  }
  const bool overflow = count > a.cap;
  const int64_t M = overflow ? 0 : (int64_t)count;
  bool done = overflow;  // an overflowed window is flagged below
  int nres = 0;
  GF_TR(1);

  if (!overflow && M <= kSelT) {
    const bool in = tid < M;
    sort_regs(L, in ? dbits(dv[0]) : ~0ull, in ? okey(ov[0]) : ~0ull, in ? (int64_t)iv[0] : INT64_MAX);
    GF_TR(4);
    nres = dedupe_topk(L, (int)M, k);
    done = true;
    GF_TR(5);
  } else if (!overflow) {
    for (int i = tid; i < kDistBins; i += kSelT) L.hist[i] = 0u;
    if (tid == 0) { L.s_cnt = 0; }
    __syncthreads();
    const int64_t bbase = dist_bin_base(T);
    // every candidate once, f(valid, d, objID, idx): the first LDS::kCap from the registers
    // loaded above, the rest from memory kU x 256 at a time with the loads issued together
    // (these passes are latency-bound: a few thousand candidates at most)
    constexpr int kU = GENERAL ? 4 : 2;
    auto each_of = [&](auto&& f, auto with_oi) {
#pragma unroll
      for (int j = 0; j < kPer; ++j) f(tid + (int64_t)j * kSelT < M, dv[j], ov[j], iv[j]);
      for (int64_t i0 = LDS::kCap; i0 < M; i0 += (int64_t)kU * kSelT) {  // block-uniform
        double d[kU];
        int64_t o[kU];
        uint32_t x[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int64_t i = i0 + (int64_t)u * kSelT + tid;
          const bool in = i < M;
          d[u] = in ? a.cand_d[i] : 0.0;
          o[u] = in && decltype(with_oi)::value ? a.cand_o[i] : 0;
          x[u] = in && decltype(with_oi)::value ? a.cand_i[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) f(i0 + (int64_t)u * kSelT + tid < M, d[u], o[u], x[u]);
      }
    };
    auto each = [&](auto&& f) { each_of(f, std::true_type{}); };
    // the distance histogram reads the distances alone (a cold window can hold ~10^6 candidates)
    each_of([&](bool v, double d, int64_t, uint32_t) {
      if (v) atomicAdd(&L.hist[dist_bin(d, bbase)], 1u);
    }, std::false_type{});
    __syncthreads();
    GF_TR(2);
    // bin holding the k-th candidate
    kth_bin(L, (uint32_t)k, 0u);
    GF_TR(3);
    const int bstar = L.s_bin;
    // Tie refinement: when the k-th bin alone overflows the sort area (points inside a query
    // polygon all have d = 0; a dense ring of equal distances), split that bin by a second
    // histogram over its own key range -- the distance bits, or the objID key when every
    // distance in it is equal -- and keep the prefix (in (d, objID) order) up to the bucket
    // of the k-th.  A prefix of the key order holds each of its objIDs' first entry, so its
    // top k distinct are the window's whenever it has k distinct.
    uint64_t cut_d = ~0ull, cut_o = ~0ull;
    if (L.s_S > (uint32_t)LDS::kCap) {  // block-uniform
      uint64_t r0 = ~0ull, r1 = 0ull, r2 = ~0ull, r3 = 0ull;
      each([&](bool v, double d, int64_t o, uint32_t) {
        if (v && dist_bin(d, bbase) == bstar) {
          const uint64_t db = dbits(d), ok = okey(o);
          r0 = db < r0 ? db : r0; r1 = db > r1 ? db : r1;
          r2 = ok < r2 ? ok : r2; r3 = ok > r3 ? ok : r3;
        }
      });
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint64_t t0 = __shfl_xor(r0, off, 64), t1 = __shfl_xor(r1, off, 64);
        const uint64_t t2 = __shfl_xor(r2, off, 64), t3 = __shfl_xor(r3, off, 64);
        r0 = t0 < r0 ? t0 : r0; r1 = t1 > r1 ? t1 : r1; r2 = t2 < r2 ? t2 : r2; r3 = t3 > r3 ? t3 : r3;
      }
      if (tid == 0) { L.s_rng[0] = ~0ull; L.s_rng[1] = 0ull; L.s_rng[2] = ~0ull; L.s_rng[3] = 0ull; }
      for (int i = tid; i < kDistBins; i += kSelT) L.hist[i] = 0u;
      __syncthreads();
      if (lane == 0) {
        atomicMin(&L.s_rng[0], r0); atomicMax(&L.s_rng[1], r1);
        atomicMin(&L.s_rng[2], r2); atomicMax(&L.s_rng[3], r3);
      }
      __syncthreads();
      const bool tie = L.s_rng[0] == L.s_rng[1];
      const uint64_t kmin = tie ? L.s_rng[2] : L.s_rng[0], span = (tie ? L.s_rng[3] : L.s_rng[1]) - kmin;
      const int bits = span ? 64 - __clzll((long long)span) : 0;
      const int shift = bits > 12 ? bits - 12 : 0;  // kDistBins = 4096 buckets
      each([&](bool v, double d, int64_t o, uint32_t) {
        if (v && dist_bin(d, bbase) == bstar) atomicAdd(&L.hist[((tie ? okey(o) : dbits(d)) - kmin) >> shift], 1u);
      });
      __syncthreads();
      const uint32_t below = L.s_below;
      kth_bin(L, (uint32_t)k - below, below);
      const int b2 = L.s_bin;
      const uint64_t cut = b2 >= kDistBins - 1 ? ~0ull : kmin + ((((uint64_t)b2 + 1ull) << shift) - 1ull);
      cut_d = tie ? L.s_rng[0] : cut;  // tie: every distance of the bin is equal
      cut_o = tie ? cut : ~0ull;
    }
    if (L.s_S <= (uint32_t)LDS::kCap) {  // survivors (bins < bstar, bin bstar up to the cut) fit
      each([&](bool v, double d, int64_t o, uint32_t x) {
        const int b = dist_bin(d, bbase);
        const uint64_t ok = okey(o);
        const bool c = v && (b < bstar || (b == bstar && dbits(d) <= cut_d && ok <= cut_o));
        lds_push(L, c, dbits(d), ok, (int64_t)x);
      });
      __syncthreads();
      GF_TR(4);
      const int cnt = L.s_cnt;
#ifdef GF_TRACE
      if (tid == 0) tr[8] = (uint64_t)cnt;
#endif
      sort_lds(L, cnt);
      nres = dedupe_topk(L, cnt, k);
      done = (nres >= k) || (cnt == M);
      GF_TR(5);
    }
    if (GENERAL && !done) {
      // every candidate, 256 at a time, against a running top-k-distinct list: once the list
      // holds k entries only keys below its k-th can change it, so a round usually adds a few
      // keys and the sort stays on the register path (many equal distances -- points inside a
      // query polygon all have d = 0 -- used to cost full LDS bitonic sorts of 1024 keys)
      int nr = 0;
      uint64_t md = ~0ull, mo = ~0ull;
      int64_t mi = INT64_MAX;
      for (int64_t i0 = 0; i0 < M; i0 += kSelT) {  // block-uniform trip count
        for (int i = tid; i < nr; i += kSelT) { L.sd[i] = L.rd[i]; L.so[i] = L.ro[i]; L.si[i] = L.ri[i]; }
        if (tid == 0) L.s_cnt = nr;
        __syncthreads();
        const int64_t i = i0 + tid;
        bool c = i < M;
        uint64_t d = 0, o = 0;
        int64_t ix = 0;
        if (c) {
          d = dbits(a.cand_d[i]);
          o = okey(a.cand_o[i]);
          ix = (int64_t)a.cand_i[i];
          c = nr < k || kless(d, o, ix, md, mo, mi);
        }
        lds_push(L, c, d, o, ix);
        __syncthreads();
        const int cnt = L.s_cnt;
        if (cnt > nr) {  // block-uniform
          sort_lds(L, cnt);
          nr = dedupe_topk(L, cnt, k);
          if (nr == k) { md = L.rd[k - 1]; mo = L.ro[k - 1]; mi = L.ri[k - 1]; }
        }
        __syncthreads();
      }
      nres = nr;
      done = true;
    }
  }
  // final iff nothing overflowed, every candidate was considered (or k found), and either k
  // distinct objIDs lie below T or T reached r
  const bool too_few = done && !overflow && nres < k && T < a.r;
  const int status = (!done || overflow || too_few) ? 1 : 0;
  GF_TR(6);
#ifdef GF_TRACE
  if (tid == 0) {
    tr[9] = a.st->tr[0]; tr[10] = a.st->tr[1]; tr[11] = a.st->tr[2];
    a.st->tr[1] = ~0ull; a.st->tr[2] = 0ull;
  }
#endif
  RecView out = rec_view(a.result, k);
  if (status == 0)
    for (int i = tid; i < nres; i += kSelT) {
      out.d[i] = from_bits(L.rd[i]); out.o[i] = from_okey(L.ro[i]); out.i[i] = L.ri[i] + a.idx_base;
    }
  if (tid == 0) {
    out.h->status = status;
    out.h->n = status ? 0 : nres;
    out.h->k = k;
    out.h->flags = overflow ? 1 : 0;
    out.h->candidates = (int64_t)count;
    out.h->threshold = T;
    a.st->count = 0ull;  // ready for the lane's next window
    a.st->maybe = 0ull;
    if (a.write_hint) {
      double h;
      if (status == 0) h = nres == k ? fmax(2.0 * from_bits(L.rd[k - 1]), 4.9e-324) : a.r;
      else if (overflow) h = T * sqrt(0.5 * (double)a.cap / (double)count);
      else if (too_few) h = 2.0 * T;
      else h = T;
      a.st->hint_T = h;
    }
  }
}

__global__ __launch_bounds__(kSelT) void knn_select_kernel(KnnSelectArgs a) {
  __shared__ SelFull L;
  knn_select_body<SelFull, true>(a, L);
}

// ---------------------------------------------------------------------------------------
// k > kMaxK (the reference's PriorityQueue takes any k, KNNQuery.java:216): every candidate
// within r is kept (T = r, capacity >= window), then two stable LSD radix sorts over 32-bit key
// fields of the candidate permutation -- (objID, d, idx) to keep each objID's first occurrence,
// then the survivors by (d, objID, idx) -- and the first k are the record.  Kernels below; the
// driver (api.cpp knn_large) reuses the K2 radix passes (k_points.hip).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t large_count(const KnnLargeArgs& a, int which) {
  const int64_t c = (int64_t)a.cnt[which];
  return c < a.m ? c : a.m;
}

// field: 0 idx, 1 d low word, 2 d high word (d >= 0: IEEE bits order as values), 3 objID low
// word, 4 objID high word with the sign bit flipped (signed order)
__global__ __launch_bounds__(kBlock) void knn_large_key_kernel(KnnLargeArgs a) {
  const int64_t m = large_count(a, a.pass);
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < m; j += (int64_t)gridDim.x * kBlock) {
    const uint32_t p = a.perm[j];
    uint32_t v;
    switch (a.field) {
      case 0: v = a.ci[p]; break;
      case 1: v = lo32(a.cd[p]); break;
      case 2: v = hi32(a.cd[p]); break;
      case 3: v = (uint32_t)(uint64_t)a.co[p]; break;
      default: v = (uint32_t)((uint64_t)a.co[p] >> 32) ^ 0x80000000u; break;
    }
    a.keys[j] = v;
  }
}

__global__ __launch_bounds__(kBlock) void knn_large_iota_kernel(KnnLargeArgs a) {
  const int64_t m = large_count(a, 0);
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < m; j += (int64_t)gridDim.x * kBlock)
    a.perm[j] = (uint32_t)j;
}

// the window's candidate count into cnt[0] (the bound of the first sort), the survivor counter
// zeroed, the lane ready for its next window (the select kernel does this on the other paths)
__global__ void knn_large_start_kernel(KnnLargeArgs a) {
  a.cnt[0] = (uint32_t)*a.lane_count;
  a.cnt[1] = 0u;
  *a.lane_count = 0ull;
  *a.lane_maybe = 0ull;
}

// in (objID, d, idx) order the first entry of every objID is its minimum -- the one the
// reference's merge keeps (KNNQuery.java:232-251); the survivors are appended in any order
// (one wave-aggregated atomic per wave step): the second sort's key (d, objID, idx) is total
__global__ __launch_bounds__(kBlock) void knn_large_first_kernel(KnnLargeArgs a) {
  const int64_t m = large_count(a, 0);
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j0 = (int64_t)blockIdx.x * kBlock + (threadIdx.x & ~63); j0 < m; j0 += stride) {  // wave-uniform
    const int64_t j = j0 + lane;
    uint32_t p = 0u;
    bool first = false;
    if (j < m) {
      p = a.perm[j];
      first = j == 0 || a.co[p] != a.co[a.perm[j - 1]];
    }
    const uint64_t bal = __ballot(first);
    if (bal == 0ull) continue;
    const int leader = __ffsll((unsigned long long)bal) - 1;
    uint32_t base = 0u;
    if (lane == leader) base = atomicAdd(&a.cnt[1], (uint32_t)__popcll(bal));
    base = __shfl(base, leader, 64);
    if (first) a.out[base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = p;
  }
}

// the record: header + the first min(k, survivors) entries in (d, objID, idx) order
__global__ __launch_bounds__(kBlock) void knn_large_record_kernel(KnnLargeArgs a) {
  gf_knn_header* h = reinterpret_cast<gf_knn_header*>(a.result);
  const int32_t k = a.k;
  const int32_t n = (int64_t)a.cnt[1] < (int64_t)k ? (int32_t)a.cnt[1] : k;
  double* rd = reinterpret_cast<double*>(h + 1);
  int64_t* ro = reinterpret_cast<int64_t*>(rd + k);
  int64_t* ri = ro + k;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n; j += (int64_t)gridDim.x * kBlock) {
    const uint32_t p = a.perm[j];
    rd[j] = a.cd[p];
    ro[j] = a.co[p];
    ri[j] = (int64_t)a.ci[p] + a.idx_base;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    h->status = 0;
    h->n = n;
    h->k = k;
    h->flags = 0;
    h->candidates = a.cnt[0];
    h->threshold = a.T;
  }
}

static unsigned large_blocks(int64_t items) {
  const int64_t b = (items + kBlock - 1) / kBlock;
  return (unsigned)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

hipError_t launch_knn_large(gf_ctx* ctx, int op, const KnnLargeArgs& a) {
  hipStream_t s = ctx->stream;
  const dim3 g(large_blocks(a.m)), b(kBlock);
  switch (op) {
    case 0: hipLaunchKernelGGL(knn_large_iota_kernel, g, b, 0, s, a); break;
    case 1: hipLaunchKernelGGL(knn_large_key_kernel, g, b, 0, s, a); break;
    case 2: hipLaunchKernelGGL(knn_large_first_kernel, g, b, 0, s, a); break;
    case 5: hipLaunchKernelGGL(knn_large_start_kernel, dim3(1), dim3(1), 0, s, a); break;
    default: hipLaunchKernelGGL(knn_large_record_kernel, dim3(large_blocks(a.k)), b, 0, s, a); break;
  }
  return hipGetLastError();
}

hipError_t launch_knn_select(gf_ctx* ctx, const KnnSelectArgs& a) {
  KTimer t(ctx, GF_K_KNN_SELECT);
  hipLaunchKernelGGL(knn_select_kernel, dim3(1), dim3(kSelT), 0, ctx->stream, a);
  return hipGetLastError();
}

// Merge of per-shard / per-pane records (nrec <= 64): whole records are appended to the
// running top-k-distinct list while they fit the sort area, then sorted and deduped.
// Top-k-distinct of a union = top-k-distinct of the parts' top-k-distinct lists, so the
// merged record equals evaluating the union directly.  The record source is a functor:
// strided (all-gathered shard records, batched over windows) or a pointer list (the panes of
// a sliding window, which wrap around the sliding engine's record ring).
struct StridedRecs {
  const char* base;
  size_t stride;
  __device__ const char* operator()(int r) const { return base + (size_t)r * stride; }
};
struct ListRecs {
  const KnnRecList* l;
  __device__ const char* operator()(int r) const { return l->rec[r]; }
};

// LDS: SelFull (merge kernels, any k) or SelLite (block 0 of the fused kernel, k <= 128 so the
// running list plus one whole record fit its 256-key sort area).
// foreign: the records come from other contexts (an all-gather across ranks), whose dictionary
// objID keys are ids in their own dictionaries -- a window holding one is refused (status 2).
template <class LDS, class Src>
__device__ void knn_merge_body(int32_t k, const Src& src, int32_t nrec, void* result, LDS& L, int foreign = 0) {
  __shared__ int s_off[kMaxMergeRecs + 1], s_status, s_foreign;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_foreign = 0;
    int off = 0, st = 0;
    for (int r = 0; r < nrec; ++r) {
      const gf_knn_header* h = (const gf_knn_header*)src(r);
      s_off[r] = off;
      off += h->status == 0 ? h->n : 0;
      st = h->status > st ? h->status : st;
    }
    s_off[nrec] = off;
    s_status = st;
  }
  __syncthreads();
  int nr = 0, r = 0;
  while (r < nrec) {  // block-uniform
    for (int i = tid; i < nr; i += kSelT) { L.sd[i] = L.rd[i]; L.so[i] = L.ro[i]; L.si[i] = L.ri[i]; }
    int cnt = nr;
    while (r < nrec && cnt + (s_off[r + 1] - s_off[r]) <= LDS::kCap) {
      RecView in = rec_view((void*)src(r), k);
      const int n = s_off[r + 1] - s_off[r];
      for (int i = tid; i < n; i += kSelT) {
        const int64_t o = in.o[i];
        L.sd[cnt + i] = dbits(in.d[i]); L.so[cnt + i] = okey(o); L.si[cnt + i] = in.i[i];
        if (foreign && o < GF_OBJID_NUMERIC_MIN && o != GF_OBJID_NULL) s_foreign = 1;
      }
      cnt += n;
      ++r;
    }
    __syncthreads();
    sort_lds(L, cnt);
    nr = dedupe_topk(L, cnt, k);
  }
  RecView out = rec_view(result, k);
  __syncthreads();  // s_foreign complete
  const int status = s_foreign ? GF_KNN_STATUS_FOREIGN_KEYS : s_status;
  if (status == 0)
    for (int i = tid; i < nr; i += kSelT) {
      out.d[i] = from_bits(L.rd[i]); out.o[i] = from_okey(L.ro[i]); out.i[i] = L.ri[i];
    }
  if (tid == 0) {
    out.h->status = status;
    out.h->n = status ? 0 : nr;
    out.h->k = k;
    out.h->flags = 0;
    out.h->candidates = s_off[nrec];
    out.h->threshold = 0.0;
  }
}

// ---------------------------------------------------------------------------------------
// Merge for k > kMaxK (KNNQuery.java:216 takes any k): the records no longer fit the LDS sort
// area, but each is already sorted by (d, objID, idx) -- distinct keys within a record -- so
// an entry's rank in the union is its position in its own record plus, for every other record,
// the number of its entries below it (a binary search; ties between records go to the lower
// record index, so ranks are a permutation).  Entries are placed by rank in global scratch,
// the first occurrence of every objID is found through a hash table (objID -> lowest rank,
// CAS insert + atomicMin), and a block scan over the keep flags emits the first k.  One
// 1024-thread block per window.
// ---------------------------------------------------------------------------------------
constexpr int kMergeAnyT = 1024;

template <class Src>
__device__ void knn_merge_any_body(int32_t k, const Src& src, int32_t nrec, void* result, char* scratch, int foreign) {
  __shared__ int s_off[kMaxMergeRecs + 1], s_status, s_foreign;
  __shared__ uint32_t s_null, s_wsum[kMergeAnyT / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) {
    s_foreign = 0;
    s_null = 0xFFFFFFFFu;
    int off = 0, st = 0;
    for (int r = 0; r < nrec; ++r) {
      const gf_knn_header* h = (const gf_knn_header*)src(r);
      s_off[r] = off;
      off += h->status == 0 ? h->n : 0;
      st = h->status > st ? h->status : st;
    }
    s_off[nrec] = off;
    s_status = st;
  }
  const int64_t E = (int64_t)nrec * k;
  const size_t H = merge_any_hash(E);
  uint64_t* ed = reinterpret_cast<uint64_t*>(scratch);
  uint64_t* eo = ed + E;
  int64_t* ei = reinterpret_cast<int64_t*>(eo + E);
  uint64_t* hkey = reinterpret_cast<uint64_t*>(ei + E);
  uint32_t* hpos = reinterpret_cast<uint32_t*>(hkey + H);
  for (size_t s = tid; s < H; s += kMergeAnyT) { hkey[s] = ~0ull; hpos[s] = 0xFFFFFFFFu; }
  __syncthreads();
  const int total = s_off[nrec];
  // (1) ranks
  for (int e = tid; e < total; e += kMergeAnyT) {
    int r = 0;
    while (s_off[r + 1] <= e) ++r;  // nrec <= 64
    const int p = e - s_off[r];
    const RecView in = rec_view((void*)src(r), k);
    const int64_t o = in.o[p];
    const uint64_t kd = dbits(in.d[p]), ko = okey(o);
    const int64_t ki = in.i[p];
    if (foreign && o < GF_OBJID_NUMERIC_MIN && o != GF_OBJID_NULL) s_foreign = 1;
    int rank = p;
    for (int q = 0; q < nrec; ++q) {
      if (q == r) continue;
      const RecView v = rec_view((void*)src(q), k);
      int lo = 0, hi = s_off[q + 1] - s_off[q];  // first entry of q not below the key
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        const uint64_t md = dbits(v.d[m]), mo = okey(v.o[m]);
        const int64_t mi = v.i[m];
        const bool below = q < r ? !kless(kd, ko, ki, md, mo, mi) : kless(md, mo, mi, kd, ko, ki);
        if (below) lo = m + 1;
        else hi = m;
      }
      rank += lo;
    }
    ed[rank] = kd; eo[rank] = ko; ei[rank] = ki;
  }
  __syncthreads();
  // (2) the lowest rank of every objID (~0 = INT64_MAX, the table's empty marker: its own minimum)
  for (int p = tid; p < total; p += kMergeAnyT) {
    const uint64_t o = eo[p];
    if (o == ~0ull) {
      atomicMin(&s_null, (uint32_t)p);
      continue;
    }
    size_t h = (size_t)((o * 0x9E3779B97F4A7C15ull) >> 20) & (H - 1);
    for (;;) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&hkey[h], ~0ull, o);
      if (prev == ~0ull || prev == o) break;
      h = (h + 1) & (H - 1);
    }
    atomicMin(&hpos[h], (uint32_t)p);
  }
  __syncthreads();
  // (3) the first k kept entries, in rank order
  RecView out = rec_view(result, k);
  const int status = s_foreign ? GF_KNN_STATUS_FOREIGN_KEYS : s_status;
  int base = 0;
  for (int p0 = 0; p0 < total && base < k; p0 += kMergeAnyT) {  // block-uniform
    const int p = p0 + tid;
    bool keep = false;
    if (p < total) {
      const uint64_t o = eo[p];
      if (o == ~0ull) {
        keep = s_null == (uint32_t)p;
      } else {
        size_t h = (size_t)((o * 0x9E3779B97F4A7C15ull) >> 20) & (H - 1);
        while (hkey[h] != o) h = (h + 1) & (H - 1);
        keep = hpos[h] == (uint32_t)p;
      }
    }
    const uint64_t m = __ballot(keep);
    if (lane == 0) s_wsum[w] = (uint32_t)__popcll(m);
    __syncthreads();
    int before = base, all = 0;
    for (int v = 0; v < kMergeAnyT / 64; ++v) {
      before += v < w ? (int)s_wsum[v] : 0;
      all += (int)s_wsum[v];
    }
    const int pos = before + __popcll(m & ((1ull << lane) - 1ull));
    if (keep && pos < k && status == 0) {
      out.d[pos] = from_bits(ed[p]); out.o[pos] = from_okey(eo[p]); out.i[pos] = ei[p];
    }
    base += all;
    __syncthreads();
  }
  if (tid == 0) {
    out.h->status = status;
    out.h->n = status ? 0 : (base < k ? base : k);
    out.h->k = k;
    out.h->flags = 0;
    out.h->candidates = total;
    out.h->threshold = 0.0;
  }
}

__global__ __launch_bounds__(kMergeAnyT) void knn_merge_any_kernel(int32_t k, const char* records, int32_t nrec,
                                                                   size_t rec_stride, size_t win_stride,
                                                                   void* result_base, size_t res_stride, int foreign,
                                                                   char* scratch, size_t scratch_stride) {
  const StridedRecs src{records + (size_t)blockIdx.x * win_stride, rec_stride};
  knn_merge_any_body(k, src, nrec, (char*)result_base + (size_t)blockIdx.x * res_stride,
                     scratch + (size_t)blockIdx.x * scratch_stride, foreign);
}

__global__ __launch_bounds__(kMergeAnyT) void knn_merge_any_list_kernel(int32_t k, KnnRecList list, int32_t nrec,
                                                                        void* result, char* scratch) {
  const ListRecs src{&list};
  knn_merge_any_body(k, src, nrec, result, scratch, 0);
}

// Fused continuous-query kernel (pipeline depth 2): blocks 1.. scan window i with the
// threshold taken from the lane's hint (set by window i-2's select) -- or, for a lane's first
// window (use_state 2), from the sample kernel launched just before; block 0, dispatched
// first, runs window i-1's select on the other lane while they stream.  One launch per window.
// Sliding windows: with m.nrec > 0, block 0 then merges the window that closed with window i-1
// (its pane records, the one just written included) into m.result -- no separate merge launch.
template <int METRIC, int NT>
__global__ __launch_bounds__(kBlock) void knn_fused_kernel(KnnScanArgs a, KnnSelectArgs prev, int has_prev,
                                                           KnnMergeArgs m) {
  __shared__ SelLite L;
  if (blockIdx.x == 0) {
    if (has_prev) knn_select_body<SelLite, false>(prev, L);
    if (m.nrec > 0) {
      __threadfence();  // the select's record stores, before the block reads them back
      __syncthreads();
      const ListRecs src{&m.list};
      knn_merge_body(prev.k, src, m.nrec, m.result, L);
    }
    return;
  }
  double T, sp;
  if (a.use_state == 2) {  // cold lane: the sample kernel just set T
    T = a.st->T;
    sp = a.st->s_pre;
  } else {
    const double h = a.st->hint_T;
    T = (h > 0.0 && h < a.T) ? h : a.T;  // a.T = r
    sp = s_prefilter(T, a.metric);
    if (blockIdx.x == 1 && threadIdx.x == 0) { a.st->T = T; a.st->s_pre = sp; }
  }
  knn_scan_body<METRIC, 1, NT>(a, sp, T, blockIdx.x - 1, gridDim.x - 1);
}

hipError_t launch_knn_fused(gf_ctx* ctx, const KnnScanArgs& a, const KnnSelectArgs& prev, int has_prev,
                            int scan_blocks, int nt, const KnnMergeArgs* merge) {
  KTimer t(ctx, GF_K_KNN_SCAN);
  const dim3 g(scan_blocks + 1), b(kBlock);
  KnnMergeArgs m{};
  if (merge && has_prev) m = *merge;
  if (a.metric == 0) {
    if (nt) hipLaunchKernelGGL((knn_fused_kernel<0, 1>), g, b, 0, ctx->stream, a, prev, has_prev, m);
    else hipLaunchKernelGGL((knn_fused_kernel<0, 0>), g, b, 0, ctx->stream, a, prev, has_prev, m);
  } else {
    if (nt) hipLaunchKernelGGL((knn_fused_kernel<1, 1>), g, b, 0, ctx->stream, a, prev, has_prev, m);
    else hipLaunchKernelGGL((knn_fused_kernel<1, 0>), g, b, 0, ctx->stream, a, prev, has_prev, m);
  }
  return hipGetLastError();
}

// Block w merges window w: its nrec records start at records + w*win_stride, rec_stride apart;
// the merged record goes to result + w*res_stride.
__global__ __launch_bounds__(kSelT) void knn_merge_kernel(int32_t k, const char* records, int32_t nrec,
                                                          size_t rec_stride, size_t win_stride, void* result_base,
                                                          size_t res_stride, int foreign) {
  __shared__ SelFull L;
  const StridedRecs src{records + (size_t)blockIdx.x * win_stride, rec_stride};
  knn_merge_body(k, src, nrec, (char*)result_base + (size_t)blockIdx.x * res_stride, L, foreign);
}

__global__ __launch_bounds__(kSelT) void knn_merge_list_kernel(int32_t k, KnnRecList list, int32_t nrec,
                                                               void* result) {
  __shared__ SelFull L;
  const ListRecs src{&list};
  knn_merge_body(k, src, nrec, result, L);
}

hipError_t launch_knn_merge(gf_ctx* ctx, int32_t k, const void* records, int32_t nrec, size_t rec_stride,
                            int32_t nwin, size_t win_stride, void* result, size_t res_stride, int foreign,
                            void* scratch) {
  KTimer t(ctx, GF_K_KNN_MERGE);
  if (k > kMaxK)
    hipLaunchKernelGGL(knn_merge_any_kernel, dim3(nwin), dim3(kMergeAnyT), 0, ctx->stream, k, (const char*)records,
                       nrec, rec_stride, win_stride, result, res_stride, foreign, (char*)scratch,
                       merge_any_bytes(nrec, k));
  else
    hipLaunchKernelGGL(knn_merge_kernel, dim3(nwin), dim3(kSelT), 0, ctx->stream, k, (const char*)records, nrec,
                       rec_stride, win_stride, result, res_stride, foreign);
  return hipGetLastError();
}

hipError_t launch_knn_merge_list(gf_ctx* ctx, int32_t k, const KnnRecList& list, int32_t nrec, void* result,
                                 void* scratch) {
  KTimer t(ctx, GF_K_KNN_MERGE);
  if (k > kMaxK)
    hipLaunchKernelGGL(knn_merge_any_list_kernel, dim3(1), dim3(kMergeAnyT), 0, ctx->stream, k, list, nrec, result,
                       (char*)scratch);
  else
    hipLaunchKernelGGL(knn_merge_list_kernel, dim3(1), dim3(kSelT), 0, ctx->stream, k, list, nrec, result);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Polygon-query kNN -- PointPolygonKNNQuery.windowBased (knn/PointPolygonKNNQuery.java:245-317):
// a point is a candidate iff its cell is in C u G of the polygon (UniformGrid.java:193-206,
// 399-411, the bbox cells as query cells) and d(p, P) <= T, d = JTS point-polygon distance
// (DistanceFunctions.java:33-36) or, approximate, the bbox distance (:150-200).  The envelope
// prefilter (env_far) skips the exact distance only where no rounding could bring it under T.
// T: the continuous-query hint or a 256K-point sample's k-th distance (as for point queries);
// the candidates then go through the same select (dedupe by objID, (d, objID) order).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool poly_pass(const KnnPolyArgs& a, double px, double py, double T, double& d) {
  if (!classify_cg(a.qr, px, py)) return false;
  if (px == px && py == py && env_far(a.bbox, px, py, T)) return false;
  d = a.approx ? point_bbox_distance(px, py, a.bbox) : polygon_distance(px, py, a.poly, 0);
  return d <= T;
}

__global__ __launch_bounds__(kBlock) void knn_poly_sample_kernel(KnnPolyArgs a) {
  __shared__ uint32_t lh[kDistBins];
  if (a.use_hint) {
    const double h = a.st->hint_T;
    if (h > 0.0) {
      if (blockIdx.x == 0 && threadIdx.x == 0) a.st->T = h < a.r ? h : a.r;
      return;
    }
  }
  for (int j = threadIdx.x; j < kDistBins; j += kBlock) lh[j] = 0u;
  __syncthreads();
  const int64_t n = a.end - a.begin;
  const int64_t stride = n / gridDim.x;  // >= kSamplePerBlock (n >= kSampleMinN)
  const int64_t p0 = a.begin + (int64_t)blockIdx.x * stride;
  const int64_t bbase = dist_bin_base(a.r);
  for (int u = threadIdx.x; u < kSamplePerBlock; u += kBlock) {
    const double px = a.x[p0 + u], py = a.y[p0 + u];
    double d;
    if (poly_pass(a, px, py, a.r, d)) atomicAdd(&lh[dist_bin(d, bbase)], 1u);
  }
  sample_finish(a.st, lh, a.k, a.r, a.poly.metric, bbase);
}

// Scan: the cheap prefilter only (cell class + envelope) -- no call to the polygon distance in
// the streaming loop, so the kernel keeps a streaming register footprint; survivors' indices go
// to maybe_i (one atomic per wave) and the refine kernel computes their exact distances.
__device__ __forceinline__ bool poly_maybe(const KnnPolyArgs& a, double px, double py, double T) {
  if (!classify_cg(a.qr, px, py)) return false;
  return !(px == px && py == py && env_far(a.bbox, px, py, T));
}

__device__ __forceinline__ void maybe_append(const KnnPolyArgs& a, bool c, int64_t i) {
  const uint64_t m = __ballot(c);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(&a.st->maybe, (unsigned long long)__popcll(m));
  base = __shfl(base, leader, 64);
  if (c) {
    const unsigned long long pos = base + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
    if (pos < a.cap) a.maybe_i[pos] = (uint32_t)i;
  }
}

// Two points per lane per iteration from 16-B loads of x and y (begin is even, x / y 16-B
// aligned), like the point scan; the odd last point in a checked tail.
__device__ __forceinline__ void knn_poly_scan_body(const KnnPolyArgs& a, double T, int64_t bid, int64_t nblk) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = nblk * kBlock;
  const int64_t pb = a.begin >> 1, pe = a.end >> 1;  // complete pairs [pb, pe)
  for (int64_t p = pb + bid * kBlock + threadIdx.x; p - lane < pe; p += stride) {
    const bool in = p < pe;
    dbl2 xv = {0.0, 0.0}, yv = {0.0, 0.0};
    if (in) {
      xv = __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(a.x) + p);
      yv = __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(a.y) + p);
    }
    const bool c0 = in && poly_maybe(a, xv.x, yv.x, T);
    const bool c1 = in && poly_maybe(a, xv.y, yv.y, T);
    if (__ballot(c0 || c1) == 0) continue;  // wave-uniform
    maybe_append(a, c0, 2 * p);
    maybe_append(a, c1, 2 * p + 1);
  }
  if ((a.end & 1) && bid == 0 && threadIdx.x < 64) {  // the odd last point, one wave
    const int64_t i = a.end - 1;
    maybe_append(a, lane == 0 && poly_maybe(a, a.x[i], a.y[i], T), i);
  }
}

__global__ __launch_bounds__(kBlock) void knn_poly_scan_kernel(KnnPolyArgs a) {
  knn_poly_scan_body(a, a.use_state ? a.st->T : a.r, blockIdx.x, gridDim.x);
}

// Polygon query at pipeline depth 2: blocks 1.. run window i's prefilter scan with the lane's
// hint threshold (use_state 2: the sample just taken), block 0 the select of window i-1 (whose
// refine ran before this launch) on the other lane -- and, for a sliding window closing with it,
// the window merge.  Window i's refine follows in its own launch; its select rides in window
// i+1's launch (or gf_knn_plan_flush).  Two launches per window instead of three.
__global__ __launch_bounds__(kBlock) void knn_poly_fused_kernel(KnnPolyArgs a, KnnSelectArgs prev, int has_prev,
                                                                KnnMergeArgs m) {
  __shared__ SelLite L;
  if (blockIdx.x == 0) {
    if (has_prev) knn_select_body<SelLite, false>(prev, L);
    if (m.nrec > 0) {
      __threadfence();
      __syncthreads();
      const ListRecs src{&m.list};
      knn_merge_body(prev.k, src, m.nrec, m.result, L);
    }
    return;
  }
  double T;
  if (a.use_state == 2) {
    T = a.st->T;
  } else {
    const double h = a.st->hint_T;
    T = (h > 0.0 && h < a.r) ? h : a.r;
    if (blockIdx.x == 1 && threadIdx.x == 0) a.st->T = T;  // the refine and the select read it
  }
  knn_poly_scan_body(a, T, blockIdx.x - 1, gridDim.x - 1);
}

// Refine: exact distance of each prefilter survivor; d <= T -> (d, idx, objID) candidates.  A
// maybe-list past capacity marks the window overflowed (count > cap) for the select.
__global__ __launch_bounds__(kBlock) void knn_poly_refine_kernel(KnnPolyArgs a) {
  const double T = a.use_state ? a.st->T : a.r;
  const unsigned long long nm = a.st->maybe;
  if (nm > a.cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&a.st->count, nm);
    return;
  }
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j - lane < (int64_t)nm; j += stride) {
    const bool in = j < (int64_t)nm;
    const int64_t i = in ? (int64_t)a.maybe_i[j] : 0;
    double d = 0.0;
    bool c = false;
    if (in) {
      const double px = a.x[i], py = a.y[i];
      d = a.approx ? point_bbox_distance(px, py, a.bbox) : polygon_distance(px, py, a.poly, 0);
      c = d <= T;
    }
    const uint64_t m = __ballot(c);
    if (m == 0) continue;
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(&a.st->count, (unsigned long long)__popcll(m));
    base = __shfl(base, leader, 64);
    if (c) {
      const unsigned long long pos = base + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
      if (pos < a.cap) {
        a.cand_d[pos] = d;
        a.cand_i[pos] = (uint32_t)i;
        a.cand_o[pos] = a.objID[i];
      }
    }
  }
}

hipError_t launch_knn_poly_sample(gf_ctx* ctx, const KnnPolyArgs& a) {
  KTimer t(ctx, GF_K_KNN_SAMPLE);
  hipLaunchKernelGGL(knn_poly_sample_kernel, dim3(kSampleBlocks), dim3(kBlock), 0, ctx->stream, a);
  return hipGetLastError();
}

hipError_t launch_knn_poly_fused(gf_ctx* ctx, const KnnPolyArgs& a, const KnnSelectArgs& prev, int has_prev,
                                 int blocks, const KnnMergeArgs* merge) {
  KnnMergeArgs m{};
  if (merge && has_prev) m = *merge;
  {
    KTimer t(ctx, GF_K_KNN_SCAN);
    hipLaunchKernelGGL(knn_poly_fused_kernel, dim3(blocks + 1), dim3(kBlock), 0, ctx->stream, a, prev, has_prev, m);
  }
  KnnPolyArgs r = a;
  r.use_state = 1;  // the refine reads the threshold the scan blocks stored
  hipLaunchKernelGGL(knn_poly_refine_kernel, dim3(256), dim3(kBlock), 0, ctx->stream, r);
  return hipGetLastError();
}

hipError_t launch_knn_poly_scan(gf_ctx* ctx, const KnnPolyArgs& a, int blocks) {
  {
    KTimer t(ctx, GF_K_KNN_SCAN);
    hipLaunchKernelGGL(knn_poly_scan_kernel, dim3(blocks), dim3(kBlock), 0, ctx->stream, a);
  }
  hipLaunchKernelGGL(knn_poly_refine_kernel, dim3(256), dim3(kBlock), 0, ctx->stream, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// kNN across ranks with String objIDs (KNNQuery.java:232-251 dedupes by String.equals; the
// in-repo caller MN_Q1.java:52 feeds gps.deviceId Strings).  A dictionary objID key is an id in
// its own rank's gf_objid_dict, so before the all-gather every rank attaches the Strings of its
// record's dictionary keys (a sidecar read from its dictionary's device arena); the merge then
// orders and dedupes by the Strings themselves: (d, String, idx) with dictionary Strings by
// their bytes (unsigned, a prefix first), dictionary Strings before canonical decimals, decimals
// by value -- the same on every rank, so every rank gets the same merged record.
// ---------------------------------------------------------------------------------------
struct StrSide {
  int32_t status;  // 0 ok; 1 the Strings did not fit cap (nbytes = what they need)
  int32_t n;
  int64_t nbytes;
};
__device__ __forceinline__ StrSide* side_of(void* rec, int32_t k) {
  return reinterpret_cast<StrSide*>((char*)rec + 32 + (size_t)24 * k);
}
__device__ __forceinline__ uint32_t* side_off(void* rec, int32_t k) { return reinterpret_cast<uint32_t*>(side_of(rec, k) + 1); }
__device__ __forceinline__ char* side_bytes(void* rec, int32_t k) { return (char*)side_off(rec, k) + str_side_off(k); }
__device__ __forceinline__ bool dict_key(int64_t o) { return o < GF_OBJID_NUMERIC_MIN; }

// block-wide exclusive scan of one u32 per thread (any block size <= 1024), returns the total
template <int NT>
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t* excl, uint32_t* ws) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    before += i < w ? ws[i] : 0u;
    tot += ws[i];
  }
  *excl = before + inc - v;
  __syncthreads();
  return tot;
}

// Strings of n entries (lengths len_of(i), sources src_of(i)) packed into a sidecar: offsets by a
// chunked block scan, bytes copied one entry per thread; status 1 when they exceed cap
template <int NT, class Len, class Src>
__device__ void side_pack(void* rec, int32_t k, int n, int64_t cap, const Len& len_of, const Src& src_of, uint32_t* ws) {
  StrSide* sd = side_of(rec, k);
  uint32_t* off = side_off(rec, k);
  char* bytes = side_bytes(rec, k);
  uint32_t carry = 0;
  for (int i0 = 0; i0 < n; i0 += NT) {  // block-uniform
    const int i = i0 + (int)threadIdx.x;
    const uint32_t l = i < n ? len_of(i) : 0u;
    uint32_t ex;
    const uint32_t tot = block_excl<NT>(l, &ex, ws);
    if (i < n) off[i] = carry + ex;
    carry += tot;
  }
  const bool fits = (int64_t)carry <= cap;
  if (fits)
    for (int i = threadIdx.x; i < n; i += NT) {
      const uint32_t l = len_of(i);
      const char* src = src_of(i);
      char* dst = bytes + off[i];
      for (uint32_t b = 0; b < l; ++b) dst[b] = src[b];
    }
  if (threadIdx.x == 0) {
    off[n] = carry;
    sd->status = fits ? 0 : 1;
    sd->n = n;
    sd->nbytes = (int64_t)carry;
  }
}

// block r: record r copied into string record r, its dictionary keys' Strings attached
__global__ __launch_bounds__(kBlock) void knn_attach_strings_kernel(int32_t k, const unsigned long long* idmap,
                                                                    const char* arena, int64_t dict_size,
                                                                    const char* records, int64_t cap, char* out) {
  __shared__ uint32_t ws[kBlock / 64];
  const size_t rb = 32 + (size_t)24 * k;
  const char* in = records + (size_t)blockIdx.x * rb;
  char* o = out + (size_t)blockIdx.x * str_record_bytes(k, cap);
  for (size_t b = (size_t)threadIdx.x * 8; b < rb; b += (size_t)kBlock * 8)
    *reinterpret_cast<uint64_t*>(o + b) = *reinterpret_cast<const uint64_t*>(in + b);
  const gf_knn_header* h = reinterpret_cast<const gf_knn_header*>(in);
  const int n = h->status == 0 ? h->n : 0;
  const RecView v = rec_view((void*)in, k);
  auto meta = [&](int i) -> unsigned long long {
    const int64_t key = v.o[i];
    if (!dict_key(key)) return 0ull;
    const uint64_t id = (uint64_t)key - (uint64_t)INT64_MIN;
    return id < (uint64_t)dict_size ? idmap[id] : 0ull;
  };
  side_pack<kBlock>(o, k, n, cap, [&](int i) { return (uint32_t)(meta(i) & kDictLenMask); },
                    [&](int i) { return arena + (meta(i) >> kDictLenBits); }, ws);
}

hipError_t launch_knn_attach_strings(gf_ctx* ctx, int32_t k, const unsigned long long* idmap, const char* arena,
                                     int64_t dict_size, const void* records, int32_t nrec, int64_t cap, void* out) {
  hipLaunchKernelGGL(knn_attach_strings_kernel, dim3(nrec), dim3(kBlock), 0, ctx->stream, k, idmap, arena, dict_size,
                     (const char*)records, cap, (char*)out);
  return hipGetLastError();
}

struct StrEnt {  // one entry of a string merge, in global scratch (structure of arrays)
  uint64_t* d;
  int64_t* o;
  int64_t* i;
  const char** s;
  uint32_t* len;
  uint32_t* slot;
};
__device__ __forceinline__ int str_cmp(const char* a, uint32_t la, const char* b, uint32_t lb) {
  const uint32_t m = la < lb ? la : lb;
  for (uint32_t j = 0; j < m; ++j) {
    const uint8_t x = (uint8_t)a[j], y = (uint8_t)b[j];
    if (x != y) return x < y ? -1 : 1;
  }
  return la == lb ? 0 : (la < lb ? -1 : 1);
}
// (d, String, idx): dictionary Strings by bytes and before decimals, decimals by value
__device__ __forceinline__ bool str_less(const StrEnt& E, uint32_t a, uint32_t b) {
  if (E.d[a] != E.d[b]) return E.d[a] < E.d[b];
  const int64_t oa = E.o[a], ob = E.o[b];
  const bool da = dict_key(oa), db = dict_key(ob);
  if (da != db) return da;
  if (da) {
    const int c = str_cmp(E.s[a], E.len[a], E.s[b], E.len[b]);
    if (c) return c < 0;
  } else if (oa != ob) {
    return oa < ob;
  }
  if (E.i[a] != E.i[b]) return E.i[a] < E.i[b];
  return a < b;  // identical entries: a total order still
}
__device__ __forceinline__ bool str_same(const StrEnt& E, uint32_t a, uint32_t b) {
  const int64_t oa = E.o[a], ob = E.o[b];
  const bool da = dict_key(oa), db = dict_key(ob);
  if (da != db) return false;
  return da ? str_cmp(E.s[a], E.len[a], E.s[b], E.len[b]) == 0 : oa == ob;
}
__device__ __forceinline__ uint64_t str_hash(const StrEnt& E, uint32_t a) {
  const int64_t o = E.o[a];
  uint64_t h;
  if (dict_key(o)) {
    h = 1469598103934665603ull;
    for (uint32_t j = 0; j < E.len[a]; ++j) h = (h ^ (uint8_t)E.s[a][j]) * 1099511628211ull;
    h ^= (uint64_t)E.len[a] << 40;
  } else {
    h = (uint64_t)o * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  }
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33;
  return h;
}

constexpr int kStrMergeT = 1024;
__global__ __launch_bounds__(kStrMergeT) void knn_merge_strings_kernel(int32_t k, int64_t cap, const char* records,
                                                                       int32_t nrec, size_t rec_stride,
                                                                       size_t win_stride, char* results,
                                                                       char* scratch_base) {
  __shared__ int s_off[kMaxMergeRecs + 1], s_status;
  __shared__ uint32_t ws[kStrMergeT / 64];
  const int tid = threadIdx.x;
  const char* recs = records + (size_t)blockIdx.x * win_stride;
  char* result = results + (size_t)blockIdx.x * str_record_bytes(k, cap);
  char* scratch = scratch_base + (size_t)blockIdx.x * strmerge_bytes(nrec, k);
  auto rec = [&](int r) { return (void*)(recs + (size_t)r * rec_stride); };
  if (tid == 0) {
    int off = 0, st = 0;
    for (int r = 0; r < nrec; ++r) {
      const gf_knn_header* h = (const gf_knn_header*)rec(r);
      s_off[r] = off;
      off += h->status == 0 ? h->n : 0;
      // a flagged input (status 1: its rank's window needs the exact re-evaluation) keeps the
      // merged record flagged (1), as gf_knn_merge_dev does, so every rank re-evaluates its
      // shard exactly and exchanges again; Strings that did not fit a sidecar cannot be merged
      // by String at all -- 2 (GF_KNN_STATUS_FOREIGN_KEYS), which wins over 1
      if (side_of(rec(r), k)->status != 0) st = GF_KNN_STATUS_FOREIGN_KEYS;
      else if (h->status != 0 && st == 0) st = h->status;
    }
    s_off[nrec] = off;
    s_status = st;
  }
  __syncthreads();
  const int total = s_off[nrec];
  const int64_t Emax = (int64_t)nrec * k;
  const size_t P = strmerge_pow2(total > 2 ? total : 2), H = strmerge_pow2(2 * (total > 1 ? total : 1));
  StrEnt E;
  E.d = reinterpret_cast<uint64_t*>(scratch);
  E.o = reinterpret_cast<int64_t*>(E.d + Emax);
  E.i = E.o + Emax;
  E.s = reinterpret_cast<const char**>(E.i + Emax);
  E.len = reinterpret_cast<uint32_t*>(E.s + Emax);
  E.slot = E.len + Emax;
  uint32_t* si = E.slot + Emax;                                  // [P] sorted entry order
  uint32_t* hent = si + strmerge_pow2(Emax > 2 ? Emax : 2);      // [H] representative entry
  uint32_t* hrank = hent + strmerge_pow2(2 * Emax);              // [H] its lowest sorted position
  uint32_t* olen = hrank + strmerge_pow2(2 * Emax);              // [k]
  const char** osrc = reinterpret_cast<const char**>(((uintptr_t)(olen + k) + 7) & ~(uintptr_t)7);  // [k]
  // entries, the sort order, the table
  for (int e = tid; e < total; e += kStrMergeT) {
    int r = 0;
    while (s_off[r + 1] <= e) ++r;
    const int p = e - s_off[r];
    void* rr = rec(r);
    const RecView v = rec_view(rr, k);
    E.d[e] = dbits(v.d[p]); E.o[e] = v.o[p]; E.i[e] = v.i[p];
    const uint32_t* off = side_off(rr, k);
    E.s[e] = side_bytes(rr, k) + off[p];
    E.len[e] = off[p + 1] - off[p];
  }
  for (size_t t = tid; t < P; t += kStrMergeT) si[t] = t < (size_t)total ? (uint32_t)t : 0xFFFFFFFFu;
  for (size_t t = tid; t < H; t += kStrMergeT) { hent[t] = 0xFFFFFFFFu; hrank[t] = 0xFFFFFFFFu; }
  __syncthreads();
  // bitonic sort of the entry order (padding ~0 sorts last)
  for (size_t size = 2; size <= P; size <<= 1)
    for (size_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (size_t t = tid; t < P / 2; t += kStrMergeT) {
        const size_t i = 2 * stride * (t / stride) + (t & (stride - 1)), j = i + stride;
        const uint32_t a = si[i], b = si[j];
        const bool up = (i & size) == 0;
        const bool j_less = b != 0xFFFFFFFFu && (a == 0xFFFFFFFFu || str_less(E, b, a));
        if (j_less == up) { si[i] = b; si[j] = a; }
      }
      __syncthreads();
    }
  // the lowest sorted position of every String (equal Strings share a slot)
  for (int p = tid; p < total; p += kStrMergeT) {
    const uint32_t e = si[p];
    size_t h = (size_t)str_hash(E, e) & (H - 1);
    for (;;) {
      const uint32_t cur = atomicCAS(&hent[h], 0xFFFFFFFFu, e);
      if (cur == 0xFFFFFFFFu || str_same(E, cur, e)) break;
      h = (h + 1) & (H - 1);
    }
    atomicMin(&hrank[h], (uint32_t)p);
    E.slot[p] = (uint32_t)h;
  }
  __syncthreads();
  // the first k kept entries in sorted order
  RecView out = rec_view(result, k);
  const int status = s_status;
  int base = 0;
  for (int p0 = 0; p0 < total && base < k; p0 += kStrMergeT) {  // block-uniform
    const int p = p0 + tid;
    const bool keep = p < total && hrank[E.slot[p]] == (uint32_t)p;
    uint32_t ex;
    const int all = (int)block_excl<kStrMergeT>(keep ? 1u : 0u, &ex, ws);
    const int pos = base + (int)ex;
    if (keep && pos < k) {
      const uint32_t e = si[p];
      out.d[pos] = from_bits(E.d[e]); out.o[pos] = E.o[e]; out.i[pos] = E.i[e];
      olen[pos] = E.len[e];
      osrc[pos] = E.s[e];
    }
    base += all;
  }
  const int n = status == 0 ? (base < k ? base : k) : 0;
  __syncthreads();
  side_pack<kStrMergeT>(result, k, n, cap, [&](int i) { return olen[i]; }, [&](int i) { return osrc[i]; }, ws);
  if (tid == 0) {
    out.h->status = status;
    out.h->n = n;
    out.h->k = k;
    out.h->flags = 0;
    out.h->candidates = total;
    out.h->threshold = 0.0;
  }
}

hipError_t launch_knn_merge_strings(gf_ctx* ctx, int32_t k, int64_t cap, const void* records, int32_t nrec,
                                    size_t rec_stride, int32_t nwin, size_t win_stride, void* results, void* scratch) {
  KTimer t(ctx, GF_K_KNN_MERGE);
  hipLaunchKernelGGL(knn_merge_strings_kernel, dim3(nwin), dim3(kStrMergeT), 0, ctx->stream, k, cap,
                     (const char*)records, nrec, rec_stride, win_stride, (char*)results, (char*)scratch);
  return hipGetLastError();
}

}  // namespace gf
