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
template <int METRIC>
__global__ __launch_bounds__(kBlock) void knn_sample_kernel(KnnSampleArgs a) {
  __shared__ uint32_t lh[kDistBins];
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ int s_last, s_bin;
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
  __syncthreads();
  for (int j = threadIdx.x; j < kDistBins; j += kBlock)
    if (lh[j]) atomicAdd(&a.st->hist[j], lh[j]);
  // last-arriving block picks the threshold (split-K style ticket, agent-scope fences)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t t = atomicAdd(&a.st->ticket, 1u);
    s_last = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  constexpr int kPer = kDistBins / kBlock;  // 16 bins per thread
  uint32_t v[kPer];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    v[j] = __hip_atomic_load(&a.st->hist[threadIdx.x * kPer + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  const uint32_t k = (uint32_t)a.k;
  if (excl < k && k <= excl + s) {
    uint32_t run = excl;
    for (int j = 0; j < kPer; ++j) {
      run += v[j];
      if (run >= k) { s_bin = threadIdx.x * kPer + j; break; }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double T = a.r;
    if (s_bin >= 0) {
      const double up = dist_bin_upper(s_bin, bbase);
      T = up < a.r ? up : a.r;
    }
    a.st->T = T;
    a.st->s_pre = s_prefilter(T, a.metric);
    a.st->ticket = 0;
  }
  for (int j = threadIdx.x; j < kDistBins; j += kBlock) a.st->hist[j] = 0u;
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
// checked one-pair-per-lane tail.
template <int METRIC, int U, int NT>
__global__ __launch_bounds__(kBlock) void knn_scan_kernel(KnnScanArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * kBlock;
  const int64_t pbeg = a.begin >> 1;
  const int64_t npf = (a.end - a.begin) >> 1;  // complete pairs
  const int64_t iters = npf / (U * wstride);    // full tiles for every wave
  const int64_t off = (int64_t)blockIdx.x * kBlock + (threadIdx.x & ~63) + lane;
  const double sp = a.use_state ? a.st->s_pre : a.s_pre;
  const double T = a.use_state ? a.st->T : a.T;
  const dbl2* px = reinterpret_cast<const dbl2*>(a.x) + pbeg + off;
  const dbl2* py = reinterpret_cast<const dbl2*>(a.y) + pbeg + off;
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
// select / merge: sort on (d bits, objID key, idx) then objID dedupe
// ---------------------------------------------------------------------------------------
constexpr int kSelThreads = 1024;

__device__ __forceinline__ bool key_gt(const uint64_t* sd, const uint64_t* so, const int64_t* si, int i, int j) {
  if (sd[i] != sd[j]) return sd[i] > sd[j];
  if (so[i] != so[j]) return so[i] > so[j];
  return si[i] > si[j];
}

__device__ void bitonic_sort(uint64_t* sd, uint64_t* so, int64_t* si, int P) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < (P >> 1); t += blockDim.x) {
        const int i = 2 * stride * (t / stride) + (t & (stride - 1));
        const int j = i + stride;
        const bool up = (i & size) == 0;
        if (key_gt(sd, so, si, i, j) == up) {
          uint64_t td = sd[i]; sd[i] = sd[j]; sd[j] = td;
          uint64_t to = so[i]; so[i] = so[j]; so[j] = to;
          int64_t ti = si[i]; si[i] = si[j]; si[j] = ti;
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

__device__ void pad_keys(uint64_t* sd, uint64_t* so, int64_t* si, int cnt, int P) {
  for (int i = cnt + threadIdx.x; i < P; i += blockDim.x) {
    sd[i] = ~0ull; so[i] = ~0ull; si[i] = INT64_MAX;
  }
}

// first k distinct objIDs of the sorted [0, cnt) -> (rd, ro, ri); returns the count (all threads)
__device__ int dedupe_first_k(const uint64_t* sd, const uint64_t* so, const int64_t* si, int cnt, int k,
                              uint64_t* rd, uint64_t* ro, int64_t* ri, int* s_n) {
  if ((threadIdx.x >> 6) == 0) {
    const int lane = threadIdx.x & 63;
    int acc = 0;
    for (int base = 0; base < cnt && acc < k; base += 64) {
      const int i = base + lane;
      const bool valid = i < cnt;
      const uint64_t o = valid ? so[i] : 0ull;
      bool dup = false;
      for (int j = 0; j < acc; ++j) dup |= (ro[j] == o);
      for (int j = 0; j < 64; ++j) {
        const uint64_t oj = __shfl(o, j, 64);
        dup |= (j < lane) && (oj == o);
      }
      const bool keep = valid && !dup;
      const uint64_t m = __ballot(keep);
      const int rank = __popcll(m & ((1ull << lane) - 1ull));
      if (keep && acc + rank < k) {
        rd[acc + rank] = sd[i]; ro[acc + rank] = o; ri[acc + rank] = si[i];
      }
      const int add = __popcll(m);
      acc = (acc + add < k) ? acc + add : k;
    }
    if (lane == 0) *s_n = acc;
  }
  __syncthreads();
  return *s_n;
}

// <= 64 entries in one wave's registers: bitonic network over __shfl_xor, then dedupe.
// Keys are unique (idx), so the compare-exchange needs no tie rule.
__device__ __forceinline__ bool kless(uint64_t ad, uint64_t ao, int64_t ai, uint64_t bd, uint64_t bo, int64_t bi) {
  if (ad != bd) return ad < bd;
  if (ao != bo) return ao < bo;
  return ai < bi;
}
__device__ int wave_sort_dedupe(uint64_t d, uint64_t o, int64_t i, int k, uint64_t* rd, uint64_t* ro, int64_t* ri) {
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
  bool dup = false;
  for (int j = 0; j < 64; ++j) {
    const uint64_t oj = __shfl(o, j, 64);
    dup |= (j < lane) && (oj == o);
  }
  const bool keep = (d != ~0ull) && !dup;
  const uint64_t m = __ballot(keep);
  const int rank = __popcll(m & ((1ull << lane) - 1ull));
  if (keep && rank < k) { rd[rank] = d; ro[rank] = o; ri[rank] = i; }
  const int n = __popcll(m);
  return n < k ? n : k;
}

// Lean select: 4 waves, 64 KB of LDS.  Up to kSelFast candidates are staged in registers
// (loaded together with the count: one memory latency), histogrammed in LDS; the survivors up
// to the k-th bin are sorted in one wave's registers (<= 64) or an LDS bitonic network.
constexpr int kSelT = 256;
constexpr int kSelFast = 1024;
static_assert(kSelFast > kMaxK, "general path needs room for the running list plus a chunk");

__global__ __launch_bounds__(kSelT) void knn_select_kernel(KnnSelectArgs a) {
  __shared__ uint64_t sd[kSelFast], so[kSelFast];
  __shared__ int64_t si[kSelFast];
  __shared__ uint64_t rd[kMaxK], ro[kMaxK];
  __shared__ int64_t ri[kMaxK];
  __shared__ uint32_t hist[kDistBins];
  __shared__ uint32_t wsum[kSelT / 64];
  __shared__ int s_cnt, s_n, s_bin;
  __shared__ uint32_t s_S;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int k = a.k;
  constexpr int kPer = kSelFast / kSelT;  // 4
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
  for (int i = tid; i < kDistBins; i += kSelT) hist[i] = 0u;
  const bool overflow = count > a.cap;
  const int64_t M = overflow ? 0 : (int64_t)count;
  int status = overflow ? 1 : 0;
  int nres = 0;
  __syncthreads();

  if (!overflow) {
    const bool staged = M <= kSelFast;
    const int64_t bbase = dist_bin_base(T);
    if (staged) {
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (tid + (int64_t)j * kSelT < M) atomicAdd(&hist[dist_bin(dv[j], bbase)], 1u);
    } else {
      for (int64_t i = tid; i < M; i += kSelT) atomicAdd(&hist[dist_bin(a.cand_d[i], bbase)], 1u);
    }
    __syncthreads();
    // bin holding the k-th candidate: 16 bins per thread, block scan over 4 waves
    constexpr int kB = kDistBins / kSelT;
    uint32_t v[kB], s = 0;
#pragma unroll
    for (int j = 0; j < kB; ++j) { v[j] = hist[kB * tid + j]; s += v[j]; }
    uint32_t inc = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t t = __shfl_up(inc, off, 64);
      if (lane >= off) inc += t;
    }
    if (lane == 63) wsum[wid] = inc;
    if (tid == 0) { s_bin = kDistBins - 1; s_S = (uint32_t)M; s_cnt = 0; }
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wid; ++w) before += wsum[w];
    const uint32_t excl = before + inc - s;
    if (excl < (uint32_t)k && (uint32_t)k <= excl + s) {
      uint32_t run = excl;
      for (int j = 0; j < kB; ++j) {
        run += v[j];
        if (run >= (uint32_t)k) { s_bin = kB * tid + j; s_S = run; break; }
      }
    }
    __syncthreads();
    const int bstar = s_bin;
    bool done = false;
    if (s_S <= (uint32_t)kSelFast) {  // fast path: survivors (bins <= bstar) fit the sort area
      if (staged) {
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          if (tid + (int64_t)j * kSelT < M && dist_bin(dv[j], bbase) <= bstar) {
            const int pos = atomicAdd(&s_cnt, 1);
            sd[pos] = dbits(dv[j]); si[pos] = iv[j]; so[pos] = okey(ov[j]);
          }
        }
      } else {
        for (int64_t i = tid; i < M; i += kSelT) {
          const double d = a.cand_d[i];
          if (dist_bin(d, bbase) <= bstar) {
            const int pos = atomicAdd(&s_cnt, 1);
            sd[pos] = dbits(d); si[pos] = a.cand_i[i]; so[pos] = okey(a.cand_o[i]);
          }
        }
      }
      __syncthreads();
      const int cnt = s_cnt;
      if (cnt <= 64 && k <= 64) {  // one wave, registers only
        if (wid == 0) {
          const bool in = lane < cnt;
          const int r = wave_sort_dedupe(in ? sd[lane] : ~0ull, in ? so[lane] : ~0ull, in ? si[lane] : INT64_MAX, k,
                                         rd, ro, ri);
          if (lane == 0) s_n = r;
        }
        __syncthreads();
        nres = s_n;
      } else {
        const int P = pow2ceil(cnt);
        pad_keys(sd, so, si, cnt, P);
        __syncthreads();
        bitonic_sort(sd, so, si, P);
        nres = dedupe_first_k(sd, so, si, cnt, k, rd, ro, ri, &s_n);
      }
      done = (nres >= k) || (cnt == M);
    }
    if (!done) {  // general path: every candidate, chunk by chunk, running top-k-distinct list
      int nr = 0;
      const int chunk = kSelFast - k;
      for (int64_t start = 0; start < M; start += chunk) {
        const int len = (int)((M - start) < chunk ? (M - start) : chunk);
        for (int i = tid; i < nr; i += kSelT) { sd[i] = rd[i]; so[i] = ro[i]; si[i] = ri[i]; }
        for (int i = tid; i < len; i += kSelT) {
          sd[nr + i] = dbits(a.cand_d[start + i]); si[nr + i] = a.cand_i[start + i];
          so[nr + i] = okey(a.cand_o[start + i]);
        }
        const int cnt = nr + len;
        const int P = pow2ceil(cnt);
        pad_keys(sd, so, si, cnt, P);
        __syncthreads();
        bitonic_sort(sd, so, si, P);
        nr = dedupe_first_k(sd, so, si, cnt, k, rd, ro, ri, &s_n);
      }
      nres = nr;
    }
    if (nres < k && T < a.r) status = 1;  // fewer than k distinct objIDs below T: re-evaluate
  }
  RecView out = rec_view(a.result, k);
  if (status == 0)
    for (int i = tid; i < nres; i += kSelT) {
      out.d[i] = from_bits(rd[i]); out.o[i] = from_okey(ro[i]); out.i[i] = ri[i] + a.idx_base;
    }
  if (tid == 0) {
    out.h->status = status;
    out.h->n = status ? 0 : nres;
    out.h->k = k;
    out.h->flags = overflow ? 1 : 0;
    out.h->candidates = (int64_t)count;
    out.h->threshold = T;
    a.st->count = 0ull;  // ready for the next window on this stream
    if (a.write_hint) {
      double h = 0.0;  // 0: sample the next window
      if (status == 0 && nres == k) h = 2.0 * from_bits(rd[k - 1]);
      else if (status == 0) h = a.r;  // fewer than k within r: the next window scans to r as well
      a.st->hint_T = h;
    }
  }
}

hipError_t launch_knn_select(gf_ctx* ctx, const KnnSelectArgs& a) {
  KTimer t(ctx, GF_K_KNN_SELECT);
  hipLaunchKernelGGL(knn_select_kernel, dim3(1), dim3(kSelT), 0, ctx->stream, a);
  return hipGetLastError();
}

// merge of per-shard records: nrec * k <= kSortCap (checked by the host)
__global__ __launch_bounds__(kSelThreads) void knn_merge_kernel(int32_t k, const char* records, int32_t nrec,
                                                                size_t rec_bytes, void* result) {
  __shared__ uint64_t sd[kSortCap], so[kSortCap];
  __shared__ int64_t si[kSortCap];
  __shared__ uint64_t rd[kMaxK], ro[kMaxK];
  __shared__ int64_t ri[kMaxK];
  __shared__ int s_off[65], s_n, s_status;
  const int tid = threadIdx.x;
  if (tid == 0) {
    int off = 0, st = 0;
    for (int r = 0; r < nrec; ++r) {
      const gf_knn_header* h = (const gf_knn_header*)(records + (size_t)r * rec_bytes);
      s_off[r] = off;
      off += h->status == 0 ? h->n : 0;
      st = h->status > st ? h->status : st;
    }
    s_off[nrec] = off;
    s_status = st;
  }
  __syncthreads();
  for (int r = 0; r < nrec; ++r) {
    RecView in = rec_view((void*)(records + (size_t)r * rec_bytes), k);
    const int n = s_off[r + 1] - s_off[r];
    for (int i = tid; i < n; i += kSelThreads) {
      sd[s_off[r] + i] = dbits(in.d[i]); so[s_off[r] + i] = okey(in.o[i]); si[s_off[r] + i] = in.i[i];
    }
  }
  const int cnt = s_off[nrec];
  const int P = pow2ceil(cnt);
  pad_keys(sd, so, si, cnt, P);
  __syncthreads();
  bitonic_sort(sd, so, si, P);
  const int nres = dedupe_first_k(sd, so, si, cnt, k, rd, ro, ri, &s_n);
  RecView out = rec_view(result, k);
  for (int i = tid; i < nres; i += kSelThreads) {
    out.d[i] = from_bits(rd[i]); out.o[i] = from_okey(ro[i]); out.i[i] = ri[i];
  }
  if (tid == 0) {
    out.h->status = s_status;
    out.h->n = s_status ? 0 : nres;
    out.h->k = k;
    out.h->flags = 0;
    out.h->candidates = cnt;
    out.h->threshold = 0.0;
  }
}

hipError_t launch_knn_merge(gf_ctx* ctx, int32_t k, const void* records, int32_t nrec, void* result) {
  const size_t rb = gf_knn_result_bytes(k);
  hipLaunchKernelGGL(knn_merge_kernel, dim3(1), dim3(kSelThreads), 0, ctx->stream, k, (const char*)records, nrec,
                     rb, result);
  return hipGetLastError();
}

}  // namespace gf
