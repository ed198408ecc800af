// k_range.hip -- window apply of the range queries:
//   PointPointRangeQuery.java:150-186   (guaranteed cell -> emit; candidate cell -> emit once
//                                         if some query point is within r; approximate: once
//                                         per query point)
//   PointPolygonRangeQuery.java:170-204 (same with JTS point-polygon distance, or the polygon
//                                         bounding-box distance in approximate mode)
// One fused HBM-bound pass: 16 B/point in (x, y), 1 bit/point out (selection bitmap, built
// from two wave ballots per 128 points), per-block hit counts (no global atomics).
//
// Classification (guaranteed / candidate / none):
//   ARITH  single query point: exact per-axis double intervals precomputed on the host from
//          the cell thresholds, so no per-point division at all.
//   TABLE  many query objects: exact cell (two fp64 divisions) + one byte from a per-cell
//          class table (L1/L2 resident), out-of-grid cells against the g == 0 extra rects.
// Testing a candidate-cell point walks that cell's object list (CSR built on the host over a
// (c+2)-cell reach, a superset of every object that can be within r).
#define GF_TU_NAME k_range_hip
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include "gf_geom.hpp"
#include "gf_internal.hpp"

// range_kernel<1, 1, 0, U> (inline polygon tests, a tuning fallback to the deferred queue): the
// inlined JTS code is too large for range_stage's tile unroll, which then stays a loop; that
// variant is slower anyway, and calls (the alternative) cost it more registers than the loop.
#pragma clang diagnostic ignored "-Wpass-failed"

namespace gf {

// DistanceOp(point, polygon) of polygon p of the plan's set (gf_geom.hpp)
__device__ __forceinline__ double point_polygon_distance(double px, double py, const RangeArgs& a, int p) {
  return polygon_distance(px, py, PolyView{a.ring_off, a.vert_off, a.vx, a.vy, a.ring_env, a.metric, a.rect}, p);
}

// ---------------- classification --------------------------------------------------------
// kInside: a candidate cell lying wholly inside a closed region whose every point is at
// distance 0 (an axis-aligned rectangle polygon, or any polygon's bbox in approximate mode);
// accepted without a test for non-NaN coordinates (d = 0 <= r, r >= 0).
constexpr int kNone = 0, kTest = 1, kAccept = 2, kInside = 3;

// Table modes: rows[cy] packs the first / last column of row cy whose class is not kNone
// (staged in LDS), so points of a row outside that span never touch the n*n class table (a
// per-point L2 gather: at 10M points the L2 request rate, not HBM, bounded the scan).
// Two phases so that a wave's table gathers overlap: cell_slot() computes the cell (-1 when
// outside the grid, -2 when outside its row's span) without touching memory; the caller then
// issues every gather of the iteration (an unconditional load from a clamped address: a load
// under a branch would be waited on inside the branch) and only then finishes the classes.
// Exact cell of an in-grid coordinate without a division: c = trunc((v - mn) / cl) computed
// with 1/cl is within one of the exact cell (relative error ~2^-52 on values < n <= 2048), and
// the exact per-axis thresholds T[c] = first_at_least(c) (host-built, staged in LDS) fix it.
__device__ __forceinline__ int32_t fast_cell(double v, double mn, double inv_cl, const double* T, int32_t n) {
  int32_t c = (int32_t)((v - mn) * inv_cl);
  c = c < 0 ? 0 : (c > n - 1 ? n - 1 : c);
  return c - (v < T[c] ? 1 : 0) + (v >= T[c + 1] ? 1 : 0);
}

// Block-local copies of the plan's lookup tables (LDS).
struct RangeLds {
  const uint32_t* rows;    // [n] span of row cy: first | last << 16 non-none column
  const uint32_t* rowoff;  // [n] offset of row cy's span in `spans`
  const uint8_t* spans;    // the class table restricted to the row spans (null: use a.table)
  const double* tx;        // [n+1] exact thresholds per axis (null: divide)
  const double* ty;
};

template <int TABLE>
__device__ __forceinline__ int32_t cell_slot(const RangeArgs& a, const RangeLds& L, double px, double py) {
  if (!TABLE) return 0;
  const int32_t n = a.grid_n;
  int32_t cx, cy;
  if (L.tx) {
    // in grid on both axes <=> T[0] <= v < T[n] (NaN fails: it takes the slow path below)
    if (!(px >= a.x_lo && px < a.x_hi && py >= a.y_lo && py < a.y_hi)) return -1;
    // in grid, column outside every row's span (T[lo] <= x < T[hi + 1] <=> lo <= cx <= hi):
    // those lanes skip the threshold / span LDS reads
    if (!(px >= a.sx_lo && px < a.sx_hi)) return -2;
    cx = fast_cell(px, a.minX, a.inv_cl, L.tx, n);
    cy = fast_cell(py, a.minY, a.inv_cl, L.ty, n);
  } else {
    cx = cell_index(px, a.minX, a.cl);
    cy = cell_index(py, a.minY, a.cl);
    if (!(cx >= 0 && cy >= 0 && cx < n && cy < n)) return -1;
  }
  const uint32_t span = L.rows[cy];
  const int32_t lo = (int32_t)(span & 0xffffu);
  if (cx < lo || cx > (int32_t)(span >> 16)) return -2;
  return L.spans ? (int32_t)L.rowoff[cy] + (cx - lo) : cy * n + cx;
}
// (the LDS read goes through an address_space(3) pointer: with one generic pointer for both
// sources the compiler merged the two loads into a FLAT load, whose wait also drains every
// outstanding global load -- the stream's prefetched tiles)
typedef const uint8_t __attribute__((address_space(3)))* lds_u8;
__device__ __forceinline__ int table_load(const RangeArgs& a, const RangeLds& L, int32_t slot) {
  const int32_t s = slot < 0 ? 0 : slot;
  if (L.spans) return ((lds_u8)L.spans)[s];
  return a.table[s];
}
template <int TABLE>
__device__ __forceinline__ int classify_finish(const RangeArgs& a, double px, double py, int32_t slot, int tv) {
  if (!TABLE) {
    const double xs = (px == px) ? px : a.qr.minX;
    const double ys = (py == py) ? py : a.qr.minY;
    if (a.qr.g_any && in_iv(a.qr.gx, xs) && in_iv(a.qr.gy, ys)) return kAccept;
    return (in_iv(a.qr.cgx, xs) && in_iv(a.qr.cgy, ys)) ? kTest : kNone;
  }
  if (slot >= 0) {
    if (tv != kInside) return tv;
    return (px == px && py == py) ? kAccept : kTest;  // NaN lands in cell 0 (Java (int)NaN == 0)
  }
  if (slot == -2) return kNone;
  const int32_t cx = cell_index(px, a.minX, a.cl);
  const int32_t cy = cell_index(py, a.minY, a.cl);
  const int32_t n = a.grid_n;
  if (cx >= 0 && cy >= 0 && cx < n && cy < n) {  // only NaN coordinates get here in grid
    const int c = a.table[cy * n + cx];
    return c == kInside ? kTest : c;
  }
  for (int e = 0; e < a.n_extra; ++e) {
    const int32_t* r = a.extra + 4 * e;
    if (cx >= r[0] && cx <= r[1] && cy >= r[2] && cy <= r[3]) return kAccept;
  }
  return kNone;
}


// OR bit i into the bitmap word this block stored during its scan: workgroup scope -- the
// atomic is performed in this XCD's L2, which holds the block's own (drained) store of the word;
// other blocks only write other words, byte-masked (device scope went past L2 for each of the
// ~5e5 accepted points of a C3 window).
__device__ __forceinline__ void bitmap_or(uint64_t* bitmap, uint32_t i) {
  __hip_atomic_fetch_or(reinterpret_cast<unsigned long long*>(bitmap) + (i >> 6), 1ull << (i & 63),
                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// d <= r for a point pair: ONE bound field (RangeArgs.thr).  Written with the two fields (s_r on
// the squared distance, r on hypot) the compiler folded the two compares into one load from a
// select of the two members' ADDRESSES, which put the whole argument block in scratch (528 B per
// lane in the 16-B-load build, plus an s_waitcnt vmcnt(0) on the scratch load that drained the
// stream's prefetched tiles).
__device__ __forceinline__ bool pp_within(const RangeArgs& a, double dx, double dy) {
  return (a.metric == 0 ? dx * dx + dy * dy : fdlibm_hypot(dx, dy)) <= a.thr;
}

// candidate-cell test: exists object within r (first hit wins, emitted once).  The answer is
// an existential over the cell's object list, so visiting order is free: polygons whose
// envelope holds the point go first, polygons whose envelope is farther than r are skipped.
template <int TABLE, int POLY>
__device__ __forceinline__ bool test_point(const RangeArgs& a, double px, double py) {
  if (!POLY && !TABLE) {  // single query point: exact s <= smax(r) for the sqrt metric
    return pp_within(a, a.qx0 - px, a.qy0 - py);
  }
  int32_t b = 0, e = POLY ? a.npoly : a.nq;
  const int32_t* lst = nullptr;
  if (a.cand_off) {
    const int32_t cell = cell_index(py, a.minY, a.cl) * a.grid_n + cell_index(px, a.minX, a.cl);
    b = a.cand_off[cell];
    e = a.cand_off[cell + 1];
    lst = a.cand_list;
  }
  if (!POLY) {
    for (int32_t t = b; t < e; ++t) {
      const int32_t o = lst ? lst[t] : t;
      if (pp_within(a, a.qx[o] - px, a.qy[o] - py)) return true;
    }
    return false;
  }
  if (a.approx) {
    for (int32_t t = b; t < e; ++t) {
      const int32_t o = lst ? lst[t] : t;
      if (point_bbox_distance(px, py, a.bbox + 4 * o) <= a.r) return true;
    }
    return false;
  }
  const bool finite = px == px && py == py;
  if (finite) {
    for (int32_t t = b; t < e; ++t) {  // pass 1: envelopes holding the point (usually a hit)
      const int32_t o = lst ? lst[t] : t;
      if (env_holds(a.bbox + 4 * o, px, py) && point_polygon_distance(px, py, a, o) <= a.r) return true;
    }
  }
  for (int32_t t = b; t < e; ++t) {  // pass 2: the rest, envelope-pruned
    const int32_t o = lst ? lst[t] : t;
    const double* bb = a.bbox + 4 * o;
    if (finite && (env_holds(bb, px, py) || env_far(bb, px, py, a.r))) continue;
    if (point_polygon_distance(px, py, a, o) <= a.r) return true;
  }
  return false;
}


// DEFER: candidate-cell points are not tested inline (a wave would serialise on its slowest
// lane's object list) but appended to the block's queue segment, drained densely at the end of
// the block (drain_own_queue).
template <int TABLE, int POLY, int DEFER>
__device__ __forceinline__ void eval_point(const RangeArgs& a, double px, double py, int cls, bool valid, bool& hit,
                                           bool& multi, bool& defer) {
  hit = false;
  multi = false;
  defer = false;
  if (!valid) return;
  if (DEFER >= 2) {  // 2: point-polygon join (every point whose key some polygon replicates to);
    defer = cls != kNone;  // 3: span prefilter (every point not ruled out by the class spans)
    return;
  }
  if (cls == kAccept) {
    hit = true;
  } else if (cls == kTest) {
    if (!POLY && a.approx) {  // approximate point-point: emitted once per query point
      hit = true;
      multi = a.nq > 1;
    } else if (DEFER) {
      defer = true;
    } else {
      hit = test_point<TABLE, POLY>(a, px, py);
    }
  }
}

// Per-block queue segments: a wave reserves slots with one LDS atomic (a single global
// counter would serialise ~10^5 wave atomics on one L2 line).
// Both halves of a wave-tile with ONE LDS reservation (the reservation's atomic return and
// the broadcast are the latency a queueing tile pays): slots [base, base + |m0|) for the first
// half, then [base + |m0|, base + |m0| + |m1|) for the second.
__device__ __forceinline__ void queue_append2(bool c0, uint32_t i0, double x0, double y0, bool c1, uint32_t i1,
                                              double x1, double y1, const RangeArgs& a, uint32_t* lcount) {
  const uint64_t m0 = __ballot(c0), m1 = __ballot(c1);
  if ((m0 | m1) == 0) return;
  const int lane = threadIdx.x & 63;
  const uint32_t n0 = (uint32_t)__popcll(m0);
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(lcount, n0 + (uint32_t)__popcll(m1));
  base = __shfl(base, 0, 64);
  const uint64_t below = (1ull << lane) - 1ull;
  const size_t seg = (size_t)blockIdx.x * a.seg_cap + base;
  if (c0) {
    const size_t pos = seg + (uint32_t)__popcll(m0 & below);
    a.queue[pos] = i0;
    a.queue_xy[2 * pos] = x0;
    a.queue_xy[2 * pos + 1] = y0;
  }
  if (c1) {
    const size_t pos = seg + n0 + (uint32_t)__popcll(m1 & below);
    a.queue[pos] = i1;
    a.queue_xy[2 * pos] = x1;
    a.queue_xy[2 * pos + 1] = y1;
  }
}

// Span prefilter (DEFER 3): the points not ruled out by span_maybe are collected in a per-wave
// LDS buffer (ballot + mbcnt, the count in a scalar register) and classified with the table 64
// at a time, one per lane, interleaved with the stream: accepted points set their bit (an atomic
// OR into the word this wave stored), candidate-cell points go to the block's queue for
// drain_own_queue at the block's end.  (Classifying them all at the end of each block cost
// 21 us of a 74 us C3 window: no block's stream overlapped it.)
// The tile's two halves are appended separately with a round in between, so the buffer holds
// < 64 left after a round + one half's 64: 128 entries (192 before r03: the whole tile at once --
// 5 KB more LDS per block, which held C3's blocks to 3 per CU).
#ifndef GF_RANGE_WAVEQ
#define GF_RANGE_WAVEQ 128
#endif
constexpr int kWaveQ = GF_RANGE_WAVEQ;
static_assert(kWaveQ >= 127, "a round leaves < 64, a half-tile adds <= 64");
static_assert((kWaveQ & (kWaveQ - 1)) == 0, "the queue is a ring indexed mod kWaveQ");
// The bitmap words of the wave's last kWaveRing tiles stay in LDS (a ring, two words per tile),
// so the bits of points the classification accepts later are OR-ed there (ds_or) and every word
// reaches global memory once, when its tile leaves the ring or at the end of the stream.  (Each
// accepted point of the span prefilter used to take a workgroup-scope atomic OR on the word the
// wave had already stored: ~5e5 L2 atomics and 21 MB of partial-line writes per C3 window.)
// Points whose tile already left the ring (sparse stretches) still take the atomic.
constexpr int kWaveRing = 32;
struct WaveQ {  // a ring: entries head .. head + cnt - 1 (mod kWaveQ)
  uint32_t* idx;
  double2* xy;
  uint32_t cnt;
  uint32_t head;
  unsigned long long* ring;  // [2 * kWaveRing]: tile k's words at 2 (k % kWaveRing) + {0, 1}
  uint32_t ntile;            // tiles pushed so far (wave-uniform)
  uint32_t t0, tstride;      // the wave's first tile and the tile stride (points)
};
// tile k of the wave leaves the ring: its words to global memory (the tail word only in range)
__device__ __forceinline__ void ring_store(const RangeArgs& a, const WaveQ& q, uint32_t k) {
  const int64_t t = (int64_t)q.t0 + (int64_t)k * q.tstride;
  const uint32_t j = k % kWaveRing;
  a.bitmap[t >> 6] = q.ring[2 * j];
  if (t + 64 < a.n) a.bitmap[(t >> 6) + 1] = q.ring[2 * j + 1];
}
template <int POLY>
__device__ __forceinline__ void waveq_round(const RangeArgs& a, const RangeLds& L, WaveQ& q, uint32_t take,
                                            uint64_t& hits, uint32_t* lcount) {
  const uint32_t lane = threadIdx.x & 63;
  const bool valid = lane < take;
  wave_lds_sync();  // the entries other lanes of this wave queued (intra-wave LDS hand-off)
  const uint32_t slot_q = (q.head + (valid ? lane : 0u)) & (uint32_t)(kWaveQ - 1);
  const uint32_t i = q.idx[slot_q];
  const double2 v = q.xy[slot_q];
  const int32_t slot = cell_slot<1>(a, L, v.x, v.y);
  // the span table is in LDS whenever the span prefilter runs (host: span_lds): with a global
  // fallback here the two reads merge into one wait on vmcnt too, draining the stream's
  // prefetched tiles at every round
  const int tv = ((lds_u8)L.spans)[slot < 0 ? 0 : slot];
  const int cls = valid ? classify_finish<1>(a, v.x, v.y, slot, tv) : kNone;
  const bool acc = cls == kAccept;
  if (acc) {
    const uint32_t k = (i - q.t0) / q.tstride;  // the point's tile of this wave
    if (k + kWaveRing >= q.ntile)               // still in the ring
      atomicOr(&q.ring[2 * (k % kWaveRing) + ((i >> 6) & 1u)], 1ull << (i & 63));
    else
      bitmap_or(a.bitmap, i);
  }
  hits += (uint64_t)__popcll(__ballot(acc));
  wave_lds_sync();  // the ring words OR-ed by other lanes, before lane 0 stores a word that left the ring
#if GF_RANGE_EXP != 4
  queue_append2(cls == kTest, i, v.x, v.y, false, 0u, 0.0, 0.0, a, lcount);
#endif
  // the ring's head moves past the round (r04 moved the rest [take, cnt) to the front instead: two
  // LDS reads and two writes per lane per round)
  q.head = (q.head + take) & (uint32_t)(kWaveQ - 1);
  q.cnt -= take;
}

// Tile layout.  Default: lane l holds t + l and t + 64 + l and the ballots ARE the bitmap words.
// kRangeVec (GF_RANGE_VEC=1, an A/B variant): lane l holds points t + 2l and t + 2l + 1, read
// with one 16-B load per coordinate (half the load instructions, twice the bytes in flight per
// outstanding load); a tile's words are the two ballots bit-interleaved (lanes 0-31 -> word w,
// lanes 32-63 -> word w + 1).  r05 A/B on one box: C1 1M 3.7 vs 4.5 us, C1 10M 32.7 vs 36.0 us,
// C3 45.5 vs 45.0 us per window -- the 8-B layout stays.
#ifndef GF_RANGE_EXP
#define GF_RANGE_EXP 0  // experiment builds only (tools/build_exp.sh): 1 no span-queue rounds, 2 nothing queued
                        // (the compiler then drops the loads: not a measurement), 3 no candidate tests at the
                        // block's end, 4 nor their queue appends
#endif
#ifndef GF_RANGE_VEC
#define GF_RANGE_VEC 0
#endif
constexpr bool kRangeVec = GF_RANGE_VEC != 0;
__device__ __forceinline__ uint64_t spread32(uint32_t v) {  // bit i -> bit 2i
  uint64_t x = v;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}
// the tile's two bitmap words from the ballots of its first / second point per lane
__device__ __forceinline__ void tile_words(uint64_t b0, uint64_t b1, uint64_t& w0, uint64_t& w1) {
  if (kRangeVec) {
    w0 = spread32((uint32_t)b0) | (spread32((uint32_t)b1) << 1);
    w1 = spread32((uint32_t)(b0 >> 32)) | (spread32((uint32_t)(b1 >> 32)) << 1);
  } else {
    w0 = b0;
    w1 = b1;
  }
}

// One wave-tile = 128 consecutive points = bitmap words w, w+1 (one 16-B store by lane 0).
template <int TABLE, int POLY, int DEFER, bool FULL>
__device__ __forceinline__ void range_tile(const RangeArgs& a, int64_t t, double x0, double y0, double x1, double y1,
                                           int c0, int c1, uint64_t& hits, uint64_t& mult, uint32_t* lcount,
                                           WaveQ& wq, const RangeLds& L) {
  const int lane = threadIdx.x & 63;
  const int64_t i0 = kRangeVec ? t + 2 * lane : t + lane, i1 = kRangeVec ? i0 + 1 : t + 64 + lane;
  const bool v0 = FULL || i0 < a.n, v1 = FULL || i1 < a.n;
  bool h0, h1, m0, m1, d0, d1;
  eval_point<TABLE, POLY, DEFER>(a, x0, y0, c0, v0, h0, m0, d0);
  eval_point<TABLE, POLY, DEFER>(a, x1, y1, c1, v1, h1, m1, d1);
  uint64_t b0, b1;
  tile_words(__ballot(h0), __ballot(h1), b0, b1);
  const int64_t w = t >> 6;
  if (DEFER == 3) {  // into the ring (the tile that leaves it goes to global memory)
    const uint32_t k = wq.ntile++;
    if (lane == 0) {
      if (k >= (uint32_t)kWaveRing) ring_store(a, wq, k - kWaveRing);
      wq.ring[2 * (k % kWaveRing)] = b0;
      wq.ring[2 * (k % kWaveRing) + 1] = b1;
    }
  } else if (DEFER != 2 && lane == 0) {  // the caller's bitmap is only 8-B aligned
    a.bitmap[w] = b0;
    if (FULL || t + 64 < a.n) a.bitmap[w + 1] = b1;
  }
  if (a.multi) {
    uint64_t e0, e1;
    tile_words(__ballot(m0), __ballot(m1), e0, e1);
    if (lane == 0) {
      a.multi[w] = e0;
      if (FULL || t + 64 < a.n) a.multi[w + 1] = e1;
    }
    mult += (uint64_t)(__popcll(e0) + __popcll(e1));
  }
  if (DEFER == 3) {  // into the wave's buffer; classify whenever 64 are collected
#if GF_RANGE_EXP == 2  // experiment build: nothing queued (the stream and the ring only)
    d0 = d1 = false;
#endif
    const uint64_t q0 = __ballot(d0), q1 = __ballot(d1);
    const uint32_t n0 = (uint32_t)__popcll(q0);
    const uint64_t below = (1ull << lane) - 1ull;
    (void)n0;
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {  // one round call site (inlined twice it spilled)
      const bool d = h ? d1 : d0;
      const uint64_t qm = h ? q1 : q0;
      if (d) {
        const uint32_t pos = (wq.head + wq.cnt + (uint32_t)__popcll(qm & below)) & (uint32_t)(kWaveQ - 1);
        wq.idx[pos] = (uint32_t)(h ? i1 : i0);
        wq.xy[pos] = h ? make_double2(x1, y1) : make_double2(x0, y0);
      }
      wq.cnt += (uint32_t)__popcll(qm);
#if GF_RANGE_EXP == 1  // experiment build: queued points dropped (no classification rounds)
      if (wq.cnt >= 64) { wq.head = (wq.head + 64) & (uint32_t)(kWaveQ - 1); wq.cnt -= 64; }
      continue;
#endif
      if (wq.cnt >= 64) waveq_round<POLY>(a, L, wq, 64u, hits, lcount);  // leaves < 64
    }
  } else if (DEFER) {
    queue_append2(d0, (uint32_t)i0, x0, y0, d1, (uint32_t)i1, x1, y1, a, lcount);
  }
  hits += (uint64_t)(__popcll(b0) + __popcll(b1));
}

// Main loop: every wave runs the same number of full U-tile iterations with unchecked
// nontemporal 16-B loads (x, y are read once); the remainder goes through the checked tail.
// All U tiles are classified (the table-mode cell-class gathers are independent loads that
// overlap) before any tile stores, so U tiles' latencies overlap instead of adding up.
// U tiles of one wave: coordinates of the lane's two points (kRangeVec: t_u + 2 lane and the
// next, one 16-B load per coordinate for a whole tile).  A partial or past-the-end tile (the
// pipeline's last prefetch, the last tile) loads per point with the index clamped to n - 1, so
// it reads valid memory and is masked afterwards.
template <int U>
struct RangeBuf {
  double xa[U], ya[U], xb[U], yb[U];
};
template <int U, bool VEC>
__device__ __forceinline__ void range_load(RangeBuf<U>& b, const RangeArgs& a, int64_t t, int64_t tstride) {
  const int lane = threadIdx.x & 63;
  if (VEC) {  // whole tiles only: the tile start is clamped to the last whole tile (a prefetch past
              // the wave's last tile reads valid memory; those tiles are never evaluated)
    typedef double v2d __attribute__((ext_vector_type(2)));
    const int64_t tmax = (a.n & ~(int64_t)127) - 128;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t tu = t + u * tstride < tmax ? t + u * tstride : tmax;
      const v2d xv = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(a.x + tu) + lane);
      const v2d yv = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(a.y + tu) + lane);
      b.xa[u] = xv.x; b.xb[u] = xv.y;
      b.ya[u] = yv.x; b.yb[u] = yv.y;
    }
    return;
  }
  const uint32_t last = (uint32_t)(a.n - 1);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t tu = t + u * tstride;
    const int64_t p0 = kRangeVec ? tu + 2 * lane : tu + lane, p1 = kRangeVec ? p0 + 1 : tu + 64 + lane;
    const uint32_t i0 = p0 < a.n ? (uint32_t)p0 : last;
    const uint32_t i1 = p1 < a.n ? (uint32_t)p1 : last;
    b.xa[u] = __builtin_nontemporal_load(a.x + i0);
    b.xb[u] = __builtin_nontemporal_load(a.x + i1);
    b.ya[u] = __builtin_nontemporal_load(a.y + i0);
    b.yb[u] = __builtin_nontemporal_load(a.y + i1);
  }
}

// One pipeline stage: classify the U tiles of `cur` (issuing the class-table gathers first),
// then issue the loads of `nxt`, then finish -- so the gathers are waited on (vmcnt is in
// order) while the next stage's tiles stay in flight.
template <int TABLE, int POLY, int DEFER, int U, bool VEC>
__device__ __forceinline__ void range_stage(const RangeArgs& a, const RangeLds& L, const RangeBuf<U>& cur, int64_t t, RangeBuf<U>& nxt,
                                            int64_t tn, int64_t tstride, uint64_t& hits, uint64_t& mult,
                                            uint32_t* lcount, WaveQ& wq) {
  int32_t s0[U], s1[U];
  int c0[U], c1[U];
  if constexpr (DEFER == 3) {  // span prefilter: no table gathers in the stream (WaveQ)
    range_load<U, VEC>(nxt, a, tn, tstride);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c0[u] = span_maybe(a, cur.xa[u], cur.ya[u]) ? kTest : kNone;
      c1[u] = span_maybe(a, cur.xb[u], cur.yb[u]) ? kTest : kNone;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t tu = t + u * tstride;
      if (tu + 128 <= a.n)
        range_tile<TABLE, POLY, DEFER, true>(a, tu, cur.xa[u], cur.ya[u], cur.xb[u], cur.yb[u], c0[u], c1[u], hits,
                                             mult, lcount, wq, L);
      else if (!VEC && tu < a.n)
        range_tile<TABLE, POLY, DEFER, false>(a, tu, cur.xa[u], cur.ya[u], cur.xb[u], cur.yb[u], c0[u], c1[u], hits,
                                              mult, lcount, wq, L);
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    s0[u] = cell_slot<TABLE>(a, L, cur.xa[u], cur.ya[u]);
    s1[u] = cell_slot<TABLE>(a, L, cur.xb[u], cur.yb[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    c0[u] = TABLE ? table_load(a, L, s0[u]) : 0;
    c1[u] = TABLE ? table_load(a, L, s1[u]) : 0;
  }
  range_load<U, VEC>(nxt, a, tn, tstride);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    c0[u] = classify_finish<TABLE>(a, cur.xa[u], cur.ya[u], s0[u], c0[u]);
    c1[u] = classify_finish<TABLE>(a, cur.xb[u], cur.yb[u], s1[u], c1[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t tu = t + u * tstride;
    if (tu + 128 <= a.n)
      range_tile<TABLE, POLY, DEFER, true>(a, tu, cur.xa[u], cur.ya[u], cur.xb[u], cur.yb[u], c0[u], c1[u], hits,
                                           mult, lcount, wq, L);
    else if (!VEC && tu < a.n)
      range_tile<TABLE, POLY, DEFER, false>(a, tu, cur.xa[u], cur.ya[u], cur.xb[u], cur.yb[u], c0[u], c1[u], hits,
                                            mult, lcount, wq, L);
  }
}

// The window's counts without a finalize launch: the last block of the window's last kernel to
// finish (atomic ticket) sums the partials of every block and resets the ticket for the next
// window.  Hand-off without fences (cdna_hip_programming.md Guideline 16, R1): each partial is
// stored write-through (agent-scope atomic store = sc1) and drained (s_waitcnt vmcnt(0)) by the
// storing lane before its ticket add; the last block reads them with agent-scope (sc1) loads.
// (__threadfence() here is an L2 write-back per block: it doubled the 10M-point scan.)
__device__ __forceinline__ void store_partial(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void finalize_counts(const RangeArgs& a, int nparts, uint32_t* flag, uint64_t* wsum) {
  uint32_t* ticket = reinterpret_cast<uint32_t*>(a.partials + kRangeTicketSlot);
  if (threadIdx.x == 0) {  // the lane that stored this block's partials
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *flag = atomicAdd(ticket, 1u) == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!*flag) return;
  uint64_t h = 0, m = 0;
  for (int b = threadIdx.x; b < nparts; b += kBlock) {
    h += __hip_atomic_load(&a.partials[2 * b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    m += __hip_atomic_load(&a.partials[2 * b + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    h += __shfl_xor(h, o, 64);
    m += __shfl_xor(m, o, 64);
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) { wsum[2 * w] = h; wsum[2 * w + 1] = m; }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t th = 0, tm = 0;
    for (int v = 0; v < kBlock / 64; ++v) { th += wsum[2 * v]; tm += wsum[2 * v + 1]; }
    a.counts[0] = (int64_t)th;
    a.counts[1] = (int64_t)tm;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One candidate object of a queued point: within r?  (envelope-pruned for exact polygons)
template <int POLY>
__device__ __forceinline__ bool test_object(const RangeArgs& a, double px, double py, int32_t o) {
  if (!POLY) {
    return pp_within(a, a.qx[o] - px, a.qy[o] - py);
  }
  if (a.approx) return point_bbox_distance(px, py, a.bbox + 4 * o) <= a.r;
  if (px == px && py == py && env_far(a.bbox + 4 * o, px, py, a.r)) return false;
  return point_polygon_distance(px, py, a, o) <= a.r;
}

#ifndef GF_RANGE_TEST_GROUP
#define GF_RANGE_TEST_GROUP 2  // lanes per queued point in drain_own_queue (1, 2, 4, 8)
// r05 A/B, C3 per window (tools/gpu_r05_c3g.sh, one box, twice): 8 lanes 45.9 / 45.5 us, 4 45.2 /
// 45.4, 2 43.1 / 43.1, 1 44.1 / 44.4.  A block's ~60 queued points take one pass of 128 pairs
// instead of two of 32 octets: each pass is a chain of dependent loads (entry, cell list,
// polygon), so fewer passes shorten the block's tail; one lane per point walks lists serially.
#endif
constexpr int kTestGroup = GF_RANGE_TEST_GROUP;
// DEFER 1 / 3: after its scan loop, a block drains its OWN queue segment (the candidate-cell points
// it queued) -- no second launch, no grid-wide prefix of the segment counts.  A queued point is a
// group of up to kTestGroup lanes that test its candidate objects in parallel (stopping once one
// hits); hits are OR-ed into the bitmap words this block stored during the scan.
// Hand-offs (r06), by construction rather than by the calling context:
//  * the entries are GLOBAL memory stored by any wave of the block during its stream, the count
//    is LDS: every wave drains its stores (s_waitcnt vmcnt(0): acknowledged by L2) and then meets
//    the workgroup barrier (__syncthreads: release + acquire at workgroup scope, and no memory
//    access moves across it), so every entry is complete before any lane reads one;
//  * nothing else crosses lanes through memory: a group shares only ballot masks;
//  * no full wave is assumed: each wave's ACTIVE lanes take points from a block cursor in LDS
//    (one atomic per wave pass, its result broadcast by readfirstlane), form groups among
//    themselves, and a point's hit is recorded by the lowest active lane of its group that found
//    one -- a partially active wave drains every point it takes (tests: gf_range_plan_set_drain_lanes).
// Returns this wave's added hits (uniform over the active lanes).
template <int POLY>
__device__ uint64_t drain_own_queue(const RangeArgs& a, const uint32_t& lcount, uint32_t* cursor) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint32_t total = lcount;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t act = __ballot(1);                     // the lanes running the drain
  const uint32_t nact = (uint32_t)__popcll(act);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
  const uint32_t G = nact < (uint32_t)kTestGroup ? nact : (uint32_t)kTestGroup;  // lanes per point
  const uint32_t ng = nact / G;                          // groups in this wave (>= 1)
  const uint32_t gi = rank / G, g = rank - gi * G;       // my group, my place in it
  const bool grouped = gi < ng;                          // (the nact % G last lanes idle)
  uint64_t gmask = 0;                                    // my group's lanes
  for (uint32_t k = 0; k < ng; ++k) {
    const uint64_t m = __ballot(grouped && gi == k);
    if (gi == k) gmask = m;
  }
  const size_t seg = (size_t)blockIdx.x * a.seg_cap;
  uint64_t hits = 0;
  for (;;) {  // uniform over the active lanes: this wave's next ng points
    uint32_t e0 = 0;
    if (rank == 0) e0 = atomicAdd(cursor, ng);
    e0 = __builtin_amdgcn_readfirstlane(e0);
    if (e0 >= total) break;
    const uint32_t e = e0 + gi;
    const bool valid = grouped && e < total;
    const size_t pos = seg + e;
    double px = 0.0, py = 0.0;
    int32_t b = 0, end = 0;
    if (valid) {
      px = a.queue_xy[2 * pos];
      py = a.queue_xy[2 * pos + 1];
      end = POLY ? a.npoly : a.nq;
      if (a.cand_off) {
        const int32_t cell = cell_index(py, a.minY, a.cl) * a.grid_n + cell_index(px, a.minX, a.cl);
        b = a.cand_off[cell];
        end = a.cand_off[cell + 1];
      }
    }
    bool hit = false;
    for (int32_t t = b + (int32_t)g;; t += (int32_t)G) {
      const uint64_t hb = __ballot(hit);
      const bool mine = valid && t < end && !(hb & gmask);
      if (!__ballot(mine)) break;  // every group of the wave is done
      if (mine) hit = test_object<POLY>(a, px, py, a.cand_off ? a.cand_list[t] : t);
    }
    const uint64_t hm = __ballot(hit) & gmask;
    const bool rec = hit && lane == (uint32_t)__builtin_ctzll(hm);  // one recorder per point
    const uint64_t won = __ballot(rec);
    if (rec) bitmap_or(a.bitmap, a.queue[pos]);
    hits += (uint64_t)__popcll(won);
  }
  return hits;
}

// Span prefilter (DEFER 3): an in-grid point whose x lies outside the union of the rows' class
// spans, or whose y lies outside the rows holding any class, is in a none cell (exact through
// the cell thresholds); every other point -- NaN and out-of-grid ones included -- is queued and
// classified with the table at the end of its block (drain_span_queue).  The stream then has
// the interval kernel's shape (two compares per point, no table gathers, a small register
// footprint), which pays when the classes cover a small part of the grid.
__device__ __forceinline__ bool span_maybe(const RangeArgs& a, double px, double py) {
  const bool in_grid = px >= a.x_lo && px < a.x_hi && py >= a.y_lo && py < a.y_hi;
  return !in_grid || (px >= a.sx_lo && px < a.sx_hi && py >= a.sy_lo && py < a.sy_hi);
}

// dynamic-LDS header of range_kernel: lcount, pad, drain cursor, pad, sh[kBlock/64], sm[kBlock/64] (16 B multiple)
constexpr int kRangeHdrWords = 4 + 2 * 2 * (kBlock / 64);
#ifndef GF_RANGE_WAVES
#define GF_RANGE_WAVES 1
#endif
template <int TABLE, int POLY, int DEFER, int U>
__device__ __forceinline__ void range_body(const RangeArgs& a) {
  const int64_t tstride = (int64_t)gridDim.x * (kBlock / 64) * 128;       // points per grid sweep
  const int64_t t0 = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 128;
  uint64_t hits = 0, mult = 0;
  // LDS = 16-byte header (lcount) | TABLE: rows[n] | rowoff[n] | (fast cells) 2 x (n+1)
  // thresholds | (small) spans.  No static __shared__: it would shift the dynamic base off
  // 8 B and every fp64 threshold read (ds_read_b64) would be replayed as misaligned.
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_base[];
  uint32_t& lcount = lds_base[0];
  uint64_t* const sh = reinterpret_cast<uint64_t*>(lds_base + 4);  // [kBlock / 64] hits
  uint64_t* const sm = sh + kBlock / 64;                           // [kBlock / 64] multiplicity
  uint32_t* const lds = lds_base + kRangeHdrWords;
  RangeLds L{nullptr, nullptr, nullptr, nullptr, nullptr};
  WaveQ wq{nullptr, nullptr, 0u, 0u, nullptr, 0u, (uint32_t)t0, (uint32_t)tstride};
  if (DEFER || TABLE) {
    if (threadIdx.x == 0) {
      lcount = 0u;
      lds_base[2] = 0u;  // drain_own_queue's cursor
    }
    if (TABLE) {
      const int n = a.grid_n;
      uint32_t* lr = lds;
      uint32_t* lo = lds + n;
      for (int j = threadIdx.x; j < n; j += kBlock) {
        lr[j] = a.rows[j];
        lo[j] = a.rowoff[j];
      }
      L.rows = lr;
      L.rowoff = lo;
      char* tail = reinterpret_cast<char*>(lds + ((2 * n + 1) & ~1));
      if (a.xt) {
        double* lt = reinterpret_cast<double*>(tail);
        for (int j = threadIdx.x; j <= n; j += kBlock) {
          lt[j] = a.xt[j];
          lt[n + 1 + j] = a.yt[j];
        }
        L.tx = lt;
        L.ty = lt + n + 1;
        tail += 2 * sizeof(double) * (n + 1);
      }
      if (a.span_lds) {
        uint32_t* ls = reinterpret_cast<uint32_t*>(tail);
        const uint32_t* gs = reinterpret_cast<const uint32_t*>(a.spans);
        for (int j = threadIdx.x; j < (a.span_bytes + 3) / 4; j += kBlock) ls[j] = gs[j];
        L.spans = reinterpret_cast<const uint8_t*>(ls);
        tail += (a.span_bytes + 3) & ~3;
      }
      if (DEFER == 3) {  // the waves' buffers (16-B aligned)
        // aligned by OFFSET from the LDS base: an integer round trip ((uintptr_t)tail + 15 & ~15)
        // loses the address space, and the queue / ring accesses then compile to FLAT
        // instructions, whose s_waitcnt vmcnt(0) lgkmcnt(0) drained the stream's prefetched tiles
        // at every ring store
        char* const lb = reinterpret_cast<char*>(lds_base);
        char* wb = lb + (((size_t)(tail - lb) + 15) & ~(size_t)15);
        const int w = threadIdx.x >> 6;
        wq.xy = reinterpret_cast<double2*>(wb) + w * kWaveQ;
        wq.idx = reinterpret_cast<uint32_t*>(reinterpret_cast<double2*>(wb) + (kBlock / 64) * kWaveQ) + w * kWaveQ;
        wq.ring = reinterpret_cast<unsigned long long*>(reinterpret_cast<double2*>(wb) + (kBlock / 64) * kWaveQ) +
                  ((size_t)(kBlock / 64) * kWaveQ * 4 + 7) / 8 + (size_t)w * 2 * kWaveRing;
      }
    }
    __syncthreads();
  }
  // this wave's tiles t0 + k * tstride, k < K; stages of U tiles, run in pairs (buffers A, B
  // alternate, so no register copies -- and no wait -- sit on the loop's back edge)
  // kRangeVec: the stages run over the wave's WHOLE tiles with 16-B loads and no load branch
  // (a branch between the loads made the waitcnt pass drain them: the prefetch was lost); the
  // window's one partial tile, if this wave owns it, follows with checked 8-B loads
  const int64_t nfull = kRangeVec ? (a.n & ~(int64_t)127) : a.n;
  const int64_t K = t0 < nfull ? (nfull - t0 + tstride - 1) / tstride : 0;
  const int64_t pairs = (K + 2 * U - 1) / (2 * U);
  const int64_t sstride = U * tstride;
  RangeBuf<U> A, B;
  if (pairs > 0) range_load<U, kRangeVec>(A, a, t0, tstride);
  for (int64_t p = 0; p < pairs; ++p) {
    const int64_t ta = t0 + 2 * p * sstride;
    range_stage<TABLE, POLY, DEFER, U, kRangeVec>(a, L, A, ta, B, ta + sstride, tstride, hits, mult, &lcount, wq);
    range_stage<TABLE, POLY, DEFER, U, kRangeVec>(a, L, B, ta + sstride, A, ta + 2 * sstride, tstride, hits, mult,
                                                  &lcount, wq);
  }
  if (kRangeVec && nfull < a.n && t0 <= nfull && (nfull - t0) % tstride == 0) {  // this wave's partial tile
    RangeBuf<1> T, Tn;
    range_load<1, false>(T, a, nfull, tstride);
    range_stage<TABLE, POLY, DEFER, 1, false>(a, L, T, nfull, Tn, nfull, tstride, hits, mult, &lcount, wq);
  }
  const uint32_t dl = (uint32_t)a.drain_lanes;  // testing: 0 = every lane drains
  const bool drainer = dl == 0 || (threadIdx.x & 63) < dl;
  if (DEFER == 1 && drainer) hits += drain_own_queue<POLY>(a, lcount, &lds_base[2]);
  if (DEFER == 3) {
    if (wq.cnt > 0) waveq_round<POLY>(a, L, wq, wq.cnt, hits, &lcount);
    // the ring's tiles to global memory (before the block's candidate tests OR into them)
    const uint32_t lane = threadIdx.x & 63, held = wq.ntile < (uint32_t)kWaveRing ? wq.ntile : kWaveRing;
    wave_lds_sync();  // ring words written by lane 0 and OR-ed by every lane, read by lane `held`
    if (lane < held) ring_store(a, wq, wq.ntile - held + lane);
#if GF_RANGE_EXP != 3 && GF_RANGE_EXP != 4  // experiment builds: 3 no candidate tests, 4 nor their queue
    if (drainer) hits += drain_own_queue<POLY>(a, lcount, &lds_base[2]);
#endif
  }
  // per-block partial counts (plain stores; summed by range_finalize)
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh[wid] = hits; sm[wid] = mult; }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t th = 0, tm = 0;
    for (int w = 0; w < kBlock / 64; ++w) { th += sh[w]; tm += sm[w]; }
    store_partial(&a.partials[2 * blockIdx.x], th);
    store_partial(&a.partials[2 * blockIdx.x + 1], th + tm * (uint64_t)(a.nq > 1 ? a.nq - 1 : 0));
    if (DEFER == 2) a.queue_count[blockIdx.x] = lcount;
  }
  // no kernel follows (the join's passes do for DEFER 2): this kernel's last block sums the
  // window's counts (sh / sm are free again after the partials, lds_base[1] is header padding)
  if (DEFER != 2 && a.counts) finalize_counts(a, gridDim.x, &lds_base[1], sh);
}

template <int TABLE, int POLY, int DEFER, int U>
__global__ __launch_bounds__(kBlock, GF_RANGE_WAVES) void range_kernel(RangeArgs a) {
  range_body<TABLE, POLY, DEFER, U>(a);
}

// A batch of windows of one plan (gf_range_run_batch): window blockIdx.y, gridDim.x blocks
// each; the window's columns, bitmaps and partials replace the single window's (wave-uniform
// scalars), everything else is the plan's.  Inline tests only (DEFER 0: no queues to share).
template <int TABLE, int POLY, int U>
__global__ __launch_bounds__(kBlock, GF_RANGE_WAVES) void range_batch_kernel(RangeArgs a, RangeBatch b) {
  const RangeWin& w = b.w[blockIdx.y];
  RangeArgs c = a;
  c.x = w.x;
  c.y = w.y;
  c.n = w.n;
  c.bitmap = w.bitmap;
  c.multi = w.multi;
  c.partials = w.partials;
  c.counts = w.counts;
  range_body<TABLE, POLY, 0, U>(c);
}

#ifndef GF_RANGE_U
#define GF_RANGE_U 2
#endif
constexpr int kRangeU = GF_RANGE_U;  // tiles (of 128 points per wave) per main-loop iteration

// =======================================================================================
// Point-polygon window join (PointPolygonJoinQuery.java:154-213).  Polygon q is replicated to
// its keys K_q = G_q u C_q (JoinQuery.java:93-115): with B_q its bbox cells (Polygon.gridIDsSet),
//   K_q = (g == 0 ? B_q : {}) u (c > 0 ? valid cells within Chebyshev c of B_q : {})
// (G_q for g > 0 lies inside the c-neighbourhood since g < c).  Point p pairs with q iff p's
// cell is in K_q and (approximate or JTS distance(p, q) <= r).  The scan (range_kernel with
// DEFER == 2) queues every point whose cell is in some K_q; the two passes below walk each
// queued point's cell list (CSR superset) with the exact key test -- count, then write at
// block-scanned offsets.  Pairs are grouped by queued point; order otherwise unspecified.
// =======================================================================================
constexpr int kJoinKeep = 4;  // pairs per queued point kept by the count pass for the write pass (a corner point of
                              // four adjacent squares has 4; more re-walk the list in the write pass)
struct JoinPolyOut {
  uint32_t* ecnt;             // [queued entries] pairs per entry (count pass -> write pass)
  uint32_t* ecand;            // [queued entries * kJoinKeep] the first pairs' polygon indices
  uint32_t* btot;             // [gridDim.x] pairs per block
  unsigned long long* total;  // pairs of the window
  uint32_t* pairs;            // caller's (point index, polygon index) pairs
  int64_t cap;
  int aligned;
};

// Block b takes scan block b's queue segment (equal point ranges -> balanced segments), one
// lane per queued point.  A lane walks its cell's polygon list 4 at a time (list and bbox-cell
// loads batched before the tests: the walk is a chain of dependent loads otherwise).
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t* total, uint32_t* ws) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; ++w) {
    before += w < wid ? ws[w] : 0u;
    tot += ws[w];
  }
  *total = tot;
  __syncthreads();
  return before + inc - v;
}

// the polygons of (px, py)'s list that pair with it, in list order: sink(rank, q)
template <class Sink>
__device__ __forceinline__ uint32_t join_ppoly_walk(const RangeArgs& a, double px, double py, Sink&& sink) {
  const int32_t cx = cell_index(px, a.minX, a.cl), cy = cell_index(py, a.minY, a.cl);
  int32_t lb = 0, le = a.npoly;
  const bool list = a.cand_off && cx >= 0 && cy >= 0 && cx < a.grid_n && cy < a.grid_n;
  if (list) {
    const int32_t cell = cy * a.grid_n + cx;
    lb = a.cand_off[cell];
    le = a.cand_off[cell + 1];
  }
  uint32_t n = 0;
  for (int32_t t = lb; t < le; t += 4) {
    int32_t q[4];
    int4 br[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = t + u < le ? (list ? a.cand_list[t + u] : t + u) : -1;
#pragma unroll
    for (int u = 0; u < 4; ++u) br[u] = reinterpret_cast<const int4*>(a.brect)[q[u] < 0 ? 0 : q[u]];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (q[u] < 0) continue;
      // p's key in K_q (see above), on the loaded bbox cells
      const int4 b = br[u];
      bool key = a.g_layers == 0 && cx >= b.x && cx <= b.y && cy >= b.z && cy <= b.w;
      const int64_t c = a.c_layers;
      key = key || (c > 0 && cx >= 0 && cy >= 0 && cx < a.grid_n && cy < a.grid_n && (int64_t)cx >= (int64_t)b.x - c &&
                    (int64_t)cx <= (int64_t)b.y + c && (int64_t)cy >= (int64_t)b.z - c && (int64_t)cy <= (int64_t)b.w + c);
      if (key && (a.approx || test_object<1>(a, px, py, q[u]))) sink(n++, q[u]);
    }
  }
  return n;
}

// Write pass: block offset = sum of the earlier blocks' counts (count pass), a block scan per
// round of kBlock queued points, then the kept pairs are stored (a point with more than
// kJoinKeep pairs walks its list again).
__global__ __launch_bounds__(kBlock) void join_ppoly_write_kernel(RangeArgs a, JoinPolyOut o) {
  __shared__ uint32_t ws[kBlock / 64];
  __shared__ unsigned long long part[kBlock / 64];
  const int lane = threadIdx.x & 63;
  const uint32_t cnt = a.queue_count[blockIdx.x];
  const size_t base = (size_t)blockIdx.x * a.seg_cap;
  unsigned long long run = 0;
  {  // this block's output offset: sum of the earlier blocks' totals
    unsigned long long sum = 0;
    for (uint32_t i = threadIdx.x; i < blockIdx.x; i += kBlock) sum += o.btot[i];
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_down(sum, off, 64);
    if (lane == 0) part[threadIdx.x >> 6] = sum;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) run += part[w];
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *o.total = run + o.btot[blockIdx.x];
  }
  for (uint32_t i0 = 0; i0 < cnt; i0 += kBlock) {  // block-uniform
    const uint32_t i = i0 + threadIdx.x;
    const bool valid = i < cnt;
    const size_t pos = base + i;
    const uint32_t c = valid ? o.ecnt[pos] : 0u;
    uint32_t tot;
    const uint32_t ex = block_scan_excl(c, &tot, ws);
    const unsigned long long at0 = run + ex;
    run += tot;
    if (c == 0) continue;
    const uint32_t pidx = a.queue[pos];
    auto put = [&](uint32_t k, int32_t q) {
      if ((int64_t)(at0 + k) < o.cap) join_store(o.pairs, o.aligned, at0 + k, make_uint2(pidx, (uint32_t)q));
    };
    if (c <= (uint32_t)kJoinKeep) {
      for (uint32_t k = 0; k < c; ++k) put(k, (int32_t)o.ecand[pos * kJoinKeep + k]);
    } else {
      join_ppoly_walk(a, a.queue_xy[2 * pos], a.queue_xy[2 * pos + 1], put);
    }
  }
}

// Count pass.  Phase A, one lane per queued point: walk the cell list with the key test, the
// envelope prune and -- for rectangles -- the closed-box test; every other surviving pair needs
// the exact JTS distance and goes to a block worklist in LDS.  Phase B: the whole block
// computes the worklist's distances densely (a lane-per-point walk would run each wave's
// distance calls once per lane that needs one).  A point whose pairs overflow the worklist is
// recounted by its own full walk.  Ranks inside a point come from LDS atomics (pair order is
// unspecified); the set equals join_ppoly_walk's.
constexpr int kJoinWork = 4 * kBlock;  // worklist entries per round
__global__ __launch_bounds__(kBlock) void join_ppoly_count_kernel(RangeArgs a, JoinPolyOut o) {
  __shared__ uint32_t ws[kBlock / 64];
  __shared__ uint32_t pcnt[kBlock];
  __shared__ uint8_t slow[kBlock];
  __shared__ double2 pxy[kBlock];
  __shared__ uint16_t wl_slot[kJoinWork];
  __shared__ int32_t wl_poly[kJoinWork];
  __shared__ uint32_t wl_n;
  const int lane = threadIdx.x & 63;
  const uint32_t cnt = a.queue_count[blockIdx.x];
  const size_t base = (size_t)blockIdx.x * a.seg_cap;
  uint32_t bsum = 0;
  for (uint32_t i0 = 0; i0 < cnt; i0 += kBlock) {  // block-uniform
    const uint32_t i = i0 + threadIdx.x;
    const bool valid = i < cnt;
    const size_t pos = base + i;
    if (threadIdx.x == 0) wl_n = 0u;
    slow[threadIdx.x] = 0;
    __syncthreads();
    uint32_t n = 0;  // pairs found without the exact distance
    bool over = false;
    double px = 0.0, py = 0.0;
    if (valid) {
      px = a.queue_xy[2 * pos];
      py = a.queue_xy[2 * pos + 1];
      pxy[threadIdx.x] = make_double2(px, py);
      const bool finite = px == px && py == py;
      const int32_t cx = cell_index(px, a.minX, a.cl), cy = cell_index(py, a.minY, a.cl);
      int32_t lb = 0, le = a.npoly;
      const bool list = a.cand_off && cx >= 0 && cy >= 0 && cx < a.grid_n && cy < a.grid_n;
      if (list) {
        const int32_t cell = cy * a.grid_n + cx;
        lb = a.cand_off[cell];
        le = a.cand_off[cell + 1];
      }
      for (int32_t t = lb; t < le; t += 4) {
        int32_t q[4];
        int4 br[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = t + u < le ? (list ? a.cand_list[t + u] : t + u) : -1;
#pragma unroll
        for (int u = 0; u < 4; ++u) br[u] = reinterpret_cast<const int4*>(a.brect)[q[u] < 0 ? 0 : q[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (q[u] < 0) continue;
          const int4 b = br[u];
          bool key = a.g_layers == 0 && cx >= b.x && cx <= b.y && cy >= b.z && cy <= b.w;
          const int64_t c = a.c_layers;
          key = key || (c > 0 && cx >= 0 && cy >= 0 && cx < a.grid_n && cy < a.grid_n &&
                        (int64_t)cx >= (int64_t)b.x - c && (int64_t)cx <= (int64_t)b.y + c &&
                        (int64_t)cy >= (int64_t)b.z - c && (int64_t)cy <= (int64_t)b.w + c);
          if (!key) continue;
          bool hit = a.approx != 0;
          if (!hit) {
            const double* bb = a.bbox + 4 * q[u];
            if (finite && env_far(bb, px, py, a.r)) continue;
            // rectangle shell: inside the closed box <=> distance 0 (<= r: keys exist only for r > 0)
            hit = a.rect && a.rect[q[u]] && env_holds(bb, px, py);
          }
          if (hit) {
            if (n < (uint32_t)kJoinKeep) o.ecand[pos * kJoinKeep + n] = (uint32_t)q[u];
            ++n;
          } else {
            const uint32_t w = atomicAdd(&wl_n, 1u);
            if (w < (uint32_t)kJoinWork) { wl_slot[w] = (uint16_t)threadIdx.x; wl_poly[w] = q[u]; }
            else over = true;
          }
        }
      }
    }
    pcnt[threadIdx.x] = n;
    if (over) slow[threadIdx.x] = 1;
    __syncthreads();
    const uint32_t nw = wl_n < (uint32_t)kJoinWork ? wl_n : (uint32_t)kJoinWork;
    for (uint32_t w = threadIdx.x; w < nw; w += kBlock) {  // phase B: dense exact distances
      const uint32_t sl = wl_slot[w];
      if (slow[sl]) continue;
      const double2 v = pxy[sl];
      const int32_t q = wl_poly[w];
      if (point_polygon_distance(v.x, v.y, a, q) <= a.r) {
        const uint32_t rk = atomicAdd(&pcnt[sl], 1u);
        if (rk < (uint32_t)kJoinKeep) o.ecand[(base + i0 + sl) * kJoinKeep + rk] = (uint32_t)q;
      }
    }
    __syncthreads();
    uint32_t total = pcnt[threadIdx.x];
    if (over)  // worklist overflow: this point's own full walk
      total = join_ppoly_walk(a, px, py, [&](uint32_t k, int32_t q) {
        if (k < (uint32_t)kJoinKeep) o.ecand[pos * kJoinKeep + k] = (uint32_t)q;
      });
    if (valid) {
      o.ecnt[pos] = total;
      bsum += total;
    }
    __syncthreads();  // pcnt / slow / worklist reused by the next round
  }
  for (int off = 32; off > 0; off >>= 1) bsum += __shfl_down(bsum, off, 64);
  if (lane == 0) ws[threadIdx.x >> 6] = bsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) t += ws[w];
    o.btot[blockIdx.x] = t;
  }
}

hipError_t launch_join_ppoly(gf_ctx* ctx, const RangeArgs& a, int blocks, int jblocks, uint32_t* ecnt, uint32_t* ecand,
                             uint32_t* btot, unsigned long long* total, uint32_t* pairs, int64_t cap, int aligned) {
  const size_t lds = 4 * kRangeHdrWords + sizeof(uint32_t) * (size_t)((2 * a.grid_n + 1) & ~1) +
                     (a.xt ? 2 * sizeof(double) * (size_t)(a.grid_n + 1) : 0) +
                     (a.span_lds ? (size_t)((a.span_bytes + 3) & ~3) : 0);
  {
    KTimer t(ctx, GF_K_RANGE_SCAN);
    hipLaunchKernelGGL((range_kernel<1, 1, 2, kRangeU>), dim3(blocks), dim3(kBlock), lds, ctx->stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  KTimer t(ctx, GF_K_RANGE_TEST);
  JoinPolyOut o{ecnt, ecand, btot, total, pairs, cap, aligned};
  (void)jblocks;  // one block per scan block's queue segment
  hipLaunchKernelGGL(join_ppoly_count_kernel, dim3(blocks), dim3(kBlock), 0, ctx->stream, a, o);
  hipLaunchKernelGGL(join_ppoly_write_kernel, dim3(blocks), dim3(kBlock), 0, ctx->stream, a, o);
  return hipGetLastError();
}

hipError_t launch_range(gf_ctx* ctx, const RangeArgs& a, int table_mode, int poly, int blocks) {
  const dim3 g(blocks), b(kBlock);
  const bool defer = a.queue != nullptr;
  const size_t lds = 4 * kRangeHdrWords + (table_mode ? sizeof(uint32_t) * (size_t)((2 * a.grid_n + 1) & ~1) +
                                           (a.xt ? 2 * sizeof(double) * (size_t)(a.grid_n + 1) : 0) +
                                           (a.span_lds ? (size_t)((a.span_bytes + 3) & ~3) : 0)
                                     : 0) +
                     (a.span_mode ? 16 + (size_t)(kBlock / 64) * (kWaveQ * (16 + 4) + 8 + 16 * kWaveRing) : 0);
  {
    KTimer t(ctx, GF_K_RANGE_SCAN);
    if (!table_mode && !poly) hipLaunchKernelGGL((range_kernel<0, 0, 0, kRangeU>), g, b, lds, ctx->stream, a);
    else if (!poly) {
      if (defer && a.span_mode) hipLaunchKernelGGL((range_kernel<1, 0, 3, kRangeU>), g, b, lds, ctx->stream, a);
      else if (defer) hipLaunchKernelGGL((range_kernel<1, 0, 1, kRangeU>), g, b, lds, ctx->stream, a);
      else hipLaunchKernelGGL((range_kernel<1, 0, 0, kRangeU>), g, b, lds, ctx->stream, a);
    } else {
      if (defer && a.span_mode) hipLaunchKernelGGL((range_kernel<1, 1, 3, kRangeU>), g, b, lds, ctx->stream, a);
      else if (defer) hipLaunchKernelGGL((range_kernel<1, 1, 1, kRangeU>), g, b, lds, ctx->stream, a);
      else hipLaunchKernelGGL((range_kernel<1, 1, 0, kRangeU>), g, b, lds, ctx->stream, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;  // deferred tests: drained by each scan block at its end (drain_own_queue)
}

hipError_t launch_range_batch(gf_ctx* ctx, const RangeArgs& a, const RangeBatch& b, int nwin, int table_mode, int poly,
                              int blocks) {
  const dim3 g(blocks, nwin), t(kBlock);
  const size_t lds = 4 * kRangeHdrWords + (table_mode ? sizeof(uint32_t) * (size_t)((2 * a.grid_n + 1) & ~1) +
                                           (a.xt ? 2 * sizeof(double) * (size_t)(a.grid_n + 1) : 0) +
                                           (a.span_lds ? (size_t)((a.span_bytes + 3) & ~3) : 0)
                                     : 0);
  KTimer k(ctx, GF_K_RANGE_SCAN);
  if (!table_mode && !poly) hipLaunchKernelGGL((range_batch_kernel<0, 0, kRangeU>), g, t, lds, ctx->stream, a, b);
  else if (!poly) hipLaunchKernelGGL((range_batch_kernel<1, 0, kRangeU>), g, t, lds, ctx->stream, a, b);
  else hipLaunchKernelGGL((range_batch_kernel<1, 1, kRangeU>), g, t, lds, ctx->stream, a, b);
  return hipGetLastError();
}

}  // namespace gf
