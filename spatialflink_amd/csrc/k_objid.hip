// k_objid.hip -- the objID dictionary: the reference's objID is a String (Point.objID,
// Deserialization.java:317 `String strOId = ...`), compared with String.equals by the kNN
// merge's objID dedupe (KNNQuery.java:232-251).  The SoA carries an int64 KEY per point that
// must be injective over Strings: canonical decimals are their value (gf_decimal.hpp), every
// other String gets INT64_MIN + its id in a device hash table (open addressing, linear probe,
// load <= 1/2) whose strings live in a device byte arena.
//
// A batch (one CSV chunk, or a host intern call) is a worklist of byte ranges with their batch
// position `line`; ids of the batch's new Strings are assigned in first-occurrence order, so
// the keys never depend on scheduling:
//   dict_probe   (rounds) one lane per pending entry: hash, probe; an empty slot is claimed
//                with one CAS and filled (bytes copied to the arena); a slot with the same tag
//                claimed in THIS round is not compared yet (its bytes may still be in flight):
//                the entry is deferred to the next round, where everything is visible.  New
//                slots keep the smallest batch position that maps to them (atomicMin).
//   dict_mark    flag[line] = 1 for the first occurrence of each new String
//   (scan)       rank = exclusive prefix of the flags
//   dict_assign  id = dictionary size + rank; idmap[id] = the slot's arena (offset, length)
//   dict_keys    key[line] = INT64_MIN + id of the line's slot
#define GF_TU_NAME k_objid_hip
#include "gf_buildtag.hpp"  // first: records this unit's command-line defines

#include "gf_internal.hpp"

namespace gf {

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// FNV-1a over the String's bytes ('"' skipped when `quotes`: the reference's
// str.replace("\"", "") runs before the split), finalised; *len = the String's length.
__device__ __forceinline__ uint64_t dict_hash(const char* src, int64_t b, int32_t n, int quotes, uint32_t* len) {
  uint64_t h = 1469598103934665603ull;
  uint32_t m = 0;
  for (int32_t i = 0; i < n; ++i) {
    const char c = src[b + i];
    if (quotes && c == '"') continue;
    h = (h ^ (uint8_t)c) * 1099511628211ull;
    ++m;
  }
  *len = m;
  return fmix64(h ^ ((uint64_t)m << 40));
}

__device__ __forceinline__ bool dict_equal(const char* arena, uint64_t meta, const char* src, int64_t b, int32_t n,
                                           int quotes, uint32_t len) {
  if ((uint32_t)(meta & kDictLenMask) != len) return false;
  const char* p = arena + (meta >> kDictLenBits);
  uint32_t k = 0;
  for (int32_t i = 0; i < n; ++i) {
    const char c = src[b + i];
    if (quotes && c == '"') continue;
    if (p[k++] != c) return false;
  }
  return true;
}

__device__ __forceinline__ void wave_append(bool c, const DictWork& w, DictWork* out, uint32_t* count) {
  const uint64_t m = __ballot(c);
  if (!m) return;
  const int lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(count, (uint32_t)__popcll(m));
  base = __shfl(base, 0, 64);
  if (c) out[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = w;
}

__global__ __launch_bounds__(kBlock) void dict_probe_kernel(DictDev d, DictBatch B) {
  const uint32_t stride = gridDim.x * kBlock;
  for (uint32_t w0 = blockIdx.x * kBlock; w0 < B.nwork; w0 += stride) {  // block-uniform
    const uint32_t wi = w0 + threadIdx.x;
    bool defer = false;
    DictWork e{0, 0, 0};
    if (wi < B.nwork) {
      e = B.work[wi];
      uint32_t len;
      const uint64_t h = dict_hash(B.src, e.b, e.n, B.quotes, &len);
      const unsigned long long tag = h | 1ull;
      uint64_t pos = (h >> 24) & d.mask;
      for (;;) {
        DictSlot* s = d.slots + pos;
        unsigned long long t = __hip_atomic_load(&s->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == 0ull) {
          t = atomicCAS(&s->tag, 0ull, tag);
          if (t == 0ull) {  // claimed: copy the String to the arena, fill the slot
            const unsigned long long off = atomicAdd(d.arena_used, (unsigned long long)len);
            char* p = d.arena + off;
            uint32_t k = 0;
            for (int32_t i = 0; i < e.n; ++i) {
              const char c = B.src[e.b + i];
              if (!(B.quotes && c == '"')) p[k++] = c;
            }
            s->meta = (off << kDictLenBits) | len;
            s->id = -1;
            s->first = e.line;
            __hip_atomic_store(&s->round, B.round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            B.slot_of[e.line] = (uint32_t)pos;
            break;
          }
        }
        if (t == tag) {
          const uint32_t r = __hip_atomic_load(&s->round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (r == 0u || r == B.round) {  // claimed in this round: compare next round
            defer = true;
            break;
          }
          if (dict_equal(d.arena, s->meta, B.src, e.b, e.n, B.quotes, len)) {
            if (r >= B.round0) atomicMin(&s->first, e.line);  // a String new in this batch
            B.slot_of[e.line] = (uint32_t)pos;
            break;
          }
        }
        pos = (pos + 1) & d.mask;
      }
    }
    wave_append(defer, e, B.pend_out, B.npend_out);
  }
}

__global__ __launch_bounds__(kBlock) void dict_mark_kernel(DictDev d, DictBatch B) {
  for (uint32_t wi = blockIdx.x * kBlock + threadIdx.x; wi < B.nwork; wi += gridDim.x * kBlock) {
    const uint32_t line = B.work[wi].line;
    const DictSlot& s = d.slots[B.slot_of[line]];
    if (s.round >= B.round0 && s.first == line) B.flag[line] = 1u;
  }
}

__global__ __launch_bounds__(kBlock) void dict_assign_kernel(DictDev d, DictBatch B) {
  for (uint32_t wi = blockIdx.x * kBlock + threadIdx.x; wi < B.nwork; wi += gridDim.x * kBlock) {
    const uint32_t line = B.work[wi].line;
    if (!B.flag[line]) continue;
    DictSlot& s = d.slots[B.slot_of[line]];
    const int64_t id = B.id_base + (int64_t)B.rank[line];
    s.id = id;
    d.idmap[id] = s.meta;
  }
}

__global__ __launch_bounds__(kBlock) void dict_keys_kernel(DictDev d, DictBatch B) {
  for (uint32_t wi = blockIdx.x * kBlock + threadIdx.x; wi < B.nwork; wi += gridDim.x * kBlock) {
    const uint32_t line = B.work[wi].line;
    B.keys[line] = INT64_MIN + d.slots[B.slot_of[line]].id;
  }
}

// re-insert ids [0, n) into a fresh (zeroed) table: every String is distinct, so no compares
__global__ __launch_bounds__(kBlock) void dict_rehash_kernel(DictDev d, int64_t n) {
  for (int64_t id = (int64_t)blockIdx.x * kBlock + threadIdx.x; id < n; id += (int64_t)gridDim.x * kBlock) {
    const uint64_t meta = d.idmap[id];
    uint32_t len;
    const uint64_t h = dict_hash(d.arena, (int64_t)(meta >> kDictLenBits), (int32_t)(meta & kDictLenMask), 0, &len);
    uint64_t pos = (h >> 24) & d.mask;
    while (atomicCAS(&d.slots[pos].tag, 0ull, (unsigned long long)(h | 1ull)) != 0ull) pos = (pos + 1) & d.mask;
    DictSlot& s = d.slots[pos];
    s.meta = meta;
    s.id = id;
    s.first = ~0u;
    s.round = 1u;  // older than every batch (batches start at round 2)
  }
}

static unsigned dict_blocks(uint64_t n) {
  const uint64_t b = (n + kBlock - 1) / kBlock;
  return (unsigned)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

hipError_t launch_dict(hipStream_t st, int stage, const DictDev& d, const DictBatch& B) {
  const unsigned g = dict_blocks(B.nwork);
  switch (stage) {
    case 0: hipLaunchKernelGGL(dict_probe_kernel, dim3(g), dim3(kBlock), 0, st, d, B); break;
    case 1: hipLaunchKernelGGL(dict_mark_kernel, dim3(g), dim3(kBlock), 0, st, d, B); break;
    case 2: hipLaunchKernelGGL(dict_assign_kernel, dim3(g), dim3(kBlock), 0, st, d, B); break;
    default: hipLaunchKernelGGL(dict_keys_kernel, dim3(g), dim3(kBlock), 0, st, d, B); break;
  }
  return hipGetLastError();
}

hipError_t launch_dict_rehash(hipStream_t st, const DictDev& d, int64_t n) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(dict_rehash_kernel, dim3(dict_blocks((uint64_t)n)), dim3(kBlock), 0, st, d, n);
  return hipGetLastError();
}

}  // namespace gf
