// kernels.hip — gfx950 (CDNA4) kernels of the Pinot segment query executor.
//
// K1 unpack      : FixedBitSVForwardIndexReaderV2.readDictIds / PinotDataBitSet.readInt
//                  (seglocal/segment/index/readers/forward/FixedBitSVForwardIndexReaderV2.java:62-96,
//                   seglocal/io/util/PinotDataBitSet.java:78-136).
// K2+K3 fused    : SVScanDocIdIterator + predicate evaluators (core/operator/dociditerators/SVScanDocIdIterator.java:56-138,
//                  RangePredicateEvaluatorFactory.java:109-193, InPredicateEvaluatorFactory.java:133-173),
//                  AndDocIdIterator/OrDocIdIterator, DictionaryBasedGroupKeyGenerator key math (:259-323),
//                  Sum/Count/Min/Max/Avg aggregateGroupBySV, GroupByCombineOperator merge.
// The path is HBM-bound integer work: no MFMA.  A lane owns 32 consecutive docs, i.e. exactly `bits` u32 words
// of a column (the read32 unit of FixedBitIntReader), decodes them with compile-time shifts (one template
// instance per bit width, selected by a wave-uniform switch) and folds the predicate into a 32-bit match mask.
// Matched docs are gathered (two-word loads; only the 128-B lines that hold matches are touched) and aggregated
// into an LDS-privatised dense group table (small key spaces), a global dense table (large) or a global open
// addressing hash table (huge/overflowing key spaces).
#include <hip/hip_runtime.h>

#include "internal.h"

namespace pgpu {

#define PGPU_HIP_OK(x) ((x) == hipSuccess ? 0 : -1)

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Value of doc `doc` in a packed column (PinotDataBitSet.readInt semantics).  The two-word window never leaves
// the allocation thanks to the padding words.
__device__ __forceinline__ uint32_t gather_id(const uint32_t* __restrict__ fwd, int bits, int64_t doc) {
  const uint64_t bit = (uint64_t)doc * (uint64_t)bits;
  const uint64_t wi = bit >> 5;
  const uint32_t sh = (uint32_t)(bit & 31);
  const uint64_t two = ((uint64_t)bswap32(fwd[wi]) << 32) | (uint64_t)bswap32(fwd[wi + 1]);
  return (uint32_t)(two >> (64 - sh - bits)) & ((1u << bits) - 1u);
}

// ---------------------------------------------------------------------------------------------- K1 unpack
__global__ void unpack_kernel(const uint32_t* __restrict__ fwd, int32_t bits, int64_t start, int64_t n,
                              int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)gather_id(fwd, bits, start + i);
}

__global__ void gather_ids_kernel(const uint32_t* __restrict__ fwd, int32_t bits, const int32_t* __restrict__ docs,
                                  int32_t n, int32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)gather_id(fwd, bits, docs[i]);
}

// ---------------------------------------------------------------------------------------------- K2 leaf masks
// 32-doc group `words` (B big-endian u32 words) -> bit i set iff doc i matches the leaf.
template <int B>
__device__ __forceinline__ uint32_t leaf_mask_b(const uint32_t* __restrict__ words, const KLeaf& L) {
  uint32_t w[B + 1];
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = bswap32(words[k]);
  w[B] = 0;
  constexpr uint32_t vmask = (1u << B) - 1u;
  uint32_t m = 0;
  if (L.kind == LEAF_RANGE) {
    const uint32_t lo = L.lo, span = L.span;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int bit = i * B, wi = bit >> 5, sh = bit & 31;
      uint32_t v;
      if (sh + B <= 32) v = (w[wi] >> (32 - sh - B)) & vmask;
      else v = ((w[wi] << (sh + B - 32)) | (w[wi + 1] >> (64 - sh - B))) & vmask;
      m |= (uint32_t)((v - lo) < span) << i;
    }
  } else {
    const uint32_t* __restrict__ set = L.set;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int bit = i * B, wi = bit >> 5, sh = bit & 31;
      uint32_t v;
      if (sh + B <= 32) v = (w[wi] >> (32 - sh - B)) & vmask;
      else v = ((w[wi] << (sh + B - 32)) | (w[wi + 1] >> (64 - sh - B))) & vmask;
      m |= ((set[v >> 5] >> (v & 31)) & 1u) << i;
    }
  }
  return L.negate ? ~m : m;
}

__device__ __noinline__ uint32_t leaf_mask(const KLeaf& L, const KCol& C, int64_t group) {
  if (L.kind == LEAF_ALL) return ~0u;
  if (L.kind == LEAF_NONE) return 0u;
  const uint32_t* words = C.fwd + group * (int64_t)C.bits;
  switch (C.bits) {
#define PGPU_CASE(B) \
  case B:            \
    return leaf_mask_b<B>(words, L);
    PGPU_CASE(1) PGPU_CASE(2) PGPU_CASE(3) PGPU_CASE(4) PGPU_CASE(5) PGPU_CASE(6) PGPU_CASE(7) PGPU_CASE(8)
    PGPU_CASE(9) PGPU_CASE(10) PGPU_CASE(11) PGPU_CASE(12) PGPU_CASE(13) PGPU_CASE(14) PGPU_CASE(15)
    PGPU_CASE(16) PGPU_CASE(17) PGPU_CASE(18) PGPU_CASE(19) PGPU_CASE(20) PGPU_CASE(21) PGPU_CASE(22)
    PGPU_CASE(23) PGPU_CASE(24) PGPU_CASE(25) PGPU_CASE(26) PGPU_CASE(27) PGPU_CASE(28) PGPU_CASE(29)
    PGPU_CASE(30) PGPU_CASE(31)
#undef PGPU_CASE
    default:
      return 0u;
  }
}

// ---------------------------------------------------------------------------------------------- helpers
struct SegView {
  const KSegHdr* hdr;
  const KCol* cols;
  const KLeaf* leaves;
};

__device__ __forceinline__ SegView seg_view(const KParams& p, int seg) {
  const uint8_t* base = p.segs + (int64_t)seg * p.seg_stride;
  SegView v;
  v.hdr = reinterpret_cast<const KSegHdr*>(base);
  v.cols = reinterpret_cast<const KCol*>(base + sizeof(KSegHdr));
  v.leaves = reinterpret_cast<const KLeaf*>(base + sizeof(KSegHdr) + sizeof(KCol) * p.num_cols);
  return v;
}

__device__ __forceinline__ int find_seg(const KParams& p, int64_t tile) {
  int lo = 0, hi = p.num_segs - 1;
  while (lo < hi) {  // last segment whose tile_base <= tile
    const int mid = (lo + hi + 1) >> 1;
    if (seg_view(p, mid).hdr->tile_base <= tile) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ uint64_t slot_init(int kind) {
  if (kind == SLOT_MIN_KEY) return (uint64_t)INT64_MAX;
  if (kind == SLOT_MAX_KEY) return (uint64_t)INT64_MIN;
  return 0ull;
}

// Evaluates the filter program for this lane's 32-doc group.
__device__ __forceinline__ uint32_t eval_filter(const KParams& p, const SegView& S, int64_t group, uint32_t mask,
                                                uint32_t* __restrict__ stack) {
  if (p.num_ops == 0) return mask;
  if (p.pure_and) {
    for (int l = 0; l < p.num_leaves; ++l) {
      if (!__any(mask != 0u)) break;  // wave-uniform early exit: AndDocIdIterator never scans past an empty child
      mask &= leaf_mask(S.leaves[l], S.cols[p.leaf_col[l]], group);
    }
    return mask;
  }
  const int tid = threadIdx.x;
  int sp = 0;
  for (int k = 0; k < p.num_ops; ++k) {
    const int op = p.ops[k] >> 16, arg = p.ops[k] & 0xFFFF;
    if (op == OP_LEAF) {
      stack[sp * kBlock + tid] = leaf_mask(S.leaves[arg], S.cols[p.leaf_col[arg]], group);
      ++sp;
    } else if (op == OP_NOT) {
      stack[(sp - 1) * kBlock + tid] = ~stack[(sp - 1) * kBlock + tid];
    } else {
      uint32_t acc = stack[(sp - arg) * kBlock + tid];
      for (int j = sp - arg + 1; j < sp; ++j) {
        const uint32_t x = stack[j * kBlock + tid];
        acc = (op == OP_AND) ? (acc & x) : (acc | x);
      }
      sp -= arg;
      stack[sp * kBlock + tid] = acc;
      ++sp;
    }
  }
  return mask & stack[tid];
}

__device__ __forceinline__ int64_t hash_slot(unsigned long long* __restrict__ keys, int64_t cap, uint64_t key) {
  uint64_t h = key * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29;
  int64_t s = (int64_t)(h & (uint64_t)(cap - 1));
  for (;;) {
    unsigned long long k = keys[s];
    if (k == key) return s;
    if (k == ~0ull) {
      const unsigned long long prev = atomicCAS(&keys[s], ~0ull, (unsigned long long)key);
      if (prev == ~0ull || prev == key) return s;
    }
    s = (s + 1) & (cap - 1);
  }
}

template <int MODE>
__device__ __forceinline__ void accumulate(uint64_t* __restrict__ base, int64_t idx, int kind, int64_t ikey,
                                           double dval) {
  unsigned long long* u = reinterpret_cast<unsigned long long*>(base + idx);
  long long* s = reinterpret_cast<long long*>(base + idx);
  switch (kind) {
    case SLOT_COUNT: atomicAdd(u, 1ull); break;
    case SLOT_SUM_I64: atomicAdd(u, (unsigned long long)ikey); break;
    case SLOT_SUM_F64: atomicAdd(reinterpret_cast<double*>(base + idx), dval); break;
    case SLOT_MIN_KEY: atomicMin(s, (long long)ikey); break;
    default: atomicMax(s, (long long)ikey); break;
  }
}

// ---------------------------------------------------------------------------------------------- K3 fused
template <int MODE>
__global__ __launch_bounds__(kBlock) void filter_groupby_kernel(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const int tid = threadIdx.x;
  const int64_t G = p.num_keys_total;
  const int64_t table_words = (MODE == MODE_LDS) ? (int64_t)p.num_slots * G : 0;
  uint32_t* stack = reinterpret_cast<uint32_t*>(lds + table_words);

  if (MODE == MODE_LDS) {
    for (int64_t i = tid; i < table_words; i += kBlock) lds[i] = slot_init(p.slot_kind[i / G]);
    __syncthreads();
  }
  uint64_t* tbl = (MODE == MODE_LDS) ? lds : p.table;

  // Contiguous chunk of tiles per workgroup: the segment cursor only moves forward.
  const int64_t T = p.num_tiles;
  const int64_t t0 = (int64_t)blockIdx.x * T / gridDim.x;
  const int64_t t1 = (int64_t)(blockIdx.x + 1) * T / gridDim.x;
  unsigned long long matched = 0;
  if (t0 < t1) {
    int seg = find_seg(p, t0);
    SegView S = seg_view(p, seg);
    for (int64_t t = t0; t < t1; ++t) {
      while (t >= (int64_t)S.hdr->tile_base + S.hdr->num_tiles) S = seg_view(p, ++seg);
      const int nd = S.hdr->num_docs;
      const int64_t group = (t - S.hdr->tile_base) * kBlock + tid;
      const int64_t ngroups = ((int64_t)nd + 31) >> 5;
      const int64_t doc0 = group << 5;
      uint32_t mask = doc0 >= nd ? 0u : (nd - doc0 >= 32 ? ~0u : ((1u << (nd - doc0)) - 1u));
      const int64_t gclamp = group < ngroups ? group : ngroups - 1;
      mask = eval_filter(p, S, gclamp, mask, stack);
      matched += __popc(mask);
      while (mask) {
        const int i = __ffs(mask) - 1;
        mask &= mask - 1u;
        const int64_t doc = doc0 + i;
        int64_t key = 0;
        for (int j = 0; j < p.num_keys; ++j) {
          const KCol& c = S.cols[p.key_col[j]];
          key += (int64_t)c.lut[gather_id(c.fwd, c.bits, doc)] * p.key_stride[j];
        }
        int64_t idx = key;
        if (MODE == MODE_HASH) idx = hash_slot(p.hash_keys, G, (uint64_t)key);
        for (int s = 0; s < p.num_slots; ++s) {
          const int kind = p.slot_kind[s];
          int64_t ikey = 0;
          double dval = 0.0;
          if (kind != SLOT_COUNT) {
            const KCol& c = S.cols[p.slot_col[s]];
            const uint32_t id = gather_id(c.fwd, c.bits, doc);
            if (kind == SLOT_SUM_F64) dval = c.dval[id];
            else ikey = c.dkey[id];
          }
          accumulate<MODE>(tbl, (int64_t)s * G + idx, kind, ikey, dval);
        }
      }
    }
  }
  // numDocsScanned: wave reduce, one atomic per wave.
  for (int off = 32; off > 0; off >>= 1) matched += __shfl_xor(matched, off);
  if ((tid & 63) == 0 && matched) atomicAdd(p.stats, matched);

  if (MODE == MODE_LDS) {
    __syncthreads();
    uint64_t* out = p.slab + (int64_t)blockIdx.x * table_words;
    for (int64_t i = tid; i < table_words; i += kBlock) out[i] = lds[i];
  }
}

// Deterministic fold of the per-workgroup slabs in workgroup order.
struct SlotKinds {
  int32_t k[kMaxSlots];
};
__global__ void reduce_slabs_kernel(const uint64_t* __restrict__ slab, SlotKinds kinds, int64_t num_keys,
                                    int32_t num_slots, int32_t num_blocks, uint64_t* __restrict__ out) {
  const int64_t words = (int64_t)num_slots * num_keys;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
    const int kind = kinds.k[i / num_keys];
    if (kind == SLOT_SUM_F64) {
      double acc = 0.0;
      for (int b = 0; b < num_blocks; ++b) acc += __longlong_as_double((long long)slab[(int64_t)b * words + i]);
      out[i] = (uint64_t)__double_as_longlong(acc);
    } else if (kind == SLOT_MIN_KEY) {
      long long acc = INT64_MAX;
      for (int b = 0; b < num_blocks; ++b) acc = min(acc, (long long)slab[(int64_t)b * words + i]);
      out[i] = (uint64_t)acc;
    } else if (kind == SLOT_MAX_KEY) {
      long long acc = INT64_MIN;
      for (int b = 0; b < num_blocks; ++b) acc = max(acc, (long long)slab[(int64_t)b * words + i]);
      out[i] = (uint64_t)acc;
    } else {
      uint64_t acc = 0;
      for (int b = 0; b < num_blocks; ++b) acc += slab[(int64_t)b * words + i];
      out[i] = acc;
    }
  }
}

__global__ void table_init_kernel(uint64_t* __restrict__ table, SlotKinds kinds, int32_t num_slots, int64_t num_keys,
                                  unsigned long long* __restrict__ hash_keys) {
  const int64_t words = (int64_t)num_slots * num_keys;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
    table[i] = slot_init(kinds.k[i / num_keys]);
    if (hash_keys && i < num_keys) hash_keys[i] = ~0ull;
  }
}

__global__ void compact_kernel(const uint64_t* __restrict__ table, const unsigned long long* __restrict__ hash_keys,
                               int32_t num_slots, int64_t num_keys, unsigned long long* __restrict__ counter,
                               uint64_t* __restrict__ out_keys, uint64_t* __restrict__ out_slots, int64_t cap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < num_keys; i += (int64_t)gridDim.x * blockDim.x) {
    if (table[i] == 0) continue;  // row 0 = COUNT
    const unsigned long long j = atomicAdd(counter, 1ull);
    if ((int64_t)j >= cap) continue;
    out_keys[j] = hash_keys ? (uint64_t)hash_keys[i] : (uint64_t)i;
    for (int s = 0; s < num_slots; ++s) out_slots[(int64_t)s * cap + j] = table[(int64_t)s * num_keys + i];
  }
}

// K2 alone: the FilterOperator's docId bitmap of the plan's first segment, one 32-bit word per lane group.
__global__ __launch_bounds__(kBlock) void filter_bitmap_kernel(const KParams p, uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  uint32_t* stack = reinterpret_cast<uint32_t*>(lds);
  const SegView S = seg_view(p, 0);
  const int nd = S.hdr->num_docs;
  const int64_t ngroups = ((int64_t)nd + 31) >> 5;
  for (int64_t base = (int64_t)blockIdx.x * kBlock; base < ngroups; base += (int64_t)gridDim.x * kBlock) {
    const int64_t group = base + threadIdx.x;
    const int64_t doc0 = group << 5;
    uint32_t mask = doc0 >= nd ? 0u : (nd - doc0 >= 32 ? ~0u : ((1u << (nd - doc0)) - 1u));
    const int64_t gclamp = group < ngroups ? group : ngroups - 1;
    mask = eval_filter(p, S, gclamp, mask, stack);
    if (group < ngroups) out[group] = mask;
  }
}

// ---------------------------------------------------------------------------------------------- generator
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void gen_positions_kernel(int32_t kind, uint64_t seed, int64_t span, const double* __restrict__ cdf,
                                     const int32_t* __restrict__ code_to_pos, int32_t n_codes, int64_t row0,
                                     int32_t num_docs, int32_t* __restrict__ pos_out, uint32_t* __restrict__ presence) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= num_docs) return;
  const uint64_t h = splitmix64(seed ^ (uint64_t)(row0 + i));
  int32_t pos;
  if (kind == 0) {
    pos = (int32_t)(h % (uint64_t)span);
  } else if (kind == 1) {
    const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
    int lo = 0, hi = n_codes - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid] > u) hi = mid;
      else lo = mid + 1;
    }
    pos = code_to_pos[lo];
  } else {
    pos = code_to_pos[(int32_t)(h % (uint64_t)n_codes)];
  }
  pos_out[i] = pos;
  atomicOr(&presence[pos >> 5], 1u << (pos & 31));
}

__global__ void gen_pack_kernel(const int32_t* __restrict__ pos, const int32_t* __restrict__ pos_to_id,
                                int32_t num_docs, int32_t bits, uint32_t* __restrict__ fwd) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t ngroups = ((int64_t)num_docs + 31) >> 5;
  if (g >= ngroups) return;
  uint64_t buf = 0;
  int nbits = 0, k = 0;
  for (int i = 0; i < 32; ++i) {
    const int64_t d = g * 32 + i;
    const uint32_t id = d < num_docs ? (uint32_t)pos_to_id[pos[d]] : 0u;
    buf = (buf << bits) | id;
    nbits += bits;
    if (nbits >= 32) {
      nbits -= 32;
      fwd[g * bits + k++] = bswap32((uint32_t)(buf >> nbits));
      buf &= (nbits ? ((1ull << nbits) - 1ull) : 0ull);
    }
  }
}

// ---------------------------------------------------------------------------------------------- launchers
static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

int launch_unpack(const uint32_t* fwd, int32_t bits, int64_t start, int64_t n, int32_t* out, void* stream) {
  if (n <= 0) return 0;
  const int64_t grid = (n + 255) / 256;
  hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), fwd, bits, start, n, out);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_gather_ids(const uint32_t* fwd, int32_t bits, const int32_t* docs, int32_t n, int32_t* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gather_ids_kernel, dim3((n + 255) / 256), dim3(256), 0, S(stream), fwd, bits, docs, n, out);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_table_init(uint64_t* table, const int32_t* slot_kind, int32_t num_slots, int64_t num_keys,
                      unsigned long long* hash_keys, void* stream) {
  SlotKinds k{};
  for (int i = 0; i < num_slots && i < kMaxSlots; ++i) k.k[i] = slot_kind[i];
  const int64_t words = (int64_t)num_slots * num_keys;
  int64_t grid = (words + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(table_init_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), table, k, num_slots, num_keys,
                     hash_keys);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_filter_groupby(const KParams& p, int mode, int grid, size_t lds_bytes, void* stream) {
  switch (mode) {
    case MODE_LDS:
      hipLaunchKernelGGL(filter_groupby_kernel<MODE_LDS>, dim3(grid), dim3(kBlock), lds_bytes, S(stream), p);
      break;
    case MODE_GLOBAL:
      hipLaunchKernelGGL(filter_groupby_kernel<MODE_GLOBAL>, dim3(grid), dim3(kBlock), lds_bytes, S(stream), p);
      break;
    default:
      hipLaunchKernelGGL(filter_groupby_kernel<MODE_HASH>, dim3(grid), dim3(kBlock), lds_bytes, S(stream), p);
      break;
  }
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_reduce_slabs(const uint64_t* slab, const int32_t* slot_kind, int32_t num_slots, int64_t num_keys,
                        int32_t num_blocks, uint64_t* out, void* stream) {
  SlotKinds k{};
  for (int i = 0; i < num_slots && i < kMaxSlots; ++i) k.k[i] = slot_kind[i];
  const int64_t words = (int64_t)num_slots * num_keys;
  int64_t grid = (words + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), slab, k, num_keys, num_slots,
                     num_blocks, out);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_compact(const uint64_t* table, const unsigned long long* hash_keys, int32_t num_slots, int64_t num_keys,
                   unsigned long long* counter, uint64_t* out_keys, uint64_t* out_slots, int64_t out_cap,
                   void* stream) {
  int64_t grid = (num_keys + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(compact_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), table, hash_keys, num_slots,
                     num_keys, counter, out_keys, out_slots, out_cap);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_filter_bitmap(const KParams& p, uint32_t* out_words, void* stream) {
  const KParams q = p;
  int64_t grid = 1;
  // The number of groups is only known on the device; the host passes num_tiles = ceil(groups / 256).
  grid = q.num_tiles > 0 ? q.num_tiles : 1;
  if (grid > 4096) grid = 4096;
  const size_t lds = (size_t)kMaxStack * kBlock * sizeof(uint32_t);
  hipLaunchKernelGGL(filter_bitmap_kernel, dim3((unsigned)grid), dim3(kBlock), lds, S(stream), q, out_words);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_gen_positions(int32_t kind, uint64_t seed, int64_t lo, int64_t span, const double* cdf,
                         const int32_t* code_to_pos, int32_t n_codes, int64_t row0, int32_t num_docs,
                         int32_t* pos_out, uint32_t* presence, void* stream) {
  (void)lo;
  if (num_docs <= 0) return 0;
  hipLaunchKernelGGL(gen_positions_kernel, dim3((num_docs + 255) / 256), dim3(256), 0, S(stream), kind, seed, span,
                     cdf, code_to_pos, n_codes, row0, num_docs, pos_out, presence);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_gen_pack(const int32_t* pos, const int32_t* pos_to_id, int32_t num_docs, int32_t bits, uint32_t* fwd_out,
                    void* stream) {
  const int64_t ngroups = ((int64_t)num_docs + 31) >> 5;
  if (ngroups <= 0) return 0;
  hipLaunchKernelGGL(gen_pack_kernel, dim3((unsigned)((ngroups + 255) / 256)), dim3(256), 0, S(stream), pos,
                     pos_to_id, num_docs, bits, fwd_out);
  return PGPU_HIP_OK(hipGetLastError());
}

}  // namespace pgpu
