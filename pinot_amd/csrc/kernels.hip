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
#include "device.h"

namespace pgpu {

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

// tile -> segment map of a plan (one workgroup per segment record).
__global__ void expand_tiles_kernel(const uint8_t* __restrict__ segs, int32_t seg_stride, int32_t num_segs,
                                    int32_t* __restrict__ tile_seg) {
  for (int s = blockIdx.x; s < num_segs; s += gridDim.x) {
    const KSegHdr* h = reinterpret_cast<const KSegHdr*>(segs + (int64_t)s * seg_stride);
    for (int i = threadIdx.x; i < h->num_tiles; i += blockDim.x) tile_seg[h->tile_base + i] = s;
  }
}

// Deterministic fold of the per-workgroup slabs in workgroup order.
struct SlotKinds {
  int32_t k[kMaxSlots];
};
// Each block folds 8 table words; the 32 lanes of a word take every 32nd slab and their partials are combined
// in lane order, so the result is bitwise reproducible run to run.
__global__ __launch_bounds__(256) void reduce_slabs_kernel(const uint64_t* __restrict__ slab, SlotKinds kinds,
                                                           int64_t num_keys, int32_t num_slots, int32_t num_blocks,
                                                           uint64_t* __restrict__ out) {
  __shared__ uint64_t part[256];
  const int64_t words = (int64_t)num_slots * num_keys;
  const int j = threadIdx.x & 31;
  const int64_t i = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int kind = i < words ? kinds.k[i / num_keys] : SLOT_COUNT;
  uint64_t acc;
  if (kind == SLOT_SUM_F64) {
    double a = 0.0;
    if (i < words)
      for (int b = j; b < num_blocks; b += 32) a += __longlong_as_double((long long)slab[(int64_t)b * words + i]);
    acc = (uint64_t)__double_as_longlong(a);
  } else if (kind == SLOT_MIN_KEY) {
    long long a = INT64_MAX;
    if (i < words)
      for (int b = j; b < num_blocks; b += 32) a = min(a, (long long)slab[(int64_t)b * words + i]);
    acc = (uint64_t)a;
  } else if (kind == SLOT_MAX_KEY) {
    long long a = INT64_MIN;
    if (i < words)
      for (int b = j; b < num_blocks; b += 32) a = max(a, (long long)slab[(int64_t)b * words + i]);
    acc = (uint64_t)a;
  } else {
    uint64_t a = 0;
    if (i < words)
      for (int b = j; b < num_blocks; b += 32) a += slab[(int64_t)b * words + i];
    acc = a;
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  if (j == 0 && i < words) {
    const uint64_t* q = part + threadIdx.x;
    if (kind == SLOT_SUM_F64) {
      double a = 0.0;
      for (int k = 0; k < 32; ++k) a += __longlong_as_double((long long)q[k]);
      out[i] = (uint64_t)__double_as_longlong(a);
    } else if (kind == SLOT_MIN_KEY) {
      long long a = INT64_MAX;
      for (int k = 0; k < 32; ++k) a = min(a, (long long)q[k]);
      out[i] = (uint64_t)a;
    } else if (kind == SLOT_MAX_KEY) {
      long long a = INT64_MIN;
      for (int k = 0; k < 32; ++k) a = max(a, (long long)q[k]);
      out[i] = (uint64_t)a;
    } else {
      uint64_t a = 0;
      for (int k = 0; k < 32; ++k) a += q[k];
      out[i] = a;
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

// Groups with COUNT > 0, entry-major: out[j * (1 + num_slots)] = key, then the slot words.
__global__ void compact_kernel(const uint64_t* __restrict__ table, const unsigned long long* __restrict__ hash_keys,
                               int32_t num_slots, int64_t num_keys, unsigned long long* __restrict__ counter,
                               uint64_t* __restrict__ out, int64_t cap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < num_keys; i += (int64_t)gridDim.x * blockDim.x) {
    if (table[i] == 0) continue;  // row 0 = COUNT
    const unsigned long long j = atomicAdd(counter, 1ull);
    if ((int64_t)j >= cap) continue;
    uint64_t* o = out + (int64_t)j * (1 + num_slots);
    o[0] = hash_keys ? (uint64_t)hash_keys[i] : (uint64_t)i;
    for (int s = 0; s < num_slots; ++s) o[1 + s] = table[(int64_t)s * num_keys + i];
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

// One object per (kernel family, mode): k_direct.hip / k_staged.hip compiled with -DPGPU_MODE=0,1,2.
int launch_direct_mode0(const KParams& p, int grid, size_t lds_bytes, void* stream);
int launch_direct_mode1(const KParams& p, int grid, size_t lds_bytes, void* stream);
int launch_direct_mode2(const KParams& p, int grid, size_t lds_bytes, void* stream);
int launch_staged_mode0(const KParams& p, int grid, size_t lds_bytes, void* stream);
int launch_staged_mode1(const KParams& p, int grid, size_t lds_bytes, void* stream);
int launch_staged_mode2(const KParams& p, int grid, size_t lds_bytes, void* stream);

int launch_startree_scan_mode0(const KStarParams& p, size_t lds_bytes, void* stream);
int launch_startree_scan_mode1(const KStarParams& p, size_t lds_bytes, void* stream);
int launch_startree_scan_mode2(const KStarParams& p, size_t lds_bytes, void* stream);

int launch_startree_scan(const KStarParams& p, int mode, size_t lds_bytes, void* stream) {
  switch (mode) {
    case MODE_LDS: return launch_startree_scan_mode0(p, lds_bytes, stream);
    case MODE_GLOBAL: return launch_startree_scan_mode1(p, lds_bytes, stream);
    default: return launch_startree_scan_mode2(p, lds_bytes, stream);
  }
}

int launch_filter_groupby(const KParams& p, int mode, int grid, size_t lds_bytes, void* stream) {
  switch (mode) {
    case MODE_LDS: return launch_direct_mode0(p, grid, lds_bytes, stream);
    case MODE_GLOBAL: return launch_direct_mode1(p, grid, lds_bytes, stream);
    default: return launch_direct_mode2(p, grid, lds_bytes, stream);
  }
}

int launch_expand_tiles(const uint8_t* segs, int32_t seg_stride, int32_t num_segs, int32_t* tile_seg, void* stream) {
  if (num_segs <= 0) return 0;
  hipLaunchKernelGGL(expand_tiles_kernel, dim3(num_segs < 4096 ? num_segs : 4096), dim3(128), 0, S(stream), segs,
                     seg_stride, num_segs, tile_seg);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_scan(const KParams& p, int mode, int grid, size_t lds_bytes, void* stream) {
  switch (mode) {
    case MODE_LDS: return launch_staged_mode0(p, grid, lds_bytes, stream);
    case MODE_GLOBAL: return launch_staged_mode1(p, grid, lds_bytes, stream);
    default: return launch_staged_mode2(p, grid, lds_bytes, stream);
  }
}

int launch_reduce_slabs(const uint64_t* slab, const int32_t* slot_kind, int32_t num_slots, int64_t num_keys,
                        int32_t num_blocks, uint64_t* out, void* stream) {
  SlotKinds k{};
  for (int i = 0; i < num_slots && i < kMaxSlots; ++i) k.k[i] = slot_kind[i];
  const int64_t words = (int64_t)num_slots * num_keys;
  const int64_t grid = (words + 7) / 8;
  if (grid < 1) return 0;
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), slab, k, num_keys, num_slots,
                     num_blocks, out);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_compact(const uint64_t* table, const unsigned long long* hash_keys, int32_t num_slots, int64_t num_keys,
                   unsigned long long* counter, uint64_t* out, int64_t out_cap, void* stream) {
  int64_t grid = (num_keys + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(compact_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), table, hash_keys, num_slots,
                     num_keys, counter, out, out_cap);
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
