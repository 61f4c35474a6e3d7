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

#include <utility>

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
// A lane's 32-doc group is B big-endian u32 words; doc i occupies bits [i*B, i*B+B) counted from the MSB of word
// 0 (FixedBitIntReader.read32 layout).  Each decoder walks the docs from 31 down to 0 and shifts the predicate
// bit in with v_alignbit (mask = mask << 1 | sign(test)), so doc i lands on bit i without materialising 1 << i.
template <int B, int I>
__device__ __forceinline__ uint32_t extract(const uint32_t (&w)[B + 1]) {
  constexpr int bit = I * B, wi = bit >> 5, sh = bit & 31;
  if constexpr (sh + B <= 32) {
    return __builtin_amdgcn_ubfe(w[wi], 32 - sh - B, B);
  } else {
    return __builtin_amdgcn_alignbit(w[wi], w[wi + 1], 64 - sh - B) & ((1u << B) - 1u);
  }
}

template <int B>
__device__ __forceinline__ void load_group(const uint32_t* __restrict__ words, uint32_t (&w)[B + 1]) {
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = bswap32(words[k]);
  w[B] = 0;
}

// value in [lo, hi): sign bit of (v - hi) & ~(v - lo)   (values, lo, hi < 2^31)
template <int B, int I>
__device__ __forceinline__ uint32_t range_step(const uint32_t (&w)[B + 1], uint32_t lo, uint32_t hi, uint32_t m) {
  const uint32_t v = extract<B, I>(w);
  const uint32_t t = (v - hi) & ~(v - lo);
  return __builtin_amdgcn_alignbit(m, t, 31);
}
// value == eq: sign bit of (v ^ eq) - 1
template <int B, int I>
__device__ __forceinline__ uint32_t eq_step(const uint32_t (&w)[B + 1], uint32_t eq, uint32_t m) {
  const uint32_t v = extract<B, I>(w);
  return __builtin_amdgcn_alignbit(m, (v ^ eq) - 1u, 31);
}

template <int B, int... I>
__device__ __forceinline__ uint32_t range_all(const uint32_t (&w)[B + 1], uint32_t lo, uint32_t hi,
                                              std::integer_sequence<int, I...>) {
  uint32_t m = 0;
  ((m = range_step<B, 31 - I>(w, lo, hi, m)), ...);
  return m;
}
template <int B, int... I>
__device__ __forceinline__ uint32_t eq_all(const uint32_t (&w)[B + 1], uint32_t eq, std::integer_sequence<int, I...>) {
  uint32_t m = 0;
  ((m = eq_step<B, 31 - I>(w, eq, m)), ...);
  return m;
}

template <int B>
__device__ __forceinline__ uint32_t leaf_range_b(const uint32_t* __restrict__ words, uint32_t lo, uint32_t span) {
  uint32_t w[B + 1];
  load_group<B>(words, w);
  if (span == 1) return eq_all<B>(w, lo, std::make_integer_sequence<int, 32>{});
  return range_all<B>(w, lo, lo + span, std::make_integer_sequence<int, 32>{});
}

template <int B>
__device__ __forceinline__ uint32_t leaf_set_b(const uint32_t* __restrict__ words, const uint32_t* __restrict__ set) {
  uint32_t w[B + 1];
  load_group<B>(words, w);
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int bit = i * B, wi = bit >> 5, sh = bit & 31;
    uint32_t v;
    if (sh + B <= 32) v = (w[wi] >> (32 - sh - B)) & ((1u << B) - 1u);
    else v = ((w[wi] << (sh + B - 32)) | (w[wi + 1] >> (64 - sh - B))) & ((1u << B) - 1u);
    m |= ((set[v >> 5] >> (v & 31)) & 1u) << i;
  }
  return m;
}

// Wave-uniform dispatch on (kind, bits) to the decoder instance; `words` = this lane's 32-doc group (global
// memory or an LDS stage buffer).
__device__ __forceinline__ uint32_t leaf_eval_words(int kind, int negate, uint32_t lo, uint32_t span,
                                                    const uint32_t* set, const uint32_t* words, int bits) {
  if (kind == LEAF_ALL) return ~0u;
  if (kind == LEAF_NONE) return 0u;
  uint32_t m = 0;
  if (kind == LEAF_RANGE) {
    switch (bits) {
#define PGPU_CASE(B) \
  case B:            \
    m = leaf_range_b<B>(words, lo, span); \
    break;
      PGPU_CASE(1) PGPU_CASE(2) PGPU_CASE(3) PGPU_CASE(4) PGPU_CASE(5) PGPU_CASE(6) PGPU_CASE(7) PGPU_CASE(8)
      PGPU_CASE(9) PGPU_CASE(10) PGPU_CASE(11) PGPU_CASE(12) PGPU_CASE(13) PGPU_CASE(14) PGPU_CASE(15)
      PGPU_CASE(16) PGPU_CASE(17) PGPU_CASE(18) PGPU_CASE(19) PGPU_CASE(20) PGPU_CASE(21) PGPU_CASE(22)
      PGPU_CASE(23) PGPU_CASE(24) PGPU_CASE(25) PGPU_CASE(26) PGPU_CASE(27) PGPU_CASE(28) PGPU_CASE(29)
      PGPU_CASE(30) PGPU_CASE(31)
#undef PGPU_CASE
      default: break;
    }
  } else {
    switch (bits) {
#define PGPU_CASE(B) \
  case B:            \
    m = leaf_set_b<B>(words, set); \
    break;
      PGPU_CASE(1) PGPU_CASE(2) PGPU_CASE(3) PGPU_CASE(4) PGPU_CASE(5) PGPU_CASE(6) PGPU_CASE(7) PGPU_CASE(8)
      PGPU_CASE(9) PGPU_CASE(10) PGPU_CASE(11) PGPU_CASE(12) PGPU_CASE(13) PGPU_CASE(14) PGPU_CASE(15)
      PGPU_CASE(16) PGPU_CASE(17) PGPU_CASE(18) PGPU_CASE(19) PGPU_CASE(20) PGPU_CASE(21) PGPU_CASE(22)
      PGPU_CASE(23) PGPU_CASE(24) PGPU_CASE(25) PGPU_CASE(26) PGPU_CASE(27) PGPU_CASE(28) PGPU_CASE(29)
      PGPU_CASE(30) PGPU_CASE(31)
#undef PGPU_CASE
      default: break;
    }
  }
  return negate ? ~m : m;
}

__device__ __forceinline__ uint32_t leaf_eval(int kind, int negate, uint32_t lo, uint32_t span, const uint32_t* set,
                                              const uint32_t* fwd, int bits, int64_t group) {
  return leaf_eval_words(kind, negate, lo, span, set, fwd + group * (int64_t)bits, bits);
}

__device__ __forceinline__ uint32_t leaf_mask(const KLeaf& L, const KCol& C, int64_t group) {
  return leaf_eval(L.kind, L.negate, L.lo, L.span, L.set, C.fwd, C.bits, group);
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

__device__ __forceinline__ uint64_t slot_init(int kind) {
  if (kind == SLOT_MIN_KEY) return (uint64_t)INT64_MAX;
  if (kind == SLOT_MAX_KEY) return (uint64_t)INT64_MIN;
  return 0ull;
}

// Leaf descriptors of the current segment held in registers (reloaded only when the segment changes).
constexpr int kFastLeaves = 4;
struct LeafReg {
  const uint32_t* fwd;
  const uint32_t* set;
  int32_t bits, kind, negate;
  uint32_t lo, span;
};

__device__ __forceinline__ uint32_t leaf_mask_reg(const LeafReg& R, int64_t group) {
  return leaf_eval(R.kind, R.negate, R.lo, R.span, R.set, R.fwd, R.bits, group);
}

__device__ __forceinline__ LeafReg load_leaf_reg(const KParams& p, const SegView& S, int l) {
  LeafReg r;
  const KLeaf& L = S.leaves[l];
  const KCol& C = S.cols[p.leaf_col[l]];
  r.fwd = C.fwd;
  r.bits = C.bits;
  r.kind = L.kind;
  r.negate = L.negate;
  r.lo = L.lo;
  r.span = L.span;
  r.set = L.set;
  return r;
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
#ifndef PGPU_MIN_WAVES
#define PGPU_MIN_WAVES 1
#endif
__global__ __launch_bounds__(kBlock, PGPU_MIN_WAVES) void filter_groupby_kernel(const KParams p) {
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

  // Each workgroup streams a contiguous range of tiles; the segment cursor only moves forward and the leaf
  // descriptors stay in registers until the segment changes (no per-tile dependent descriptor loads).
  unsigned long long matched = 0;
  const int64_t T = p.num_tiles;
  const int64_t t0 = (int64_t)blockIdx.x * T / gridDim.x;
  const int64_t t1 = (int64_t)(blockIdx.x + 1) * T / gridDim.x;
  const bool fast = p.pure_and && p.num_leaves <= kFastLeaves;
  if (t0 < t1) {
    int seg = p.tile_seg[t0];
    SegView S = seg_view(p, seg);
    int64_t tile_base = S.hdr->tile_base, tile_end = tile_base + S.hdr->num_tiles;
    int nd = S.hdr->num_docs;
    // named registers, not an array: a runtime-guarded array of structs lands in scratch
    LeafReg R0{}, R1{}, R2{}, R3{};
    const int nl = p.num_leaves;
#define PGPU_LOAD_LEAVES()                      \
  do {                                          \
    if (nl > 0) R0 = load_leaf_reg(p, S, 0);    \
    if (nl > 1) R1 = load_leaf_reg(p, S, 1);    \
    if (nl > 2) R2 = load_leaf_reg(p, S, 2);    \
    if (nl > 3) R3 = load_leaf_reg(p, S, 3);    \
  } while (0)
    if (fast) PGPU_LOAD_LEAVES();
    for (int64_t t = t0; t < t1; ++t) {
      if (t >= tile_end) {
        S = seg_view(p, ++seg);
        tile_base = S.hdr->tile_base;
        tile_end = tile_base + S.hdr->num_tiles;
        nd = S.hdr->num_docs;
        if (fast) PGPU_LOAD_LEAVES();
      }
      const int64_t group = (t - tile_base) * kBlock + tid;
      const int64_t ngroups = ((int64_t)nd + 31) >> 5;
      const int64_t doc0 = group << 5;
      uint32_t mask = doc0 >= nd ? 0u : (nd - doc0 >= 32 ? ~0u : ((1u << (nd - doc0)) - 1u));
      const int64_t gclamp = group < ngroups ? group : ngroups - 1;
      if (fast) {
        for (int l = 0; l < nl; ++l) {
          if (!__any(mask != 0u)) break;  // AndDocIdIterator never scans past an empty child
          const LeafReg& r = l == 0 ? R0 : l == 1 ? R1 : l == 2 ? R2 : R3;
          mask &= leaf_mask_reg(r, gclamp);
        }
      } else {
        mask = eval_filter(p, S, gclamp, mask, stack);
      }
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

// ---------------------------------------------------------------------------------------------- K3 staged
// The scan kernel of the path.  Per 8192-doc tile, the filter columns' packed words are copied HBM -> LDS with
// global_load_lds_dwordx4 (1 KB per wave instruction, no VGPR staging) one tile ahead of the decode, so the
// bytes in flight do not depend on register occupancy.  Lanes decode their 32-doc groups from LDS.  Matched
// docs are appended to an LDS queue and aggregated in batches (the sparse gathers of group-by / metric columns
// then overlap the next tile's copy instead of stalling every tile); a tile with more matches than the queue
// holds is aggregated in place.
//
// LDS: [group table (MODE_LDS)] [filter stack (general programs)] [4 wave totals] [queue] [2 stage buffers]

// Uniform (scalar) copies of the current segment's scan descriptors.  Loaded with ordinary loads only when the
// segment changes and made wave-uniform with readfirstlane, so the steady-state tile loop issues no vector
// load besides the LDS-DMA (a vector load's s_waitcnt would also drain the in-flight prefetch).
__device__ __forceinline__ uint32_t ufl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
template <class T>
__device__ __forceinline__ const T* ufl_ptr(const T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  return reinterpret_cast<const T*>(((uint64_t)ufl((uint32_t)(v >> 32)) << 32) | ufl((uint32_t)v));
}

struct StageRegs {
  int32_t num_docs, tile_base, num_tiles;
  const uint32_t *f0, *f1, *f2, *f3;   // staged columns' forward indexes
  int32_t b0, b1, b2, b3;              // their bit widths
  int32_t o1, o2, o3;                  // their word offsets inside a stage buffer (o0 = 0)
};
struct LeafRegs {
  int32_t kind, negate;
  uint32_t lo, span;
  const uint32_t* set;
};

__device__ __forceinline__ StageRegs load_stage_regs(const KParams& p, int seg) {
  const SegView S = seg_view(p, seg);
  StageRegs r;
  r.num_docs = (int32_t)ufl((uint32_t)S.hdr->num_docs);
  r.tile_base = (int32_t)ufl((uint32_t)S.hdr->tile_base);
  r.num_tiles = (int32_t)ufl((uint32_t)S.hdr->num_tiles);
  r.f0 = r.f1 = r.f2 = r.f3 = nullptr;
  r.b0 = r.b1 = r.b2 = r.b3 = 0;
  const int ns = p.num_stage;
  if (ns > 0) { r.f0 = ufl_ptr(S.cols[p.stage_col[0]].fwd); r.b0 = (int32_t)ufl((uint32_t)S.cols[p.stage_col[0]].bits); }
  if (ns > 1) { r.f1 = ufl_ptr(S.cols[p.stage_col[1]].fwd); r.b1 = (int32_t)ufl((uint32_t)S.cols[p.stage_col[1]].bits); }
  if (ns > 2) { r.f2 = ufl_ptr(S.cols[p.stage_col[2]].fwd); r.b2 = (int32_t)ufl((uint32_t)S.cols[p.stage_col[2]].bits); }
  if (ns > 3) { r.f3 = ufl_ptr(S.cols[p.stage_col[3]].fwd); r.b3 = (int32_t)ufl((uint32_t)S.cols[p.stage_col[3]].bits); }
  r.o1 = kBlock * r.b0;
  r.o2 = r.o1 + kBlock * r.b1;
  r.o3 = r.o2 + kBlock * r.b2;
  return r;
}

__device__ __forceinline__ LeafRegs load_leaf_regs(const KParams& p, int seg, int l) {
  const KLeaf& L = seg_view(p, seg).leaves[l];
  LeafRegs r;
  r.kind = (int32_t)ufl((uint32_t)L.kind);
  r.negate = (int32_t)ufl((uint32_t)L.negate);
  r.lo = ufl(L.lo);
  r.span = ufl(L.span);
  r.set = ufl_ptr(L.set);
  return r;
}

__device__ __forceinline__ void issue_column(const uint32_t* fwd, int b, int off, int64_t tile_in_seg, uint32_t* buf,
                                             int& k, int wave, int lane) {
  const uint32_t* src = fwd + tile_in_seg * (int64_t)(kBlock * b);
  for (int j = 0; j < b; ++j, ++k) {
    if ((k & 3) == wave)
      __builtin_amdgcn_global_load_lds(src + j * 256 + lane * 4,
                                       (__attribute__((address_space(3))) void*)(buf + off + j * 256), 16, 0, 0);
  }
}

__device__ __forceinline__ void issue_tile(const KParams& p, const StageRegs& R, int64_t tile_in_seg, uint32_t* buf,
                                           int wave, int lane) {
  int k = 0;
  const int ns = p.num_stage;
  if (ns > 0) issue_column(R.f0, R.b0, 0, tile_in_seg, buf, k, wave, lane);
  if (ns > 1) issue_column(R.f1, R.b1, R.o1, tile_in_seg, buf, k, wave, lane);
  if (ns > 2) issue_column(R.f2, R.b2, R.o2, tile_in_seg, buf, k, wave, lane);
  if (ns > 3) issue_column(R.f3, R.b3, R.o3, tile_in_seg, buf, k, wave, lane);
}

__device__ __forceinline__ uint32_t staged_leaf(const StageRegs& R, int sidx, const LeafRegs& L, const uint32_t* sbuf,
                                                int tid) {
  const int b = sidx == 0 ? R.b0 : sidx == 1 ? R.b1 : sidx == 2 ? R.b2 : R.b3;
  const int off = sidx == 0 ? 0 : sidx == 1 ? R.o1 : sidx == 2 ? R.o2 : R.o3;
  return leaf_eval_words(L.kind, L.negate, L.lo, L.span, L.set, sbuf + off + tid * b, b);
}

template <int MODE>
__device__ __forceinline__ void aggregate_doc(const KParams& p, const SegView& S, int64_t doc, uint64_t* tbl,
                                              int64_t G) {
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

__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void scan_kernel(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t G = p.num_keys_total;
  const int table_words = MODE == MODE_LDS ? p.lds_table_words : 0;
  const int stack_words = p.pure_and ? 0 : kMaxStack * kBlock;
  uint32_t* stack = reinterpret_cast<uint32_t*>(lds + table_words);
  uint32_t* wtot = stack + stack_words;
  uint2* queue = reinterpret_cast<uint2*>(wtot + 4);
  uint32_t* stage = reinterpret_cast<uint32_t*>(queue + kQueueCap);
  uint64_t* tbl = (MODE == MODE_LDS) ? lds : p.table;

  if (MODE == MODE_LDS) {
    for (int64_t i = tid; i < (int64_t)p.num_slots * G; i += kBlock) lds[i] = slot_init(p.slot_kind[i / G]);
  }
  __syncthreads();

  unsigned long long matched = 0;
  const int64_t T = p.num_tiles;
  const int64_t t0 = (int64_t)blockIdx.x * T / gridDim.x;
  const int64_t t1 = (int64_t)(blockIdx.x + 1) * T / gridDim.x;
  const int uwave = (int)ufl((uint32_t)wave);
  const int nl = p.num_leaves;
  uint32_t qc = 0;  // queue fill, identical in every thread of the workgroup
  if (t0 < t1) {
    int seg = (int)ufl((uint32_t)p.tile_seg[t0]);
    StageRegs R = load_stage_regs(p, seg);
    LeafRegs L0{}, L1{}, L2{}, L3{};
#define PGPU_LOAD_LEAF_REGS()                                \
    do {                                                     \
      if (p.pure_and) {                                      \
        if (nl > 0) L0 = load_leaf_regs(p, seg, 0);          \
        if (nl > 1) L1 = load_leaf_regs(p, seg, 1);          \
        if (nl > 2) L2 = load_leaf_regs(p, seg, 2);          \
        if (nl > 3) L3 = load_leaf_regs(p, seg, 3);          \
      }                                                      \
    } while (0)
    PGPU_LOAD_LEAF_REGS();
    issue_tile(p, R, t0 - R.tile_base, stage, uwave, lane);
    for (int64_t t = t0; t < t1; ++t) {
      const int cur = (int)((t - t0) & 1);
      uint32_t* sbuf = stage + cur * p.stage_words;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of tile t have landed
      __builtin_amdgcn_s_barrier();                     // ... and every other wave's
      // prefetch tile t + 1 (possibly the first tile of the next segment) into the other buffer
      const bool next_seg = t + 1 < t1 && t + 1 >= (int64_t)R.tile_base + R.num_tiles;
      if (t + 1 < t1) {
        if (next_seg) {
          const StageRegs Rn = load_stage_regs(p, seg + 1);
          issue_tile(p, Rn, t + 1 - Rn.tile_base, stage + (cur ^ 1) * p.stage_words, uwave, lane);
        } else {
          issue_tile(p, R, t + 1 - R.tile_base, stage + (cur ^ 1) * p.stage_words, uwave, lane);
        }
      }
      // decode tile t
      const int nd = R.num_docs;
      const int64_t group = (t - R.tile_base) * kBlock + tid;
      const int64_t doc0 = group << 5;
      uint32_t mask = doc0 >= nd ? 0u : (nd - doc0 >= 32 ? ~0u : ((1u << (nd - doc0)) - 1u));
      if (p.num_ops > 0) {
        if (p.pure_and) {
          if (nl > 0 && __any(mask != 0u)) mask &= staged_leaf(R, p.leaf_stage[0], L0, sbuf, tid);
          if (nl > 1 && __any(mask != 0u)) mask &= staged_leaf(R, p.leaf_stage[1], L1, sbuf, tid);
          if (nl > 2 && __any(mask != 0u)) mask &= staged_leaf(R, p.leaf_stage[2], L2, sbuf, tid);
          if (nl > 3 && __any(mask != 0u)) mask &= staged_leaf(R, p.leaf_stage[3], L3, sbuf, tid);
        } else {
          int sp = 0;
          for (int k = 0; k < p.num_ops; ++k) {
            const int op = p.ops[k] >> 16, arg = p.ops[k] & 0xFFFF;
            if (op == OP_LEAF) {
              const LeafRegs Lk = load_leaf_regs(p, seg, arg);
              stack[sp * kBlock + tid] = staged_leaf(R, p.leaf_stage[arg], Lk, sbuf, tid);
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
          mask &= stack[tid];
        }
      }
      // matched docs: block-wide prefix of the per-lane counts
      const uint32_t cnt = __popc(mask);
      matched += cnt;
      const uint32_t incl = wave_inclusive_scan(cnt, lane);
      if (lane == 63) wtot[wave] = incl;
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      const uint32_t w0 = wtot[0], w1 = wtot[1], w2 = wtot[2], w3 = wtot[3];
      const uint32_t total = ufl(w0 + w1 + w2 + w3);
      if (total > 0) {
        if (qc + total > (uint32_t)kQueueCap) {  // flush the queue first
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_s_barrier();
          for (uint32_t i = tid; i < qc; i += kBlock) {
            const uint2 e = queue[i];
            aggregate_doc<MODE>(p, seg_view(p, (int)e.x), (int64_t)e.y, tbl, G);
          }
          qc = 0;
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_s_barrier();
        }
        if (total > (uint32_t)kQueueCap) {  // dense tile: aggregate in place
          const SegView S = seg_view(p, seg);
          uint32_t m = mask;
          while (m) {
            const int i = __ffs(m) - 1;
            m &= m - 1u;
            aggregate_doc<MODE>(p, S, doc0 + i, tbl, G);
          }
        } else {
          uint32_t pos = qc + (wave > 0 ? w0 : 0) + (wave > 1 ? w1 : 0) + (wave > 2 ? w2 : 0) + incl - cnt;
          uint32_t m = mask;
          while (m) {
            const int i = __ffs(m) - 1;
            m &= m - 1u;
            queue[pos++] = make_uint2((uint32_t)seg, (uint32_t)(doc0 + i));
          }
          qc += total;
        }
      }
      if (next_seg) {  // advance the cursor (re-reads descriptors once per segment)
        ++seg;
        R = load_stage_regs(p, seg);
        PGPU_LOAD_LEAF_REGS();
      }
    }
#undef PGPU_LOAD_LEAF_REGS
  }
  // drain the queue
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();
  for (uint32_t i = tid; i < qc; i += kBlock) {
    const uint2 e = queue[i];
    aggregate_doc<MODE>(p, seg_view(p, (int)e.x), (int64_t)e.y, tbl, G);
  }
  for (int off = 32; off > 0; off >>= 1) matched += __shfl_xor(matched, off);
  if (lane == 0 && matched) atomicAdd(p.stats, matched);
  if (MODE == MODE_LDS) {
    __syncthreads();
    uint64_t* out = p.slab + (int64_t)blockIdx.x * p.num_slots * G;
    for (int64_t i = tid; i < (int64_t)p.num_slots * G; i += kBlock) out[i] = lds[i];
  }
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

int launch_expand_tiles(const uint8_t* segs, int32_t seg_stride, int32_t num_segs, int32_t* tile_seg, void* stream) {
  if (num_segs <= 0) return 0;
  hipLaunchKernelGGL(expand_tiles_kernel, dim3(num_segs < 4096 ? num_segs : 4096), dim3(128), 0, S(stream), segs,
                     seg_stride, num_segs, tile_seg);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_scan(const KParams& p, int mode, int grid, size_t lds_bytes, void* stream) {
  switch (mode) {
    case MODE_LDS:
      hipLaunchKernelGGL(scan_kernel<MODE_LDS>, dim3(grid), dim3(kBlock), lds_bytes, S(stream), p);
      break;
    case MODE_GLOBAL:
      hipLaunchKernelGGL(scan_kernel<MODE_GLOBAL>, dim3(grid), dim3(kBlock), lds_bytes, S(stream), p);
      break;
    default:
      hipLaunchKernelGGL(scan_kernel<MODE_HASH>, dim3(grid), dim3(kBlock), lds_bytes, S(stream), p);
      break;
  }
  return PGPU_HIP_OK(hipGetLastError());
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
