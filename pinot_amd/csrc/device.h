// device.h — device-side building blocks shared by the gfx950 kernels: the MSB-first fixed-bit decoders
// (PinotDataBitSet / FixedBitIntReader layout), predicate leaf masks, segment-record views, accumulators and
// the batched group-by aggregation.  Included by every kernel translation unit (one object per kernel family and
// accumulator mode, compiled in parallel).
#pragma once
#include <hip/hip_runtime.h>

#include <utility>

#include "internal.h"

namespace pgpu {

#define PGPU_HIP_OK(x) ((x) == hipSuccess ? 0 : -1)

// Reads through the global address space.  Pointers read out of the packed segment / star-tree records are generic
// to the compiler, which then emits FLAT loads: those also count in lgkmcnt, so every wait for an LDS access (match
// queues, LDS tables, LUT caches) waits for all outstanding column loads too.  Every pointer passed here points into
// device memory (hipMalloc), never into LDS.
template <typename T>
using gmem = const __attribute__((address_space(1))) T;
template <typename T>
__device__ __forceinline__ gmem<T>* gp(const T* p) { return (gmem<T>*)p; }
// Reads of the plan's segment records and tile map, which no kernel writes: through the constant address space, so
// their wave-uniform loads stay scalar loads (SMEM) whatever the kernel stores elsewhere.  Through generic or global
// pointers the compiler proves a load unclobbered only when no store or atomic can run before it, so a global atomic
// ahead of the tile loop (the run-time tile claims) had turned them into vector loads: the sparse scan instances went
// 112 -> 145 VGPRs (3 waves per SIMD instead of 4).
template <typename T>
using cmem = const __attribute__((address_space(4))) T;
using KColC = cmem<KCol>;
using KLeafC = cmem<KLeaf>;
template <typename T>
__device__ __forceinline__ cmem<T>* cp(const T* p) { return (cmem<T>*)p; }

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// PGPU_SADDR (default off): gathers from a wave-uniform base take a 32-bit byte offset, so they compile to the
// global_load SADDR form (base in SGPRs, one offset VGPR per load instead of a 64-bit VGPR address pair).  Measured
// on MI355X (r04, interleaved A/B of two libraries): the dense instance keeps 168 VGPRs either way, and C2's scan
// ran 605 / 604 us with it against 578 / 573 without (C3 and C1 flat), so it stays off.
#ifndef PGPU_SADDR
#define PGPU_SADDR 0
#endif
template <typename T>
__device__ __forceinline__ const T* wave_uniform(const T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const T*>(((uint64_t)hi << 32) | lo);
}
template <typename T>
__device__ __forceinline__ T load_off(const T* ubase, uint32_t byte_off) {
  using GC = const __attribute__((address_space(1))) char;
  return *reinterpret_cast<gmem<T>*>(reinterpret_cast<GC*>(gp(ubase)) + byte_off);
}

// The query's end time (KParams.deadline: a wall_clock64() value, 0 = none) has passed.  wall_clock64 is a scalar
// read of the constant-rate device clock, so the answer is uniform across a wave.
__device__ __forceinline__ bool past_deadline(uint64_t deadline) {
  return deadline != 0 && (uint64_t)wall_clock64() > deadline;
}
// stats[5] != 0: some workgroup stopped at the deadline (the group table is partial; the host reports the timeout).
__device__ __forceinline__ void flag_timeout(unsigned long long* stats) { atomicOr(stats + 5, 1ull); }

// Value of doc `doc` in a packed column (PinotDataBitSet.readInt semantics).  The two-word window never leaves
// the allocation thanks to the padding words.
__device__ __forceinline__ uint32_t gather_id(const uint32_t* __restrict__ fwd, int bits, int64_t doc) {
  const uint64_t bit = (uint64_t)doc * (uint64_t)bits;
  const uint64_t wi = bit >> 5;
  const uint32_t sh = (uint32_t)(bit & 31);
  gmem<uint32_t>* f = gp(fwd);
  const uint64_t two = ((uint64_t)bswap32(f[wi]) << 32) | (uint64_t)bswap32(f[wi + 1]);
  return (uint32_t)(two >> (64 - sh - bits)) & ((1u << bits) - 1u);
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

// G: `words` is in global memory (else LDS).
template <int B, bool G = true>
__device__ __forceinline__ void load_group(const uint32_t* __restrict__ words, uint32_t (&w)[B + 1]) {
  if constexpr (G) {
    gmem<uint32_t>* g = gp(words);
    // plain loads: word k of every lane is B words apart, so a line is finished by the next instructions; measured
    // on MI355X, non-temporal loads here cost C3 44% (775 -> 1115 us) and C2 2% (the L2 must keep the lines)
#pragma unroll
    for (int k = 0; k < B; ++k) w[k] = bswap32(g[k]);
  } else {
#pragma unroll
    for (int k = 0; k < B; ++k) w[k] = bswap32(words[k]);
  }
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

template <int B, bool G>
__device__ __forceinline__ uint32_t leaf_range_b(const uint32_t* __restrict__ words, uint32_t lo, uint32_t span) {
  uint32_t w[B + 1];
  load_group<B, G>(words, w);
  if (span == 1) return eq_all<B>(w, lo, std::make_integer_sequence<int, 32>{});
  return range_all<B>(w, lo, lo + span, std::make_integer_sequence<int, 32>{});
}

template <int B, bool G>
__device__ __forceinline__ uint32_t leaf_set_b(const uint32_t* __restrict__ words, const uint32_t* __restrict__ set) {
  uint32_t w[B + 1];
  load_group<B, G>(words, w);
  gmem<uint32_t>* gs = gp(set);
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int bit = i * B, wi = bit >> 5, sh = bit & 31;
    uint32_t v;
    if (sh + B <= 32) v = (w[wi] >> (32 - sh - B)) & ((1u << B) - 1u);
    else v = ((w[wi] << (sh + B - 32)) | (w[wi + 1] >> (64 - sh - B))) & ((1u << B) - 1u);
    m |= ((gs[v >> 5] >> (v & 31)) & 1u) << i;
  }
  return m;
}

// Wave-uniform dispatch on (kind, bits) to the decoder instance; `words` = this lane's 32-doc group (global
// memory, G = true, or an LDS stage buffer).
template <bool G = true>
__device__ __forceinline__ uint32_t leaf_eval_words(int kind, int negate, uint32_t lo, uint32_t span,
                                                    const uint32_t* set, const uint32_t* words, int bits) {
  if (kind == LEAF_ALL) return ~0u;
  if (kind == LEAF_NONE) return 0u;
  uint32_t m = 0;
  if (kind == LEAF_RANGE) {
    switch (bits) {
#define PGPU_CASE(B) \
  case B:            \
    m = leaf_range_b<B, G>(words, lo, span); \
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
    m = leaf_set_b<B, G>(words, set); \
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

// Docs [32*group, 32*group + 32) inside [lo, lo + span): bit i = doc 32*group + i.
__device__ __forceinline__ uint32_t docrange_mask(int64_t group, uint32_t lo, uint32_t span) {
  const int64_t doc0 = group << 5;
  int64_t a = (int64_t)lo - doc0, b = (int64_t)lo + span - doc0;
  a = a < 0 ? 0 : (a > 32 ? 32 : a);
  b = b < 0 ? 0 : (b > 32 ? 32 : b);
  if (b <= a) return 0u;
  const uint32_t upto_b = b >= 32 ? ~0u : ((1u << b) - 1u);
  const uint32_t below_a = a >= 32 ? ~0u : ((1u << a) - 1u);
  return upto_b & ~below_a;
}

// One 32-doc group of a Roaring ARRAY container read in place (LEAF_BITDIR directory entry with bit 0 set: payload
// pointer in bits 1..47, entry count in bits 48..63): the container's sorted u16 doc offsets are binary-searched for
// the group's first doc, then the group's entries (at most 32) set their bits.  ARRAY containers hold < 4096 docs of
// their 65536 (RoaringBitmap's ARRAY / BITMAP threshold), e.g. the partial last block of a segment.
__device__ __forceinline__ uint32_t array_group_mask(uint64_t e, int64_t group) {
  gmem<uint16_t>* __restrict__ a = gp(reinterpret_cast<const uint16_t*>(e & 0x0000FFFFFFFFFFFEull));
  const int n = (int)(e >> 48);
  const uint32_t lo = (uint32_t)(group & 2047) << 5;
  int l = 0, h = n;
  while (l < h) {
    const int mid = (l + h) >> 1;
    if ((uint32_t)a[mid] < lo) l = mid + 1;
    else h = mid;
  }
  uint32_t m = 0;
  for (int i = l; i < n; ++i) {
    const uint32_t v = (uint32_t)a[i] - lo;
    if (v >= 32u) break;
    m |= 1u << v;
  }
  return m;
}

// One 32-doc group of a LEAF_BITDIR leaf from its block's directory entry (0: no docs; a BITMAP container's address;
// an ARRAY container's address | 1 with its count in bits 48-63).
__device__ __forceinline__ uint32_t bitdir_mask(uint64_t e, int negate, int64_t group) {
  const uint32_t m = (e & 1ull) ? array_group_mask(e, group) : e ? gp(reinterpret_cast<const uint32_t*>(e))[group & 2047] : 0u;
  return negate ? ~m : m;
}

// A LEAF_BITDIR leaf (an inverted index read in place) beside a LEAF_RANGE scan of B-bit dictIds, evaluated
// together: the scan column's words and the container word are requested together (the block's directory entry `e`
// comes from the caller, which keeps it across the 8 tiles of a 65536-doc block), so a tile waits one memory round
// trip instead of three.  Both masks come back; the caller applies them in Pinot's order (index leaf, then the scan
// on its survivors).
template <int B>
__device__ __forceinline__ void bitdir_range_b(const uint32_t* __restrict__ words, uint32_t lo, uint32_t span,
                                               uint64_t e, int neg0, int64_t group, uint32_t& m0, uint32_t& m1) {
  uint32_t w[B + 1];
  load_group<B, true>(words, w);
  m0 = bitdir_mask(e, neg0, group);
  m1 = span == 1 ? eq_all<B>(w, lo, std::make_integer_sequence<int, 32>{})
                 : range_all<B>(w, lo, lo + span, std::make_integer_sequence<int, 32>{});
}
__device__ __forceinline__ void bitdir_range(const uint32_t* fwd, int bits, uint32_t lo, uint32_t span, int neg1,
                                             uint64_t e, int neg0, int64_t group, uint32_t& m0, uint32_t& m1) {
  const uint32_t* words = fwd + group * (int64_t)bits;
  m0 = 0;
  m1 = 0;
  switch (bits) {
#define PGPU_CASE(B)                                                 \
  case B:                                                            \
    bitdir_range_b<B>(words, lo, span, e, neg0, group, m0, m1); \
    break;
    PGPU_CASE(1) PGPU_CASE(2) PGPU_CASE(3) PGPU_CASE(4) PGPU_CASE(5) PGPU_CASE(6) PGPU_CASE(7) PGPU_CASE(8)
    PGPU_CASE(9) PGPU_CASE(10) PGPU_CASE(11) PGPU_CASE(12) PGPU_CASE(13) PGPU_CASE(14) PGPU_CASE(15)
    PGPU_CASE(16) PGPU_CASE(17) PGPU_CASE(18) PGPU_CASE(19) PGPU_CASE(20) PGPU_CASE(21) PGPU_CASE(22)
    PGPU_CASE(23) PGPU_CASE(24) PGPU_CASE(25) PGPU_CASE(26) PGPU_CASE(27) PGPU_CASE(28) PGPU_CASE(29)
    PGPU_CASE(30) PGPU_CASE(31)
#undef PGPU_CASE
    default: break;
  }
  if (neg1) m1 = ~m1;
}

__device__ __forceinline__ uint32_t leaf_eval(int kind, int negate, uint32_t lo, uint32_t span, const uint32_t* set,
                                              const uint32_t* fwd, int bits, int64_t group) {
  if (kind == LEAF_DOCRANGE) {
    const uint32_t m = docrange_mask(group, lo, span);
    return negate ? ~m : m;
  }
  if (kind == LEAF_BITMAP) {
    const uint32_t m = gp(set)[group];
    return negate ? ~m : m;
  }
  if (kind == LEAF_BITDIR) {
    const uint64_t e = gp(reinterpret_cast<const uint64_t*>(set))[group >> 11];
    const uint32_t m = (e & 1ull) ? array_group_mask(e, group) : e ? gp(reinterpret_cast<const uint32_t*>(e))[group & 2047] : 0u;
    return negate ? ~m : m;
  }
  return leaf_eval_words(kind, negate, lo, span, set, fwd + group * (int64_t)bits, bits);
}

// Raw-value leaf test of one 32-doc group (raw_leaf_bitmap_kernel): the docs' int64 keys (contiguous: the compiler
// pairs the loads into 16-byte ones) against inclusive bounds [lo, hi] (LEAF_RAW_RANGE) or the `hi` sorted keys at
// set_keys (LEAF_RAW_IN).
__device__ __forceinline__ uint32_t raw_group_mask(int kind, int64_t lo, int64_t hi, const int64_t* set_keys,
                                                   const int64_t* keys, int64_t group) {
  gmem<int64_t>* __restrict__ s = gp(set_keys);
  gmem<int64_t>* __restrict__ v = gp(keys) + group * 32;
  uint32_t m = 0;
  if (kind == LEAF_RAW_RANGE) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int64_t x = v[i];
      m |= (uint32_t)(lo <= x && x <= hi) << i;
    }
  } else {
    const int n = (int)hi;
    for (int i = 0; i < 32; ++i) {
      const int64_t key = v[i];
      int a = 0, b = n;  // first set key >= key
      while (a < b) {
        const int mid = (a + b) >> 1;
        if (s[mid] < key) a = mid + 1;
        else b = mid;
      }
      m |= (uint32_t)(a < n && s[a] == key) << i;
    }
  }
  return m;
}

__device__ __forceinline__ uint32_t leaf_mask(KLeafC& L, KColC& C, int64_t group) {
  return leaf_eval(L.kind, L.negate, L.lo, L.span, L.set, C.fwd, C.bits, group);
}

// ---------------------------------------------------------------------------------------------- helpers
struct SegView {
  cmem<KSegHdr>* hdr;
  KColC* cols;
  KLeafC* leaves;
};

// Index of local dictId `id` in a column's value arrays (KCol.dkey / dval): the id itself, or -- table-global value
// arrays -- id + the global ids missing from the segment's dictionary below it.  Threshold k is t_k + k (t_k the local
// id above the k-th missing value, rt_dict.cpp ensure_value_map), so the running index is compared, no memory access.
__device__ __forceinline__ uint32_t vidx(KColC& c, uint32_t id) {
  for (int k = 0; k < c.ngaps; ++k) id += id >= c.gaps[k] ? 1u : 0u;
  return id;
}
// The same for N ids of one segment (c wave-uniform: the thresholds are scalar operands).
template <int N>
__device__ __forceinline__ void vidx_n(KColC& c, uint32_t (&ids)[N]) {
  const int ng = c.ngaps;
  for (int k = 0; k < ng; ++k) {
    const uint32_t g = c.gaps[k];
#pragma unroll
    for (int i = 0; i < N; ++i) ids[i] += ids[i] >= g ? 1u : 0u;
  }
}

__device__ __forceinline__ SegView seg_view(const KParams& p, int seg) {
  const uint8_t* base = p.segs + (int64_t)seg * p.seg_stride;
  SegView v;
  v.hdr = cp(reinterpret_cast<const KSegHdr*>(base));
  v.cols = cp(reinterpret_cast<const KCol*>(base + sizeof(KSegHdr)));
  v.leaves = cp(reinterpret_cast<const KLeaf*>(base + sizeof(KSegHdr) + sizeof(KCol) * p.num_cols));
  return v;
}

// Word j of a compact slot column at `width` bytes (two's complement, little-endian).
__device__ __forceinline__ void put_compact(uint8_t* o, int64_t j, int width, uint64_t v) {
  switch (width) {
    case 1: o[j] = (uint8_t)v; break;
    case 2: reinterpret_cast<uint16_t*>(o)[j] = (uint16_t)v; break;
    case 3:
      o[3 * j] = (uint8_t)v;
      o[3 * j + 1] = (uint8_t)(v >> 8);
      o[3 * j + 2] = (uint8_t)(v >> 16);
      break;
    case 4: reinterpret_cast<uint32_t*>(o)[j] = (uint32_t)v; break;
    default: reinterpret_cast<uint64_t*>(o)[j] = v; break;
  }
}

__device__ __forceinline__ uint64_t slot_init(int kind) {
  if (kind == SLOT_MIN_KEY) return (uint64_t)INT64_MAX;
  if (kind == SLOT_MAX_KEY) return (uint64_t)INT64_MIN;
  return 0ull;
}
// An LDS table word's start value (KParams.narrow: 32-bit min / max on the low half).
__device__ __forceinline__ uint64_t slot_init_lds(int kind, bool narrow) {
  if (narrow) return kind == SLOT_MIN_KEY ? 0xFFFFFFFFull : 0ull;
  return slot_init(kind);
}

// Leaf descriptors of the current segment held in registers (reloaded only when the segment changes).
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
  KLeafC& L = S.leaves[l];
  KColC& C = S.cols[p.leaf_col[l]];
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

// Slot of `key` in an open-addressing table of `cap` (a power of two) slots, inserted if absent; linear probing,
// at most `cap` probes: a full table returns -1 and sets *full (stats[4]; the host reports the error) instead of
// spinning.  Tables are sized for a load <= 1/2 of the groups the plan can produce, so this never happens in a
// correct plan -- it only bounds every wave's loop.
__device__ __forceinline__ int64_t hash_slot(unsigned long long* __restrict__ keys, int64_t cap, uint64_t key,
                                             unsigned long long* full) {
  uint64_t h = key * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29;
  int64_t s = (int64_t)(h & (uint64_t)(cap - 1));
  for (int64_t probes = 0; probes < cap; ++probes) {
    unsigned long long k = keys[s];
    if (k == key) return s;
    if (k == ~0ull) {
      const unsigned long long prev = atomicCAS(&keys[s], ~0ull, (unsigned long long)key);
      if (prev == ~0ull || prev == key) return s;
    }
    s = (s + 1) & (cap - 1);
  }
  if (full) atomicOr(full, 1ull);
  return -1;
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

// ---- single-row tables (aggregation-only queries, G == 1): every matched doc updates the same word, so each
// lane folds its docs, the wave folds its lanes (xor butterfly) and one lane issues the atomic.  Requires the
// whole wave to be converged at the call.
__device__ __forceinline__ int64_t wave_sum_i64(int64_t x) {
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}
__device__ __forceinline__ double wave_sum_f64(double x) {
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t x) {
  for (int off = 32; off > 0; off >>= 1) { const int64_t y = __shfl_xor(x, off); x = y < x ? y : x; }
  return x;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t x) {
  for (int off = 32; off > 0; off >>= 1) { const int64_t y = __shfl_xor(x, off); x = y > x ? y : x; }
  return x;
}

// Per-workgroup statistics counters: the waves' partial sums meet in LDS and one atomic per workgroup and counter
// reaches global memory (a thousand waves' atomics on one address serialise in a kernel's tail: 70 us on C3's
// 125-segment scan, measured).  Call from every thread of the workgroup; v holds the lane's partial of counter k.
template <int N, int BLOCK = kBlock>
__device__ __forceinline__ void block_stats_add(unsigned long long* __restrict__ stats, const int (&idx)[N],
                                                unsigned long long (&v)[N]) {
  __shared__ unsigned long long red[BLOCK / 64][N];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
    if (lane == 0) red[wave][k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k)  // constant k: idx[] and v[] stay in registers (a dynamic index would use scratch)
    if (threadIdx.x == k) {
      unsigned long long t = 0;
      for (int w = 0; w < BLOCK / 64; ++w) t += red[w][k];
      if (t) atomicAdd(stats + idx[k], t);
    }
}

// Lane partials of one slot (cnt docs; isum / fsum sums; imin / imax extremes) -> one atomic on `word`.
__device__ __forceinline__ void accumulate_wave(uint64_t* __restrict__ word, int kind, int64_t cnt, int64_t ival,
                                                double fval) {
  const bool leader = (threadIdx.x & 63) == 0;
  const int64_t total = wave_sum_i64(cnt);
  if (total == 0) return;  // wave-uniform
  switch (kind) {
    case SLOT_COUNT:
      if (leader) atomicAdd(reinterpret_cast<unsigned long long*>(word), (unsigned long long)total);
      break;
    case SLOT_SUM_I64: {
      const int64_t v = wave_sum_i64(ival);
      if (leader) atomicAdd(reinterpret_cast<unsigned long long*>(word), (unsigned long long)v);
      break;
    }
    case SLOT_SUM_F64: {
      const double v = wave_sum_f64(fval);
      if (leader) atomicAdd(reinterpret_cast<double*>(word), v);
      break;
    }
    case SLOT_MIN_KEY: {
      const int64_t v = wave_min_i64(ival);
      if (leader) atomicMin(reinterpret_cast<long long*>(word), (long long)v);
      break;
    }
    default: {
      const int64_t v = wave_max_i64(ival);
      if (leader) atomicMax(reinterpret_cast<long long*>(word), (long long)v);
      break;
    }
  }
}
// Identity of a slot's lane partial.
__device__ __forceinline__ int64_t slot_identity(int kind) {
  return kind == SLOT_MIN_KEY ? INT64_MAX : kind == SLOT_MAX_KEY ? INT64_MIN : 0;
}
__device__ __forceinline__ int64_t slot_fold(int kind, int64_t a, int64_t v) {
  return kind == SLOT_MIN_KEY ? (v < a ? v : a) : kind == SLOT_MAX_KEY ? (v > a ? v : a) : a + v;
}

// Aggregates NB docs per lane (doc b of segment S[b]) with their gathers interleaved: every dependent level
// (segment record -> forward-index words -> dictId -> LUT / dictionary value) is issued for all NB docs before any
// is consumed, so a batch pays each memory round trip once.  Docs with ok[b] == false read doc 0 of their segment
// (always in bounds) and add nothing.
// SIMPLE (KParams of a "simple" dense plan, plan_create_impl): every group-by column's dictionary is a contiguous run of
// the global one in every segment (no LUT), every aggregated column is an integer of consecutive values (no
// dictionary lookup) and no slot sums doubles -- the gathers compile away, and with them their registers.
template <int MODE, int NB, bool SIMPLE = false>
__device__ __forceinline__ void aggregate_batch(const KParams& p, const SegView (&S)[NB], const int64_t (&doc)[NB],
                                                const bool (&ok)[NB], uint64_t* __restrict__ tbl, int64_t G) {
  int64_t key[NB];
  bool live[NB];  // ok, and (hash mode) a slot was found
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    key[b] = -p.key_bias;  // filter-restricted key space (0 for hash / staged keys)
    live[b] = ok[b];
  }
  int st = 0;  // MODE_HASH key stages (key spaces beyond 64 bits)
  for (int j = 0; j < p.num_keys; ++j) {
    const int kc = p.key_col[j];
    uint32_t id[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      KColC& c = S[b].cols[kc];
      id[b] = gather_id(c.fwd, c.bits, ok[b] ? doc[b] : 0);
    }
    int32_t g[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {  // the lanes' docs may come from different segments: per-lane select
      KColC& c = S[b].cols[kc];
      g[b] = !SIMPLE && c.lut ? gp(c.lut)[id[b]] : (int32_t)id[b] + c.lut_off;
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) key[b] += (int64_t)g[b] * p.key_stride[j];
    if (MODE == MODE_HASH && st < p.num_stages && j + 1 == p.stage_end[st]) {  // wave-uniform
      // the group's key -> its slot in stage table st (a dense id), the base of the next group's key
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int64_t slot = live[b] ? hash_slot(p.stage_keys + p.stage_off[st], p.stage_cap[st], (uint64_t)key[b],
                                                 p.stats + 4) : 0;
        live[b] = live[b] && slot >= 0;
        key[b] = live[b] ? slot * p.stage_mult[st] : 0;
      }
      ++st;
    }
  }
  int64_t idx[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    idx[b] = key[b];
    if (MODE == MODE_HASH && live[b]) {
      idx[b] = hash_slot(p.hash_keys, G, (uint64_t)key[b], p.stats + 4);
      live[b] = idx[b] >= 0;
    }
  }
  uint32_t id[NB], vi[NB];  // dictIds, and their indexes in the value arrays (vidx)
  int prev_col = -1;
  for (int s = 0; s < p.num_slots; ++s) {
    const int kind = p.slot_kind[s];
    int64_t ikey[NB];
    double dval[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) { ikey[b] = 0; dval[b] = 0.0; }
    if (kind != SLOT_COUNT) {
      const int col = p.slot_col[s];
      if (col != prev_col) {  // SUM/MIN/MAX of one column share the dictId gather
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          KColC& c = S[b].cols[col];
          id[b] = gather_id(c.fwd, c.bits, ok[b] ? doc[b] : 0);
        }
        if (!SIMPLE) {
#pragma unroll
          for (int b = 0; b < NB; ++b) vi[b] = vidx(S[b].cols[col], id[b]);
        }
        prev_col = col;
      }
      if (!SIMPLE && kind == SLOT_SUM_F64) {
#pragma unroll
        for (int b = 0; b < NB; ++b) dval[b] = gp(S[b].cols[col].dval)[vi[b]];
      } else {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          KColC& c = S[b].cols[col];
          ikey[b] = !SIMPLE && c.dkey ? gp(c.dkey)[vi[b]] : c.key_base + (int64_t)id[b];
        }
      }
    }
    if (G == 1) {  // single row: fold the lane's docs, then the wave
      int64_t cnt = 0, iacc = slot_identity(kind);
      double facc = 0.0;
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (ok[b]) { ++cnt; iacc = slot_fold(kind, iacc, ikey[b]); facc += dval[b]; }
      accumulate_wave(tbl + s, kind, cnt, iacc, facc);
      continue;
    }
    if ((MODE == MODE_LDS || MODE == MODE_HASH) && p.pack_slot >= 0) {  // KParams.pack_slot: the pack slot adds both
      if (kind == SLOT_COUNT) continue;
      if (s == p.pack_slot) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
          if (live[b])
            atomicAdd(reinterpret_cast<unsigned long long*>(tbl + (int64_t)s * G + idx[b]),
                      (1ull << p.pack_shift) | (unsigned long long)ikey[b]);
        continue;
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if (live[b]) accumulate<MODE>(tbl, (int64_t)s * G + idx[b], kind, ikey[b], dval[b]);
  }
}

// ---------------------------------------------------------------------------------------------- dense groups
// Dense tiles: every 128-B line of the group-by / aggregated columns holds matches, so instead of per-doc gathers
// each lane streams its whole 32-doc group of each such column (the same coalesced B-word read as a filter leaf),
// decodes the 32 dictIds with compile-time shifts into registers, and issues the 32 dictionary / LUT lookups of a
// column together (one memory round trip per column instead of one per doc pair).
template <int B, int H, int... I>
__device__ __forceinline__ void decode_half(const uint32_t (&w)[B + 1], uint32_t (&ids)[16],
                                            std::integer_sequence<int, I...>) {
  ((ids[I] = extract<B, H + I>(w)), ...);
}

template <int B, int H>
__device__ __forceinline__ void decode_group_b(const uint32_t* __restrict__ words, uint32_t (&ids)[16]) {
  uint32_t w[B + 1];
  load_group<B, true>(words, w);
  decode_half<B, H>(w, ids, std::make_integer_sequence<int, 16>{});
}
// The same from a wave-uniform column base and the group's byte offset (PGPU_SADDR).
template <int B, int H>
__device__ __forceinline__ void decode_group_ob(const uint32_t* __restrict__ ubase, uint32_t off, uint32_t (&ids)[16]) {
  uint32_t w[B + 1];
#pragma unroll
  for (int k = 0; k < B; ++k) w[k] = bswap32(load_off(ubase, off + 4u * k));
  w[B] = 0;
  decode_half<B, H>(w, ids, std::make_integer_sequence<int, 16>{});
}

// dictIds of docs [32*group + H, 32*group + H + 16) (PinotDataBitSet.readInt).
template <int H>
__device__ __forceinline__ void decode_group(const uint32_t* __restrict__ fwd, int bits, int64_t group,
                                             uint32_t (&ids)[16]) {
#if PGPU_SADDR
  const uint32_t* ubase = wave_uniform(fwd);
  const uint32_t off = (uint32_t)group * (uint32_t)bits * 4u;  // a segment's forward index is < 4 GB
#define PGPU_DECODE(B) decode_group_ob<B, H>(ubase, off, ids)
#else
  const uint32_t* words = fwd + group * (int64_t)bits;
#define PGPU_DECODE(B) decode_group_b<B, H>(words, ids)
#endif
  switch (bits) {
#define PGPU_CASE(B) \
  case B:            \
    PGPU_DECODE(B); \
    break;
    PGPU_CASE(1) PGPU_CASE(2) PGPU_CASE(3) PGPU_CASE(4) PGPU_CASE(5) PGPU_CASE(6) PGPU_CASE(7) PGPU_CASE(8)
    PGPU_CASE(9) PGPU_CASE(10) PGPU_CASE(11) PGPU_CASE(12) PGPU_CASE(13) PGPU_CASE(14) PGPU_CASE(15)
    PGPU_CASE(16) PGPU_CASE(17) PGPU_CASE(18) PGPU_CASE(19) PGPU_CASE(20) PGPU_CASE(21) PGPU_CASE(22)
    PGPU_CASE(23) PGPU_CASE(24) PGPU_CASE(25) PGPU_CASE(26) PGPU_CASE(27) PGPU_CASE(28) PGPU_CASE(29)
    PGPU_CASE(30) PGPU_CASE(31)
#undef PGPU_CASE
#undef PGPU_DECODE
    default:
#pragma unroll
      for (int i = 0; i < 16; ++i) ids[i] = 0;
      break;
  }
}

// The 16 docs of a half-group into one slot row of the table.  In LDS the atomics are issued for every doc, the
// unmatched ones with the kind's neutral value at key 0: no per-doc exec-mask branch and no per-doc switch on the
// slot kind (measured on C2: SALU instructions outnumbered VALU ones with the branches), and an LDS atomic costs the
// same with 32 or 64 lanes active.  Global tables keep the branches (a neutral global atomic is real traffic).
template <int MODE>
__device__ __forceinline__ void accumulate16_i(uint64_t* __restrict__ row, const int32_t (&key)[16], uint32_t m,
                                               int kind, const int64_t (&v)[16], bool narrow = false,
                                               uint64_t addend = 0) {
  if (MODE == MODE_LDS) {
    unsigned long long* u = reinterpret_cast<unsigned long long*>(row);
    long long* l = reinterpret_cast<long long*>(row);
    uint32_t* w32 = reinterpret_cast<uint32_t*>(row);  // narrow: the word's low half (little-endian)
    switch (kind) {
      case SLOT_SUM_I64:
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((m >> i) & 1u) atomicAdd(u + key[i], (unsigned long long)v[i] + addend);
        break;
      case SLOT_MIN_KEY:
        if (narrow) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((m >> i) & 1u) atomicMin(w32 + 2 * key[i], (uint32_t)v[i]);
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((m >> i) & 1u) atomicMin(l + key[i], (long long)v[i]);
        }
        break;
      default:
        if (narrow) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((m >> i) & 1u) atomicMax(w32 + 2 * key[i], (uint32_t)v[i]);
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((m >> i) & 1u) atomicMax(l + key[i], (long long)v[i]);
        }
        break;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) accumulate<MODE>(row, key[i], kind, v[i], 0.0);
  }
}
template <int MODE>
__device__ __forceinline__ void accumulate16_count(uint64_t* __restrict__ row, const int32_t (&key)[16], uint32_t m) {
  if (MODE == MODE_LDS) {
    unsigned long long* u = reinterpret_cast<unsigned long long*>(row);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) atomicAdd(u + key[i], 1ull);
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) accumulate<MODE>(row, key[i], SLOT_COUNT, 0, 0.0);
  }
}
template <int MODE>
__device__ __forceinline__ void accumulate16_f(uint64_t* __restrict__ row, const int32_t (&key)[16], uint32_t m,
                                               const double (&v)[16]) {
  if (MODE == MODE_LDS) {
    double* d = reinterpret_cast<double*>(row);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) atomicAdd(d + key[i], v[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) accumulate<MODE>(row, key[i], SLOT_SUM_F64, 0, v[i]);
  }
}

// One half (docs H..H+15 of the lane's group) of aggregate_group.
template <int MODE, int H, bool SIMPLE = false>
__device__ __forceinline__ void aggregate_half(const KParams& p, const SegView& S, int64_t group, uint32_t mask,
                                               uint64_t* __restrict__ tbl, int64_t G) {
  const uint32_t m = (mask >> H) & 0xFFFFu;
  uint32_t ids[16];
  int32_t key[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) key[i] = -(int32_t)p.key_bias;  // dense key spaces: < 2^31 after the bias
  for (int j = 0; j < p.num_keys; ++j) {
    KColC& c = S.cols[p.key_col[j]];
    decode_group<H>(c.fwd, c.bits, group, ids);
    const int32_t stride = (int32_t)p.key_stride[j];
    if (!SIMPLE && c.lut) {  // segment-uniform: the whole wave reads one segment here
      int32_t g[16];
#if PGPU_SADDR
      const int32_t* lut = wave_uniform(c.lut);
#pragma unroll
      for (int i = 0; i < 16; ++i) g[i] = load_off(lut, ids[i] << 2);
#else
      gmem<int32_t>* __restrict__ lut = gp(c.lut);
#pragma unroll
      for (int i = 0; i < 16; ++i) g[i] = lut[ids[i]];
#endif
#pragma unroll
      for (int i = 0; i < 16; ++i) key[i] += g[i] * stride;
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) key[i] += ((int32_t)ids[i] + c.lut_off) * stride;
    }
  }
  // Slots in runs of one column (SUM/MIN/MAX of a column share the decode and the dictionary lookups).
  for (int s = 0; s < p.num_slots;) {
    const int kind = p.slot_kind[s];
    if (kind == SLOT_COUNT) {
      uint64_t* __restrict__ row = tbl + (int64_t)s * G;
      if (G == 1) accumulate_wave(row, SLOT_COUNT, __popc(m), 0, 0.0);
      else if (MODE != MODE_LDS || p.pack_slot < 0) accumulate16_count<MODE>(row, key, m);  // else: with the sum
      ++s;
      continue;
    }
    const int col = p.slot_col[s];
    int e = s + 1;
    bool need_i = kind != SLOT_SUM_F64, need_f = kind == SLOT_SUM_F64;
    while (e < p.num_slots && p.slot_kind[e] != SLOT_COUNT && p.slot_col[e] == col) {
      need_i |= p.slot_kind[e] != SLOT_SUM_F64;
      need_f |= p.slot_kind[e] == SLOT_SUM_F64;
      ++e;
    }
    KColC& c = S.cols[col];
    decode_group<H>(c.fwd, c.bits, group, ids);
    if (!SIMPLE) vidx_n(c, ids);  // table-global value arrays (one segment): dictIds -> their indexes
    if (need_i) {  // the 16 lookups in flight together, then every integer-keyed slot of the run
      int64_t v[16];
      if (!SIMPLE && c.dkey) {
#if PGPU_SADDR
        const int64_t* dk = wave_uniform(c.dkey);
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? load_off(dk, ids[i] << 3) : 0;
#else
        gmem<int64_t>* __restrict__ dk = gp(c.dkey);
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? dk[ids[i]] : 0;
#endif
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? c.key_base + (int64_t)ids[i] : 0;
      }
      for (int r = s; r < e; ++r) {
        const int kr = p.slot_kind[r];
        if (kr == SLOT_SUM_F64) continue;
        uint64_t* __restrict__ row = tbl + (int64_t)r * G;
        if (G == 1) {
          int64_t acc = slot_identity(kr);
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((m >> i) & 1u) acc = slot_fold(kr, acc, v[i]);
          accumulate_wave(row, kr, __popc(m), acc, 0.0);
          continue;
        }
        // KParams.pack_slot: the COUNT rides in the high bits of the sum; narrow: 32-bit min / max
        accumulate16_i<MODE>(row, key, m, kr, v, MODE == MODE_LDS && ((p.narrow >> r) & 1u),
                             MODE == MODE_LDS && r == p.pack_slot ? (1ull << kLdsPackShift) : 0ull);
      }
    }
    if (!SIMPLE && need_f) {
      double v[16];
#if PGPU_SADDR
      const double* dv = wave_uniform(c.dval);
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? load_off(dv, ids[i] << 3) : 0.0;
#else
      gmem<double>* __restrict__ dv = gp(c.dval);
#ifdef PGPU_DIAG_NO_DVAL_GATHER  // diagnostic build only (wrong sums): the dictionary gathers' share of the traffic
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? (double)ids[i] : 0.0;
      (void)dv;
#elif defined(PGPU_DIAG_SHARED_DVAL)  // diagnostic build only (wrong sums): every segment gathers from segment 0's
      // dictionary (in bounds: ids below 2^16), i.e. the access pattern of one table-global dictionary array
      gmem<double>* __restrict__ dv0 = gp(seg_view(p, 0).cols[col].dval);
      (void)dv;
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? dv0[ids[i] & 0xFFFFu] : 0.0;
#else
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? dv[ids[i]] : 0.0;
#endif
#endif
      for (int r = s; r < e; ++r) {
        if (p.slot_kind[r] != SLOT_SUM_F64) continue;
        uint64_t* __restrict__ row = tbl + (int64_t)r * G;
        if (G == 1) {
          double acc = 0.0;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((m >> i) & 1u) acc += v[i];
          accumulate_wave(row, SLOT_SUM_F64, __popc(m), 0, acc);
          continue;
        }
        accumulate16_f<MODE>(row, key, m, v);
      }
    }
    s = e;
  }
}

// Aggregates the matched docs (bits of `mask`) of this lane's 32-doc group `group` of segment S, 16 docs at a
// time.  Dense key spaces only (MODE_LDS / MODE_GLOBAL: composite keys < 2^31).  Docs beyond numDocs decode from
// the zero padding to dictId 0 (in bounds) and are never in `mask`.
template <int MODE, bool SIMPLE = false>
__device__ __forceinline__ void aggregate_group(const KParams& p, const SegView& S, int64_t group, uint32_t mask,
                                                uint64_t* __restrict__ tbl, int64_t G) {
  // wave-uniform conditions: the single-row (G == 1) fold inside uses cross-lane shuffles
  if (__any((mask & 0xFFFFu) != 0u)) aggregate_half<MODE, 0, SIMPLE>(p, S, group, mask, tbl, G);
  if (__any((mask >> 16) != 0u)) aggregate_half<MODE, 16, SIMPLE>(p, S, group, mask, tbl, G);
}

// Drains a wave's queue of matched (segment, doc) entries: 2 per lane per batch.
template <int MODE, bool SIMPLE = false>
__device__ __forceinline__ void flush_wave_queue(const KParams& p, const uint32_t* qd, const uint32_t* qs, uint32_t qn,
                                                 int lane, uint64_t* __restrict__ tbl, int64_t G) {
  for (uint32_t base = 0; base < qn; base += 128) {
    const uint32_t i0 = base + lane, i1 = base + 64 + lane;
    int64_t doc[2];
    bool ok[2];
    ok[0] = i0 < qn;
    ok[1] = i1 < qn;
    doc[0] = ok[0] ? qd[i0] : 0;
    doc[1] = ok[1] ? qd[i1] : 0;
    const SegView S[2] = {seg_view(p, ok[0] ? (int)qs[i0] : (int)qs[0]), seg_view(p, ok[1] ? (int)qs[i1] : (int)qs[0])};
    aggregate_batch<MODE, 2, SIMPLE>(p, S, doc, ok, tbl, G);
  }
}

}  // namespace pgpu
