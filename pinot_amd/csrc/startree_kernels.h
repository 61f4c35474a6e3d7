// startree_kernels.h — star-tree query kernels (K5 traversal, K6 residual scan + aggregation of the
// pre-aggregated documents).  Instantiated per accumulator mode in k_startree.hip.
//
// K5 restates StarTreeFilterOperator.traverseStarTree (core/startree/operator/StarTreeFilterOperator.java:234-338)
// as a level-synchronous BFS, one workgroup per segment: an entry whose remaining predicate and group-by dims are
// all consumed contributes the node's aggregated document; a leaf contributes its [startDocId, endDocId) and its
// remaining predicate dims (the residual filter, :201-223); otherwise the next dimension's children are expanded —
// the children matching the predicate's dictIds, all non-star children for a group-by dimension, else the star
// child when there is one.
// K6 restates the residual filter (BitmapBasedFilterOperator AND the remaining leaf scans, :194-225) and
// StarTreeGroupByExecutor.aggregate (core/startree/executor/StarTreeGroupByExecutor.java:60-71): the documents of
// every emitted range are split over persistent workgroups; metrics come from the pre-aggregated
// "fn__col" arrays (COUNT adds count__*: CountAggregationFunction.java:97-104).
#pragma once
#include <type_traits>

#include "device.h"

namespace pgpu {

__device__ __forceinline__ int64_t double_key_dev(double d) {  // order-preserving int64 of an IEEE double
  const int64_t b = __double_as_longlong(d);
  return b >= 0 ? b : (b ^ INT64_MAX);
}

#if PGPU_MODE == 0  // one definition: the mode-0 object
__global__ __launch_bounds__(256) void startree_traverse_kernel(const KStarSeg* __restrict__ segs,
                                                                int64_t* __restrict__ seg_total, uint64_t deadline,
                                                                unsigned long long* __restrict__ stats) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && past_deadline(deadline)) flag_timeout(stats);  // read by K6
  const KStarSeg& S = segs[blockIdx.x];
  __shared__ int cur_n, next_n, nr, rem;
  // the BFS frontiers in LDS when the tree is small enough (C4: ~100 nodes per segment): a level's expansion then
  // costs no global round trip; larger trees use the global scratch
  // ... and the node array itself (7 ints per node, one coalesced copy): every level's node and child reads are
  // then LDS reads instead of dependent global round trips
  constexpr int kLdsFront = 1024;
  __shared__ int lfront[2][3 * kLdsFront];
  __shared__ int lnodes[7 * kLdsFront];
  const int tid = threadIdx.x;
  const bool in_lds = S.num_nodes <= kLdsFront;
  if (in_lds) {
    for (int i = tid; i < 7 * S.num_nodes; i += blockDim.x) lnodes[i] = S.nodes[i];
  }
  const int* __restrict__ nodes = in_lds ? lnodes : S.nodes;
  int* fa = in_lds ? lfront[0] : S.frontier;
  int* fb = in_lds ? lfront[1] : S.frontier + 3 * S.num_nodes;
  if (tid == 0) {
    fa[0] = 0;  // root
    fa[1] = S.pred_mask;
    fa[2] = S.group_mask;
    cur_n = S.num_nodes > 0 ? 1 : 0;
    nr = 0;
    rem = 0;
  }
  __syncthreads();
  for (;;) {
    const int n = cur_n;
    if (n == 0) break;
    __syncthreads();
    if (tid == 0) next_n = 0;
    __syncthreads();
    // one wave per frontier entry, its children over the wave's lanes (the root of a group-by dimension has as many
    // children as the dimension has values -- C4's d1: 100 -- which one thread used to push one by one)
    const int lane = tid & 63, nwaves = (int)blockDim.x >> 6;
    for (int i = tid >> 6; i < n; i += nwaves) {
      const int node = fa[3 * i], rp = fa[3 * i + 1], rg = fa[3 * i + 2];
      const int* N = nodes + 7 * (int64_t)node;
      const int first = N[5], last = N[6];
      if (rp == 0 && rg == 0) {  // all predicates and group-by dims matched: the aggregated document
        if (lane == 0) {
          const int r = atomicAdd(&nr, 1);
          S.ranges[2 * r] = N[4];
          S.ranges[2 * r + 1] = N[4] + 1;
        }
      } else if (first < 0) {  // leaf: its documents, with the remaining predicates as a residual filter
        if (lane == 0) {
          const int r = atomicAdd(&nr, 1);
          S.ranges[2 * r] = N[2];
          S.ranges[2 * r + 1] = N[3];
          atomicOr(&rem, rp);
        }
      } else {
        const int cd = nodes[7 * (int64_t)first];  // getChildDimensionId
        const int bit = 1 << cd;
        const bool pred = (rp & bit) != 0;
        // neither predicate nor group-by: the star child when it exists, else every non-star child
        if (!pred && !(rg & bit) && nodes[7 * (int64_t)first + 1] == -1) {
          if (lane == 0) {
            const int k = atomicAdd(&next_n, 1);
            fb[3 * k] = first;
            fb[3 * k + 1] = rp;
            fb[3 * k + 2] = rg;
          }
        } else {
          // predicate: the children whose dictId matches; group-by (or no star child): every non-star child
          const int nrp = pred ? rp & ~bit : rp, nrg = pred ? rg : rg & ~bit;
          const uint32_t* m = S.match[cd];
          for (int c0 = first; c0 <= last; c0 += 64) {
            const int c = c0 + lane;
            bool take = false;
            if (c <= last) {
              const int v = nodes[7 * (int64_t)c + 1];
              take = pred ? (v >= 0 && ((m[v >> 5] >> (v & 31)) & 1u)) : v != -1;
            }
            const uint64_t bal = __ballot(take);
            int base = 0;
            if (lane == 0 && bal) base = atomicAdd(&next_n, __popcll(bal));
            base = __shfl(base, 0);
            if (take) {
              const int k = base + __popcll(bal & ((1ull << lane) - 1ull));
              fb[3 * k] = c;
              fb[3 * k + 1] = nrp;
              fb[3 * k + 2] = nrg;
            }
          }
        }
      }
    }
    __syncthreads();
    int* t = fa;
    fa = fb;
    fb = t;
    if (tid == 0) cur_n = next_n;
    __syncthreads();
  }
  // Prefix sums of the ranges' 32-doc groups (K6's unit of work; a range [start, end) covers groups start/32 ..
  // (end-1)/32), block-wide in chunks of blockDim.x ranges.
  __shared__ int64_t part[256];
  __shared__ int64_t carry;
  const int total = nr;
  if (tid == 0) { carry = 0; S.prefix[0] = 0; }
  __syncthreads();
  for (int base = 0; base < total; base += blockDim.x) {
    const int r = base + tid;
    int64_t v = 0;
    if (r < total) {
      const int a = S.ranges[2 * r], b = S.ranges[2 * r + 1];
      v = b > a ? ((b - 1) >> 5) - (a >> 5) + 1 : 0;
    }
    part[tid] = v;
    __syncthreads();
    for (int off = 1; off < (int)blockDim.x; off <<= 1) {
      const int64_t x = tid >= off ? part[tid - off] : 0;
      __syncthreads();
      part[tid] += x;
      __syncthreads();
    }
    if (r < total) S.prefix[r + 1] = carry + part[tid];
    __syncthreads();
    if (tid == blockDim.x - 1) carry += part[tid];
    __syncthreads();
  }
  if (tid == 0) {
    S.out[0] = nr;
    S.out[1] = rem;
    seg_total[blockIdx.x] = carry;
  }
}
#endif

// K6 block size: MODE_LDS workgroups share one LDS table, so they are large (16 waves) to hide memory latency
// with few workgroups per CU.
template <int MODE>
struct StarBlock { static constexpr int value = MODE == MODE_LDS ? 1024 : 256; };

// dictIds of docs [32 g + H, 32 g + H + 16) of a star-tree dimension (MSB-first, whole 32-doc groups padded).
template <int H>
__device__ __forceinline__ void star_decode(const uint32_t* __restrict__ fwd, int bits, int64_t g, uint32_t (&ids)[16]) {
  decode_group<H>(fwd, bits, g, ids);
}

// Aggregates the docs of `mask` (bits H..H+15 of the lane's group g) of star-tree segment S.
// sectors: 64-byte sectors of the metric arrays holding a matched doc, for the bytes model (statistics word 7).
template <int MODE, int H>
__device__ __forceinline__ void star_aggregate_half(const KStarParams& p, const KStarSeg& S, int64_t g, uint32_t mask,
                                                    const int32_t* __restrict__ cache, bool cached,
                                                    uint64_t* __restrict__ tbl, int64_t G,
                                                    unsigned long long& sectors) {
  uint32_t m = (mask >> H) & 0xFFFFu;
  // dense key spaces (MODE_LDS / MODE_GLOBAL) stay below 2^31: 32-bit keys
  using KeyT = typename std::conditional<MODE == MODE_HASH, int64_t, int32_t>::type;
  KeyT key[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) key[i] = -(KeyT)p.key_bias;  // filter-restricted key space (KParams.key_bias)
  int koff = 0;
  for (int j = 0; j < p.num_keys; ++j) {
    const int d = S.key_dim[j];
    uint32_t ids[16];
    star_decode<H>(S.dim_fwd[d], S.dim_bits[d], g, ids);
    const KeyT stride = (KeyT)p.key_stride[j];
    if (cached) {
#pragma unroll
      for (int i = 0; i < 16; ++i) key[i] += (KeyT)cache[koff + (int)ids[i]] * stride;
    } else {
      gmem<int32_t>* __restrict__ lut = gp(S.key_lut[j]);
      int32_t v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? lut[ids[i]] : 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) key[i] += (KeyT)v[i] * stride;
    }
    koff += S.dim_card[d];
  }
  if (MODE == MODE_HASH) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) {
        const int64_t slot = hash_slot(p.hash_keys, G, (uint64_t)key[i], p.stats + 4);
        if (slot < 0) m &= ~(1u << i);
        key[i] = (KeyT)(slot < 0 ? 0 : slot);
      }
  }
  const int64_t d0 = g * 32 + H;
  // a half's 16 docs: one 64-B sector of an int32 array, two of an 8-byte one
  const unsigned sec4 = m != 0u, sec8 = ((m & 0xFFu) != 0u) + ((m >> 8) != 0u);
  for (int s = 0; s < p.num_slots; ++s) {
    const int kind = p.slot_kind[s];
    uint64_t* __restrict__ row = tbl + (int64_t)s * G;
    if (kind == SLOT_COUNT) {  // COUNT adds the pre-aggregated count (1 per document when the tree has none)
      const bool has = S.src_c[0] != nullptr;
      const bool nar = (S.narrow >> 31) & 1u;
      int64_t c[16];
      if (nar) {
        gmem<int32_t>* __restrict__ src = gp(reinterpret_cast<const int32_t*>(S.src_c[0]));
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = has && ((m >> i) & 1u) ? (int64_t)src[d0 + i] : 1;
      } else {
        gmem<int64_t>* __restrict__ src = gp(S.src_c[0]);
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = has && ((m >> i) & 1u) ? src[d0 + i] : 1;
      }
#ifndef PGPU_STAR_NO_SECTORS
      if (has) sectors += nar ? sec4 : sec8;
#endif
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if ((m >> i) & 1u) atomicAdd(reinterpret_cast<unsigned long long*>(row + key[i]), (unsigned long long)c[i]);
      continue;
    }
    double v[16];
    if ((S.narrow >> s) & 1u) {  // integral values of int32 range: exact as doubles
      gmem<int32_t>* __restrict__ src = gp(reinterpret_cast<const int32_t*>(S.src_f[s]));
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? (double)src[d0 + i] : 0.0;
#ifndef PGPU_STAR_NO_SECTORS
      sectors += sec4;
#endif
    } else {
      gmem<double>* __restrict__ src = gp(S.src_f[s]);
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? src[d0 + i] : 0.0;
#ifndef PGPU_STAR_NO_SECTORS
      sectors += sec8;
#endif
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (!((m >> i) & 1u)) continue;
      int64_t ikey = 0;
      double dval = 0.0;
      if (kind == SLOT_SUM_F64) dval = v[i];
      else if (kind == SLOT_SUM_I64) ikey = (int64_t)v[i];  // sums of integers are exact in double (< 2^53)
      else ikey = p.slot_int[s] ? (int64_t)v[i] : double_key_dev(v[i]);
      accumulate<MODE>(row, key[i], kind, ikey, dval);
    }
  }
}

// Residual-filter bits H..H+15 of group g for dim d (match set in LDS when cached).
template <int H>
__device__ __forceinline__ uint32_t star_match_half(const KStarSeg& S, int d, int64_t g, const int32_t* __restrict__ mset,
                                                    const uint32_t* __restrict__ gset) {
  uint32_t ids[16];
  star_decode<H>(S.dim_fwd[d], S.dim_bits[d], g, ids);
  uint32_t w[16];
  if (mset) {
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = (uint32_t)mset[ids[i] >> 5];
  } else {
    gmem<uint32_t>* g = gp(gset);
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = g[ids[i] >> 5];
  }
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) m |= ((w[i] >> (ids[i] & 31)) & 1u) << (H + i);
  return m;
}

// K6: persistent workgroups over the concatenated 32-doc groups of every segment's emitted ranges (each workgroup a
// contiguous run, so it crosses at most a few segment boundaries and flushes its table slab once).  Per segment the
// workgroup stages the key LUTs, residual match sets and the ranges with their group prefix in LDS; each lane then
// takes one group at a time, decodes the residual dims into a 32-bit match mask, decodes the group-by dims of the
// matching docs 16 at a time and adds their pre-aggregated metrics.
template <int MODE>
__global__ __launch_bounds__(StarBlock<MODE>::value) void startree_scan_kernel(const KStarParams p) {
  constexpr int BLOCK = StarBlock<MODE>::value;
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  __shared__ int64_t wsum[BLOCK / 64];
  const int tid = threadIdx.x;
  if (p.deadline && p.stats[5]) return;  // end time passed before the traversal ran (K5 set the flag)
  const int64_t G = p.num_keys_total;
  const int64_t words = MODE == MODE_LDS ? (int64_t)p.num_slots * G : 0;
  if (MODE == MODE_LDS)
    for (int64_t i = tid; i < words; i += BLOCK) lds[i] = slot_init(p.slot_kind[i / G]);
  uint64_t* tbl = MODE == MODE_LDS ? lds : p.table;
  // LDS after the table: group prefix over segments [num_segs + 1], then per segment the ranges' group prefix
  // [range_cache + 1] and (start, end) pairs [range_cache], then the LUT / match-set cache
  int64_t* segpre = reinterpret_cast<int64_t*>(lds + ((words + 1) & ~int64_t(1)));
  int64_t* rpre = segpre + ((p.num_segs + 2) & ~1);
  int32_t* rdoc = reinterpret_cast<int32_t*>(rpre + ((p.range_cache + 2) & ~1));
  int32_t* cache = rdoc + ((2 * p.range_cache + 3) & ~3);
  // segment prefix: per thread a slice, wave sums, then the block
  {
    const int per = (p.num_segs + BLOCK - 1) / BLOCK;
    const int s0 = tid * per;
    int64_t acc = 0;
    for (int i = 0; i < per && s0 + i < p.num_segs; ++i) acc += gp(p.seg_total)[s0 + i];
    int64_t inc = acc;  // inclusive scan within the wave
    const int lane = tid & 63;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    int64_t wbase = 0;
    for (int w = 0; w < (tid >> 6); ++w) wbase += wsum[w];
    int64_t run = wbase + inc - acc;  // exclusive prefix of this thread's slice
    if (tid == 0) segpre[0] = 0;
    for (int i = 0; i < per && s0 + i < p.num_segs; ++i) {
      run += gp(p.seg_total)[s0 + i];
      segpre[s0 + i + 1] = run;
    }
  }
  __syncthreads();
  const int64_t total = segpre[p.num_segs];
  const int64_t glo = (int64_t)blockIdx.x * total / p.num_wgs, ghi = (int64_t)(blockIdx.x + 1) * total / p.num_wgs;
  unsigned long long matched = 0, scanned = 0, read = 0;  // read: star-tree documents of the emitted ranges
  unsigned long long sectors = 0;  // metric-array sectors holding a matched doc (bytes model)
  // first segment of the run: binary search over the LDS prefix
  int seg = 0;
  {
    int b = p.num_segs - 1;
    while (seg < b) {
      const int mid = (seg + b + 1) >> 1;
      if (segpre[mid] <= glo) seg = mid;
      else b = mid - 1;
    }
  }
  for (; seg < p.num_segs && segpre[seg] < ghi; ++seg) {
    const int64_t lo = max(glo, segpre[seg]) - segpre[seg], hi = min(ghi, segpre[seg + 1]) - segpre[seg];
    if (lo >= hi) continue;  // workgroup-uniform
    const KStarSeg& S = p.segs[seg];
    const int nr = S.out[0], rem = S.out[1];
    const bool ranges_lds = nr <= p.range_cache;
    const bool cached = p.cache_ints > 0;
    int match_base = 0;
    for (int j = 0; j < p.num_keys; ++j) match_base += S.dim_card[S.key_dim[j]];
    __syncthreads();  // the previous segment's LDS copies are no longer read
    if (ranges_lds) {
      for (int r = tid; r <= nr; r += BLOCK) rpre[r] = gp(S.prefix)[r];
      for (int r = tid; r < 2 * nr; r += BLOCK) rdoc[r] = gp(S.ranges)[r];
    }
    if (cached) {
      int off = 0;
      for (int j = 0; j < p.num_keys; ++j) {
        const int card = S.dim_card[S.key_dim[j]];
        for (int i = tid; i < card; i += BLOCK) cache[off + i] = gp(S.key_lut[j])[i];
        off += card;
      }
      for (int r = rem; r; r &= r - 1) {
        const int d = __ffs(r) - 1;
        const int nw = (S.dim_card[d] + 31) >> 5;
        for (int i = tid; i < nw; i += BLOCK) cache[off + i] = (int32_t)gp(S.match[d])[i];
        off += nw;
      }
    }
    __syncthreads();
    // ranges from LDS when staged, else from global memory (two typed reads: no FLAT access)
    gmem<int64_t>* gpre = gp(S.prefix);
    gmem<int32_t>* grng = gp(S.ranges);
    auto pre = [&](int i) -> int64_t { return ranges_lds ? rpre[i] : gpre[i]; };
    auto rng = [&](int i) -> int32_t { return ranges_lds ? rdoc[i] : grng[i]; };
    const int nrem = __popc(rem);
    // the lane's range cursor only moves forward: one binary search, then registers
    int a = 0;
    int64_t next = INT64_MAX, first = 0;
    int32_t rb = 0, re = 0;
    if (lo + tid < hi) {
      int b = nr - 1;
      const int64_t pos = lo + tid;
      while (a < b) {
        const int mid = (a + b + 1) >> 1;
        if (pre(mid) <= pos) a = mid;
        else b = mid - 1;
      }
      rb = rng(2 * a);
      re = rng(2 * a + 1);
      first = pre(a);
      next = a + 1 < nr ? pre(a + 1) : INT64_MAX;
    }
    for (int64_t base = lo; base < hi; base += BLOCK) {
      const int64_t pos = base + tid;
      uint32_t mask = 0;
      int64_t g = 0;
      if (pos < hi) {
        while (pos >= next) {
          ++a;
          rb = rng(2 * a);
          re = rng(2 * a + 1);
          first = next;
          next = a + 1 < nr ? pre(a + 1) : INT64_MAX;
        }
        g = (rb >> 5) + (pos - first);
        const int64_t d0 = g * 32;
        const int64_t lo_doc = rb > d0 ? rb - d0 : 0, hi_doc = re - d0 < 32 ? re - d0 : 32;
        mask = hi_doc > lo_doc
                   ? (uint32_t)((hi_doc - lo_doc == 32 ? ~0ull : ((1ull << (hi_doc - lo_doc)) - 1)) << lo_doc)
                   : 0u;
      }
      const int in_range = __popc(mask);
      read += in_range;
      scanned += (unsigned long long)in_range * nrem;
      int moff = match_base;
      for (int r = rem; r; r &= r - 1) {
        const int d = __ffs(r) - 1;
        const int32_t* mset = cached ? cache + moff : nullptr;
        const uint32_t m =
            star_match_half<0>(S, d, g, mset, S.match[d]) | star_match_half<16>(S, d, g, mset, S.match[d]);
        mask &= m;
        moff += (S.dim_card[d] + 31) >> 5;
      }
      matched += __popc(mask);
      if (__any((mask & 0xFFFFu) != 0u)) star_aggregate_half<MODE, 0>(p, S, g, mask, cache, cached, tbl, G, sectors);
      if (__any((mask >> 16) != 0u)) star_aggregate_half<MODE, 16>(p, S, g, mask, cache, cached, tbl, G, sectors);
    }
  }
  {
    const int idx[4] = {0, 1, 3, 7};
    unsigned long long v[4] = {(unsigned long long)matched, (unsigned long long)scanned, (unsigned long long)read,
                               sectors};
    block_stats_add<4, BLOCK>(p.stats, idx, v);
  }
  if (MODE == MODE_LDS) {
    __syncthreads();
    uint64_t* o = p.slab + (int64_t)blockIdx.x * words;
    for (int64_t i = tid; i < words; i += BLOCK) o[i] = lds[i];
  }
}

}  // namespace pgpu
