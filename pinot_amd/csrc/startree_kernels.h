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
// every emitted range are split over `chunks_per_seg` workgroups per segment; metrics come from the pre-aggregated
// "fn__col" arrays (COUNT adds count__*: CountAggregationFunction.java:97-104).
#pragma once
#include "device.h"

namespace pgpu {

__device__ __forceinline__ int64_t double_key_dev(double d) {  // order-preserving int64 of an IEEE double
  const int64_t b = __double_as_longlong(d);
  return b >= 0 ? b : (b ^ INT64_MAX);
}

#if PGPU_MODE == 0  // one definition: the mode-0 object
__global__ __launch_bounds__(256) void startree_traverse_kernel(const KStarSeg* __restrict__ segs) {
  const KStarSeg& S = segs[blockIdx.x];
  __shared__ int cur_n, next_n, nr, rem;
  const int tid = threadIdx.x;
  const int* __restrict__ nodes = S.nodes;
  int* fa = S.frontier;
  int* fb = S.frontier + 3 * S.num_nodes;
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
    for (int i = tid; i < n; i += blockDim.x) {
      const int node = fa[3 * i], rp = fa[3 * i + 1], rg = fa[3 * i + 2];
      const int* N = nodes + 7 * (int64_t)node;
      const int first = N[5], last = N[6];
      if (rp == 0 && rg == 0) {  // all predicates and group-by dims matched: the aggregated document
        const int r = atomicAdd(&nr, 1);
        S.ranges[2 * r] = N[4];
        S.ranges[2 * r + 1] = N[4] + 1;
      } else if (first < 0) {  // leaf: its documents, with the remaining predicates as a residual filter
        const int r = atomicAdd(&nr, 1);
        S.ranges[2 * r] = N[2];
        S.ranges[2 * r + 1] = N[3];
        atomicOr(&rem, rp);
      } else {
        const int cd = nodes[7 * (int64_t)first];  // getChildDimensionId
        const int bit = 1 << cd;
        if (rp & bit) {  // predicate on the next dimension: children whose dictId matches
          const uint32_t* m = S.match[cd];
          for (int c = first; c <= last; ++c) {
            const int v = nodes[7 * (int64_t)c + 1];
            if (v >= 0 && ((m[v >> 5] >> (v & 31)) & 1u)) {
              const int k = atomicAdd(&next_n, 1);
              fb[3 * k] = c;
              fb[3 * k + 1] = rp & ~bit;
              fb[3 * k + 2] = rg;
            }
          }
        } else {
          int nrg = rg;
          bool expand = true;
          if (!(rg & bit)) {  // neither predicate nor group-by: the star child when it exists
            if (nodes[7 * (int64_t)first + 1] == -1) {
              const int k = atomicAdd(&next_n, 1);
              fb[3 * k] = first;
              fb[3 * k + 1] = rp;
              fb[3 * k + 2] = rg;
              expand = false;
            }
          } else {
            nrg = rg & ~bit;
          }
          if (expand)
            for (int c = first; c <= last; ++c) {
              if (nodes[7 * (int64_t)c + 1] == -1) continue;
              const int k = atomicAdd(&next_n, 1);
              fb[3 * k] = c;
              fb[3 * k + 1] = rp;
              fb[3 * k + 2] = nrg;
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
  if (tid == 0) {
    int64_t acc = 0;
    S.prefix[0] = 0;
    for (int r = 0; r < nr; ++r) {
      acc += S.ranges[2 * r + 1] - S.ranges[2 * r];
      S.prefix[r + 1] = acc;
    }
    S.out[0] = nr;
    S.out[1] = rem;
  }
}
#endif

template <int MODE>
__global__ __launch_bounds__(256) void startree_scan_kernel(const KStarParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const int tid = threadIdx.x;
  const int64_t G = p.num_keys_total;
  const int64_t words = (int64_t)p.num_slots * G;
  if (MODE == MODE_LDS) {
    for (int64_t i = tid; i < words; i += blockDim.x) lds[i] = slot_init(p.slot_kind[i / G]);
    __syncthreads();
  }
  uint64_t* tbl = MODE == MODE_LDS ? lds : p.table;
  const int seg = blockIdx.x / p.chunks_per_seg, chunk = blockIdx.x % p.chunks_per_seg;
  const KStarSeg& S = p.segs[seg];
  const int nr = S.out[0], rem = S.out[1];
  const int64_t T = S.prefix[nr];
  const int64_t lo = (int64_t)chunk * T / p.chunks_per_seg, hi = (int64_t)(chunk + 1) * T / p.chunks_per_seg;
  unsigned long long matched = 0, scanned = 0, read = 0;  // read: star-tree documents of the emitted ranges
  const int nrem = __popc(rem);
  // Each lane walks positions lo + tid + k * 256 in batches of NB, every dependent level (range -> doc ->
  // residual dictIds -> group keys / pre-aggregated values) issued for the whole batch before it is consumed.
  // The range index only moves forward, so the binary search runs once per lane.
  constexpr int NB = 4;
  int a = 0;
  {
    int b = nr - 1;
    const int64_t pos = lo + tid;
    while (a < b) {
      const int mid = (a + b + 1) >> 1;
      if (S.prefix[mid] <= pos) a = mid;
      else b = mid - 1;
    }
  }
  for (int64_t base = lo + tid; base < hi; base += (int64_t)NB * blockDim.x) {
    int64_t doc[NB];
    bool ok[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int64_t pos = base + (int64_t)k * blockDim.x;
      ok[k] = pos < hi;
      if (ok[k]) {
        while (a + 1 < nr && S.prefix[a + 1] <= pos) ++a;
        doc[k] = S.ranges[2 * a] + (pos - S.prefix[a]);
      } else {
        doc[k] = S.ranges[0];
      }
      scanned += ok[k] ? nrem : 0;
      read += ok[k] ? 1 : 0;
    }
    for (int r = rem; r; r &= r - 1) {
      const int d = __ffs(r) - 1;
      uint32_t id[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) id[k] = gather_id(S.dim_fwd[d], S.dim_bits[d], doc[k]);
#pragma unroll
      for (int k = 0; k < NB; ++k) ok[k] = ok[k] && ((S.match[d][id[k] >> 5] >> (id[k] & 31)) & 1u) != 0;
    }
    int64_t key[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) { key[k] = 0; matched += ok[k] ? 1 : 0; }
    for (int j = 0; j < p.num_keys; ++j) {
      const int d = S.key_dim[j];
      uint32_t id[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) id[k] = gather_id(S.dim_fwd[d], S.dim_bits[d], doc[k]);
#pragma unroll
      for (int k = 0; k < NB; ++k) key[k] += (int64_t)S.key_lut[j][id[k]] * p.key_stride[j];
    }
    int64_t idx[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      idx[k] = key[k];
      if (MODE == MODE_HASH && ok[k]) idx[k] = hash_slot(p.hash_keys, G, (uint64_t)key[k]);
    }
    for (int s = 0; s < p.num_slots; ++s) {
      const int kind = p.slot_kind[s];
      if (kind == SLOT_COUNT) {
        // COUNT adds the pre-aggregated count (1 per document when the tree has none)
        int64_t c[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) c[k] = S.src_c[0] ? S.src_c[0][doc[k]] : 1;
#pragma unroll
        for (int k = 0; k < NB; ++k)
          if (ok[k]) atomicAdd(reinterpret_cast<unsigned long long*>(tbl + (int64_t)s * G + idx[k]), (unsigned long long)c[k]);
        continue;
      }
      double v[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) v[k] = S.src_f[s][doc[k]];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        if (!ok[k]) continue;
        int64_t ikey = 0;
        double dval = 0.0;
        if (kind == SLOT_SUM_F64) dval = v[k];
        else if (kind == SLOT_SUM_I64) ikey = (int64_t)v[k];  // sums of integers are exact in double (< 2^53)
        else ikey = p.slot_int[s] ? (int64_t)v[k] : double_key_dev(v[k]);
        accumulate<MODE>(tbl, (int64_t)s * G + idx[k], kind, ikey, dval);
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    matched += __shfl_xor(matched, off);
    scanned += __shfl_xor(scanned, off);
    read += __shfl_xor(read, off);
  }
  if ((tid & 63) == 0) {
    if (matched) atomicAdd(p.stats, matched);
    if (scanned) atomicAdd(p.stats + 1, scanned);
    if (read) atomicAdd(p.stats + 3, read);
  }
  if (MODE == MODE_LDS) {
    __syncthreads();
    uint64_t* o = p.slab + (int64_t)blockIdx.x * words;
    for (int64_t i = tid; i < words; i += blockDim.x) o[i] = lds[i];
  }
}

}  // namespace pgpu
