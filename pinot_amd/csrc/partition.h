// partition.h — partitioned group-by for large dense key spaces (C5: ~10M groups, a 160 MB table).
//
// Random 64-bit atomics into a table far larger than L2 execute at the memory side, one 64-B request per lane
// (MI355X_MICROARCH.md, "Global float atomics"), which made the direct kernel's C5 scan ~20x slower than its
// bytes.  Instead the matched docs are radix-partitioned by the high bits of their composite key, and each
// partition (a key range whose accumulators fit in LDS) is aggregated by one workgroup with LDS atomics and
// written to the dense table with plain coalesced stores:
//
//   K8a part_count    : filter + key per matched doc; per-workgroup LDS histogram over partitions; each
//                       workgroup reserves its run in every partition with one atomic per non-empty partition.
//   K8b (scan)        : exclusive scan of the partition totals (compact_scan_kernel).
//   K8c part_scatter  : the same docs again (same tile assignment); each record (key mod partition width as u16,
//                       one 8-byte operand per value stream) goes to its partition run via an LDS cursor.
//   K8d part_aggregate: one workgroup per partition: LDS table, LDS atomics over its records, then the
//                       partition's slice of every table row stored whole (no table init, no global atomics).
//
// Replaces the same reference code as the direct kernel (DictionaryBasedGroupKeyGenerator INT_MAP holder +
// aggregateGroupBySV + GroupByCombineOperator merge); results are identical (integer
// accumulators exact; double sums within the path's 1e-9 relative bound — their order is not fixed).
#pragma once
#include "device.h"

namespace pgpu {

// KPartParams: internal.h.

// Static tile range of workgroup b (K8a and K8c must visit the same docs in the same order).
__device__ __forceinline__ void part_tiles(int64_t T, int64_t& t0, int64_t& t1) {
  t0 = (int64_t)blockIdx.x * T / gridDim.x;
  t1 = (int64_t)(blockIdx.x + 1) * T / gridDim.x;
}

// Composite keys of docs [32*group + H, +16) of segment S.
template <int H>
__device__ __forceinline__ void part_keys(const KParams& p, const SegView& S, int64_t group, int32_t (&key)[16]) {
  uint32_t ids[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) key[i] = 0;
  for (int j = 0; j < p.num_keys; ++j) {
    const KCol& c = S.cols[p.key_col[j]];
    decode_group<H>(c.fwd, c.bits, group, ids);
    const int32_t* __restrict__ lut = c.lut;
    const int32_t stride = (int32_t)p.key_stride[j];
    int32_t g[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) g[i] = lut[ids[i]];
#pragma unroll
    for (int i = 0; i < 16; ++i) key[i] += g[i] * stride;
  }
}

template <int H>
__device__ __forceinline__ void part_scatter_half(const KPartParams& pp, const SegView& S, int64_t group,
                                                  uint32_t m, uint32_t* cursor) {
  const KParams& p = pp.base;
  int32_t key[16];
  part_keys<H>(p, S, group, key);
  uint32_t pos[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    pos[i] = 0;
    if ((m >> i) & 1u) {
      pos[i] = atomicAdd(&cursor[key[i] >> pp.pshift], 1u);
      pp.rec_key[pos[i]] = (uint16_t)(key[i] & ((1 << pp.pshift) - 1));
    }
  }
  uint32_t ids[16];
  for (int s = 0; s < pp.num_streams; ++s) {
    const KCol& c = S.cols[pp.stream_col[s]];
    decode_group<H>(c.fwd, c.bits, group, ids);
    uint64_t* __restrict__ out = pp.rec_val + (int64_t)s * pp.rec_cap;
    if (pp.stream_f64[s]) {
      const double* __restrict__ dv = c.dval;
      double v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? dv[ids[i]] : 0.0;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if ((m >> i) & 1u) out[pos[i]] = (uint64_t)__double_as_longlong(v[i]);
    } else {
      const int64_t* __restrict__ dk = c.dkey;
      int64_t v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? dk[ids[i]] : 0;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if ((m >> i) & 1u) out[pos[i]] = (uint64_t)v[i];
    }
  }
}

template <int H>
__device__ __forceinline__ void part_count_half(const KPartParams& pp, const SegView& S, int64_t group, uint32_t m,
                                                uint32_t* hist) {
  int32_t key[16];
  part_keys<H>(pp.base, S, group, key);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((m >> i) & 1u) atomicAdd(&hist[key[i] >> pp.pshift], 1u);
}

// K8a (SCATTER = false) / K8c (SCATTER = true).  LDS: [num_parts u32 histogram / cursors] [filter stack].
template <bool SCATTER>
__global__ __launch_bounds__(kBlock) void part_pass_kernel(const KPartParams pp) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const KParams& p = pp.base;
  const int tid = threadIdx.x;
  uint32_t* hist = reinterpret_cast<uint32_t*>(lds);
  uint32_t* stack = hist + ((pp.num_parts + 3) & ~3);
  for (int i = tid; i < pp.num_parts; i += kBlock)
    hist[i] = SCATTER ? pp.part_start[i] + pp.block_off[(int64_t)blockIdx.x * pp.num_parts + i] : 0u;
  __syncthreads();
  int64_t t0, t1;
  part_tiles(p.num_tiles, t0, t1);
  unsigned long long matched = 0;
  int seg = -1;
  SegView S{};
  int64_t tile_base = 0;
  int nd = 0;
  for (int64_t t = t0; t < t1; ++t) {
    const int cur = p.tile_seg[t];
    if (cur != seg) {
      seg = cur;
      S = seg_view(p, seg);
      tile_base = S.hdr->tile_base;
      nd = S.hdr->num_docs;
    }
    const int64_t group = (t - tile_base) * kBlock + tid;
    const int64_t ngroups = ((int64_t)nd + 31) >> 5;
    const int64_t doc0 = group << 5;
    uint32_t mask = doc0 >= nd ? 0u : (nd - doc0 >= 32 ? ~0u : ((1u << (nd - doc0)) - 1u));
    const int64_t gclamp = group < ngroups ? group : ngroups - 1;
    mask = eval_filter(p, S, gclamp, mask, stack);
    matched += __popc(mask);
    if (!__any(mask != 0u)) continue;
    if (SCATTER) {
      if (__any((mask & 0xFFFFu) != 0u)) part_scatter_half<0>(pp, S, gclamp, mask & 0xFFFFu, hist);
      if (__any((mask >> 16) != 0u)) part_scatter_half<16>(pp, S, gclamp, mask >> 16, hist);
    } else {
      if (__any((mask & 0xFFFFu) != 0u)) part_count_half<0>(pp, S, gclamp, mask & 0xFFFFu, hist);
      if (__any((mask >> 16) != 0u)) part_count_half<16>(pp, S, gclamp, mask >> 16, hist);
    }
  }
  if (!SCATTER) {
    for (int off = 32; off > 0; off >>= 1) matched += __shfl_xor(matched, off);
    if ((tid & 63) == 0 && matched) atomicAdd(p.stats, matched);
    __syncthreads();
    // reserve this workgroup's run inside every partition it touches
    for (int i = tid; i < pp.num_parts; i += kBlock) {
      const uint32_t h = hist[i];
      pp.block_off[(int64_t)blockIdx.x * pp.num_parts + i] = h ? atomicAdd(&pp.part_start[i], h) : 0u;
    }
  }
}

// K8d: partition blockIdx.x -> its key range of every table row.  LDS: [num_slots][1 << pshift] u64.
__global__ __launch_bounds__(kBlock) void part_aggregate_kernel(const KPartParams pp) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const KParams& p = pp.base;
  const int tid = threadIdx.x;
  const int PR = 1 << pp.pshift;
  const int ns = p.num_slots;
  for (int i = tid; i < ns * PR; i += kBlock) lds[i] = slot_init(p.slot_kind[i / PR]);
  __syncthreads();
  const uint32_t r0 = pp.part_start[blockIdx.x], r1 = pp.part_start[blockIdx.x + 1];
  for (uint32_t r = r0 + tid; r < r1; r += kBlock) {
    const int k = pp.rec_key[r];
    for (int s = 0; s < ns; ++s) {
      const int kind = p.slot_kind[s];
      const int st = pp.slot_stream[s];
      const uint64_t w = st >= 0 ? pp.rec_val[(int64_t)st * pp.rec_cap + r] : 0ull;
      accumulate<MODE_LDS>(lds + (int64_t)s * PR, k, kind, (int64_t)w, __longlong_as_double((long long)w));
    }
  }
  __syncthreads();
  const int64_t G = p.num_keys_total;
  const int64_t k0 = (int64_t)blockIdx.x * PR;
  const int n = (int)(G - k0 < PR ? G - k0 : PR);
  for (int s = 0; s < ns; ++s)
    for (int i = tid; i < n; i += kBlock) p.table[(int64_t)s * G + k0 + i] = lds[(int64_t)s * PR + i];
}

}  // namespace pgpu
