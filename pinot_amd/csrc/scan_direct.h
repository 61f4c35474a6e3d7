// scan_direct.h — the fused filter / group-by / aggregation scan (K1+K2+K3) with direct loads: the kernel of
// the path.  Instantiated once per accumulator mode in k_direct.hip.
#pragma once
#include "device.h"

namespace pgpu {

// numEntriesScannedInFilter of an AND of two scans A, B (AndDocIdIterator.java:40-67 over SVScanDocIdIterators):
// the iterators hand the scan back and forth, so each doc is scanned once, plus once more when the scanner at that
// doc matches it (the other iterator then evaluates the same doc).  Scanner state after a doc: B after a doc A
// matches and B does not, A after a doc B matches, unchanged otherwise.  The lane builds that state for its 32 docs
// with a 5-step segmented fill (for both possible entry states), the wave composes its 64 lanes in order, and
// lane 0 stores the wave's map (leap2_compose_kernel chains the maps of a segment).
__device__ __forceinline__ void leap2_wave_map(uint64_t* __restrict__ maps, int64_t slot, int lane, uint32_t a,
                                               uint32_t b, uint32_t v) {
  a &= v;
  b &= v;
  const uint32_t e = a | b;
  uint32_t fill = a & ~b, seen = e;  // state after doc i: B (1) / A (0) where some event at or before i
#pragma unroll
  for (int k = 1; k < 32; k <<= 1) {
    fill |= (fill << k) & ~seen;
    seen |= seen << k;
  }
  const uint32_t before_a = fill << 1;                       // state before each doc, entering in A
  const uint32_t before_b = ((fill | ~seen) << 1) | 1u;      // ... entering in B
  const uint32_t nv = __popc(v);
  uint32_t c0 = nv + __popc((a & ~before_a) | (b & before_a));
  uint32_t c1 = nv + __popc((a & ~before_b) | (b & before_b));
  uint32_t ex = e ? ((fill >> 31) & 1u) * 3u : 2u;           // bit s: exit state from entry s
  for (int off = 1; off < 64; off <<= 1) {                   // ordered composition: left = this lane's range
    const uint32_t r0 = __shfl_down(c0, off), r1 = __shfl_down(c1, off), re = __shfl_down(ex, off);
    const uint32_t m0 = ex & 1u, m1 = (ex >> 1) & 1u;
    const uint32_t n0 = c0 + (m0 ? r1 : r0), n1 = c1 + (m1 ? r1 : r0);
    const uint32_t ne = ((re >> m0) & 1u) | (((re >> m1) & 1u) << 1);
    if ((lane & (2 * off - 1)) == 0) { c0 = n0; c1 = n1; ex = ne; }
  }
  if (lane == 0) maps[slot] = (uint64_t)c0 | ((uint64_t)c1 << 24) | ((uint64_t)ex << 48);
}

// ---------------------------------------------------------------------------------------------- K3 fused
// DENSE: the plan expects dense tiles (estimated selectivity >= 1/16): wave-tiles with >= kDenseGroupMin matches
// decode whole groups of the group-by / aggregated columns (aggregate_group).  A separate instance because that
// path needs ~45 more VGPRs, which would halve the occupancy of the sparse path.
template <int MODE, bool DENSE>
#ifndef PGPU_MIN_WAVES
#define PGPU_MIN_WAVES 1
#endif
__global__ __launch_bounds__(kBlock, DENSE ? 3 : PGPU_MIN_WAVES) void filter_groupby_kernel(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t G = p.num_keys_total;
  const int64_t table_words = (MODE == MODE_LDS) ? (int64_t)p.num_slots * G : 0;
  uint32_t* stack = reinterpret_cast<uint32_t*>(lds + table_words);
  // per-wave queue of sparse matches ((doc, segment) pairs), after the filter stack
  uint32_t* wq = stack + (p.pure_and ? 0 : kMaxStack * kBlock) + wave * 2 * kWaveQ;
  uint32_t* wqs = wq + kWaveQ;
  uint32_t qn = 0;  // wave-uniform fill

  if (MODE == MODE_LDS) {
    for (int64_t i = tid; i < table_words; i += kBlock) lds[i] = slot_init(p.slot_kind[i / G]);
    __syncthreads();
  }
  uint64_t* tbl = (MODE == MODE_LDS) ? lds : p.table;

  // XCD-aware tile order: workgroups b and b+8 share an XCD (round-robin dispatch; speed only, never correctness),
  // so XCD x sweeps its own contiguous eighth of the tile space with its workgroups side by side, one tile each.
  // The tiles in flight on an XCD then come from ~one segment at a time and that segment's dictionaries / LUTs
  // (the targets of the gathers) stay in the XCD's 4 MiB L2.
  unsigned long long matched = 0;
  uint32_t in_filter = 0;  // STATS_CHAIN entries of this lane (< 2^32: at most 4 leaves x 32 docs x tiles)
  const int64_t T = p.num_tiles;
  int64_t t_begin, t_end, t_step;
  if (gridDim.x >= 64 && (gridDim.x & 7) == 0) {
    const int64_t x = blockIdx.x & 7;
    t_begin = x * T / 8 + (blockIdx.x >> 3);
    t_end = (x + 1) * T / 8;
    t_step = gridDim.x >> 3;
  } else {
    t_begin = (int64_t)blockIdx.x * T / gridDim.x;
    t_end = (int64_t)(blockIdx.x + 1) * T / gridDim.x;
    t_step = 1;
  }
  const bool fast = p.pure_and && p.num_leaves <= kFastLeaves;
  if (t_begin < t_end) {
    int seg = -1;
    SegView S{};
    int64_t tile_base = 0;
    int nd = 0;
    int stats = 0;  // the segment's KSegHdr.stats
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
    int next_seg = p.tile_seg[t_begin];
    for (int64_t t = t_begin; t < t_end; t += t_step) {
      const int cur_seg = next_seg;
      if (t + t_step < t_end) next_seg = p.tile_seg[t + t_step];  // one tile ahead
      if (cur_seg != seg) {
        seg = cur_seg;
        S = seg_view(p, seg);
        tile_base = S.hdr->tile_base;
        nd = S.hdr->num_docs;
        stats = S.hdr->stats;
        if (fast) PGPU_LOAD_LEAVES();
      }
      const int64_t group = (t - tile_base) * kBlock + tid;
      const int64_t ngroups = ((int64_t)nd + 31) >> 5;
      const int64_t doc0 = group << 5;
      uint32_t mask = doc0 >= nd ? 0u : (nd - doc0 >= 32 ? ~0u : ((1u << (nd - doc0)) - 1u));
      const int64_t gclamp = group < ngroups ? group : ngroups - 1;
      if (fast && (stats & 3) == KSTATS_LEAP2) {
        // two scans in leap-frog: both masks are needed for the entry count, no early exit
        const uint32_t v = mask;
        const int la = (stats >> 8) & 3, lb = (stats >> 10) & 3;
        uint32_t ma = 0, mb = 0;
        for (int l = 0; l < nl; ++l) {
          const LeafReg& r = l == 0 ? R0 : l == 1 ? R1 : l == 2 ? R2 : R3;
          const uint32_t m = leaf_mask_reg(r, gclamp);
          ma = l == la ? m : ma;
          mb = l == lb ? m : mb;
          mask &= m;
        }
        leap2_wave_map(p.leap_maps, t * (kBlock / 64) + wave, lane, ma, mb, v);
      } else if (fast) {
        for (int l = 0; l < nl; ++l) {
          if (!__any(mask != 0u)) break;  // AndDocIdIterator never scans past an empty child
          // applyAnd of a scan after the index leaves (AndDocIdSet.java:124-126): its input docs are its entries
          if ((stats >> (4 + l)) & 1) in_filter += __popc(mask);
          const LeafReg& r = l == 0 ? R0 : l == 1 ? R1 : l == 2 ? R2 : R3;
          mask &= leaf_mask_reg(r, gclamp);
        }
      } else {
        mask = eval_filter(p, S, gclamp, mask, stack);
      }
      const uint32_t cnt = __popc(mask);
      matched += cnt;
      uint32_t wave_cnt = 0;
      if (DENSE && MODE != MODE_HASH) {
        wave_cnt = cnt;
        for (int off = 32; off > 0; off >>= 1) wave_cnt += __shfl_xor(wave_cnt, off);
      }
      if (DENSE && MODE != MODE_HASH && wave_cnt >= (uint32_t)kDenseGroupMin) {
        // dense tile: whole-group decode of the group-by / aggregated columns
        aggregate_group<MODE>(p, S, gclamp, mask, tbl, G);
      } else if (__any(cnt > 2u)) {
        // dense: the lane's own 32-doc group, 2 matched docs per batch (the lines are already cached)
        while (__any(mask != 0u)) {
          int64_t doc[2];
          bool ok[2];
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            ok[b] = mask != 0u;
            doc[b] = ok[b] ? doc0 + (__ffs(mask) - 1) : 0;
            mask &= mask - 1u;
          }
          const SegView SS[2] = {S, S};
          aggregate_batch<MODE, 2>(p, SS, doc, ok, tbl, G);
        }
      } else if (__any(mask != 0u)) {
        // sparse: append to the wave's queue (<= 2 per lane, so <= 128 per tile), aggregate in batches
        while (__any(mask != 0u)) {
          const bool has = mask != 0u;
          const uint64_t bal = __ballot(has);
          if (has) {
            const uint32_t pos = qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            wq[pos] = (uint32_t)(doc0 + (__ffs(mask) - 1));
            wqs[pos] = (uint32_t)seg;
            mask &= mask - 1u;
          }
          qn += (uint32_t)__popcll(bal);
        }
        if (qn >= (uint32_t)kFlushAt) {
          flush_wave_queue<MODE>(p, wq, wqs, qn, lane, tbl, G);
          qn = 0;
        }
      }
    }
    if (qn) flush_wave_queue<MODE>(p, wq, wqs, qn, lane, tbl, G);
  }
  // numDocsScanned: wave reduce, one atomic per wave.
  for (int off = 32; off > 0; off >>= 1) matched += __shfl_xor(matched, off);
  if ((tid & 63) == 0 && matched) atomicAdd(p.stats, matched);
  unsigned long long entries = in_filter;
  for (int off = 32; off > 0; off >>= 1) entries += __shfl_xor(entries, off);
  if ((tid & 63) == 0 && entries) atomicAdd(p.stats + 2, entries);

  if (MODE == MODE_LDS) {
    __syncthreads();
    uint64_t* out = p.slab + (int64_t)blockIdx.x * table_words;
    for (int64_t i = tid; i < table_words; i += kBlock) out[i] = lds[i];
  }
}

}  // namespace pgpu
