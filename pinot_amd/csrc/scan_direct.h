// scan_direct.h — the fused filter / group-by / aggregation scan (K1+K2+K3) with direct loads: the kernel of
// the path.  Instantiated once per accumulator mode in k_direct.hip.
#pragma once
#include "device.h"

namespace pgpu {

// numEntriesScannedInFilter of an AND of two scans A, B (AndDocIdIterator.java:40-67 over SVScanDocIdIterators):
// the iterators hand the scan back and forth, so each doc is scanned once, plus once more when the scanner at that
// doc matches it (the other iterator then evaluates the same doc).  Scanner after a doc: B after a doc A matches
// and B does not, A after a doc B matches, unchanged otherwise -- so only a group's first matching doc depends on
// the scanner the group is entered with.  Each lane builds the scanner state over its 32 docs (5-step segmented
// fill), counts its entries with the entry state the wave's ballots give it (the exit of the previous lane with a
// match), and the wave stores one byte for the rest: whether it has a match, its exit state, and the count
// difference at its first match between entering in B and in A (leap2_compose_kernel chains the bytes of a
// segment in doc order).  The byte goes to the workgroup's LDS list (one per tile and wave), stored to global
// memory once after the tile loop.  Returns the lane's entries (entering the wave in A).
__device__ __forceinline__ uint32_t leap2_entries(uint8_t* __restrict__ maps, int64_t slot, int lane, uint32_t a,
                                                  uint32_t b, uint32_t v) {
  a &= v;
  b &= v;
  const uint32_t e = a | b;
  // scanner after doc i: B (1) where the last matching doc <= i matched A only, A (0) otherwise -- the A-only docs'
  // ones carried up through the docs B does not match, by one addition (a set bit p of y inside a run of ~b ones
  // flips the run from p up, so (~b + y) ^ ~b marks it; y's own bits are put back for runs holding several)
  const uint32_t y = a & ~b, nb = ~b;
  const uint32_t fill = (nb & ((nb + y) ^ nb)) | y;
  const uint32_t before = fill << 1;  // scanner before each doc, entering in A
  uint32_t c = __popc(v) + __popc((a & ~before) | (b & before));
  const int f = e ? __builtin_ctz(e) : 0;
  const int d = e ? (int)((b >> f) & 1u) - (int)((a >> f) & 1u) : 0;  // entering in B instead, at the first match
  // wave-wide state from ballots only (scalar masks, no lane shuffles, no divergent branch)
  const uint64_t evm = __ballot(e != 0u), exm = __ballot(e != 0u && (fill >> 31));
  const uint64_t below = evm & ((1ull << lane) - 1ull);
  if (below && ((exm >> (63 - __builtin_clzll(below))) & 1ull)) c += d;
  uint32_t m = 0;
  if (evm) {
    const int first = __builtin_ctzll(evm), last = 63 - __builtin_clzll(evm);
    const int df = __builtin_amdgcn_readlane(d, first);  // the first matching lane's difference
    m = 1u | (uint32_t)(((exm >> last) & 1ull) << 1) | ((uint32_t)(df + 1) << 2);
  }
  if (lane == 0) maps[slot] = (uint8_t)m;  // an LDS slot: global stores inside the tile loop cost the loop registers
  return c;
}

// ---------------------------------------------------------------------------------------------- K3 fused
// DENSE: the plan expects dense tiles (estimated selectivity >= 1/4, rt_plan.cpp): wave-tiles with >= kDenseGroupMin matches
// decode whole groups of the group-by / aggregated columns (aggregate_group).  A separate instance because that
// path needs ~45 more VGPRs, which would halve the occupancy of the sparse path.
// LANE_BATCH: matched docs per aggregate_batch where a lane's 32-doc group has more than 2 -- 4 in the pure-AND sparse
// instance for plans of estimated selectivity >= 1/16 (C4's scan path at 15 %: 174 -> 150 us), 2 elsewhere (4 cost
// C3, where that path is rare, 1.5 % -- 710 -> 722 us -- and the dense instance's C2 2 %).
template <int MODE, bool DENSE, bool SIMPLE = false, bool PAIR = false, bool FAST = false, int LANE_BATCH = 2>
#ifndef PGPU_MIN_WAVES
#define PGPU_MIN_WAVES 1
#endif
#ifndef PGPU_DENSE_MIN_WAVES
#define PGPU_DENSE_MIN_WAVES 4
#endif
#ifndef PGPU_SIMPLE_MIN_WAVES
#define PGPU_SIMPLE_MIN_WAVES 4
#endif
__global__ __launch_bounds__(kBlock, DENSE ? (SIMPLE ? PGPU_SIMPLE_MIN_WAVES : PGPU_DENSE_MIN_WAVES) : PGPU_MIN_WAVES) void filter_groupby_kernel(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t G = p.num_keys_total;
  // MODE_LDS with KParams.pack_slot: no COUNT row in LDS (slot s at row s - 1; the COUNT rides in the pack slot)
  const int lds_row0 = (MODE == MODE_LDS && p.pack_slot >= 0) ? 1 : 0;
  const int64_t table_words = (MODE == MODE_LDS) ? (int64_t)(p.num_slots - lds_row0) * G : 0;
  uint32_t* stack = reinterpret_cast<uint32_t*>(lds + table_words);
  // per-wave queue of sparse matches ((doc, segment) pairs), after the filter stack
  uint32_t* wq = stack + (p.pure_and ? 0 : kMaxStack * kBlock) + wave * 2 * kWaveQ;
  uint32_t* wqs = wq + kWaveQ;
  uint32_t qn = 0;  // wave-uniform fill
  // STATS_LEAP2 bytes of this workgroup's tiles, [tile k of the workgroup][wave], after the match queues
  uint8_t* lmaps = reinterpret_cast<uint8_t*>(stack + (p.pure_and ? 0 : kMaxStack * kBlock) + (kBlock / 64) * 2 * kWaveQ);
  int kk = 0;  // tiles of this workgroup so far
  // The query's end time had passed when the launch came up (expand_tiles_kernel, run just before on the stream,
  // read the device clock and set stats[5]): take no tile.  No clock read in this kernel -- even one outside the
  // tile loop changes the sparse instance's register allocation (108 -> 134 VGPRs, one wave less per SIMD; an
  // in-loop check cost 18% on C3, measured).  A scan already running is abandoned by the host (wait_plan).
  if (p.deadline && p.stats[5]) return;
#ifdef PGPU_SLOT_PRIO
  // (A/B build) the later-dispatched workgroups' waves get the higher issue priority: the SIMDs otherwise issue the
  // oldest wave first and equal shares end in dispatch-slot order
  {
    const int pr = (int)((blockIdx.x * 4u) / gridDim.x);
    if (pr == 1) __builtin_amdgcn_s_setprio(1);
    else if (pr == 2) __builtin_amdgcn_s_setprio(2);
    else if (pr >= 3) __builtin_amdgcn_s_setprio(3);
  }
#endif
#ifdef PGPU_DIAG_WG_TIMES
  const unsigned long long diag_t0 = wall_clock64();
  unsigned long long diag_t1 = 0;
#endif

  if (MODE == MODE_LDS) {
    for (int64_t i = tid; i < table_words; i += kBlock) {
      const int s = (int)(i / G) + lds_row0;
      lds[i] = slot_init_lds(p.slot_kind[s], DENSE && ((p.narrow >> s) & 1u));
    }
    __syncthreads();
  }
  // slot s's row at tbl + s * G; with a packed COUNT, row 0 (tbl itself) is never addressed
  uint64_t* tbl = (MODE == MODE_LDS) ? lds - lds_row0 * G : p.table;

  // XCD-aware tile order: workgroups b and b+8 share an XCD (round-robin dispatch; speed only, never correctness),
  // so XCD x sweeps its own contiguous eighth of the tile space with its workgroups side by side, one tile each.
  // The tiles in flight on an XCD then come from ~one segment at a time and that segment's dictionaries / LUTs
  // (the targets of the gathers) stay in the XCD's 4 MiB L2.
  unsigned long long matched = 0;
  uint32_t in_filter = 0;  // STATS_CHAIN entries of this lane (< 2^32: at most 4 leaves x 32 docs x tiles)
  const int64_t T = p.num_tiles;
  int64_t t_begin, t_end, t_step;
  // run-time claims (chunked plans): the static runs end at claim_base, the rest goes claim_tiles at a time to the
  // workgroups that finish first.  The next claim is issued before the run it follows, so its atomic's round trip
  // overlaps that run's loads; one barrier per run hands it to the other waves.
#ifdef PGPU_TILE_CLAIMS
  const bool dyn = p.claim != nullptr && gridDim.x >= 64 && (gridDim.x & 7) == 0 && p.tile_chunks;
#else
  constexpr bool dyn = false;  // (set_tile_claims, rt_exec.cpp: an A/B build's option, not the default)
#endif
  __shared__ uint32_t claim_at[2];
  uint32_t next_claim = 0;
  if (dyn && tid == 0) next_claim = atomicAdd(p.claim, (uint32_t)p.claim_tiles);
  if (gridDim.x >= 64 && (gridDim.x & 7) == 0 && p.tile_chunks) {
    // chunked: each workgroup a contiguous run of its XCD's eighth -- consecutive tiles of one segment, so the
    // segment's records are read once per run instead of once per tile (plans without per-doc gathers)
    const int64_t TS = dyn ? p.claim_base : T;
    const int64_t x = blockIdx.x & 7, i = blockIdx.x >> 3, nx = gridDim.x >> 3;
    const int64_t lo = x * TS / 8, len = (x + 1) * TS / 8 - lo;
    if (p.slot_n > 1) {
      // weighted by CU slot (KParams.slot_w): the XCD's workgroups i of slot s are i in [nx s / n, nx (s+1) / n)
      auto cum = [&](int64_t j) {  // total weight of the XCD's workgroups [0, j)
        int64_t c = 0;
        for (int s = 0; s < p.slot_n; ++s) {
          const int64_t a = nx * s / p.slot_n, e = nx * (s + 1) / p.slot_n;
          c += (j <= a ? 0 : j < e ? j - a : e - a) * (int64_t)p.slot_w[s];
        }
        return c;
      };
      const int64_t tot = cum(nx);
      t_begin = lo + len * cum(i) / tot;
      t_end = lo + len * cum(i + 1) / tot;
    } else {
      t_begin = lo + i * len / nx;
      t_end = lo + (i + 1) * len / nx;
    }
    t_step = 1;
  } else if (gridDim.x >= 64 && (gridDim.x & 7) == 0) {
    const int64_t x = blockIdx.x & 7;
    t_begin = x * T / 8 + (blockIdx.x >> 3);
    t_end = (x + 1) * T / 8;
    t_step = gridDim.x >> 3;
  } else {
    t_begin = (int64_t)blockIdx.x * T / gridDim.x;
    t_end = (int64_t)(blockIdx.x + 1) * T / gridDim.x;
    t_step = 1;
  }
  // FAST: an instance for plans whose filter is a pure AND of at most kFastLeaves leaves (the general program
  // evaluator compiled out)
  const bool fast = FAST || (p.pure_and && p.num_leaves <= kFastLeaves);
#ifdef PGPU_DIAG_WG_TIMES
  const int64_t diag_first = t_begin;
  int diag_tiles = 0;
#endif
  for (int run = 0;; ++run) {
  if (t_begin < t_end) {
    int seg = -1;
    SegView S{};
    int64_t tile_base = 0;
    int nd = 0;
    int stats = 0;  // the segment's KSegHdr.stats
    // PAIR: the index leaf's directory entry of the current 65536-doc block (8 tiles), wave-uniform
    int32_t pair_blk = -1;
    uint64_t pair_e = 0;
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
    int next_seg = cp(p.tile_seg)[t_begin];
    for (int64_t t = t_begin; t < t_end; t += t_step) {
      const int cur_seg = next_seg;
      if (t + t_step < t_end) next_seg = cp(p.tile_seg)[t + t_step];  // one tile ahead
      if (cur_seg != seg) {
        seg = cur_seg;
        S = seg_view(p, seg);
        tile_base = S.hdr->tile_base;
        nd = S.hdr->num_docs;
        stats = S.hdr->stats;
        pair_blk = -1;
        if (fast) PGPU_LOAD_LEAVES();
      }
      const int64_t lt = t - tile_base;
      const int64_t group = (lt >> p.tile_shift) * kBlock + tid;
      const int64_t ngroups = ((int64_t)nd + 31) >> 5;
      const int64_t doc0 = group << 5;
      uint32_t mask = doc0 >= nd ? 0u : (nd - doc0 >= 32 ? ~0u : ((1u << (nd - doc0)) - 1u));
      if (p.tile_shift) {  // a split tile: this lane's 32 / 2^shift docs of its group
        const int w = 32 >> p.tile_shift;
        mask &= (0xFFFFFFFFu >> (32 - w)) << (w * (int)(lt & ((1 << p.tile_shift) - 1)));
      }
      const int64_t gclamp = group < ngroups ? group : ngroups - 1;
      if (fast) {
        // STATS_LEAP2 (two scans in leap-frog): both masks are needed for the entry count, no early exit
#ifdef PGPU_DIAG_NO_LEAP  // diagnostics build only (wrong numEntriesScannedInFilter): the leap-frog statistics' cost
        const bool leap = false;
#else
        const bool leap = (stats & 3) == KSTATS_LEAP2;
#endif
        const uint32_t v = mask;
        const int la = (stats >> 8) & 3, lb = (stats >> 10) & 3;
        uint32_t ma = 0, mb = 0;
        // (PAIR: a separate instance for plans with index leaves -- compiled into the plain sparse instance, this
        // branch cost C3's scan 1.6 %)
        if (PAIR && !DENSE && !leap && nl == 2 && R0.kind == LEAF_BITDIR && R1.kind == LEAF_RANGE && p.pair_leaves) {
          // index leaf + scan leaf (the indexed C3 shape): both requested together (bitdir_range), applied in order
          uint32_t m0, m1;
          // a tile lies inside one block (256 of its 2048 groups): the block and its entry are wave-uniform
          const int32_t blk = __builtin_amdgcn_readfirstlane((int32_t)(gclamp >> 11));
          if (blk != pair_blk) {
            pair_blk = blk;
            pair_e = reinterpret_cast<const uint64_t*>(R0.set)[blk];
          }
          bitdir_range(R1.fwd, R1.bits, R1.lo, R1.span, R1.negate, pair_e, R0.negate, gclamp, m0, m1);
          if (__any(mask != 0u)) {
            if ((stats >> 4) & 1) in_filter += __popc(mask);
            mask &= m0;
            if (__any(mask != 0u)) {
              if ((stats >> 5) & 1) in_filter += __popc(mask);
              mask &= m1;
            }
          }
        } else
        for (int l = 0; l < nl; ++l) {
          if (!leap && !__any(mask != 0u)) break;  // AndDocIdIterator never scans past an empty child
          // applyAnd of a scan after the index leaves (AndDocIdSet.java:124-126): its input docs are its entries
          if ((stats >> (4 + l)) & 1) in_filter += __popc(mask);
          const LeafReg& r = l == 0 ? R0 : l == 1 ? R1 : l == 2 ? R2 : R3;
          const uint32_t m = leaf_mask_reg(r, gclamp);
          ma = l == la ? m : ma;
          mb = l == lb ? m : mb;
          mask &= m;
        }
        if (leap) in_filter += leap2_entries(lmaps, kk * (kBlock / 64) + wave, lane, ma, mb, v);
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
        aggregate_group<MODE, SIMPLE>(p, S, gclamp, mask, tbl, G);
      } else if (__any(cnt > 2u)) {
        // dense: the lane's own 32-doc group, LANE_BATCH matched docs per batch (the lines are already cached)
        constexpr int LB = LANE_BATCH;
        while (__any(mask != 0u)) {
          int64_t doc[LB];
          bool ok[LB];
#pragma unroll
          for (int b = 0; b < LB; ++b) {
            ok[b] = mask != 0u;
            doc[b] = ok[b] ? doc0 + (__ffs(mask) - 1) : 0;
            mask &= mask - 1u;
          }
          SegView SS[LB];
#pragma unroll
          for (int b = 0; b < LB; ++b) SS[b] = S;
          aggregate_batch<MODE, LB, SIMPLE>(p, SS, doc, ok, tbl, G);
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
          flush_wave_queue<MODE, SIMPLE>(p, wq, wqs, qn, lane, tbl, G);
          qn = 0;
        }
      }
      ++kk;
#ifdef PGPU_DIAG_WG_TIMES
      ++diag_tiles;
#endif
    }
    if (p.leap_maps)  // each wave stores its own bytes (tiles of other segments hold don't-care values)
      for (int k = lane; k < kk; k += 64)
        p.leap_maps[(t_begin + (int64_t)k * t_step) * (kBlock / 64) + wave] = lmaps[k * (kBlock / 64) + wave];
    kk = 0;
  }
    if (!dyn) break;
    if (tid == 0) claim_at[run & 1] = next_claim;
    __syncthreads();
    // (readfirstlane: a value read from LDS is not known to be wave-uniform, and divergent loop bounds would move the
    // loop's scalars into VGPRs -- 112 -> 149 in the sparse instances)
    const int64_t c0 = (int64_t)p.claim_base + (uint32_t)__builtin_amdgcn_readfirstlane((int)claim_at[run & 1]);
    if (c0 >= T) break;
    if (tid == 0) next_claim = atomicAdd(p.claim, (uint32_t)p.claim_tiles);
    t_begin = c0;
    t_end = c0 + p.claim_tiles < T ? c0 + p.claim_tiles : T;
    t_step = 1;
  }
  if (qn) flush_wave_queue<MODE, SIMPLE>(p, wq, wqs, qn, lane, tbl, G);
#ifdef PGPU_DIAG_WG_TIMES
  diag_t1 = wall_clock64();
#endif
  // numDocsScanned / numEntriesScannedInFilter: one atomic per workgroup (block_stats_add)
#if PGPU_STATS_PER_WAVE
  for (int off = 32; off > 0; off >>= 1) matched += __shfl_xor(matched, off);
  unsigned long long entries = in_filter;
  for (int off = 32; off > 0; off >>= 1) entries += __shfl_xor(entries, off);
  if ((tid & 63) == 0 && matched) atomicAdd(p.stats, matched);
  if ((tid & 63) == 0 && entries) atomicAdd(p.stats + 2, entries);
  if (MODE == MODE_LDS) __syncthreads();
#else
  {
    const int idx[2] = {0, 2};
    unsigned long long v[2] = {matched, (unsigned long long)in_filter};
    block_stats_add<2>(p.stats, idx, v);
  }
#endif

  if (MODE == MODE_LDS) {
    // the slab in the plan's full layout ([num_slots][G]): a packed word splits into the COUNT row and its sum
    __syncthreads();
    uint64_t* out = p.slab + (int64_t)blockIdx.x * p.num_slots * G;
    if (lds_row0) {
      const int ps = p.pack_slot;
      for (int64_t i = tid; i < table_words; i += kBlock) {
        const int s = (int)(i / G) + 1;
        const int64_t k = i - (int64_t)(s - 1) * G;
        const uint64_t w = lds[i];
        if (s == ps) {
          out[k] = w >> kLdsPackShift;
          out[(int64_t)s * G + k] = w & ((1ull << kLdsPackShift) - 1);
        } else {
          out[(int64_t)s * G + k] = w;
        }
      }
    } else {
      for (int64_t i = tid; i < table_words; i += kBlock) out[i] = lds[i];
    }
  }
#ifdef PGPU_DIAG_WG_TIMES
  if (tid == 0 && p.diag_times) {
    unsigned long long* d = p.diag_times + 8 * (int64_t)blockIdx.x;
    d[0] = diag_t0;
    d[1] = diag_t1;
    d[2] = wall_clock64();
    d[3] = (unsigned long long)diag_tiles | ((unsigned long long)diag_first << 32);
    // hardware registers HW_ID (wave / SIMD / CU / SH / SE ids) and XCC_ID: which CU and XCD ran the workgroup
    d[4] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    d[5] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
#endif
}

}  // namespace pgpu
