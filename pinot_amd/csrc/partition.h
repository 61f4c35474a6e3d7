// partition.h — partitioned group-by for large dense key spaces (C5: ~10M groups, a 160 MB table).
//
// Random 64-bit atomics into a table far larger than L2 execute at the memory side, one 64-B request per lane
// (MI355X_MICROARCH.md, "Global float atomics"), which made the direct kernel's C5 scan ~20x slower than its
// bytes.  Instead the matched docs are radix-partitioned by the high bits of their composite key, and each
// partition (a key range whose accumulators fit in LDS) is aggregated by one workgroup with LDS atomics and
// written to the dense table with plain coalesced stores:
//
//   K8a part_count    : filter + key per matched doc; per-workgroup LDS histogram over partitions; partition
//                       totals by one atomic per non-empty partition; each workgroup reserves its run inside every
//                       coarse partition (2^cshift consecutive partitions).
//   K8b (scan)        : exclusive scan of the partition totals (compact_scan_kernel): the final layout, in which
//                       a coarse partition is the contiguous run of its partitions.
//   K8c part_scatter  : the same docs again (same tile assignment); each record (key within its coarse range,
//                       one 8-byte operand per value stream) goes to its coarse run via an LDS cursor.  With <= 64
//                       coarse runs, every workgroup's open output lines fit in L2 and fill before eviction (2442
//                       single-level runs did not: partial-line write-backs made this pass 3 ms on C5).
//   K8e part_split    : per coarse run (split over several workgroups): LDS histogram over its partitions,
//                       reservation, and the records rewritten into the final layout (u16 key within partition).
//   K8d part_aggregate: one workgroup per partition: LDS table, LDS atomics over its records, then the
//                       partition's slice of every table row stored whole (no table init, no global atomics).
//
// Hashed partitions (KPartParams.hashed; sparse key spaces of MODE_HASH plans, e.g. 10^7 groups in a 10^9-key
// space): the same passes with the partition taken from the top bits of a multiplicative hash of the key and the
// whole key carried in the records; instead of K8d,
//   K8h part_hash_aggregate: one workgroup per partition: an LDS hash table (keys + slot words) over its records;
//                       records whose key finds no slot within kHashPartProbes probes are compacted in place and
//                       aggregated by the next round; each round appends its (key, slot words) records to out_rec
//                       (the compacted form of the global hash table, DictionaryBasedGroupKeyGenerator's LONG_MAP
//                       holder at :644-746) -- no table init, no random global atomics.
//
// Replaces the same reference code as the direct kernel (DictionaryBasedGroupKeyGenerator INT_MAP holder +
// aggregateGroupBySV + GroupByCombineOperator merge); results are identical (integer
// accumulators exact; double sums within the path's 1e-9 relative bound — their order is not fixed).
#pragma once
#include <type_traits>

#include "device.h"

namespace pgpu {

// KPartParams: internal.h.

// Static tile range of workgroup b (K8a and K8c must visit the same docs in the same order).
__device__ __forceinline__ void part_tiles(int64_t T, int64_t& t0, int64_t& t1) {
  t0 = (int64_t)blockIdx.x * T / gridDim.x;
  t1 = (int64_t)(blockIdx.x + 1) * T / gridDim.x;
}

// Hashed partitions: records carry hk = part_hash(key), a bijection of u32 (the constant is odd), so the key comes
// back as hk * kHashInv.  hk's top pbits name the partition, the next sbits the start slot of the LDS table; since
// keys are < 2^31, hk is never ~0u (the preimage of ~0u is 0xF174D0AF), which stays free as the empty / padding mark.
constexpr uint32_t kHashMul = 0x9E3779B1u, kHashInv = 0x0E8B2F51u;
__device__ __forceinline__ uint32_t part_hash(uint32_t key) { return key * kHashMul; }
__device__ __forceinline__ uint32_t hpart(const KPartParams& pp, uint32_t hk) {
  return pp.pbits ? hk >> (32 - pp.pbits) : 0u;
}

// A value stream's dictIds -> their indexes in its value arrays (KCol.gaps; a no-op for the segment's own arrays).
__device__ __forceinline__ void map_value_ids(KColC& c, uint32_t (&ids)[16]) { vidx_n(c, ids); }

// Composite keys of docs [32*group + H, +16) of segment S.
template <int H>
__device__ __forceinline__ void part_keys(const KParams& p, const SegView& S, int64_t group, int32_t (&key)[16]) {
  uint32_t ids[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) key[i] = -(int32_t)p.key_bias;
  for (int j = 0; j < p.num_keys; ++j) {
    KColC& c = S.cols[p.key_col[j]];
    decode_group<H>(c.fwd, c.bits, group, ids);
    const int32_t stride = (int32_t)p.key_stride[j];
    if (c.lut) {
      gmem<int32_t>* __restrict__ lut = gp(c.lut);
      int32_t g[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) g[i] = lut[ids[i]];
#pragma unroll
      for (int i = 0; i < 16; ++i) key[i] += g[i] * stride;
    } else {  // contiguous run of the global dictionary: no lookup
#pragma unroll
      for (int i = 0; i < 16; ++i) key[i] += ((int32_t)ids[i] + c.lut_off) * stride;
    }
  }
}

template <int H>
__device__ __forceinline__ void part_scatter_half(const KPartParams& pp, const SegView& S, int64_t group,
                                                  uint32_t m, uint32_t* cursor) {
  const KParams& p = pp.base;
  int32_t key[16];
  part_keys<H>(p, S, group, key);
  const int cbits = pp.pshift + pp.cshift;  // key bits within a coarse partition
  const bool two = pp.cshift > 0;
  if (pp.pack_bits) {  // one integer stream, packed above the key bits: one u32 per record
    KColC& c = S.cols[pp.stream_col[0]];
    uint32_t ids[16];
    decode_group<H>(c.fwd, c.bits, group, ids);
    map_value_ids(c, ids);
    int64_t v[16];
    if (c.dkey) {
      gmem<int64_t>* __restrict__ dk = gp(c.dkey);
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? dk[ids[i]] : pp.pack_min;
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = c.key_base + (int64_t)ids[i];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) {
        const uint32_t pos = atomicAdd(&cursor[key[i] >> cbits], 1u);
        pp.mid_key[pos] = (uint32_t)(key[i] & ((1 << cbits) - 1)) | ((uint32_t)(v[i] - pp.pack_min) << cbits);
      }
    return;
  }
  if (pp.mid_pair) {  // hashed, one u32 value: (hk | value << 32) in one 8-byte word, one scattered store per record
    KColC& c = S.cols[pp.stream_col[0]];
    uint32_t ids[16];
    decode_group<H>(c.fwd, c.bits, group, ids);
    map_value_ids(c, ids);
    uint32_t v[16];
    if (c.dkey) {
      gmem<int64_t>* __restrict__ dk = gp(c.dkey);
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? (uint32_t)dk[ids[i]] : 0u;
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = (uint32_t)(c.key_base + (int64_t)ids[i]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) {
        const uint32_t hk = part_hash((uint32_t)key[i]);
        const uint32_t at = atomicAdd(&cursor[hpart(pp, hk) >> pp.cshift], 1u);
        pp.mid_val[at] = (uint64_t)hk | ((uint64_t)v[i] << 32);
      }
    return;
  }
  uint32_t pos[16];
  if (pp.hashed) {  // the coarse run of the key's hashed partition; the whole hashed key stored
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      pos[i] = 0;
      if ((m >> i) & 1u) {
        const uint32_t hk = part_hash((uint32_t)key[i]);
        pos[i] = atomicAdd(&cursor[hpart(pp, hk) >> pp.cshift], 1u);
        if (two) pp.mid_key[pos[i]] = hk;
        else pp.rec_key32[pos[i]] = hk;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      pos[i] = 0;
      if ((m >> i) & 1u) {
        pos[i] = atomicAdd(&cursor[key[i] >> cbits], 1u);
        if (two) pp.mid_key[pos[i]] = (uint32_t)(key[i] & ((1 << cbits) - 1));
        else pp.rec_key[pos[i]] = (uint16_t)(key[i] & ((1 << pp.pshift) - 1));
      }
    }
  }
  uint32_t ids[16];
  for (int s = 0; s < pp.num_streams; ++s) {
    KColC& c = S.cols[pp.stream_col[s]];
    decode_group<H>(c.fwd, c.bits, group, ids);
    map_value_ids(c, ids);
    uint64_t* __restrict__ out = (two ? pp.mid_val : pp.rec_val) + (int64_t)s * pp.rec_cap;
    if (pp.stream_f64[s]) {
      gmem<double>* __restrict__ dv = gp(c.dval);
      double v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? dv[ids[i]] : 0.0;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if ((m >> i) & 1u) out[pos[i]] = (uint64_t)__double_as_longlong(v[i]);
    } else {
      int64_t v[16];
      if (c.dkey) {
        gmem<int64_t>* __restrict__ dk = gp(c.dkey);
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? dk[ids[i]] : 0;
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? c.key_base + (int64_t)ids[i] : 0;
      }
      if (pp.val32) {
        uint32_t* __restrict__ o32 = reinterpret_cast<uint32_t*>(two ? pp.mid_val : pp.rec_val) + (int64_t)s * pp.rec_cap;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((m >> i) & 1u) o32[pos[i]] = (uint32_t)v[i];
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if ((m >> i) & 1u) out[pos[i]] = (uint64_t)v[i];
      }
    }
  }
}

// Wave-scope ordering of LDS accesses (the LDS unit serves one wave's instructions in order; this keeps the compiler
// from moving them across the point).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// u32 words of a wave's K8c staging region (part_scatter_half_staged): run counters / starts [64], store offsets
// [64], run of each staged record [1024 u8], staged records [1024 u32 or u64].
constexpr int kStageWaveWords32 = 64 + 64 + 256 + 1024;
constexpr int kStageWaveWords64 = 64 + 64 + 256 + 2048;

// K8c, staged (one u32 or u64 word per record, <= 64 coarse runs): the records of a wave's half-group (<= 1024: 64
// lanes x 16 docs) are counting-sorted by coarse run in the wave's own LDS region -- rank within the run by a wave-local
// counter, one workgroup-cursor reservation per run and wave (lane r reserves run r), an exclusive scan of the runs'
// counts -- and then stored in run order: consecutive lanes store consecutive positions of one run, so a store
// instruction touches a few lines instead of one line per lane.
//   W64 = false: pack_bits records, (key within its coarse run) | (value - pack_min) << cbits, to mid_key;
//   W64 = true : mid_pair records, hk | value << 32, to mid_val.
template <int H, bool W64>
__device__ __forceinline__ void part_scatter_half_staged(const KPartParams& pp, const SegView& S, int64_t group,
                                                         uint32_t m, uint32_t* cursor, uint32_t* ws) {
  const KParams& p = pp.base;
  const int lane = threadIdx.x & 63;
  uint32_t* wcnt = ws;                                          // per run: count, then local start
  int32_t* wdelta = reinterpret_cast<int32_t*>(ws + 64);        // per run: global position - local start
  uint8_t* bkt = reinterpret_cast<uint8_t*>(ws + 128);          // per staged record: its run
  int32_t key[16];
  part_keys<H>(p, S, group, key);
  KColC& c = S.cols[pp.stream_col[0]];
  uint32_t ids[16];
  decode_group<H>(c.fwd, c.bits, group, ids);
  map_value_ids(c, ids);
  int64_t v[16];
  if (c.dkey) {
    gmem<int64_t>* __restrict__ dk = gp(c.dkey);
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = ((m >> i) & 1u) ? dk[ids[i]] : pp.pack_min;
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = c.key_base + (int64_t)ids[i];
  }
  using Word = typename std::conditional<W64, uint64_t, uint32_t>::type;
  Word word[16];
  uint32_t run[16];
  if (!W64) {
    const int cbits = pp.pshift + pp.cshift;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      run[i] = (uint32_t)key[i] >> cbits;
      word[i] = (Word)((uint32_t)(key[i] & ((1 << cbits) - 1)) | ((uint32_t)(v[i] - pp.pack_min) << cbits));
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t hk = part_hash((uint32_t)key[i]);
      run[i] = hpart(pp, hk) >> pp.cshift;
      word[i] = (Word)((uint64_t)hk | ((uint64_t)(uint32_t)v[i] << 32));
    }
  }
  wcnt[lane] = 0u;
  wave_sync();
  uint32_t rank[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) rank[i] = ((m >> i) & 1u) ? atomicAdd(&wcnt[run[i]], 1u) : 0u;
  wave_sync();
  const uint32_t cnt = wcnt[lane];
  const uint32_t g = cnt ? atomicAdd(&cursor[lane], cnt) : 0u;  // run `lane`'s positions in the workgroup's run
  uint32_t incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  const uint32_t excl = incl - cnt;
  const uint32_t total = __shfl(incl, 63);
  wdelta[lane] = (int32_t)(g - excl);
  wcnt[lane] = excl;
  wave_sync();
  Word* words = reinterpret_cast<Word*>(ws + 128 + 256);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((m >> i) & 1u) {
      const uint32_t slot = wcnt[run[i]] + rank[i];
      bkt[slot] = (uint8_t)run[i];
      words[slot] = word[i];
    }
  wave_sync();
  Word* __restrict__ out = W64 ? reinterpret_cast<Word*>(pp.mid_val) : reinterpret_cast<Word*>(pp.mid_key);
  for (uint32_t s = lane; s < total; s += 64) out[(uint32_t)((int32_t)s + wdelta[bkt[s]])] = words[s];
  wave_sync();  // the region is free for the next half-group
}

template <int H>
__device__ __forceinline__ void part_count_half(const KPartParams& pp, const SegView& S, int64_t group, uint32_t m,
                                                uint32_t* hist) {
  int32_t key[16];
  part_keys<H>(pp.base, S, group, key);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((m >> i) & 1u) atomicAdd(&hist[pp.hashed ? hpart(pp, part_hash((uint32_t)key[i])) : (uint32_t)key[i] >> pp.pshift], 1u);
}

// K8a (SCATTER = false) / K8c (SCATTER = true; STAGE 0: each record stored from its lane, 1 / 2: the u32 / u64
// one-word records staged per wave, part_scatter_half_staged).  LDS: [u32 histogram of num_parts (K8a) / cursors of
// num_coarse (K8c)] [filter stack] and, staged, from u32 word pp.stage_off one region of kStageWaveWords32 / 64 words
// per wave (part_pass_lds).
// K8a / K8c held to 4 waves per SIMD (128 VGPRs): the staged K8c compiled to 130 and ran 3 (C5: K8c 403 -> 355 us,
// K8a 147 -> 126 us with the larger grid they share; r05 session zc)
#ifndef PGPU_PART_PASS_MIN_WAVES
#define PGPU_PART_PASS_MIN_WAVES 4
#endif
template <bool SCATTER, int STAGE = 0>
__global__ __launch_bounds__(kBlock, PGPU_PART_PASS_MIN_WAVES) void part_pass_kernel(const KPartParams pp) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const KParams& p = pp.base;
  const int tid = threadIdx.x;
  uint32_t* hist = reinterpret_cast<uint32_t*>(lds);
  uint32_t* stack = hist + (((SCATTER ? pp.num_coarse : pp.num_parts) + 3) & ~3);
  uint32_t* ws = reinterpret_cast<uint32_t*>(lds) + pp.stage_off +
                 (tid >> 6) * (STAGE == 2 ? kStageWaveWords64 : kStageWaveWords32);
  // Deadline: the flag expand_tiles_kernel set when the query's end time had passed before this launch.  Every
  // pass reads it at its start and it cannot change while they run, so K8c scatters exactly the docs K8a counted
  // (its cursors run inside K8a's reservations) or nothing, like K8e / K8d.
  if (p.deadline && p.stats[5]) return;
  if (SCATTER) {
    for (int c = tid; c < pp.num_coarse; c += kBlock)
      hist[c] = pp.part_start[c << pp.cshift] + pp.block_off[(int64_t)blockIdx.x * pp.num_coarse + c];
  } else {
    for (int i = tid; i < pp.num_parts; i += kBlock) hist[i] = 0u;
  }
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
    if (SCATTER && STAGE) {
      if (__any((mask & 0xFFFFu) != 0u)) part_scatter_half_staged<0, STAGE == 2>(pp, S, gclamp, mask & 0xFFFFu, hist, ws);
      if (__any((mask >> 16) != 0u)) part_scatter_half_staged<16, STAGE == 2>(pp, S, gclamp, mask >> 16, hist, ws);
    } else if (SCATTER) {
      if (__any((mask & 0xFFFFu) != 0u)) part_scatter_half<0>(pp, S, gclamp, mask & 0xFFFFu, hist);
      if (__any((mask >> 16) != 0u)) part_scatter_half<16>(pp, S, gclamp, mask >> 16, hist);
    } else {
      if (__any((mask & 0xFFFFu) != 0u)) part_count_half<0>(pp, S, gclamp, mask & 0xFFFFu, hist);
      if (__any((mask >> 16) != 0u)) part_count_half<16>(pp, S, gclamp, mask >> 16, hist);
    }
  }
  if (!SCATTER) {
    {
      const int idx[1] = {0};
      unsigned long long v[1] = {matched};
      block_stats_add<1>(p.stats, idx, v);
    }
    __syncthreads();
    // partition totals, and this workgroup's run inside every coarse partition it touches
    for (int i = tid; i < pp.num_parts; i += kBlock)
      if (hist[i]) atomicAdd(&pp.part_start[i], hist[i]);
    for (int c = tid; c < pp.num_coarse; c += kBlock) {
      const int p0 = c << pp.cshift, p1 = min(pp.num_parts, (c + 1) << pp.cshift);
      uint32_t h = 0;
      for (int i = p0; i < p1; ++i) h += hist[i];
      pp.block_off[(int64_t)blockIdx.x * pp.num_coarse + c] = h ? atomicAdd(&pp.coarse_fill[c], h) : 0u;
    }
  }
}

// K8e: workgroup (coarse run c, chunk j) moves its share of run c into the final per-partition layout,
// pp.split_batch records at a time: a batch is sorted by partition in LDS -- histogram, prefix, one global atomic
// per non-empty partition reserving the batch's run in it, each record placed at its bucket slot with the global
// position it will take -- and then the sorted batch is written back out in LDS
// order, so consecutive lanes store consecutive positions of one partition's run (coalesced u16 keys and u64
// values) instead of 64 lanes scattering over 2^cshift open runs.  LDS: counters / cursors / batch histogram /
// bucket starts [2^cshift each], then the staged batch (pp.split_batch records: a multiple of kBlock, at most
// kSplitBatch, smaller with many value streams): values u64 per stream, positions u32, keys u16.
__global__ __launch_bounds__(kBlock) void part_split_kernel(const KPartParams pp) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const int tid = threadIdx.x;
  if (pp.base.deadline && pp.base.stats[5]) return;  // K8a timed out: its counts cover only part of the docs
  const int c = blockIdx.x / pp.chunks_per_coarse, j = blockIdx.x % pp.chunks_per_coarse;
  const int p0 = c << pp.cshift, p1 = min(pp.num_parts, (c + 1) << pp.cshift), np = p1 - p0;
  const int NP = 1 << pp.cshift;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(lds);  // per partition: the batch's first global position
  uint32_t* hist = cnt + NP;                          // batch histogram, then the batch's running rank
  uint32_t* bstart = hist + NP;                       // batch bucket starts (exclusive prefix of hist)
  const int batch = pp.split_batch;
  uint64_t* sval = reinterpret_cast<uint64_t*>(bstart + NP + (NP & 1));
  uint32_t* spos = reinterpret_cast<uint32_t*>(sval + (size_t)pp.num_streams * batch);
  uint16_t* skey = reinterpret_cast<uint16_t*>(spos + batch);
  uint32_t* skey32 = reinterpret_cast<uint32_t*>(spos + batch);  // hashed: whole keys (part_split_lds key_bytes 4)
  __shared__ uint32_t wtot[kBlock / 64];
  const uint32_t cs = pp.part_start[p0], ce = pp.part_start[p1];
  const uint32_t r0 = cs + (uint32_t)((uint64_t)(ce - cs) * j / pp.chunks_per_coarse);
  const uint32_t r1 = cs + (uint32_t)((uint64_t)(ce - cs) * (j + 1) / pp.chunks_per_coarse);
  const int cbits = pp.pshift + pp.cshift;
  const uint32_t kmask = pp.pack_bits ? (1u << cbits) - 1u : ~0u;  // the key bits of a packed mid_key word
  constexpr int NB = kSplitBatch / kBlock;  // records per lane per batch
  const uint32_t low = (1u << pp.pshift) - 1u;
  const int per = (NP + kBlock - 1) / kBlock;  // prefix: each thread a contiguous slice of the buckets
  for (uint32_t b0 = r0; b0 < r1; b0 += batch) {
    const uint32_t n = min((uint32_t)batch, r1 - b0);
    for (int i = tid; i < NP; i += kBlock) hist[i] = 0u;
    __syncthreads();  // (also: the previous batch's write-out has read the staged arrays)
    uint32_t k[NB], rank[NB];
    uint64_t v0[NB];  // stream 0's values, loaded with the keys so they are in flight through the sort
    if (pp.mid_pair) {  // (hashed key, u32 value) words
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const uint32_t i = tid + b * kBlock;
        const uint64_t w = pp.mid_val[b0 + (i < n ? i : 0u)];
        k[b] = i < n ? (uint32_t)w : ~0u;
        v0[b] = (uint64_t)(uint32_t)(w >> 32);
      }
    } else {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const uint32_t i = tid + b * kBlock;
        k[b] = i < n ? pp.mid_key[b0 + i] : ~0u;
      }
    }
    if (pp.pack_bits) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        v0[b] = (uint64_t)(pp.pack_min + (int64_t)(k[b] >> cbits));  // as the u32 record the aggregate reads
        k[b] = tid + b * kBlock < n ? k[b] & kmask : ~0u;  // (a packed word may be all ones)
      }
    } else if (!pp.mid_pair) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const uint32_t r = b0 + min(tid + b * kBlock, n - 1u);
        v0[b] = pp.num_streams == 0 ? 0ull
                : pp.val32          ? (uint64_t)reinterpret_cast<const uint32_t*>(pp.mid_val)[r]
                                    : pp.mid_val[r];
      }
    }
    uint32_t part[NB];  // the record's partition within this coarse run
#pragma unroll
    for (int b = 0; b < NB; ++b)
      part[b] = pp.hashed ? hpart(pp, k[b]) & (uint32_t)(NP - 1) : k[b] >> pp.pshift;
#pragma unroll
    for (int b = 0; b < NB; ++b) rank[b] = k[b] != ~0u ? atomicAdd(&hist[part[b]], 1u) : 0u;
    __syncthreads();
    {  // exclusive prefix of the batch histogram: slices, wave scan of the slice sums, wave totals
      const int lane = tid & 63, w = tid >> 6;
      uint32_t acc = 0;
      for (int i = tid * per; i < min(NP, (tid + 1) * per); ++i) acc += hist[i];
      uint32_t incl = acc;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      if (lane == 63) wtot[w] = incl;
      __syncthreads();
      uint32_t run = incl - acc;
      for (int v = 0; v < w; ++v) run += wtot[v];
      for (int i = tid * per; i < min(NP, (tid + 1) * per); ++i) {
        bstart[i] = run;
        const uint32_t h = hist[i];
        run += h;
        // the batch's run inside partition p0 + i: reserved now (no counting pass over the coarse run first)
        cnt[i] = h ? pp.part_start[p0 + i] + atomicAdd(&pp.fine_fill[p0 + i], h) : 0u;
      }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (k[b] == ~0u) continue;
      const uint32_t l = bstart[part[b]] + rank[b];
      spos[l] = cnt[part[b]] + rank[b];
      if (pp.hashed) skey32[l] = k[b];
      else skey[l] = (uint16_t)(k[b] & low);
      const int64_t r = b0 + tid + b * kBlock;
      if (pp.num_streams > 0) sval[l] = v0[b];
      for (int s = 1; s < pp.num_streams; ++s)
        sval[(size_t)s * batch + l] = pp.val32 ? (uint64_t)reinterpret_cast<const uint32_t*>(pp.mid_val)[s * pp.rec_cap + r]
                                               : pp.mid_val[s * pp.rec_cap + r];
    }
    __syncthreads();
    if (pp.fine_pack) {  // one u32 per record: key | (value - pack_min) << pshift
      uint32_t* __restrict__ r32 = reinterpret_cast<uint32_t*>(pp.rec_val);
      if (pp.hashed) {  // hk below its partition bits | (value - pack_min) << (32 - pbits)
        const int lb = 32 - pp.pbits;
        const uint32_t hlow = (1u << lb) - 1u;
        for (uint32_t i = tid; i < n; i += kBlock)
          r32[spos[i]] = (skey32[i] & hlow) | ((uint32_t)((int64_t)sval[i] - pp.pack_min) << lb);
        continue;
      }
      for (uint32_t i = tid; i < n; i += kBlock)
        r32[spos[i]] = (uint32_t)skey[i] | ((uint32_t)((int64_t)sval[i] - pp.pack_min) << pp.pshift);
      continue;
    }
    for (uint32_t i = tid; i < n; i += kBlock) {  // in bucket order: runs of consecutive positions
      const uint32_t pos = spos[i];
      if (pp.hashed) pp.rec_key32[pos] = skey32[i];
      else pp.rec_key[pos] = skey[i];
      if (pp.val32)
        for (int s = 0; s < pp.num_streams; ++s)
          reinterpret_cast<uint32_t*>(pp.rec_val)[(int64_t)s * pp.rec_cap + pos] = (uint32_t)sval[(size_t)s * batch + i];
      else
        for (int s = 0; s < pp.num_streams; ++s) pp.rec_val[(int64_t)s * pp.rec_cap + pos] = sval[(size_t)s * batch + i];
    }
  }
}

// K8e, one final u32 word per record (KPartParams.fine_pack: C5's packed records, c5_hash's hashed ones): the same
// batch sort with the record's final word computed in registers at load time, so the staging holds 8 bytes per record
// (word, position) instead of 14-16, batches are twice as large (half the reservation round trips per record), and
// the next batch's records are loaded while the current one is placed and written out.  HASHED: hk below the
// partition bits | (value - pack_min) << (32 - pbits), from mid_pair words or mid_key + u32 mid_val; else the key
// within the partition | (value - pack_min) << pshift, from pack_bits mid_key words.  LDS: counters / histogram /
// bucket starts [2^cshift each], then kSplitWordsBatch words and positions.
constexpr int kSplitWordsBatch = 4096;
constexpr size_t part_split_words_lds(int cshift) {
  return (size_t)3 * ((size_t)1 << cshift) * 4 + (size_t)kSplitWordsBatch * 8;
}
template <bool HASHED>
__global__ __launch_bounds__(kBlock) void part_split_words_kernel(const KPartParams pp) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const int tid = threadIdx.x;
  if (pp.base.deadline && pp.base.stats[5]) return;
  const int c = blockIdx.x / pp.chunks_per_coarse, j = blockIdx.x % pp.chunks_per_coarse;
  const int p0 = c << pp.cshift, p1 = min(pp.num_parts, (c + 1) << pp.cshift);
  const int NP = 1 << pp.cshift;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(lds);
  uint32_t* hist = cnt + NP;
  uint32_t* bstart = hist + NP;
  uint32_t* sword = bstart + NP;
  uint32_t* spos = sword + kSplitWordsBatch;
  __shared__ uint32_t wtot[kBlock / 64];
  const uint32_t cs = pp.part_start[p0], ce = pp.part_start[p1];
  const uint32_t r0 = cs + (uint32_t)((uint64_t)(ce - cs) * j / pp.chunks_per_coarse);
  const uint32_t r1 = cs + (uint32_t)((uint64_t)(ce - cs) * (j + 1) / pp.chunks_per_coarse);
  const int cbits = pp.pshift + pp.cshift;
  const uint32_t kmask = (1u << cbits) - 1u, low = (1u << pp.pshift) - 1u;
  const int lb = 32 - pp.pbits;
  const uint32_t hlow = HASHED ? (1u << lb) - 1u : 0u;
  constexpr int NB = kSplitWordsBatch / kBlock;
  const int per = (NP + kBlock - 1) / kBlock;
  uint32_t part[NB], word[NB];
  // batch b0's records -> (partition within the run, final word); part = ~0u past the batch's end
  auto load = [&](uint32_t b0) {
    const uint32_t n = b0 < r1 ? min((uint32_t)kSplitWordsBatch, r1 - b0) : 0u;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const uint32_t i = tid + b * kBlock;
      const uint32_t r = b0 + (i < n ? i : 0u);
      if (HASHED) {
        uint32_t hk, v;
        if (pp.mid_pair) {
          const uint64_t w = n ? pp.mid_val[r] : 0ull;
          hk = (uint32_t)w;
          v = (uint32_t)(w >> 32);
        } else {
          hk = n ? pp.mid_key[r] : 0u;
          v = n ? reinterpret_cast<const uint32_t*>(pp.mid_val)[r] : 0u;
        }
        part[b] = i < n ? hpart(pp, hk) & (uint32_t)(NP - 1) : ~0u;
        word[b] = (hk & hlow) | ((uint32_t)((int64_t)v - pp.pack_min) << lb);
      } else {
        const uint32_t w = n ? pp.mid_key[r] : 0u;
        const uint32_t kk = w & kmask;
        part[b] = i < n ? kk >> pp.pshift : ~0u;
        word[b] = (kk & low) | ((w >> cbits) << pp.pshift);
      }
    }
  };
  load(r0);
  uint32_t* __restrict__ r32 = reinterpret_cast<uint32_t*>(pp.rec_val);
  for (uint32_t b0 = r0; b0 < r1; b0 += kSplitWordsBatch) {
    const uint32_t n = min((uint32_t)kSplitWordsBatch, r1 - b0);
    for (int i = tid; i < NP; i += kBlock) hist[i] = 0u;
    __syncthreads();  // (also: the previous batch's write-out has read the staged words)
    uint32_t rank[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) rank[b] = part[b] != ~0u ? atomicAdd(&hist[part[b]], 1u) : 0u;
    __syncthreads();
    {  // exclusive prefix of the batch histogram; the batch's run in each partition reserved with one atomic
      const int lane = tid & 63, w = tid >> 6;
      uint32_t acc = 0;
      for (int i = tid * per; i < min(NP, (tid + 1) * per); ++i) acc += hist[i];
      uint32_t incl = acc;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      if (lane == 63) wtot[w] = incl;
      __syncthreads();
      uint32_t run = incl - acc;
      for (int v = 0; v < w; ++v) run += wtot[v];
      for (int i = tid * per; i < min(NP, (tid + 1) * per); ++i) {
        bstart[i] = run;
        const uint32_t h = hist[i];
        run += h;
        cnt[i] = h && p0 + i < p1 ? pp.part_start[p0 + i] + atomicAdd(&pp.fine_fill[p0 + i], h) : 0u;
      }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (part[b] == ~0u) continue;
      const uint32_t l = bstart[part[b]] + rank[b];
      sword[l] = word[b];
      spos[l] = cnt[part[b]] + rank[b];
    }
    load(b0 + kSplitWordsBatch);  // the next batch in flight while this one is written out
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kBlock) r32[spos[i]] = sword[i];
  }
}

// K8d: partition blockIdx.x -> its key range of every table row.  LDS: [num_slots][1 << pshift] u64.
__global__ __launch_bounds__(kBlock) void part_aggregate_kernel(const KPartParams pp) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const KParams& p = pp.base;
  const int tid = threadIdx.x;
  if (p.deadline && p.stats[5]) return;
  const int PR = 1 << pp.pshift;
  const int ns = p.num_slots;
  // cs_pack: one word per key (LDS of PR words, part_aggregate_lds), COUNT + SUM from 0; else every slot's row
  for (int i = tid; i < (pp.cs_pack ? PR : ns * PR); i += kBlock) lds[i] = pp.cs_pack ? 0ull : slot_init(p.slot_kind[i / PR]);
  __syncthreads();
  const uint32_t r0 = pp.part_start[blockIdx.x], r1 = pp.part_start[blockIdx.x + 1];
  // COUNT + SUM in one LDS word per key (the table is PR words, 32 KB for C5: four workgroups per CU instead of
  // two), over chunks of records small enough that every key's count stays below 2^24 and its sum of offsets below
  // 2^40; the first chunk stores the partition's slice of both rows, later ones (a partition of more than ~10^9
  // offsets' worth of records) add to it -- the partition is this workgroup's alone.
  if (pp.cs_pack) {
    constexpr int NB = 16;
    const uint32_t* __restrict__ r32 = reinterpret_cast<const uint32_t*>(pp.rec_val);
    const uint32_t low = (1u << pp.pshift) - 1u;
    unsigned long long* w64 = reinterpret_cast<unsigned long long*>(lds);  // slot 0's words
    const uint64_t by_sum = (1ull << 40) / (uint64_t)(pp.pack_range > 0 ? pp.pack_range : 1);
    const uint32_t lim = (uint32_t)(by_sum < (1ull << 24) - 1 ? (by_sum > 0 ? by_sum : 1) : (1ull << 24) - 1);
    const int64_t G = p.num_keys_total;
    const int64_t k0 = (int64_t)blockIdx.x * PR;
    const int n = (int)(G - k0 < PR ? G - k0 : PR);
    uint32_t c0 = r0;
    do {
      const uint32_t c1 = r1 - c0 > lim ? c0 + lim : r1;
      if (c0 != r0) {
        for (int i = tid; i < PR; i += kBlock) lds[i] = 0ull;
        __syncthreads();
      }
      for (uint32_t base = c0 + tid; base < c1; base += NB * kBlock) {
        uint32_t wr[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const uint32_t r = base + b * kBlock;
          wr[b] = r32[r < c1 ? r : c0];
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
          if (base + b * kBlock < c1)
            atomicAdd(w64 + (wr[b] & low), (1ull << 40) | (unsigned long long)(wr[b] >> pp.pshift));
      }
      __syncthreads();
      const bool last = c1 >= r1;
      uint32_t present = 0;
      long long mn[2] = {INT64_MAX, INT64_MAX}, mx[2] = {INT64_MIN, INT64_MIN};
      for (int i = tid; i < n; i += kBlock) {
        const uint64_t w = lds[i];
        uint64_t cnt = w >> 40;
        uint64_t sum = (uint64_t)((int64_t)(w & ((1ull << 40) - 1)) + (int64_t)cnt * pp.pack_min);
        if (c0 == r0) {
          p.table[k0 + i] = cnt;      // COUNT (slot 0)
          p.table[G + k0 + i] = sum;  // SUM
        } else {
          cnt += p.table[k0 + i];
          sum += p.table[G + k0 + i];
          p.table[k0 + i] = cnt;
          p.table[G + k0 + i] = sum;
        }
        if (last && pp.chunk_cnt && cnt) {  // the compaction's count pass, from the words in hand
          ++present;
          mn[0] = min(mn[0], (long long)cnt);
          mx[0] = max(mx[0], (long long)cnt);
          mn[1] = min(mn[1], (long long)sum);
          mx[1] = max(mx[1], (long long)sum);
        }
      }
      if (last && pp.chunk_cnt) {  // workgroup-uniform
        __shared__ unsigned long long red_cnt[kBlock / 64];
        __shared__ long long red_mm[kBlock / 64][4];
        const int lane = tid & 63, wv = tid >> 6;
        unsigned long long c = present;
        for (int off = 32; off > 0; off >>= 1) {
          c += __shfl_xor(c, off);
          for (int s = 0; s < 2; ++s) {
            mn[s] = min(mn[s], (long long)__shfl_xor(mn[s], off));
            mx[s] = max(mx[s], (long long)__shfl_xor(mx[s], off));
          }
        }
        if (lane == 0) {
          red_cnt[wv] = c;
          red_mm[wv][0] = mn[0];
          red_mm[wv][1] = mn[1];
          red_mm[wv][2] = mx[0];
          red_mm[wv][3] = mx[1];
        }
        __syncthreads();
        if (tid < 4) {
          long long v = tid < 2 ? INT64_MAX : INT64_MIN;
          for (int w = 0; w < kBlock / 64; ++w) v = tid < 2 ? min(v, red_mm[w][tid]) : max(v, red_mm[w][tid]);
          pp.chunk_mm[4 * (int64_t)blockIdx.x + tid] = v;
        }
        if (tid == 0) {
          unsigned long long t = 0;
          for (int w = 0; w < kBlock / 64; ++w) t += red_cnt[w];
          pp.chunk_cnt[blockIdx.x] = (uint32_t)t;
        }
      }
      __syncthreads();  // the words are read before the next chunk clears them
      c0 = c1;
    } while (c0 < r1);
    return;
  }
  // Two workgroups per CU (the LDS table), so latency is hidden by loads in flight per lane: NB records per lane
  // per step, every load issued unconditionally (records past r1 re-read record r0 and are not accumulated).
  constexpr int NB = 16;
  for (uint32_t base = r0 + tid; base < r1; base += NB * kBlock) {
    uint32_t ri[NB];
    int k[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const uint32_t r = base + b * kBlock;
      ri[b] = r < r1 ? r : r0;
    }
    int64_t pv[NB];  // fine_pack: the records' values
    if (pp.fine_pack) {
      const uint32_t* __restrict__ r32 = reinterpret_cast<const uint32_t*>(pp.rec_val);
      const uint32_t low = (1u << pp.pshift) - 1u;
      uint32_t wr[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) wr[b] = r32[ri[b]];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        k[b] = (int)(wr[b] & low);
        pv[b] = pp.pack_min + (int64_t)(wr[b] >> pp.pshift);
      }
    } else {
#pragma unroll
      for (int b = 0; b < NB; ++b) k[b] = pp.rec_key[ri[b]];
    }
    for (int s = 0; s < ns; ++s) {
      const int kind = p.slot_kind[s];
      const int st = pp.slot_stream[s];
      uint64_t w[NB];
      if (st < 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) w[b] = 0ull;
      } else if (pp.fine_pack) {
#pragma unroll
        for (int b = 0; b < NB; ++b) w[b] = (uint64_t)pv[b];
      } else if (pp.val32) {
        const int32_t* __restrict__ r32 = reinterpret_cast<const int32_t*>(pp.rec_val) + (int64_t)st * pp.rec_cap;
#pragma unroll
        for (int b = 0; b < NB; ++b) w[b] = (uint64_t)(int64_t)r32[ri[b]];
      } else {
        const uint64_t* __restrict__ r64 = pp.rec_val + (int64_t)st * pp.rec_cap;
#pragma unroll
        for (int b = 0; b < NB; ++b) w[b] = r64[ri[b]];
      }
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (base + b * kBlock < r1)
          accumulate<MODE_LDS>(lds + (int64_t)s * PR, k[b], kind, (int64_t)w[b], __longlong_as_double((long long)w[b]));
    }
  }
  __syncthreads();
  const int64_t G = p.num_keys_total;
  const int64_t k0 = (int64_t)blockIdx.x * PR;
  const int n = (int)(G - k0 < PR ? G - k0 : PR);
  for (int s = 0; s < ns; ++s)
    for (int i = tid; i < n; i += kBlock) p.table[(int64_t)s * G + k0 + i] = lds[(int64_t)s * PR + i];
}

// Slot of hashed key `hk` in an LDS hash table of 2^sbits u32 entries (empty = ~0u), inserted if absent, or -1
// after kHashPartProbes probes.  Start slot: the sbits of hk below the partition's pbits.
__device__ __forceinline__ int lds_hash_slot(uint32_t* keys, uint32_t key, int pbits, int sbits) {
  const uint32_t mask = (1u << sbits) - 1u;
  uint32_t s = (key << pbits) >> (32 - sbits);
  const int probes = kHashPartProbes < (1 << sbits) ? kHashPartProbes : (1 << sbits);
  for (int i = 0; i < probes; ++i) {
    const uint32_t k = keys[s];
    if (k == key) return (int)s;
    if (k == ~0u) {
      const uint32_t prev = atomicCAS(&keys[s], ~0u, key);
      if (prev == ~0u || prev == key) return (int)s;
    }
    s = (s + 1u) & mask;
  }
  return -1;
}

// K8h: partition blockIdx.x -> its groups' compacted records.  LDS: [num_slots][2^sbits] u64 words, then
// [2^sbits] u32 keys.  Each round aggregates the partition's pending records (those of round 0: its whole run);
// a record whose key finds no slot is written back at the front of the run (in place: every record of a batch is
// loaded before any of the batch is written, and the write position never passes the records read) and waits for
// the next round, so every round places at least one new key and the loop ends.
__global__ __launch_bounds__(kBlock) void part_hash_aggregate_kernel(const KPartParams pp) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const KParams& p = pp.base;
  const int tid = threadIdx.x, lane = tid & 63;
  if (p.deadline && p.stats[5]) return;
  const int S = 1 << pp.sbits;
  const int ns = p.num_slots, nst = pp.num_streams;
  uint32_t* keys = reinterpret_cast<uint32_t*>(lds + (size_t)ns * S);
  __shared__ uint32_t pending;
  __shared__ uint32_t wave_tot[kBlock / 64];
  __shared__ unsigned long long blk_base;
  // this partition's range of every slot's words over all rounds (order-preserving u64: min at [s], max at [ns + s])
  __shared__ unsigned long long blk_mm[2 * kMaxSlots];
  if (pp.out_mm)
    for (int i = tid; i < 2 * ns; i += kBlock) blk_mm[i] = i < ns ? ~0ull : 0ull;
  const uint32_t r0 = pp.part_start[blockIdx.x];
  uint32_t n = pp.part_start[blockIdx.x + 1] - r0;
  const int64_t cap = pp.rec_cap;
  constexpr int NB = 8;
  // COUNT + SUM in one LDS word (slot 0's row) when the partition's records bound both halves (uniform per
  // workgroup): (1 << 40) | (value - pack_min) per record, split when the round's groups are written
  const bool cs = pp.cs_pack && n < (1u << 24) && (uint64_t)n * (uint64_t)pp.pack_range < (1ull << 40);
  while (n > 0) {
    for (int i = tid; i < S; i += kBlock) keys[i] = ~0u;
    for (int i = tid; i < ns * S; i += kBlock) lds[i] = slot_init(p.slot_kind[i >> pp.sbits]);
    if (tid == 0) pending = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += NB * kBlock) {
      uint32_t key[NB];  // hashed keys
      uint64_t v[NB][kHashPartStreams];
      uint32_t w32[NB];  // fine_pack: the packed records as read (written back as they are when left pending)
      if (pp.fine_pack) {
        const uint32_t* __restrict__ r32 = reinterpret_cast<const uint32_t*>(pp.rec_val);
        const int lb = 32 - pp.pbits;
        const uint32_t hi = (uint32_t)blockIdx.x << lb, hlow = (1u << lb) - 1u;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const uint32_t i = base + b * kBlock + tid;
          w32[b] = r32[r0 + (i < n ? i : 0u)];
          key[b] = i < n ? hi | (w32[b] & hlow) : ~0u;
          v[b][0] = (uint64_t)(pp.pack_min + (int64_t)(w32[b] >> lb));
#pragma unroll
          for (int st = 1; st < kHashPartStreams; ++st) v[b][st] = 0ull;
        }
      } else {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const uint32_t i = base + b * kBlock + tid;
          const uint32_t r = r0 + (i < n ? i : 0u);
          w32[b] = 0;
          key[b] = i < n ? pp.rec_key32[r] : ~0u;
#pragma unroll
          for (int st = 0; st < kHashPartStreams; ++st)
            v[b][st] = st >= nst ? 0ull
                       : pp.val32 ? (uint64_t)(int64_t)reinterpret_cast<const int32_t*>(pp.rec_val)[st * cap + r]
                                  : pp.rec_val[st * cap + r];
        }
      }
      __syncthreads();  // the batch is in registers before any record of it is overwritten by a pending one
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if (key[b] == ~0u) continue;
        const int slot = lds_hash_slot(keys, key[b], pp.pbits, pp.sbits);
        if (slot < 0) {
          const uint32_t at = r0 + atomicAdd(&pending, 1u);
          if (pp.fine_pack) {
            reinterpret_cast<uint32_t*>(pp.rec_val)[at] = w32[b];
            continue;
          }
          pp.rec_key32[at] = key[b];
#pragma unroll
          for (int st = 0; st < kHashPartStreams; ++st)
            if (st < nst) {
              if (pp.val32) reinterpret_cast<uint32_t*>(pp.rec_val)[st * cap + at] = (uint32_t)v[b][st];
              else pp.rec_val[st * cap + at] = v[b][st];
            }
          continue;
        }
        if (cs) {
          atomicAdd(reinterpret_cast<unsigned long long*>(lds) + slot,
                    (1ull << 40) | (unsigned long long)((int64_t)v[b][0] - pp.pack_min));
          continue;
        }
        for (int s = 0; s < ns; ++s) {
          const int st = pp.slot_stream[s];
          uint64_t w = 0;
#pragma unroll
          for (int j = 0; j < kHashPartStreams; ++j)
            if (j == st) w = v[b][j];
          accumulate<MODE_LDS>(lds + (int64_t)s * S, slot, p.slot_kind[s], (int64_t)w,
                               __longlong_as_double((long long)w));
        }
      }
    }
    __syncthreads();
    // append this round's groups with one reservation per workgroup (a single global counter: per-wave atomics
    // would queue 4 x 2^sbits / 256 of them per partition at one address): waves count their entries by ballot, the
    // workgroup reserves their sum, each wave writes a contiguous run
    uint32_t mine = 0;
    for (int i0 = 0; i0 < S; i0 += kBlock) {
      const int i = i0 + tid;
      mine += (uint32_t)__popcll(__ballot(i < S && keys[i] != ~0u));
    }
    if (lane == 0) wave_tot[tid >> 6] = mine;
    __syncthreads();
    if (tid == 0) {
      uint32_t tot = 0;
      for (int w = 0; w < kBlock / 64; ++w) tot += wave_tot[w];
      blk_base = tot ? atomicAdd(pp.out_count, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    uint64_t at = blk_base;
    for (int w = 0; w < (tid >> 6); ++w) at += wave_tot[w];
    // the slot ranges of the groups written, tracked in registers while writing them when there are few slots (the
    // compact result's widths; order-preserving u64), else by a pass over the table below
    constexpr int kMmRegs = 4;
    const bool mm_regs = pp.out_mm && ns <= kMmRegs;
    unsigned long long rlo[kMmRegs], rhi[kMmRegs];
#pragma unroll
    for (int s = 0; s < kMmRegs; ++s) {
      rlo[s] = ~0ull;
      rhi[s] = 0ull;
    }
    for (int i0 = 0; i0 < S; i0 += kBlock) {
      const int i = i0 + tid;
      const bool occ = i < S && keys[i] != ~0u;
      const uint64_t bal = __ballot(occ);
      if (occ) {
        const uint64_t r = at + (uint64_t)__popcll(bal & ((1ull << lane) - 1ull));
        uint64_t* o = pp.out_rec + r * (uint64_t)(1 + ns);
        const bool in_cap = r < (uint64_t)pp.out_cap;  // past it: counted, not written; finalize reports the overflow
        if (in_cap) o[0] = (uint64_t)(keys[i] * kHashInv);  // the composite key back from its hash
        if (cs) {
          const uint64_t w = lds[i], c = w >> 40;
          const uint64_t sum = (uint64_t)((int64_t)(w & ((1ull << 40) - 1)) + (int64_t)c * pp.pack_min);
          if (in_cap) {
            o[1] = c;
            o[2] = sum;
          }
          rlo[0] = min(rlo[0], (unsigned long long)(c ^ (1ull << 63)));
          rhi[0] = max(rhi[0], (unsigned long long)(c ^ (1ull << 63)));
          rlo[1] = min(rlo[1], (unsigned long long)(sum ^ (1ull << 63)));
          rhi[1] = max(rhi[1], (unsigned long long)(sum ^ (1ull << 63)));
        } else if (mm_regs) {
#pragma unroll
          for (int s = 0; s < kMmRegs; ++s)
            if (s < ns) {
              const uint64_t w = lds[(int64_t)s * S + i];
              if (in_cap) o[1 + s] = w;
              rlo[s] = min(rlo[s], (unsigned long long)(w ^ (1ull << 63)));
              rhi[s] = max(rhi[s], (unsigned long long)(w ^ (1ull << 63)));
            }
        } else if (in_cap) {
          for (int s = 0; s < ns; ++s) o[1 + s] = lds[(int64_t)s * S + i];
        }
      }
      at += (uint64_t)__popcll(bal);
    }
    if (mm_regs) {
#pragma unroll
      for (int s = 0; s < kMmRegs; ++s) {
        if (s >= ns) continue;
        unsigned long long lo = rlo[s], hi = rhi[s];
        for (int o = 32; o > 0; o >>= 1) {
          const unsigned long long a = (unsigned long long)__shfl_xor((long long)lo, o);
          const unsigned long long b = (unsigned long long)__shfl_xor((long long)hi, o);
          lo = a < lo ? a : lo;
          hi = b > hi ? b : hi;
        }
        if (lane == 0) {
          atomicMin(&blk_mm[s], lo);
          atomicMax(&blk_mm[ns + s], hi);
        }
      }
    } else if (pp.out_mm) {  // many slots: per slot a pass over the round's entries, per wave one LDS atomic each
      for (int s = 0; s < ns; ++s) {
        unsigned long long lo = ~0ull, hi = 0ull;
        for (int i = tid; i < S; i += kBlock) {
          if (keys[i] == ~0u) continue;
          uint64_t w;
          if (cs) {
            const uint64_t x = lds[i], c = x >> 40;
            w = s == 0 ? c : (uint64_t)((int64_t)(x & ((1ull << 40) - 1)) + (int64_t)c * pp.pack_min);
          } else {
            w = lds[(int64_t)s * S + i];
          }
          const unsigned long long o = w ^ (1ull << 63);
          lo = o < lo ? o : lo;
          hi = o > hi ? o : hi;
        }
        for (int o = 32; o > 0; o >>= 1) {
          const unsigned long long a = (unsigned long long)__shfl_xor((long long)lo, o);
          const unsigned long long b = (unsigned long long)__shfl_xor((long long)hi, o);
          lo = a < lo ? a : lo;
          hi = b > hi ? b : hi;
        }
        if (lane == 0) {
          atomicMin(&blk_mm[s], lo);
          atomicMax(&blk_mm[ns + s], hi);
        }
      }
    }
    __syncthreads();
    n = pending;
    __syncthreads();
  }
  if (pp.out_mm)
    for (int i = tid; i < 2 * ns; i += kBlock) pp.out_mm[(int64_t)blockIdx.x * 2 * ns + i] = blk_mm[i];
}

}  // namespace pgpu
