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

// BitmapBasedFilterOperator's OR of the matching dictIds' bitmaps (BitmapBasedFilterOperator.java:85-98), one
// workgroup per 65536-doc block of a docbits region: BITMAP containers are ORed into registers (thread t owns words
// t, t + 256, ...), ARRAY containers set bits in an LDS copy of the block, and the block is stored once, coalesced
// -- no global atomics and no separate zero fill.
__global__ void __launch_bounds__(256) inv_materialize_kernel(const KBitBlock* __restrict__ blocks, int64_t num_blocks,
                                                              const KBitTask* __restrict__ tasks,
                                                              uint32_t* __restrict__ docbits) {
  __shared__ uint32_t lds[kContainerWords];
  constexpr int kPer = kContainerWords / 256;
  for (int64_t b = blockIdx.x; b < num_blocks; b += gridDim.x) {
    const KBitBlock B = blocks[b];
    uint32_t acc[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      acc[k] = 0u;
      lds[threadIdx.x + 256 * k] = 0u;
    }
    __syncthreads();
    for (int32_t i = 0; i < B.num_tasks; ++i) {
      const KBitTask T = tasks[B.task_begin + i];
      if (T.type == CONT_BITMAP) {
#pragma unroll
        for (int k = 0; k < kPer; ++k) acc[k] |= T.payload[threadIdx.x + 256 * k];
      } else {
        for (int j = threadIdx.x; j < T.n; j += 256) {
          const uint32_t v = (T.payload[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu;
          atomicOr(&lds[v >> 5], 1u << (v & 31));
        }
      }
    }
    __syncthreads();
    uint32_t* dst = docbits + B.dst;
#pragma unroll
    for (int k = 0; k < kPer; ++k) dst[threadIdx.x + 256 * k] = acc[k] | lds[threadIdx.x + 256 * k];
    __syncthreads();
  }
}

// tile -> segment map of a plan (one workgroup per segment record); also the deadline gate of the scan launch
// that follows (the scan kernels read stats[5] instead of the clock).
__global__ void expand_tiles_kernel(const uint8_t* __restrict__ segs, int32_t seg_stride, int32_t num_segs,
                                    int32_t* __restrict__ tile_seg, uint64_t deadline,
                                    unsigned long long* __restrict__ stats) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && past_deadline(deadline)) flag_timeout(stats);
  for (int s = blockIdx.x; s < num_segs; s += gridDim.x) {
    const KSegHdr* h = reinterpret_cast<const KSegHdr*>(segs + (int64_t)s * seg_stride);
    for (int i = threadIdx.x; i < h->num_tiles; i += blockDim.x) tile_seg[h->tile_base + i] = s;
  }
}

// The deadline gate alone (launches from a cached plan's device image, whose tile map needs no expansion).
__global__ void deadline_gate_kernel(uint64_t deadline, unsigned long long* __restrict__ stats) {
  if (threadIdx.x == 0 && past_deadline(deadline)) flag_timeout(stats);
}

// Deterministic fold of the per-workgroup slabs in workgroup order.
struct SlotKinds {
  int32_t k[kMaxSlots];
};
// Each block folds 8 table words; the 32 lanes of a word take every 32nd slab and their partials are combined
// in lane order: the fold itself has a fixed order, but the LDS slabs it reads were summed with atomicAdd(double),
// so FLOAT/DOUBLE sums vary in their last bits from run to run (integer slots are exact).
__device__ __forceinline__ void reduce_slabs_block(int64_t blk, const uint64_t* __restrict__ slab,
                                                   const SlotKinds& kinds, int64_t num_keys, int32_t num_slots,
                                                   int32_t num_blocks, uint64_t* __restrict__ out) {
  __shared__ uint64_t part[256];
  const int64_t words = (int64_t)num_slots * num_keys;
  const int j = threadIdx.x & 31;
  const int64_t i = blk * 8 + (threadIdx.x >> 5);
  const int kind = i < words ? kinds.k[i / num_keys] : SLOT_COUNT;
  // every 32nd slab of word i, 8 loads in flight per step (independent partial folds, combined in a fixed order)
  constexpr int U = 8;
  uint64_t acc;
  if (kind == SLOT_SUM_F64) {
    double a[U] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (i < words)
      for (int b = j; b < num_blocks; b += 32 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int bb = b + 32 * u;
          if (bb < num_blocks) a[u] += __longlong_as_double((long long)slab[(int64_t)bb * words + i]);
        }
      }
    double t = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) t += a[u];
    acc = (uint64_t)__double_as_longlong(t);
  } else {
    const int64_t init = kind == SLOT_MIN_KEY ? INT64_MAX : kind == SLOT_MAX_KEY ? INT64_MIN : 0;
    int64_t a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = init;
    if (i < words)
      for (int b = j; b < num_blocks; b += 32 * U) {
        int64_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int bb = b + 32 * u;
          v[u] = bb < num_blocks ? (int64_t)slab[(int64_t)bb * words + i] : init;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          a[u] = kind == SLOT_MIN_KEY ? min(a[u], v[u])
                 : kind == SLOT_MAX_KEY ? max(a[u], v[u])
                                        : (int64_t)((uint64_t)a[u] + (uint64_t)v[u]);  // COUNT / int SUM: wrap-free
      }
    int64_t t = init;
#pragma unroll
    for (int u = 0; u < U; ++u)
      t = kind == SLOT_MIN_KEY ? min(t, a[u]) : kind == SLOT_MAX_KEY ? max(t, a[u]) : (int64_t)((uint64_t)t + (uint64_t)a[u]);
    acc = (uint64_t)t;
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

__global__ __launch_bounds__(256) void reduce_slabs_kernel(const uint64_t* __restrict__ slab, SlotKinds kinds,
                                                           int64_t num_keys, int32_t num_slots, int32_t num_blocks,
                                                           uint64_t* __restrict__ out) {
  reduce_slabs_block(blockIdx.x, slab, kinds, num_keys, num_slots, num_blocks, out);
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
// Unordered compaction of a hash table: each workgroup takes kHashCompactChunk slots, counts its groups by ballot,
// reserves their run with one atomic and writes it (an atomic per group -- or per wave -- on the one counter
// serialised at the memory side: ~10^7 groups queued there).
constexpr int kHashCompactChunk = 4096;
__global__ __launch_bounds__(256) void compact_kernel(const uint64_t* __restrict__ table,
                                                      const unsigned long long* __restrict__ hash_keys,
                                                      int32_t num_slots, int64_t num_keys,
                                                      unsigned long long* __restrict__ counter,
                                                      uint64_t* __restrict__ out, int64_t cap) {
  __shared__ uint32_t wave_tot[4];
  __shared__ unsigned long long blk_base;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kHashCompactChunk;
  uint32_t mine = 0;
  for (int r = 0; r < kHashCompactChunk / 256; ++r) {
    const int64_t i = base + r * 256 + threadIdx.x;
    mine += (uint32_t)__popcll(__ballot(i < num_keys && table[i] != 0));  // row 0 = COUNT
  }
  if (lane == 0) wave_tot[wave] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
    blk_base = tot ? atomicAdd(counter, (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
  unsigned long long at = blk_base;
  for (int w = 0; w < wave; ++w) at += wave_tot[w];
  for (int r = 0; r < kHashCompactChunk / 256; ++r) {
    const int64_t i = base + r * 256 + threadIdx.x;
    const bool f = i < num_keys && table[i] != 0;
    const uint64_t bal = __ballot(f);
    if (f) {
      const unsigned long long j = at + (unsigned long long)__popcll(bal & ((1ull << lane) - 1ull));
      if ((int64_t)j < cap) {
        uint64_t* o = out + (int64_t)j * (1 + num_slots);
        o[0] = hash_keys ? (uint64_t)hash_keys[i] : (uint64_t)i;
        for (int s = 0; s < num_slots; ++s) o[1 + s] = table[(int64_t)s * num_keys + i];
      }
    }
    at += (unsigned long long)__popcll(bal);
  }
}

// Ordered compaction of a dense table (AggregationGroupByResult iteration in ascending key order, deterministic):
// count per chunk -> one-workgroup exclusive scan -> scatter in key order.  Columnar output: keys[cap] then
// slot s at out + (1 + s) * cap.
constexpr int kCompactChunk = kCompactChunkKeys;  // keys per workgroup (16 rounds of 256)

// minmax (optional, [2][num_slots] int64, pre-set to 0x7F.. / 0x80.. bytes): the range of every slot's words over
// the present groups, from which the dense-bitmap scatter picks each slot's byte width.
__global__ __launch_bounds__(256) void compact_count_kernel(const uint64_t* __restrict__ table, int64_t num_keys,
                                                            uint32_t* __restrict__ chunk_cnt, int32_t num_slots,
                                                            long long* __restrict__ minmax) {
  __shared__ uint32_t wsum[4];
  __shared__ long long smm[2 * kMaxSlots];
  const int64_t base = (int64_t)blockIdx.x * kCompactChunk;
  uint32_t c = 0;
  if (minmax) {
    if (threadIdx.x < 2 * num_slots) smm[threadIdx.x] = threadIdx.x < num_slots ? INT64_MAX : INT64_MIN;
    __syncthreads();
  }
  if (!minmax) {
    for (int r = 0; r < kCompactChunk / 256; ++r) {
      const int64_t k = base + r * 256 + threadIdx.x;
      c += (k < num_keys && table[k] != 0) ? 1u : 0u;  // row 0 = COUNT
    }
  } else {
    // one slot at a time: the lane folds its 16 keys, then one wave reduction per slot
    for (int s = 0; s < num_slots; ++s) {
      long long lo = INT64_MAX, hi = INT64_MIN;
      for (int r = 0; r < kCompactChunk / 256; ++r) {
        const int64_t k = base + r * 256 + threadIdx.x;
        const bool f = k < num_keys && table[k] != 0;
        if (s == 0) c += f ? 1u : 0u;
        if (f) {
          const long long v = (long long)table[(int64_t)s * num_keys + k];
          lo = min(lo, v);
          hi = max(hi, v);
        }
      }
      for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, (long long)__shfl_xor(lo, off));
        hi = max(hi, (long long)__shfl_xor(hi, off));
      }
      if ((threadIdx.x & 63) == 0 && lo <= hi) {
        atomicMin(&smm[s], lo);
        atomicMax(&smm[num_slots + s], hi);
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  // the chunk's ranges to its own row (reduced by compact_minmax_kernel): thousands of chunks' atomics on the same
  // few words serialised at the memory side and took most of this kernel's time
  if (minmax && threadIdx.x < 2 * num_slots) minmax[(int64_t)blockIdx.x * 2 * num_slots + threadIdx.x] = smm[threadIdx.x];
}

// Per slot, the min / max over the chunks' rows (compact_count_kernel) into minmax[2][num_slots].
__global__ __launch_bounds__(256) void compact_minmax_kernel(const long long* __restrict__ rows, int64_t nch,
                                                             int32_t num_slots, long long* __restrict__ minmax) {
  __shared__ long long part[4];
  for (int s = 0; s < 2 * num_slots; ++s) {
    const bool is_min = s < num_slots;
    long long v = is_min ? INT64_MAX : INT64_MIN;
    for (int64_t c = threadIdx.x; c < nch; c += blockDim.x) {
      const long long x = rows[c * 2 * num_slots + s];
      v = is_min ? min(v, x) : max(v, x);
    }
    for (int off = 32; off > 0; off >>= 1) {
      const long long y = __shfl_xor(v, off);
      v = is_min ? min(v, y) : max(v, y);
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < 4; ++w) v = is_min ? min(v, part[w]) : max(v, part[w]);
      minmax[s] = v;
    }
    __syncthreads();
  }
}

// Byte width of a slot's words in the compact form: the narrowest two's-complement width holding [lo, hi], 1-4 or 8
// bytes (float64 sums always 8).  3 bytes (r05): C5's SUM(m) needs 17 bits -- 10 MB less over PCIe per query.
__device__ __host__ inline int slot_width(long long lo, long long hi, int kind) {
  if (kind == SLOT_SUM_F64) return 8;
  if (lo >= -128 && hi <= 127) return 1;
  if (lo >= -32768 && hi <= 32767) return 2;
  if (lo >= -(1ll << 23) && hi < (1ll << 23)) return 3;
  if (lo >= (long long)INT32_MIN && hi <= (long long)INT32_MAX) return 4;
  return 8;
}


// Compact form of a dense table (large key spaces where most keys are present, C5): a presence bitmap over the
// keys (bit k of word k / 64; one ballot per 64 keys) and each slot's words of the present keys in key order at the
// width slot_width picks from the count kernel's ranges -- keys need no bytes at all, and narrow words cut the
// copy to the host (the AggregationGroupByResult iterator decodes keys from the holder's raw keys in the same way).
// out: [ceil(num_keys / 64) u64 bitmap] then slot s at out_slots + s * cap * 8 (narrow values from its start).
__global__ __launch_bounds__(256) void compact_dense_scatter_kernel(const uint64_t* __restrict__ table,
                                                                    int32_t num_slots, int64_t num_keys,
                                                                    const uint32_t* __restrict__ chunk_off,
                                                                    SlotKinds kinds,
                                                                    const long long* __restrict__ minmax,
                                                                    uint64_t* __restrict__ bitmap,
                                                                    uint8_t* __restrict__ out_slots, int64_t cap) {
  __shared__ uint32_t wcnt[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kCompactChunk;
  int width[kMaxSlots];
  for (int s = 0; s < num_slots; ++s) width[s] = slot_width(minmax[s], minmax[num_slots + s], kinds.k[s]);
  uint32_t pos = chunk_off[blockIdx.x];
  for (int r = 0; r < kCompactChunk / 256; ++r) {
    const int64_t k = base + r * 256 + threadIdx.x;
    const bool f = k < num_keys && table[k] != 0;
    const unsigned long long bal = __ballot(f);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    if (lane == 0) {
      wcnt[wave] = (uint32_t)__popcll(bal);
      const int64_t wk = base + r * 256 + wave * 64;  // first key of this wave: a multiple of 64
      if (wk < num_keys) bitmap[wk >> 6] = bal;
    }
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wave; ++w) before += wcnt[w];
    const uint32_t round_total = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if (f) {
      const int64_t j = (int64_t)pos + before + rank;
      if (j < cap) {
        for (int s = 0; s < num_slots; ++s) {
          const uint64_t v = table[(int64_t)s * num_keys + k];
          put_compact(out_slots + (int64_t)s * cap * 8, j, width[s], v);
        }
      }
    }
    pos += round_total;
    __syncthreads();
  }
}

// One workgroup: exclusive prefix of chunk_cnt (in place) and the total into *total.
__global__ __launch_bounds__(1024) void compact_scan_kernel(uint32_t* __restrict__ chunk, int32_t n,
                                                            unsigned long long* __restrict__ total) {
  __shared__ uint32_t wsum[16];
  __shared__ unsigned long long carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int base = 0; base < n; base += 1024) {
    const int i = base + threadIdx.x;
    const uint32_t v = i < n ? chunk[i] : 0u;
    uint32_t x = v;  // inclusive wave scan
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    const unsigned long long c = carry;
    if (i < n) chunk[i] = (uint32_t)(c + before + x - v);
    __syncthreads();
    if (threadIdx.x == 1023) carry = c + before + x;
    __syncthreads();
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

// Output (columnar, stride cap): group-by dictIds gid[j] = (key / stride[j]) % card[j] as int32 rows [num_keys][cap],
// then the slot words as u64 rows [num_slots][cap] starting at byte offset num_keys * cap * 4 (8-aligned cap).
struct KeyDecode {
  int64_t stride[kMaxKeys];
  int64_t card[kMaxKeys];
  int64_t off[kMaxKeys];  // first global id of each key digit
  int64_t base;  // composite key of table column 0 (a key-range shard of the table)
  int32_t n;
};
__global__ __launch_bounds__(256) void compact_scatter_kernel(const uint64_t* __restrict__ table, int32_t num_slots,
                                                              int64_t num_keys, const uint32_t* __restrict__ chunk_off,
                                                              const KeyDecode kd, uint8_t* __restrict__ out,
                                                              int64_t cap) {
  __shared__ uint32_t wcnt[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kCompactChunk;
  int32_t* gid = reinterpret_cast<int32_t*>(out);
  uint64_t* words = reinterpret_cast<uint64_t*>(out + (int64_t)kd.n * cap * 4);
  uint32_t pos = chunk_off[blockIdx.x];
  for (int r = 0; r < kCompactChunk / 256; ++r) {
    const int64_t k = base + r * 256 + threadIdx.x;
    const bool f = k < num_keys && table[k] != 0;
    const unsigned long long bal = __ballot(f);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    if (lane == 0) wcnt[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wave; ++w) before += wcnt[w];
    const uint32_t round_total = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if (f) {
      const int64_t j = (int64_t)pos + before + rank;
      if (j < cap) {
        for (int c = 0; c < kd.n; ++c)
          gid[(int64_t)c * cap + j] = (int32_t)(((kd.base + k) / kd.stride[c]) % kd.card[c] + kd.off[c]);
        for (int s = 0; s < num_slots; ++s) words[(int64_t)s * cap + j] = table[(int64_t)s * num_keys + k];
      }
    }
    pos += round_total;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------- cross-GPU exchange
// Hash-mode group tables across GPUs (GroupByOrderByCombineOperator's IndexedTable.upsert merge,
// core/operator/combine/GroupByOrderByCombineOperator.java:170-181, as a hash-partitioned all-to-all): every rank
// splits its table's groups by owner rank (a mix of the global composite key, so every rank sends each key to the same
// owner), the records travel over RCCL, and the owner merges what it receives into a fresh table of its own.
constexpr int kMaxExchangeParts = 64;
__device__ __forceinline__ int32_t exchange_part(uint64_t key, int32_t nparts) {
  uint64_t h = key * 0xD6E8FEB86659FD93ull;
  h ^= h >> 32;
  return (int32_t)(h % (uint64_t)nparts);
}

// Per-owner group counts: block-local LDS histogram, one global atomic per (block, owner).
__global__ __launch_bounds__(256) void exchange_count_kernel(const uint64_t* __restrict__ table,
                                                             const unsigned long long* __restrict__ hash_keys,
                                                             int64_t num_keys, int32_t nparts,
                                                             unsigned long long* __restrict__ counts) {
  __shared__ uint32_t h[kMaxExchangeParts];
  if (threadIdx.x < kMaxExchangeParts) h[threadIdx.x] = 0u;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < num_keys; i += (int64_t)gridDim.x * blockDim.x)
    if (table[i] != 0) atomicAdd(&h[exchange_part((uint64_t)hash_keys[i], nparts)], 1u);  // row 0 = COUNT
  __syncthreads();
  if (threadIdx.x < nparts && h[threadIdx.x]) atomicAdd(counts + threadIdx.x, (unsigned long long)h[threadIdx.x]);
}

// Records [key, slot words] grouped by owner: cursor[p] starts at owner p's first record.  A wave reserves its
// records of one owner with one atomic (ballot per owner), so the few hot cursors see one update per wave and owner.
// conv bit s: slot s is an int64 SUM whose agreed cross-rank kind is float64 (one rank's sum could overflow int64):
// its word leaves as the double of the value.
__global__ __launch_bounds__(256) void exchange_scatter_kernel(const uint64_t* __restrict__ table,
                                                               const unsigned long long* __restrict__ hash_keys,
                                                               int64_t num_keys, int32_t num_slots, int32_t nparts,
                                                               uint32_t conv, unsigned long long* __restrict__ cursor,
                                                               uint64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < num_keys; base += stride) {  // wave-uniform trip count
    const int64_t i = base + threadIdx.x;
    const bool f = i < num_keys && table[i] != 0;
    const uint64_t key = f ? (uint64_t)hash_keys[i] : 0ull;
    const int32_t part = f ? exchange_part(key, nparts) : -1;
    int64_t j = -1;
    for (int p = 0; p < nparts; ++p) {
      const unsigned long long m = __ballot(part == p);
      if (!m) continue;
      unsigned long long b = 0;
      const int leader = __builtin_ctzll(m);
      if (lane == leader) b = atomicAdd(cursor + p, (unsigned long long)__popcll(m));
      b = __shfl(b, leader);
      if (part == p)
        j = (int64_t)b + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    }
    if (j >= 0) {
      uint64_t* o = out + j * (1 + num_slots);
      o[0] = key;
      for (int s = 0; s < num_slots; ++s) {
        uint64_t w = table[(int64_t)s * num_keys + i];
        if ((conv >> s) & 1u) w = (uint64_t)__double_as_longlong((double)(long long)w);
        o[1 + s] = w;
      }
    }
  }
}

// The owner's merge: every received record is upserted into the (freshly initialised) hash table, its words folded
// per slot kind -- AggregationFunction.merge of SUM / COUNT / MIN / MAX (MIN / MAX on order-preserving keys).
__global__ __launch_bounds__(256) void merge_records_kernel(const uint64_t* __restrict__ rec, int64_t n,
                                                            int32_t num_slots, SlotKinds kinds,
                                                            uint64_t* __restrict__ table,
                                                            unsigned long long* __restrict__ hash_keys,
                                                            int64_t num_keys) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* e = rec + r * (1 + num_slots);
    const int64_t slot = hash_slot(hash_keys, num_keys, e[0], nullptr);  // 2 x n slots: never full
    if (slot < 0) continue;
    for (int s = 0; s < num_slots; ++s) {
      uint64_t* w = table + (int64_t)s * num_keys + slot;
      const uint64_t v = e[1 + s];
      switch (kinds.k[s]) {
        case SLOT_COUNT: case SLOT_SUM_I64: atomicAdd(reinterpret_cast<unsigned long long*>(w), (unsigned long long)v); break;
        case SLOT_SUM_F64: atomicAdd(reinterpret_cast<double*>(w), __longlong_as_double((long long)v)); break;
        case SLOT_MIN_KEY: atomicMin(reinterpret_cast<long long*>(w), (long long)v); break;
        default: atomicMax(reinterpret_cast<long long*>(w), (long long)v); break;
      }
    }
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

// ---------------------------------------------------------------------------------------------- filter stats
// numEntriesScannedInFilter of STATS_LEAP2 segments (AndDocIdIterator over two SVScanDocIdIterators,
// AndDocIdIterator.java:40-67): the scan kernel counted every entry assuming each wave-tile is entered with scan A
// running, and left one byte per (tile, wave) (bit 0: a doc matches, bit 1: scanner after it, bits 2-3: count
// difference at its first match when entered with B running, + 1).  One wave per segment chains the bytes in doc
// order from the initial state (scan A at doc 0), 512 at a time (8 per lane): a byte's entry state is the exit of the nearest
// earlier byte with a match (ballots), or the state carried from the previous 64.
__device__ __forceinline__ void leap2_compose_block(int blk, const uint8_t* __restrict__ segs, int32_t seg_stride,
                                                    int32_t num_segs, const uint8_t* __restrict__ maps,
                                                    unsigned long long* __restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const int s = blk * (blockDim.x / 64) + (threadIdx.x >> 6);
  // (no early return: the block's waves meet at the barrier below)
  const KSegHdr* h = s < num_segs ? reinterpret_cast<const KSegHdr*>(segs + (int64_t)s * seg_stride) : nullptr;
  const bool leap = h && (h->stats & 3) == KSTATS_LEAP2;  // wave-uniform
  const uint8_t* m = leap ? maps + (int64_t)h->tile_base * (kBlock / 64) : maps;
  const int64_t n = leap ? (int64_t)h->num_tiles * (kBlock / 64) : 0;
  long long total = 0;
  uint32_t carry = 0;  // scanner state entering this batch (0 = A)
  // 512 bytes per step (a 1M-doc segment's 492 in one): lane l holds bytes [8l, 8l + 8), all loads in flight
  // together, folded in the lane, then one ballot pass hands each lane the state entering its first match.
  for (int64_t base = 0; base < n; base += 512) {
    uint32_t b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t i = base + 8 * lane + k;
      b[k] = i < n ? m[i] : 0u;
    }
    long long t = 0;
    int first_diff = 0;
    bool has = false;
    uint32_t st = 0;  // exit state of the lane's latest matching byte
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (b[k] & 1u) {
        const int d = (int)((b[k] >> 2) & 3u) - 1;
        if (has) t += st ? d : 0;
        else first_diff = d;
        st = (b[k] >> 1) & 1u;
        has = true;
      }
    }
    const uint64_t hasm = __ballot(has), exm = __ballot(has && st);
    const uint64_t below = hasm & ((1ull << lane) - 1ull);
    const uint32_t entry = below ? (uint32_t)((exm >> (63 - __builtin_clzll(below))) & 1ull) : carry;
    if (has && entry) t += first_diff;
    total += t;
    if (hasm) carry = (uint32_t)((exm >> (63 - __builtin_clzll(hasm))) & 1ull);
  }
  for (int off = 32; off > 0; off >>= 1) total += __shfl_xor(total, off);
  // one atomic per block, not per segment: same-address atomics serialize (~11 ns each), and 1 000 segments' adds
  // took ~9 us of the epilogue
  __shared__ long long wsum[4];
  if (lane == 0) wsum[threadIdx.x >> 6] = total;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int w = 0; w < (int)(blockDim.x / 64) && w < 4; ++w) t += wsum[w];
    if (t) atomicAdd(stats + 2, (unsigned long long)t);
  }
}

__global__ __launch_bounds__(256) void leap2_compose_kernel(const uint8_t* __restrict__ segs, int32_t seg_stride,
                                                           int32_t num_segs, const uint8_t* __restrict__ maps,
                                                           unsigned long long* __restrict__ stats) {
  leap2_compose_block(blockIdx.x, segs, seg_stride, num_segs, maps, stats);
}

// The epilogue of a one-launch LDS-table plan in one launch: the slab fold's blocks, then the leap-frog statistics'
// blocks (independent work; one launch gap and one kernel tail less per query).  host_out (small tables): the last
// block to finish copies the table and the statistics words into pinned host memory, which finalize reads once the
// stream has completed -- no copy launch behind the epilogue -- and re-arms the block counter `done` for the next use.
__global__ __launch_bounds__(256) void epilogue_kernel(const uint64_t* __restrict__ slab, SlotKinds kinds,
                                                       int64_t num_keys, int32_t num_slots, int32_t num_blocks,
                                                       uint64_t* __restrict__ out, int32_t reduce_blocks,
                                                       const uint8_t* __restrict__ segs, int32_t seg_stride,
                                                       int32_t num_segs, const uint8_t* __restrict__ maps,
                                                       unsigned long long* __restrict__ stats,
                                                       uint64_t* __restrict__ host_out, unsigned int* __restrict__ done) {
  if ((int)blockIdx.x < reduce_blocks)  // block-uniform
    reduce_slabs_block(blockIdx.x, slab, kinds, num_keys, num_slots, num_blocks, out);
  else
    leap2_compose_block((int)blockIdx.x - reduce_blocks, segs, seg_stride, num_segs, maps, stats);
  if (!host_out) return;
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();  // this block's table words and statistics adds before its count
    last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  const int64_t words = (int64_t)num_slots * num_keys;
  for (int64_t i = threadIdx.x; i < words + 6; i += blockDim.x) {
    const uint64_t v = i < words ? __hip_atomic_load(out + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : (uint64_t)__hip_atomic_load(stats + (i - words), __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(host_out + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The leaves' match bitmaps of STATS_GENERIC segments (the replay of filter_stats.cpp runs on the host).
__global__ __launch_bounds__(kBlock) void leaf_masks_kernel(const KParams p, const KMaskJob* __restrict__ jobs,
                                                           uint32_t* __restrict__ out) {
  const KMaskJob J = jobs[blockIdx.x];
  const SegView S = seg_view(p, J.rec);
  const int64_t ngroups = ((int64_t)S.hdr->num_docs + 31) >> 5;
  const int64_t g = (int64_t)J.group0 + threadIdx.x;
  if (g >= ngroups) return;
  for (int l = 0; l < p.num_leaves; ++l)
    out[J.out_word + (int64_t)l * ngroups + g] = leaf_mask(S.leaves[l], S.cols[p.leaf_col[l]], g);
}

// One reading of the device's constant-rate wall clock (host calibration of query deadlines).
__global__ void read_clock_kernel(uint64_t* out) {
  if (threadIdx.x == 0) out[0] = (uint64_t)wall_clock64();
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

// Raw-value filter leaves: one thread per 32-doc group writes its docbits word (raw_group_mask, negated for
// NOT_EQ / NOT_IN, bits past numDocs cleared).  The scans then read the leaf as a LEAF_BITMAP.
__global__ __launch_bounds__(256) void raw_leaf_bitmap_kernel(const KRawJob* __restrict__ jobs,
                                                              const KRawTask* __restrict__ tasks,
                                                              const int64_t* __restrict__ raw_vals,
                                                              uint32_t* __restrict__ docbits) {
  const KRawJob J = jobs[blockIdx.x];
  const KRawTask T = tasks[J.task];
  const int64_t g = (int64_t)J.group0 + threadIdx.x;
  const int64_t ngroups = ((int64_t)T.num_docs + 31) >> 5;
  if (g >= ngroups) return;
  uint32_t m = raw_group_mask(T.kind, T.lo, T.hi, T.kind == LEAF_RAW_IN ? raw_vals + T.lo : nullptr, T.keys, g);
  if (T.negate) m = ~m;
  const int64_t rem = (int64_t)T.num_docs - (g << 5);
  if (rem < 32) m &= (1u << rem) - 1u;
  docbits[T.dst + g] = m;
}

int launch_raw_leaf_bitmaps(const KRawJob* jobs, int64_t num_jobs, const KRawTask* tasks, const int64_t* raw_vals,
                            uint32_t* docbits, void* stream) {
  if (num_jobs <= 0) return 0;
  if (num_jobs > INT32_MAX) return -1;
  hipLaunchKernelGGL(raw_leaf_bitmap_kernel, dim3((unsigned)num_jobs), dim3(256), 0, S(stream), jobs, tasks, raw_vals,
                     docbits);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_inv_materialize(const KBitBlock* blocks, int64_t num_blocks, const KBitTask* tasks, uint32_t* docbits,
                           void* stream) {
  if (num_blocks <= 0) return 0;
  const int64_t grid = num_blocks < 65536 ? num_blocks : 65536;
  hipLaunchKernelGGL(inv_materialize_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), blocks, num_blocks, tasks,
                     docbits);
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

// Largest dictId of a pinned fixed-bit forward index (pgpu_pin_segment): a value >= the column's cardinality would
// index past its dictionary / translation arrays in every later scan, so the pin rejects it (Pinot's reader would
// throw ArrayIndexOutOfBoundsException on the first such doc).  Byte reads of the big-endian bit stream; pin-time only.
__global__ __launch_bounds__(256) void fwd_max_kernel(const uint8_t* __restrict__ fwd, int64_t n, int32_t bits,
                                                      unsigned int* __restrict__ out) {
  uint32_t m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t bit = (uint64_t)i * (uint64_t)bits;
    const int64_t byte = (int64_t)(bit >> 3);
    const int sh = (int)(bit & 7);
    const int nb = (sh + bits + 7) >> 3;
    uint64_t w = 0;
    for (int k = 0; k < nb; ++k) w = (w << 8) | fwd[byte + k];
    const uint32_t v = (uint32_t)((w >> (nb * 8 - sh - bits)) & ((1ull << bits) - 1));
    m = v > m ? v : m;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t x = (uint32_t)__shfl_xor((int)m, o);
    m = x > m ? x : m;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

int launch_fwd_max(const void* d_fwd, int64_t n, int32_t bits, unsigned int* d_out, void* stream) {
  if (n <= 0) return 0;
  if (bits < 1 || bits > 31) return -1;
  int64_t grid = (n + 255) / 256;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(fwd_max_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream),
                     reinterpret_cast<const uint8_t*>(d_fwd), n, bits, d_out);
  return PGPU_HIP_OK(hipGetLastError());
}

// KParams.pack_slot of a hash plan: every occupied slot's pack word holds (count << shift) | sum; split it into the
// COUNT row (slot 0) and the SUM row so finalize, combine and compaction read the plain table layout.
__global__ __launch_bounds__(256) void hash_unpack_kernel(uint64_t* __restrict__ table,
                                                          const unsigned long long* __restrict__ keys, int64_t cap,
                                                          int32_t pack_slot, int32_t shift) {
  const uint64_t mask = (1ull << shift) - 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
    if (keys[i] == ~0ull) continue;
    const uint64_t w = table[(int64_t)pack_slot * cap + i];
    table[i] = w >> shift;
    table[(int64_t)pack_slot * cap + i] = w & mask;
  }
}

int launch_hash_unpack(uint64_t* table, const unsigned long long* hash_keys, int64_t cap, int32_t pack_slot,
                       int32_t shift, void* stream) {
  if (cap <= 0) return 0;
  if (pack_slot <= 0 || pack_slot >= kMaxSlots || shift <= 0 || shift >= 64) return -1;
  int64_t grid = (cap + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(hash_unpack_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), table, hash_keys, cap,
                     pack_slot, shift);
  return PGPU_HIP_OK(hipGetLastError());
}

// One object per (kernel family, mode): k_direct.hip / k_startree.hip compiled with -DPGPU_MODE=0,1,2.
int launch_direct_mode0(const KParams& p, int variant, int grid, size_t lds_bytes, void* stream);
int launch_direct_mode1(const KParams& p, int variant, int grid, size_t lds_bytes, void* stream);
int launch_direct_mode2(const KParams& p, int variant, int grid, size_t lds_bytes, void* stream);
int occupancy_direct_mode0(int variant, size_t lds_bytes);
int occupancy_direct_mode1(int variant, size_t lds_bytes);
int occupancy_direct_mode2(int variant, size_t lds_bytes);

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

int launch_filter_groupby(const KParams& p, int mode, int variant, int grid, size_t lds_bytes, void* stream) {
  switch (mode) {
    case MODE_LDS: return launch_direct_mode0(p, variant, grid, lds_bytes, stream);
    case MODE_GLOBAL: return launch_direct_mode1(p, variant, grid, lds_bytes, stream);
    default: return launch_direct_mode2(p, variant, grid, lds_bytes, stream);
  }
}

int occupancy_filter_groupby(int mode, int variant, size_t lds_bytes) {
  switch (mode) {
    case MODE_LDS: return occupancy_direct_mode0(variant, lds_bytes);
    case MODE_GLOBAL: return occupancy_direct_mode1(variant, lds_bytes);
    default: return occupancy_direct_mode2(variant, lds_bytes);
  }
}

int launch_expand_tiles(const uint8_t* segs, int32_t seg_stride, int32_t num_segs, int32_t* tile_seg,
                        uint64_t deadline, unsigned long long* stats, void* stream) {
  if (num_segs <= 0) return 0;
  hipLaunchKernelGGL(expand_tiles_kernel, dim3(num_segs < 4096 ? num_segs : 4096), dim3(128), 0, S(stream), segs,
                     seg_stride, num_segs, tile_seg, deadline, stats);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_deadline_gate(uint64_t deadline, unsigned long long* stats, void* stream) {
  hipLaunchKernelGGL(deadline_gate_kernel, dim3(1), dim3(64), 0, S(stream), deadline, stats);
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
  int64_t grid = (num_keys + kHashCompactChunk - 1) / kHashCompactChunk;
  if (grid < 1) grid = 1;
  if (grid > INT32_MAX) return -1;
  hipLaunchKernelGGL(compact_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), table, hash_keys, num_slots,
                     num_keys, counter, out, out_cap);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_exchange_count(const uint64_t* table, const unsigned long long* hash_keys, int64_t num_keys, int32_t nparts,
                          unsigned long long* counts, void* stream) {
  if (nparts < 1 || nparts > kMaxExchangeParts) return -1;
  int64_t grid = (num_keys + 255) / 256;
  grid = grid < 1 ? 1 : grid > 2048 ? 2048 : grid;
  hipLaunchKernelGGL(exchange_count_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), table, hash_keys, num_keys,
                     nparts, counts);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_exchange_scatter(const uint64_t* table, const unsigned long long* hash_keys, int64_t num_keys,
                            int32_t num_slots, int32_t nparts, uint32_t conv, unsigned long long* cursor, uint64_t* out,
                            void* stream) {
  if (nparts < 1 || nparts > kMaxExchangeParts || num_slots > kMaxSlots) return -1;
  int64_t grid = (num_keys + 255) / 256;
  grid = grid < 1 ? 1 : grid > 2048 ? 2048 : grid;
  hipLaunchKernelGGL(exchange_scatter_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), table, hash_keys, num_keys,
                     num_slots, nparts, conv, cursor, out);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_merge_records(const uint64_t* rec, int64_t n, int32_t num_slots, const int32_t* slot_kind, uint64_t* table,
                         unsigned long long* hash_keys, int64_t num_keys, void* stream) {
  if (n <= 0) return 0;
  if (num_slots > kMaxSlots) return -1;
  SlotKinds k{};
  for (int i = 0; i < num_slots; ++i) k.k[i] = slot_kind[i];
  int64_t grid = (n + 255) / 256;
  grid = grid > 4096 ? 4096 : grid;
  hipLaunchKernelGGL(merge_records_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), rec, n, num_slots, k, table,
                     hash_keys, num_keys);
  return PGPU_HIP_OK(hipGetLastError());
}

// Cross-GPU combine: an int64 SUM row of a dense table rewritten as float64 words in place, when another rank's sum of
// the same slot is float64 (the ranks' overflow guards differ); grid-stride, one word per lane.
__global__ void i64_to_f64_kernel(uint64_t* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (uint64_t)__double_as_longlong((double)(long long)p[i]);
}

int launch_i64_to_f64(uint64_t* p, int64_t n, void* stream) {
  if (n <= 0) return 0;
  int64_t grid = (n + 255) / 256;
  grid = grid > 4096 ? 4096 : grid;
  hipLaunchKernelGGL(i64_to_f64_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), p, n);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_exclusive_scan_u32(uint32_t* data, int32_t n, void* stream) {
  if (n < 1) return 0;
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, S(stream), data, n,
                     static_cast<unsigned long long*>(nullptr));
  return PGPU_HIP_OK(hipGetLastError());
}

int64_t compact_ordered_chunks(int64_t num_keys) { return (num_keys + kCompactChunk - 1) / kCompactChunk; }
size_t compact_scratch_bytes(int64_t num_keys, int32_t num_slots) {
  const int64_t nch = std::max<int64_t>(compact_ordered_chunks(num_keys), 1);
  return (size_t)((nch * 4 + 7) & ~int64_t(7)) + (size_t)nch * 2 * num_slots * 8;
}

int launch_compact_ordered(const uint64_t* table, int32_t num_slots, int64_t num_keys, int64_t key_base,
                           const int64_t* key_stride, const int64_t* key_card, const int64_t* key_off,
                           int32_t num_key_cols, uint32_t* chunk_scratch,
                           unsigned long long* total, void* out, int64_t cap, void* stream) {
  const int64_t nch = compact_ordered_chunks(num_keys);
  if (nch < 1 || nch > INT32_MAX || num_key_cols > kMaxKeys || (cap & 1)) return -1;
  KeyDecode kd{};
  kd.n = num_key_cols;
  kd.base = key_base;
  for (int j = 0; j < num_key_cols; ++j) {
    kd.stride[j] = key_stride[j];
    kd.card[j] = key_card[j];
    kd.off[j] = key_off[j];
  }
  hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)nch), dim3(256), 0, S(stream), table, num_keys, chunk_scratch,
                     num_slots, static_cast<long long*>(nullptr));
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, S(stream), chunk_scratch, (int32_t)nch, total);
  hipLaunchKernelGGL(compact_scatter_kernel, dim3((unsigned)nch), dim3(256), 0, S(stream), table, num_slots, num_keys,
                     chunk_scratch, kd, reinterpret_cast<uint8_t*>(out), cap);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_compact_dense_count(const uint64_t* table, int32_t num_slots, int64_t num_keys, uint32_t* chunk_scratch,
                               unsigned long long* total, long long* minmax, void* stream, bool counted) {
  const int64_t nch = compact_ordered_chunks(num_keys);
  if (nch < 1 || nch > INT32_MAX || num_slots > kMaxSlots) return -1;
  // per-chunk ranges after the counts in chunk_scratch (compact_scratch_bytes), reduced into minmax
  long long* rows = reinterpret_cast<long long*>(reinterpret_cast<uint8_t*>(chunk_scratch) + ((nch * 4 + 7) & ~int64_t(7)));
  if (!counted)
    hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)nch), dim3(256), 0, S(stream), table, num_keys,
                       chunk_scratch, num_slots, minmax ? rows : nullptr);
  if (minmax)
    hipLaunchKernelGGL(compact_minmax_kernel, dim3(1), dim3(256), 0, S(stream), rows, nch, num_slots, minmax);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, S(stream), chunk_scratch, (int32_t)nch, total);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_compact_dense_scatter(const uint64_t* table, int32_t num_slots, int64_t num_keys, const int32_t* slot_kind,
                                 const uint32_t* chunk_scratch, const long long* minmax, uint64_t* bitmap,
                                 void* out_slots, int64_t cap, void* stream) {
  const int64_t nch = compact_ordered_chunks(num_keys);
  if (nch < 1 || nch > INT32_MAX || num_slots > kMaxSlots) return -1;
  SlotKinds k{};
  for (int i = 0; i < num_slots; ++i) k.k[i] = slot_kind[i];
  hipLaunchKernelGGL(compact_dense_scatter_kernel, dim3((unsigned)nch), dim3(256), 0, S(stream), table, num_slots,
                     num_keys, chunk_scratch, k, minmax, bitmap, reinterpret_cast<uint8_t*>(out_slots), cap);
  return PGPU_HIP_OK(hipGetLastError());
}

int compact_slot_width(long long lo, long long hi, int kind) { return slot_width(lo, hi, kind); }
int launch_compact_ordered_scatter(const uint64_t* table, int32_t num_slots, int64_t num_keys, int64_t key_base,
                                   const int64_t* key_stride, const int64_t* key_card, const int64_t* key_off,
                                   int32_t num_key_cols, const uint32_t* chunk_scratch, void* out, int64_t cap,
                                   void* stream) {
  const int64_t nch = compact_ordered_chunks(num_keys);
  if (nch < 1 || nch > INT32_MAX || num_key_cols > kMaxKeys || (cap & 1)) return -1;
  KeyDecode kd{};
  kd.n = num_key_cols;
  kd.base = key_base;
  for (int j = 0; j < num_key_cols; ++j) {
    kd.stride[j] = key_stride[j];
    kd.card[j] = key_card[j];
    kd.off[j] = key_off[j];
  }
  hipLaunchKernelGGL(compact_scatter_kernel, dim3((unsigned)nch), dim3(256), 0, S(stream), table, num_slots, num_keys,
                     chunk_scratch, kd, reinterpret_cast<uint8_t*>(out), cap);
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

int launch_epilogue(const uint64_t* slab, const int32_t* slot_kind, int32_t num_slots, int64_t num_keys,
                    int32_t num_blocks, uint64_t* out, const uint8_t* segs, int32_t seg_stride, int32_t num_segs,
                    const uint8_t* maps, unsigned long long* stats, uint64_t* host_out, unsigned int* done,
                    void* stream) {
  SlotKinds k{};
  for (int i = 0; i < num_slots && i < kMaxSlots; ++i) k.k[i] = slot_kind[i];
  const int64_t reduce_blocks = ((int64_t)num_slots * num_keys + 7) / 8;
  const int64_t leap_blocks = num_segs > 0 ? (num_segs + 3) / 4 : 0;
  if (reduce_blocks + leap_blocks < 1) return 0;
  hipLaunchKernelGGL(epilogue_kernel, dim3((unsigned)(reduce_blocks + leap_blocks)), dim3(256), 0, S(stream), slab, k,
                     num_keys, num_slots, num_blocks, out, (int32_t)reduce_blocks, segs, seg_stride, num_segs, maps,
                     stats, host_out, done);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_leap2_compose(const uint8_t* segs, int32_t seg_stride, int32_t num_segs, const uint8_t* maps,
                         unsigned long long* stats, void* stream) {
  if (num_segs <= 0) return 0;
  hipLaunchKernelGGL(leap2_compose_kernel, dim3((num_segs + 3) / 4), dim3(256), 0, S(stream), segs, seg_stride,
                     num_segs, maps, stats);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_leaf_masks(const KParams& p, const KMaskJob* jobs, int32_t num_jobs, uint32_t* out, void* stream) {
  if (num_jobs <= 0) return 0;
  hipLaunchKernelGGL(leaf_masks_kernel, dim3(num_jobs), dim3(kBlock), 0, S(stream), p, jobs, out);
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

int launch_read_clock(uint64_t* out, void* stream) {
  hipLaunchKernelGGL(read_clock_kernel, dim3(1), dim3(64), 0, S(stream), out);
  return PGPU_HIP_OK(hipGetLastError());
}

}  // namespace pgpu
