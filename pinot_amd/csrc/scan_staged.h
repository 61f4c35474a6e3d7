// scan_staged.h — the LDS-DMA staged variant of the scan (A/B alternative, PGPU_SCAN=1).
#pragma once
#include "device.h"

namespace pgpu {

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
                                                int tid, int64_t group) {
  if (L.kind == LEAF_DOCRANGE) {
    const uint32_t m = docrange_mask(group, L.lo, L.span);
    return L.negate ? ~m : m;
  }
  if (L.kind == LEAF_BITMAP) {
    const uint32_t m = gp(L.set)[group];
    return L.negate ? ~m : m;
  }
  const int b = sidx == 0 ? R.b0 : sidx == 1 ? R.b1 : sidx == 2 ? R.b2 : R.b3;
  const int off = sidx == 0 ? 0 : sidx == 1 ? R.o1 : sidx == 2 ? R.o2 : R.o3;
  return leaf_eval_words<false>(L.kind, L.negate, L.lo, L.span, L.set, sbuf + off + tid * b, b);
}

template <int MODE>
__device__ __forceinline__ void aggregate_doc(const KParams& p, const SegView& S, int64_t doc, uint64_t* tbl,
                                              int64_t G) {
  int64_t key = 0;
  for (int j = 0; j < p.num_keys; ++j) {
    const KCol& c = S.cols[p.key_col[j]];
    key += (int64_t)gp(c.lut)[gather_id(c.fwd, c.bits, doc)] * p.key_stride[j];
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
      if (kind == SLOT_SUM_F64) dval = gp(c.dval)[id];
      else ikey = gp(c.dkey)[id];
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
          if (nl > 0 && __any(mask != 0u)) mask &= staged_leaf(R, p.leaf_stage[0], L0, sbuf, tid, group);
          if (nl > 1 && __any(mask != 0u)) mask &= staged_leaf(R, p.leaf_stage[1], L1, sbuf, tid, group);
          if (nl > 2 && __any(mask != 0u)) mask &= staged_leaf(R, p.leaf_stage[2], L2, sbuf, tid, group);
          if (nl > 3 && __any(mask != 0u)) mask &= staged_leaf(R, p.leaf_stage[3], L3, sbuf, tid, group);
        } else {
          int sp = 0;
          for (int k = 0; k < p.num_ops; ++k) {
            const int op = p.ops[k] >> 16, arg = p.ops[k] & 0xFFFF;
            if (op == OP_LEAF) {
              const LeafRegs Lk = load_leaf_regs(p, seg, arg);
              stack[sp * kBlock + tid] = staged_leaf(R, p.leaf_stage[arg], Lk, sbuf, tid, group);
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

}  // namespace pgpu
