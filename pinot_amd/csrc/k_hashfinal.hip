// k_hashfinal.hip — finalize of a hash-mode group table on the device: the compacted records (one per group:
// composite key, slot words; in hash / partition order) are decoded into the result's columnar layout (int32 dictIds
// per group-by column, then the u64 slot words) or narrowed into the compact form, in one streaming pass, so the host
// copies one buffer instead of decoding millions of rows (AggregationGroupByResult iteration,
// DictionaryBasedGroupKeyGenerator.getKeys, core/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:
// 608-624 for the LONG_MAP holder).  No sort: the LONG_MAP holder iterates its groups in fastutil hash order
// (:693, :719) and no consumer of a group-by result depends on group order (ORDER BY / trims sort the rows they keep).
#include "device.h"

namespace pgpu {

struct KeyDecode {
  int64_t stride[kMaxKeys];
  int64_t card[kMaxKeys];
  int64_t off[kMaxKeys];
};

// Record r's dictIds (key / stride % card + off per column) and slot words, at row r of the columnar result.
__global__ __launch_bounds__(256) void hash_decode_kernel(const uint64_t* __restrict__ rec, int64_t n, int32_t num_slots,
                                                          int32_t num_keys, KeyDecode kd, int32_t* __restrict__ gid,
                                                          uint64_t* __restrict__ slots) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* e = rec + r * (1 + num_slots);
    const uint64_t key = e[0];
    for (int j = 0; j < num_keys; ++j)
      gid[(int64_t)j * n + r] = (int32_t)((key / (uint64_t)kd.stride[j]) % (uint64_t)kd.card[j] + kd.off[j]);
    for (int s = 0; s < num_slots; ++s) slots[(int64_t)s * n + r] = e[1 + s];
  }
}

// Per slot, the range of the words of the first min(*count, cap) records (the compact result form picks each
// slot's width from it): signed values stored order-preserving as u64 (v ^ 2^63) in mm[s] (min, preset to ~0)
// and mm[num_slots + s] (max, preset to 0).  The record count is read on the device, so this launches before the
// host has seen it.
__global__ __launch_bounds__(256) void hash_minmax_kernel(const uint64_t* __restrict__ rec,
                                                          const unsigned long long* __restrict__ count, int64_t cap,
                                                          int32_t num_slots, unsigned long long* __restrict__ mm) {
  __shared__ unsigned long long part[2][256 / 64];
  const int64_t n = (int64_t)(*count < (unsigned long long)cap ? *count : (unsigned long long)cap);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int s = 0; s < num_slots; ++s) {
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
      const unsigned long long v = rec[r * (1 + num_slots) + 1 + s] ^ (1ull << 63);
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long a = (unsigned long long)__shfl_xor((long long)lo, o);
      const unsigned long long b = (unsigned long long)__shfl_xor((long long)hi, o);
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    if (lane == 0) {
      part[0][wave] = lo;
      part[1][wave] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // one atomic per workgroup and bound (a few hundred at each address, not thousands)
      for (int w = 1; w < 256 / 64; ++w) {
        lo = part[0][w] < lo ? part[0][w] : lo;
        hi = part[1][w] > hi ? part[1][w] : hi;
      }
      atomicMin(&mm[s], lo);
      atomicMax(&mm[num_slots + s], hi);
    }
    __syncthreads();
  }
}

struct SlotWidths {
  int32_t w[kMaxSlots];
  int64_t off[kMaxSlots];  // byte offset of slot s's narrow words in `out`
};

// Record r in the compact form: its composite key (u32 when key_width is 4) at out + r * key_width, and each slot's
// word narrowed to its width (two's complement; the host sign-extends them back) at out + sw.off[s].
__global__ __launch_bounds__(256) void hash_compact_kernel(const uint64_t* __restrict__ rec, int64_t n,
                                                           int32_t num_slots, int32_t key_width, SlotWidths sw,
                                                           uint8_t* __restrict__ out) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* e = rec + r * (1 + num_slots);
    if (key_width == 4) reinterpret_cast<uint32_t*>(out)[r] = (uint32_t)e[0];
    else reinterpret_cast<uint64_t*>(out)[r] = e[0];
    for (int s = 0; s < num_slots; ++s) {
      const uint64_t v = e[1 + s];
      put_compact(out + sw.off[s], r, sw.w[s], v);
    }
  }
}

// The slot ranges of a K8h plan from its partitions' ranges (part_mm: [num_parts][2][num_slots] order-preserving u64,
// min then max, written by part_hash_aggregate_kernel), folded into mm (preset as hash_minmax_kernel's) with one
// atomic per workgroup and bound.
__global__ __launch_bounds__(256) void hash_minmax_parts_kernel(const unsigned long long* __restrict__ part_mm,
                                                                int32_t num_parts, int32_t num_slots,
                                                                unsigned long long* __restrict__ mm) {
  __shared__ unsigned long long part[2][256 / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int s = 0; s < num_slots; ++s) {
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < num_parts; p += gridDim.x * blockDim.x) {
      const unsigned long long a = part_mm[(int64_t)p * 2 * num_slots + s];
      const unsigned long long b = part_mm[(int64_t)p * 2 * num_slots + num_slots + s];
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long a = (unsigned long long)__shfl_xor((long long)lo, o);
      const unsigned long long b = (unsigned long long)__shfl_xor((long long)hi, o);
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    if (lane == 0) {
      part[0][wave] = lo;
      part[1][wave] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < 256 / 64; ++w) {
        lo = part[0][w] < lo ? part[0][w] : lo;
        hi = part[1][w] > hi ? part[1][w] : hi;
      }
      atomicMin(&mm[s], lo);
      atomicMax(&mm[num_slots + s], hi);
    }
    __syncthreads();
  }
}

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

int launch_hash_minmax(const uint64_t* rec, const unsigned long long* count, int64_t cap, int32_t num_slots,
                       unsigned long long* mm, void* stream) {
  if (num_slots <= 0 || num_slots > kMaxSlots) return -1;
  if (hipMemsetAsync(mm, 0xFF, (size_t)num_slots * 8, S(stream)) != hipSuccess) return -1;
  if (hipMemsetAsync(mm + num_slots, 0, (size_t)num_slots * 8, S(stream)) != hipSuccess) return -1;
  int64_t grid = (cap + 255) / 256;
  grid = grid > 512 ? 512 : (grid < 1 ? 1 : grid);
  hipLaunchKernelGGL(hash_minmax_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), rec, count, cap, num_slots, mm);
  return PGPU_HIP_OK(hipGetLastError());
}

int launch_hash_minmax_parts(const unsigned long long* part_mm, int32_t num_parts, int32_t num_slots,
                             unsigned long long* mm, void* stream) {
  if (num_slots <= 0 || num_slots > kMaxSlots || num_parts <= 0) return -1;
  if (hipMemsetAsync(mm, 0xFF, (size_t)num_slots * 8, S(stream)) != hipSuccess) return -1;
  if (hipMemsetAsync(mm + num_slots, 0, (size_t)num_slots * 8, S(stream)) != hipSuccess) return -1;
  const int grid = (num_parts + 255) / 256 < 64 ? (num_parts + 255) / 256 : 64;
  hipLaunchKernelGGL(hash_minmax_parts_kernel, dim3(grid), dim3(256), 0, S(stream), part_mm, num_parts, num_slots, mm);
  return PGPU_HIP_OK(hipGetLastError());
}

// Compact form: rec's n records written as [n keys of key_width bytes, 8-aligned] and slot s's words at width[s]
// bytes from slot_off[s].
int launch_hash_compact(const uint64_t* rec, int64_t n, int32_t num_slots, int32_t key_width, const int32_t* width,
                        const int64_t* slot_off, uint8_t* out, void* stream) {
  if (n <= 0) return 0;
  if (num_slots > kMaxSlots || (key_width != 4 && key_width != 8)) return -1;
  SlotWidths sw{};
  for (int s = 0; s < num_slots; ++s) {
    sw.w[s] = width[s];
    sw.off[s] = slot_off[s];
  }
  int64_t grid = (n + 255) / 256;
  grid = grid > 8192 ? 8192 : grid;
  hipLaunchKernelGGL(hash_compact_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), rec, n, num_slots, key_width,
                     sw, out);
  return PGPU_HIP_OK(hipGetLastError());
}

// Columnar form: out = [num_keys][n] int32 dictIds, then at slot_off bytes [num_slots][n] u64.
int launch_hash_decode(const uint64_t* rec, int64_t n, int32_t num_slots, int32_t num_keys, const int64_t* stride,
                       const int64_t* card, const int64_t* off, uint8_t* out, size_t slot_off, void* stream) {
  if (n <= 0) return 0;
  if (num_keys > kMaxKeys || num_slots > kMaxSlots) return -1;
  KeyDecode kd{};
  for (int j = 0; j < num_keys; ++j) {
    kd.stride[j] = stride[j];
    kd.card[j] = card[j];
    kd.off[j] = off[j];
  }
  int64_t grid = (n + 255) / 256;
  grid = grid > 8192 ? 8192 : grid;
  hipLaunchKernelGGL(hash_decode_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), rec, n, num_slots, num_keys,
                     kd, reinterpret_cast<int32_t*>(out), reinterpret_cast<uint64_t*>(out + slot_off));
  return PGPU_HIP_OK(hipGetLastError());
}

}  // namespace pgpu
