// k_hashsort.hip — finalize of a hash-mode group table on the device: the compacted records (unordered, one per
// group: composite key, slot words) are radix-sorted by key and decoded into the result's columnar layout (int32
// dictIds per group-by column, then the u64 slot words), so the host copies one buffer instead of sorting and
// decoding millions of rows (AggregationGroupByResult iteration, DictionaryBasedGroupKeyGenerator.getKeys,
// core/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:608-624 for the LONG_MAP holder).
#include <hipcub/hipcub.hpp>

#include "device.h"

namespace pgpu {

struct KeyDecode {
  int64_t stride[kMaxKeys];
  int64_t card[kMaxKeys];
  int64_t off[kMaxKeys];
};

__global__ __launch_bounds__(256) void hash_keys_kernel(const uint64_t* __restrict__ rec, int64_t n, int32_t rec_words,
                                                        uint64_t* __restrict__ keys, uint32_t* __restrict__ idx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = rec[i * rec_words];
    idx[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(256) void hash_keys32_kernel(const uint64_t* __restrict__ rec, int64_t n, int32_t rec_words,
                                                          uint32_t* __restrict__ keys, uint32_t* __restrict__ idx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = (uint32_t)rec[i * rec_words];
    idx[i] = (uint32_t)i;
  }
}

// Row r of the sorted order: its dictIds (key / stride % card + off per column) and slot words.
__global__ __launch_bounds__(256) void hash_decode_kernel(const uint64_t* __restrict__ rec, int64_t n, int32_t num_slots,
                                                          int32_t num_keys, const uint64_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ idx, KeyDecode kd,
                                                          int32_t* __restrict__ gid, uint64_t* __restrict__ slots) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[r];
    for (int j = 0; j < num_keys; ++j)
      gid[(int64_t)j * n + r] = (int32_t)((key / (uint64_t)kd.stride[j]) % (uint64_t)kd.card[j] + kd.off[j]);
    const uint64_t* e = rec + (int64_t)idx[r] * (1 + num_slots);
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

// Row r of the sorted order in the compact form: its composite key (u32 when key_width is 4) at out + 8-aligned
// key area, and each slot's word narrowed to its width (two's complement; the host sign-extends them back).
__global__ __launch_bounds__(256) void hash_compact_kernel(const uint64_t* __restrict__ rec, int64_t n,
                                                           int32_t num_slots, const uint64_t* __restrict__ keys,
                                                           const uint32_t* __restrict__ idx, int32_t key_width,
                                                           SlotWidths sw, uint8_t* __restrict__ out) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    if (key_width == 4) reinterpret_cast<uint32_t*>(out)[r] = reinterpret_cast<const uint32_t*>(keys)[r];
    else reinterpret_cast<uint64_t*>(out)[r] = keys[r];
    const uint64_t* e = rec + (int64_t)idx[r] * (1 + num_slots);
    for (int s = 0; s < num_slots; ++s) {
      const uint64_t v = e[1 + s];
      uint8_t* o = out + sw.off[s];
      switch (sw.w[s]) {
        case 1: o[r] = (uint8_t)v; break;
        case 2: reinterpret_cast<uint16_t*>(o)[r] = (uint16_t)v; break;
        case 4: reinterpret_cast<uint32_t*>(o)[r] = (uint32_t)v; break;
        default: reinterpret_cast<uint64_t*>(o)[r] = v; break;
      }
    }
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

// Sorted compact form: rec's n records sorted by key (as launch_hash_sort_decode), then written as [n keys of
// key_width bytes, 8-aligned] and slot s's words at width[s] bytes from slot_off[s].
int launch_hash_sort_compact(const uint64_t* rec, int64_t n, int32_t num_slots, int key_bits, int32_t key_width,
                             const int32_t* width, const int64_t* slot_off, void* tmp, size_t temp_bytes,
                             uint64_t* keys_a, uint64_t* keys_b, uint32_t* idx_a, uint32_t* idx_b, uint8_t* out,
                             void* stream) {
  if (n <= 0) return 0;
  if (n > INT32_MAX || num_slots > kMaxSlots || (key_width != 4 && key_width != 8)) return -1;
  int64_t grid = (n + 255) / 256;
  grid = grid > 4096 ? 4096 : grid;
  size_t tb = temp_bytes;
  if (key_width == 4) {  // key spaces below 2^32: u32 keys (the sort moves 8 bytes per element and pass, not 12)
    uint32_t* ka = reinterpret_cast<uint32_t*>(keys_a);
    uint32_t* kb = reinterpret_cast<uint32_t*>(keys_b);
    hipLaunchKernelGGL(hash_keys32_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), rec, n, 1 + num_slots, ka,
                       idx_a);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, ka, kb, idx_a, idx_b, (int)n, 0, key_bits, S(stream)) !=
        hipSuccess)
      return -1;
  } else {
    hipLaunchKernelGGL(hash_keys_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), rec, n, 1 + num_slots, keys_a,
                       idx_a);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys_a, keys_b, idx_a, idx_b, (int)n, 0, key_bits, S(stream)) !=
        hipSuccess)
      return -1;
  }
  SlotWidths sw{};
  for (int s = 0; s < num_slots; ++s) {
    sw.w[s] = width[s];
    sw.off[s] = slot_off[s];
  }
  hipLaunchKernelGGL(hash_compact_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), rec, n, num_slots, keys_b,
                     idx_b, key_width, sw, out);
  return PGPU_HIP_OK(hipGetLastError());
}

// Temporary storage of the key sort: the larger of the u64-key and (key spaces below 2^32) u32-key sorts.
int hash_sort_temp_bytes(int64_t n, int key_bits, size_t* bytes) {
  *bytes = 0;
  if (n <= 0) return 0;
  size_t b64 = 0, b32 = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, b64, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, key_bits) != hipSuccess)
    return -1;
  if (key_bits <= 32 &&
      hipcub::DeviceRadixSort::SortPairs(nullptr, b32, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, key_bits) != hipSuccess)
    return -1;
  *bytes = b64 > b32 ? b64 : b32;
  return 0;
}


// rec: n records of 1 + num_slots words; work: keys_a/keys_b (u64) and idx_a/idx_b (u32), n each; tmp: temp_bytes;
// out: [num_keys][n] int32 then, at slot_off bytes, [num_slots][n] u64.
int launch_hash_sort_decode(const uint64_t* rec, int64_t n, int32_t num_slots, int32_t num_keys, const int64_t* stride,
                            const int64_t* card, const int64_t* off, int key_bits, void* tmp, size_t temp_bytes,
                            uint64_t* keys_a, uint64_t* keys_b, uint32_t* idx_a, uint32_t* idx_b, uint8_t* out,
                            size_t slot_off, void* stream) {
  if (n <= 0) return 0;
  if (num_keys > kMaxKeys || n > INT32_MAX) return -1;
  int64_t grid = (n + 255) / 256;
  grid = grid > 4096 ? 4096 : grid;
  hipLaunchKernelGGL(hash_keys_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), rec, n, 1 + num_slots, keys_a,
                     idx_a);
  if (hipGetLastError() != hipSuccess) return -1;
  size_t tb = temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys_a, keys_b, idx_a, idx_b, (int)n, 0, key_bits, S(stream)) !=
      hipSuccess)
    return -1;
  KeyDecode kd{};
  for (int j = 0; j < num_keys; ++j) {
    kd.stride[j] = stride[j];
    kd.card[j] = card[j];
    kd.off[j] = off[j];
  }
  hipLaunchKernelGGL(hash_decode_kernel, dim3((unsigned)grid), dim3(256), 0, S(stream), rec, n, num_slots, num_keys,
                     keys_b, idx_b, kd, reinterpret_cast<int32_t*>(out), reinterpret_cast<uint64_t*>(out + slot_off));
  return PGPU_HIP_OK(hipGetLastError());
}

}  // namespace pgpu
