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

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

int hash_sort_temp_bytes(int64_t n, int key_bits, size_t* bytes) {
  *bytes = 0;
  if (n <= 0) return 0;
  return PGPU_HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, *bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                        (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0,
                                                        key_bits));
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
