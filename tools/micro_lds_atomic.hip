// micro_lds_atomic.hip — measurement harness (not product code): throughput of LDS group-table updates on
// gfx950 for the dense group-by path (C1/C2 shapes: G = 16 / 100 groups, random keys per lane).
//   hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics -o tools/micro_lds_atomic tools/micro_lds_atomic.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kBlock = 256;
constexpr int kIters = 4096;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// VARIANT: 0 ds_add_u64 random key, 1 ds_add_u32 random key, 2 ds_add_u64 key = lane (no conflicts),
// 3 ds_add_f64 random key, 4 lane-private u32 RMW (no atomics; table [G][64] per wave), 5 ds_min_i64 random,
// 6 ds_add_u32 random key with a per-wave table copy.
template <int VARIANT>
__global__ __launch_bounds__(kBlock) void k(int G, unsigned long long* out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int words = (VARIANT == 4) ? G * 64 * 4 : (VARIANT == 6 ? G * 4 : G);
  for (int i = tid; i < words; i += kBlock) lds[i] = 0;
  __syncthreads();
  uint32_t s = mix(blockIdx.x * kBlock + tid + 1);
  uint32_t* l32 = reinterpret_cast<uint32_t*>(lds);
  double* lf = reinterpret_cast<double*>(lds);
  long long* li = reinterpret_cast<long long*>(lds);
  for (int it = 0; it < kIters; ++it) {
    s = s * 1664525u + 1013904223u;
    const int key = (int)((s >> 8) % (uint32_t)G);
    if (VARIANT == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&lds[key]), 1ull);
    if (VARIANT == 1) atomicAdd(&l32[key], 1u);
    if (VARIANT == 2) atomicAdd(reinterpret_cast<unsigned long long*>(&lds[lane]), 1ull);
    if (VARIANT == 3) atomicAdd(&lf[key], 1.0);
    if (VARIANT == 4) { uint32_t* p = l32 + (wave * G + key) * 64 + lane; *p = *p + 1u; }
    if (VARIANT == 5) atomicMin(&li[key], (long long)(s & 0xffff));
    if (VARIANT == 6) atomicAdd(&l32[wave * G + key], 1u);
  }
  __syncthreads();
  if (tid == 0) atomicAdd(out, lds[0]);
}

template <int V>
float run(int G, unsigned long long* d) {
  const size_t lds = (V == 4) ? (size_t)G * 64 * 4 * 4 : (V == 6 ? (size_t)G * 4 * 4 : (size_t)G * 8);
  const int grid = 256 * 4;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(k<V>, dim3(grid), dim3(kBlock), lds, 0, G, d);
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<V>, dim3(grid), dim3(kBlock), lds, 0, G, d);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double ops = 5.0 * grid * kBlock * kIters;
  printf("variant %d G=%4d: %.3f ms, %.3f G lane-ops/s, %.2f lane-ops/CU/cycle@2.4GHz\n", V, G, ms / 5, ops / (ms * 1e6),
         ops / (ms * 1e-3) / 256 / 2.4e9);
  return ms;
}

int main() {
  unsigned long long* d;
  CHECK(hipMalloc(&d, 8));
  for (int G : {16, 100, 1000}) {
    run<0>(G, d);
    run<1>(G, d);
    run<2>(G, d);
    run<3>(G, d);
    if (G <= 100) run<4>(G, d);
    run<5>(G, d);
    run<6>(G, d);
  }
  return 0;
}
