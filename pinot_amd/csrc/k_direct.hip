// k_direct.hip — one accumulator mode of the direct-load scan kernel (compiled with -DPGPU_MODE=0|1|2).
#include "scan_direct.h"

#ifndef PGPU_MODE
#error "compile with -DPGPU_MODE=0 (LDS), 1 (GLOBAL) or 2 (HASH)"
#endif
#define PGPU_CAT2(a, b) a##b
#define PGPU_CAT(a, b) PGPU_CAT2(a, b)

namespace pgpu {

int PGPU_CAT(launch_direct_mode, PGPU_MODE)(const KParams& p, int grid, size_t lds_bytes, void* stream) {
  hipLaunchKernelGGL(filter_groupby_kernel<PGPU_MODE>, dim3(grid), dim3(kBlock), lds_bytes,
                     reinterpret_cast<hipStream_t>(stream), p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace pgpu
