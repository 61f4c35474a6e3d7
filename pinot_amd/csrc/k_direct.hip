// k_direct.hip — one accumulator mode of the direct-load scan kernel (compiled with -DPGPU_MODE=0|1|2).
#include "scan_direct.h"

#ifndef PGPU_MODE
#error "compile with -DPGPU_MODE=0 (LDS), 1 (GLOBAL) or 2 (HASH)"
#endif
#define PGPU_CAT2(a, b) a##b
#define PGPU_CAT(a, b) PGPU_CAT2(a, b)

namespace pgpu {

int PGPU_CAT(launch_direct_mode, PGPU_MODE)(const KParams& p, bool dense, int grid, size_t lds_bytes, void* stream) {
  if (dense)
    hipLaunchKernelGGL((filter_groupby_kernel<PGPU_MODE, true>), dim3(grid), dim3(kBlock), lds_bytes,
                       reinterpret_cast<hipStream_t>(stream), p);
  else
    hipLaunchKernelGGL((filter_groupby_kernel<PGPU_MODE, false>), dim3(grid), dim3(kBlock), lds_bytes,
                       reinterpret_cast<hipStream_t>(stream), p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Resident workgroups per CU of the instance (registers and LDS): the persistent grid is sized to exactly fill
// the chip, since its tile ranges are assigned statically.
int PGPU_CAT(occupancy_direct_mode, PGPU_MODE)(bool dense, size_t lds_bytes) {
  int n = 0;
  const hipError_t e = dense ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                   &n, filter_groupby_kernel<PGPU_MODE, true>, kBlock, lds_bytes)
                             : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                   &n, filter_groupby_kernel<PGPU_MODE, false>, kBlock, lds_bytes);
  return e == hipSuccess ? n : -1;
}

}  // namespace pgpu
