// k_direct.hip — one accumulator mode of the direct-load scan kernel (compiled with -DPGPU_MODE=0|1|2).
#include "scan_direct.h"

#ifndef PGPU_MODE
#error "compile with -DPGPU_MODE=0 (LDS), 1 (GLOBAL) or 2 (HASH)"
#endif
#define PGPU_CAT2(a, b) a##b
#define PGPU_CAT(a, b) PGPU_CAT2(a, b)

namespace pgpu {

// variant: 0 the sparse instance, 1 the dense one, 2 the dense one for "simple" plans (aggregate_batch's SIMPLE),
// 3 the sparse one with the index + scan pair (bitdir_range), 4 the sparse one for pure-AND plans (FAST), 5 that one
// with 4-doc lane batches (plans of estimated selectivity >= 1/16).
int PGPU_CAT(launch_direct_mode, PGPU_MODE)(const KParams& p, int variant, int grid, size_t lds_bytes, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (variant == 5)
    hipLaunchKernelGGL((filter_groupby_kernel<PGPU_MODE, false, false, false, true, 4>), dim3(grid), dim3(kBlock),
                       lds_bytes, s, p);
  else if (variant == 4)
    hipLaunchKernelGGL((filter_groupby_kernel<PGPU_MODE, false, false, false, true>), dim3(grid), dim3(kBlock),
                       lds_bytes, s, p);
  else if (variant == 3)
    hipLaunchKernelGGL((filter_groupby_kernel<PGPU_MODE, false, false, true>), dim3(grid), dim3(kBlock), lds_bytes, s,
                       p);
  else if (variant == 2)
    hipLaunchKernelGGL((filter_groupby_kernel<PGPU_MODE, true, true>), dim3(grid), dim3(kBlock), lds_bytes, s, p);
  else if (variant == 1)
    hipLaunchKernelGGL((filter_groupby_kernel<PGPU_MODE, true>), dim3(grid), dim3(kBlock), lds_bytes, s, p);
  else
    hipLaunchKernelGGL((filter_groupby_kernel<PGPU_MODE, false>), dim3(grid), dim3(kBlock), lds_bytes, s, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Resident workgroups per CU of the instance (registers and LDS): the persistent grid is sized to exactly fill
// the chip, since its tile ranges are assigned statically.
int PGPU_CAT(occupancy_direct_mode, PGPU_MODE)(int variant, size_t lds_bytes) {
  int n = 0;
  const hipError_t e =
      variant == 5 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                         &n, filter_groupby_kernel<PGPU_MODE, false, false, false, true, 4>, kBlock, lds_bytes)
      : variant == 4 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                         &n, filter_groupby_kernel<PGPU_MODE, false, false, false, true>, kBlock, lds_bytes)
      : variant == 3 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, filter_groupby_kernel<PGPU_MODE, false, false, true>,
                                                                   kBlock, lds_bytes)
      : variant == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, filter_groupby_kernel<PGPU_MODE, true, true>, kBlock,
                                                                   lds_bytes)
      : variant == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, filter_groupby_kernel<PGPU_MODE, true>, kBlock,
                                                                     lds_bytes)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, filter_groupby_kernel<PGPU_MODE, false>, kBlock,
                                                                    lds_bytes);
  return e == hipSuccess ? n : -1;
}

}  // namespace pgpu
