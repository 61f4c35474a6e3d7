// k_startree.hip — star-tree kernels for one accumulator mode (compiled with -DPGPU_MODE=0|1|2); the traversal
// (mode-independent) lives in the mode-0 object.
#include "startree_kernels.h"

#ifndef PGPU_MODE
#error "compile with -DPGPU_MODE=0 (LDS), 1 (GLOBAL) or 2 (HASH)"
#endif
#define PGPU_CAT2(a, b) a##b
#define PGPU_CAT(a, b) PGPU_CAT2(a, b)

namespace pgpu {

int PGPU_CAT(launch_startree_scan_mode, PGPU_MODE)(const KStarParams& p, size_t lds_bytes, void* stream) {
  const int grid = p.num_wgs;
  if (grid <= 0 || p.num_segs <= 0) return 0;
  hipLaunchKernelGGL(startree_scan_kernel<PGPU_MODE>, dim3(grid), dim3(StarBlock<PGPU_MODE>::value), lds_bytes,
                     reinterpret_cast<hipStream_t>(stream), p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

#if PGPU_MODE == 0
int launch_startree_traverse(const KStarSeg* segs, int32_t num_segs, int64_t* seg_total, uint64_t deadline,
                             unsigned long long* stats, void* stream) {
  if (num_segs <= 0) return 0;
  hipLaunchKernelGGL(startree_traverse_kernel, dim3(num_segs), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     segs, seg_total, deadline, stats);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif

}  // namespace pgpu
