// k_partition.hip — launchers of the partitioned group-by (partition.h).
#include "partition.h"

namespace pgpu {

int occupancy_part_pass(size_t lds_bytes) {
  int n = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, part_pass_kernel<true>, kBlock, lds_bytes) == hipSuccess
             ? n
             : -1;
}

int launch_partitioned(const KPartParams& pp, int grid, size_t pass_lds, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(pp.part_start, 0, (size_t)(pp.num_parts + 1) * 4, s) != hipSuccess) return -1;
  if (hipMemsetAsync(pp.coarse_fill, 0, (size_t)pp.num_coarse * 4, s) != hipSuccess) return -1;
  hipLaunchKernelGGL(part_pass_kernel<false>, dim3(grid), dim3(kBlock), pass_lds, s, pp);
  if (launch_exclusive_scan_u32(pp.part_start, pp.num_parts + 1, stream)) return -1;
  hipLaunchKernelGGL(part_pass_kernel<true>, dim3(grid), dim3(kBlock), pass_lds, s, pp);
  if (pp.cshift > 0) {
    if (hipMemsetAsync(pp.fine_fill, 0, (size_t)pp.num_parts * 4, s) != hipSuccess) return -1;
    hipLaunchKernelGGL(part_split_kernel, dim3(pp.num_coarse * pp.chunks_per_coarse), dim3(kBlock),
                       part_split_lds(pp.cshift, pp.num_streams, pp.split_batch, pp.hashed ? 4 : 2), s, pp);
  }
  if (pp.hashed) {
    if (pp.num_streams > kHashPartStreams || pp.sbits < 8 || pp.sbits > 14) return -1;
    hipLaunchKernelGGL(part_hash_aggregate_kernel, dim3(pp.num_parts), dim3(kBlock),
                       part_hash_lds(pp.sbits, pp.base.num_slots), s, pp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const size_t agg_lds = (size_t)pp.base.num_slots * ((size_t)1 << pp.pshift) * 8;
  hipLaunchKernelGGL(part_aggregate_kernel, dim3(pp.num_parts), dim3(kBlock), agg_lds, s, pp);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace pgpu
