// k_partition.hip — launchers of the partitioned group-by (partition.h).
#include "partition.h"

namespace pgpu {

// LDS of K8c from the pass LDS (K8a's: a num_parts histogram + the filter stack): num_coarse cursors instead of the
// histogram, and, staged (1 / 2: u32 / u64 records), one staging region per wave from u32 word *stage_off.
size_t part_scatter_lds(size_t pass_lds, int num_parts, int num_coarse, int staged, int32_t* stage_off) {
  const size_t base = pass_lds - (size_t)((num_parts + 3) & ~3) * 4 + (size_t)((num_coarse + 3) & ~3) * 4;
  const size_t at = (base + 7) & ~size_t(7);
  if (stage_off) *stage_off = (int32_t)(at / 4);
  return staged ? at + (size_t)(kBlock / 64) * 4 * (staged == 2 ? kStageWaveWords64 : kStageWaveWords32) : base;
}

// Workgroups per CU of K8c (K8a shares its grid: both walk the same static tile ranges), direct or staged.
int occupancy_part_pass(size_t pass_lds, int num_parts, int num_coarse, int staged) {
  const size_t lds = part_scatter_lds(pass_lds, num_parts, num_coarse, staged, nullptr);
  int n = 0;
  hipError_t e;
  if (staged == 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, part_pass_kernel<true, 1>, kBlock, lds);
  else if (staged == 2) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, part_pass_kernel<true, 2>, kBlock, lds);
  else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, part_pass_kernel<true, 0>, kBlock, lds);
  return e == hipSuccess ? n : -1;
}

int launch_partitioned(const KPartParams& pp, int grid, size_t pass_lds, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(pp.part_start, 0, (size_t)(pp.num_parts + 1) * 4, s) != hipSuccess) return -1;
  if (hipMemsetAsync(pp.coarse_fill, 0, (size_t)pp.num_coarse * 4, s) != hipSuccess) return -1;
  hipLaunchKernelGGL((part_pass_kernel<false, 0>), dim3(grid), dim3(kBlock), pass_lds, s, pp);
  if (launch_exclusive_scan_u32(pp.part_start, pp.num_parts + 1, stream)) return -1;
  KPartParams pc = pp;
  const size_t scatter_lds = part_scatter_lds(pass_lds, pp.num_parts, pp.num_coarse, pp.staged, &pc.stage_off);
  if (pp.staged == 1)
    hipLaunchKernelGGL((part_pass_kernel<true, 1>), dim3(grid), dim3(kBlock), scatter_lds, s, pc);
  else if (pp.staged == 2)
    hipLaunchKernelGGL((part_pass_kernel<true, 2>), dim3(grid), dim3(kBlock), scatter_lds, s, pc);
  else
    hipLaunchKernelGGL((part_pass_kernel<true, 0>), dim3(grid), dim3(kBlock), scatter_lds, s, pc);
  if (pp.cshift > 0) {
    if (hipMemsetAsync(pp.fine_fill, 0, (size_t)pp.num_parts * 4, s) != hipSuccess) return -1;
    const dim3 sgrid(pp.num_coarse * pp.chunks_per_coarse);
#ifndef PGPU_PART_NO_SPLIT_WORDS  // (defined only by an A/B build of the library)
    if (pp.fine_pack && pp.hashed)
      hipLaunchKernelGGL(part_split_words_kernel<true>, sgrid, dim3(kBlock), part_split_words_lds(pp.cshift), s, pp);
    else if (pp.fine_pack)
      hipLaunchKernelGGL(part_split_words_kernel<false>, sgrid, dim3(kBlock), part_split_words_lds(pp.cshift), s, pp);
    else
#endif
      hipLaunchKernelGGL(part_split_kernel, sgrid, dim3(kBlock),
                         part_split_lds(pp.cshift, pp.num_streams, pp.split_batch, pp.hashed ? 4 : 2), s, pp);
  }
  if (pp.hashed) {
    if (pp.num_streams > kHashPartStreams || pp.sbits < 8 || pp.sbits > 14) return -1;
    hipLaunchKernelGGL(part_hash_aggregate_kernel, dim3(pp.num_parts), dim3(kBlock),
                       part_hash_lds(pp.sbits, pp.base.num_slots), s, pp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  // cs_pack: COUNT + SUM in one word per key (part_aggregate_kernel)
#ifndef PGPU_PART_CS_FULL_LDS  // (defined only by an A/B build: the LDS of every slot's row, two workgroups per CU)
  const size_t agg_lds = (pp.cs_pack ? (size_t)1 : (size_t)pp.base.num_slots) * ((size_t)1 << pp.pshift) * 8;
#else
  const size_t agg_lds = (size_t)pp.base.num_slots * ((size_t)1 << pp.pshift) * 8;
#endif
  hipLaunchKernelGGL(part_aggregate_kernel, dim3(pp.num_parts), dim3(kBlock), agg_lds, s, pp);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace pgpu
