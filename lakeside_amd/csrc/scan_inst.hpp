// Instantiations of the fused scan kernel (scan_kernel.hpp) for one aggregate; included by scan_<agg>.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "kernels.hpp"
#include "scan_kernel.hpp"

namespace lk {

template <int AGG, bool HASH>
static void launch_agg(const QParams& P, dim3 grid, hipStream_t st) {
  const dim3 block(BLOCK);
  if (P.lean_split) {   // lean tiles first (lean_kernel.hpp), by late string columns
    switch (P.nstr * 2 + (P.late_chunk ? 1 : 0)) {
      case 2: hipLaunchKernelGGL((scan_lean<AGG, HASH, 0>), grid, block, 0, st, P); break;
      case 3: hipLaunchKernelGGL((scan_lean<AGG, HASH, 0, true>), grid, block, 0, st, P); break;   // dense codes
      case 4: hipLaunchKernelGGL((scan_lean<AGG, HASH, 1>), grid, block, 0, st, P); break;
      case 5: hipLaunchKernelGGL((scan_lean<AGG, HASH, 1, true>), grid, block, 0, st, P); break;
      case 6: hipLaunchKernelGGL((scan_lean<AGG, HASH, 2>), grid, block, 0, st, P); break;
      default: hipLaunchKernelGGL((scan_lean<AGG, HASH, 2, true>), grid, block, 0, st, P); break;
    }
  }
  if (P.lean_split == 2) return;                                   // no other tile: scan_tiles need not run
  if (!P.truth) {   // > TT_MAX_LEAVES leaves: one generic instantiation interprets the Kleene program per row
    hipLaunchKernelGGL((scan_tiles<AGG, MAXSTR, false, HASH>), grid, block, 0, st, P);
    return;
  }
  // lean min / max / count with group dims: the SLIM LDS layout (twice the cells)
  if constexpr (AGG != AGG_SUM) {
    if (P.lean && P.nstr >= 2) {
    switch (P.nstr) {
      case 2: hipLaunchKernelGGL((scan_tiles<AGG, 2, true, HASH, true>), grid, block, 0, st, P); return;
      case 3: hipLaunchKernelGGL((scan_tiles<AGG, 3, true, HASH, true>), grid, block, 0, st, P); return;
      case 4: hipLaunchKernelGGL((scan_tiles<AGG, 4, true, HASH, true>), grid, block, 0, st, P); return;
      case 5: hipLaunchKernelGGL((scan_tiles<AGG, 5, true, HASH, true>), grid, block, 0, st, P); return;
      case 6: hipLaunchKernelGGL((scan_tiles<AGG, 6, true, HASH, true>), grid, block, 0, st, P); return;
      case 7: hipLaunchKernelGGL((scan_tiles<AGG, 7, true, HASH, true>), grid, block, 0, st, P); return;
      default: hipLaunchKernelGGL((scan_tiles<AGG, 8, true, HASH, true>), grid, block, 0, st, P); return;
    }
    }
  }
  switch (P.nstr) {
    case 1: hipLaunchKernelGGL((scan_tiles<AGG, 1, true, HASH>), grid, block, 0, st, P); break;
    case 2: hipLaunchKernelGGL((scan_tiles<AGG, 2, true, HASH>), grid, block, 0, st, P); break;
    case 3: hipLaunchKernelGGL((scan_tiles<AGG, 3, true, HASH>), grid, block, 0, st, P); break;
    case 4: hipLaunchKernelGGL((scan_tiles<AGG, 4, true, HASH>), grid, block, 0, st, P); break;
    case 5: hipLaunchKernelGGL((scan_tiles<AGG, 5, true, HASH>), grid, block, 0, st, P); break;
    case 6: hipLaunchKernelGGL((scan_tiles<AGG, 6, true, HASH>), grid, block, 0, st, P); break;
    case 7: hipLaunchKernelGGL((scan_tiles<AGG, 7, true, HASH>), grid, block, 0, st, P); break;
    default: hipLaunchKernelGGL((scan_tiles<AGG, 8, true, HASH>), grid, block, 0, st, P); break;
  }
}

template <int AGG>
void launch_scan_agg(const QParams& P, dim3 grid, hipStream_t st) {
  if (P.hkeys) launch_agg<AGG, true>(P, grid, st);
  else launch_agg<AGG, false>(P, grid, st);
}

}  // namespace lk
