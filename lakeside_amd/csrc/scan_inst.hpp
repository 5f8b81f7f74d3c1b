// Instantiations of the fused scan kernels (scan_kernel.hpp, lean_kernel.hpp) and their host dispatch; included by the
// scan_<agg>_<lean|tiles>_<d|h>.hip units and (dispatch only) by kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "kernels.hpp"
#if defined(LK_INST_LEAN) || defined(LK_INST_TILES)
#include "scan_kernel.hpp"
#endif

namespace lk {

// The fused kernels are instantiated per (aggregate, table mode, kernel family) in their own translation units
// (scan_<agg>_<lean|tiles>_<d|h>.hip), so the build runs them in parallel and an edit of one family's header rebuilds
// only that family's objects: each unit includes this header with LK_INST_LEAN or LK_INST_TILES defined.
template <int AGG, bool HASH>
void launch_lean(const QParams& P, dim3 grid, hipStream_t st);    // lean tiles (lean_kernel.hpp), by late columns
template <int AGG, bool HASH>
void launch_tiles(const QParams& P, dim3 grid, hipStream_t st);   // every other tile (scan_kernel.hpp)

#ifdef LK_INST_LEAN
template <int AGG, bool HASH>
void launch_lean(const QParams& P, dim3 grid, hipStream_t st) {
  const dim3 block(BLOCK);
  switch (P.nstr * 2 + (P.late_chunk ? 1 : 0)) {
    case 2: hipLaunchKernelGGL((scan_lean<AGG, HASH, 0>), grid, block, 0, st, P); break;
    case 3: hipLaunchKernelGGL((scan_lean<AGG, HASH, 0, true>), grid, block, 0, st, P); break;   // dense codes
    case 4: hipLaunchKernelGGL((scan_lean<AGG, HASH, 1>), grid, block, 0, st, P); break;
    case 5: hipLaunchKernelGGL((scan_lean<AGG, HASH, 1, true>), grid, block, 0, st, P); break;
    case 6: hipLaunchKernelGGL((scan_lean<AGG, HASH, 2>), grid, block, 0, st, P); break;
    default: hipLaunchKernelGGL((scan_lean<AGG, HASH, 2, true>), grid, block, 0, st, P); break;
  }
}
#endif

#ifdef LK_INST_TILES
template <int AGG, bool HASH>
void launch_tiles(const QParams& P, dim3 grid, hipStream_t st) {
  const dim3 block(BLOCK);
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
#endif

// Host dispatch (no kernel code): lean tiles first, then the general kernel unless every tile was lean.
template <int AGG, bool HASH>
void launch_agg(const QParams& P, dim3 grid, hipStream_t st) {
  if (P.lean_split) launch_lean<AGG, HASH>(P, grid, st);
  if (P.lean_split == 2) return;                                   // no other tile: scan_tiles need not run
  launch_tiles<AGG, HASH>(P, grid, st);
}

template <int AGG>
void launch_scan_agg(const QParams& P, dim3 grid, hipStream_t st) {
  if (P.hkeys) launch_agg<AGG, true>(P, grid, st);
  else launch_agg<AGG, false>(P, grid, st);
}

}  // namespace lk
