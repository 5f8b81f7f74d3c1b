// Register / scratch / LDS probe of the scan_lean shapes the bench queries run (C2: <SUM,0>, C4/C5: <SUM,1>,
// C3: <MAX,2>, tag: <COUNT,1>) without building every instantiation: `make lean-res` (device assembly only).
#include "../lakeside_amd/csrc/scan_kernel.hpp"

namespace lk {
template __global__ void scan_lean<AGG_SUM, false, 0, false>(QParams);
template __global__ void scan_lean<AGG_SUM, false, 1, false>(QParams);
template __global__ void scan_lean<AGG_MAX, false, 2, false>(QParams);
template __global__ void scan_lean<AGG_COUNT, false, 1, false>(QParams);
}  // namespace lk
namespace lk {
template __global__ void scan_lean<AGG_COUNT, false, 0, false>(QParams);
}  // namespace lk
