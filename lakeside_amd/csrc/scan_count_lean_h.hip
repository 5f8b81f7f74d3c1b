// scan_lean instantiations for AGG_COUNT, hash-mode tables (see scan_inst.hpp).
#define LK_INST_LEAN
#include "scan_inst.hpp"

namespace lk {
template void launch_lean<AGG_COUNT, true>(const QParams& P, dim3 grid, hipStream_t st);
}  // namespace lk
