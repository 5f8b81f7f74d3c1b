// scan_tiles instantiations for AGG_SUM, hash-mode tables (see scan_inst.hpp).
#define LK_INST_TILES
#include "scan_inst.hpp"

namespace lk {
template void launch_tiles<AGG_SUM, true>(const QParams& P, dim3 grid, hipStream_t st);
}  // namespace lk
