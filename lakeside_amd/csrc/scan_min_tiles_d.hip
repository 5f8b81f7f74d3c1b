// scan_tiles instantiations for AGG_MIN, dense tables (see scan_inst.hpp).
#define LK_INST_TILES
#include "scan_inst.hpp"

namespace lk {
template void launch_tiles<AGG_MIN, false>(const QParams& P, dim3 grid, hipStream_t st);
}  // namespace lk
