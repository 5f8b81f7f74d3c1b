// scan_tiles instantiations for AGG_COUNT (dense and hash-mode tables, every string-column count).
#include "scan_inst.hpp"

namespace lk {
template void launch_scan_agg<AGG_COUNT>(const QParams& P, dim3 grid, hipStream_t st);
}  // namespace lk
