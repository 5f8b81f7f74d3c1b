// scan_tiles instantiations for AGG_SUM (dense and hash-mode tables, every string-column count).
#include "scan_inst.hpp"

namespace lk {
template void launch_scan_agg<AGG_SUM>(const QParams& P, dim3 grid, hipStream_t st);
}  // namespace lk
