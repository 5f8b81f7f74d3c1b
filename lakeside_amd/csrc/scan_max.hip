// scan_tiles instantiations for AGG_MAX (dense and hash-mode tables, every string-column count).
#include "scan_inst.hpp"

namespace lk {
template void launch_scan_agg<AGG_MAX>(const QParams& P, dim3 grid, hipStream_t st);
}  // namespace lk
