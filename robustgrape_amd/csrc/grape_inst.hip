// grape_inst.hip -- the small-d engine's kernels and launch sequences for ONE
// compile-time dimension (-DGRAPE_INST_DIM=D); the build compiles one object per
// D in parallel and links them with grape_engine.hip (the C ABI).
#include "grape_launch.hpp"

#ifndef GRAPE_INST_DIM
#error "compile with -DGRAPE_INST_DIM=<d>"
#endif

namespace grape_host {
GRAPE_DECLARE_DIM(GRAPE_INST_DIM, )
#if GRAPE_INST_DIM == 4
GRAPE_DECLARE_SCAN_PAIR()
#endif
}  // namespace grape_host
