// gemm_pp3_kernel instances for A MN-contiguous, B MN-contiguous (gemm_pp3.h).
#include "gemm_pp3.h"

namespace gvl {
int gemm_pp3_launch_tt(const GemmP& p, hipStream_t s) { return launch_pp3_epi<4, true, true>(p, s); }
}  // namespace gvl
