// gemm_pp3_kernel instances for A K-contiguous, B K-contiguous (gemm_pp3.h).
#include "gemm_pp3.h"

namespace gvl {
int gemm_pp3_launch_ff(const GemmP& p, hipStream_t s) { return launch_pp3_epi<4, false, false>(p, s); }
}  // namespace gvl
