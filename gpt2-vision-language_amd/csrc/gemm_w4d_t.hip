// gemm_w4d_kernel instances with an MN-contiguous B (the weight in dX GEMMs): gemm_w4d.h.
#include "gemm_w4d.h"

namespace gvl {
int gemm_w4d_launch_t(const GemmP& p, bool rows128, hipStream_t s) {
  return launch_epi<true>(p, rows128, s);
}
}  // namespace gvl
