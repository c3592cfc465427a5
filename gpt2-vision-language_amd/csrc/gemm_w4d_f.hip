// gemm_w4d_kernel instances with a K-contiguous B (the weight in forward GEMMs) and the
// routing of the direct-A variant: gemm_w4d.h.
#include "gemm_w4d.h"

namespace gvl {

int gemm_w4d_launch_t(const GemmP& p, bool rows128, hipStream_t s);  // gemm_w4d_t.hip

// A shape the four-wave planner accepted runs on the direct-A kernel when K is a multiple of
// six 64-deep steps, its epilogue is instantiated and the tiles are 192 rows.  128-row tiles
// stay on gemm_w4m_kernel: with 32 rows per wave the B fragment reads (all 128 columns per
// wave) fill the LDS again and the direct variant measured slower there (cross-att step:
// dX 24.4 vs 21.4 us; 192-row dX 35.9 vs 38.6 us, profiles/r3/w4d_ab_r3s2.txt).
// GVL_W4D=0: never (A/B); 2: also 128-row tiles (tests).
bool gemm_w4d_ok(const GemmP& p) {
  static const int mode = [] {
    const char* e = getenv("GVL_W4D");
    return e ? atoi(e) : 1;
  }();
  return mode != 0 && p.K % (6 * D_KS) == 0 && p.lda % 8 == 0 &&
         epi_supported(gemm_epi_kind(p)) && (mode == 2 || !gemm_w4_rows128(p));
}

int gemm_w4d_launch(const GemmP& p, int b_mn, bool rows128, hipStream_t s) {
  return b_mn ? gemm_w4d_launch_t(p, rows128, s) : launch_epi<false>(p, rows128, s);
}

}  // namespace gvl
