// Plain GEMMs (no epilogue operand, no activation, bf16 out) on hipBLASLt where the library's
// kernel is measured faster than this library's own: the task's rule is hand-written kernels
// for the fused hot ops and hipBLASLt only for plain library GEMMs, and on the N = 768
// products of both steps (the dX GEMMs c_fc.dX / c_attn.dX / attn.c_proj.dX, M = 8064 and
// 16384) hipBLASLt's 4-wave 192x256x64 / 128x192x64 kernels run 17-28 % faster than the
// persistent and direct-A kernels (profiles/r4/wgrad_and_n768_diag_r4f.txt,
// profiles/r4/hipblaslt_n768_r4i.txt).
// Every fused GEMM (bias, GELU, dGELU, residual, dropout, accumulate) stays on gvl's kernels.
//
// Row-major C[M,N] = op(A) op(B) is the column-major product C^T = op(B)^T op(A)^T, so the
// library's "A" is gvl's B and its "B" is gvl's A; per shape (and device) the matmul
// descriptor, the three layouts and the heuristic's first algorithm are built once and cached
// (the first call of a shape happens in the eager warm-up steps, before any graph capture).
// No workspace: the chosen kernels need none, and the split-K workspace gvl_gemm receives may
// be in use by a launch on another stream.
#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "capi_util.h"
#include "../../include/gvl.h"

namespace gvl {
namespace {

struct LibPlan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  bool ok = false;
};

using LibKey = std::tuple<int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int>;

std::mutex g_mu;
std::map<LibKey, LibPlan> g_plans;
hipblasLtHandle_t g_handle[64] = {};

int lib_mode_env() {
  const char* e = getenv("GVL_GEMM_LIB");
  return e ? atoi(e) : 1;
}
int g_mode = lib_mode_env();  // 0: never, 1: the measured shapes, 2: every plain GEMM (tests)

bool plain(const gvl_gemm_desc* d) {
  return !d->bias && !d->act && !d->dact && !d->residual && !d->pre_in && !d->pre_out &&
         !d->gate && d->drop_p == 0.f && !d->c_fp32 && !d->alpha_ptr;
}

// The shapes measured faster on hipBLASLt (see the header): N = 768 outputs with K in
// [768, 4096] at M >= 12288, K >= 3072 below (at M = 8064 the direct-A kernel is as fast or
// faster for K = 768 / 2304: 17.5 vs 20.1 us, 36.5 vs 36.4, profiles/r4/pp3_epilogue_diag_r4a.txt).
// The M = 16384 ones reach gvl_gemm's AGPR four-wave kernel first (gemm_w4x.hip), which runs
// them as fast (profiles/r4/w4x_shapes_r4o.txt).  (The lm_head forward, also faster there, is not routed: its
// first routed run hit an illegal address inside the library (session r4j) and the cause
// is not established.)
bool measured_faster(const gvl_gemm_desc* d) {
  return d->m >= 4096 && d->n == 768 && d->k <= 4096 && (d->k >= 3072 || (d->m >= 12288 && d->k >= 768));
}

LibPlan build(hipblasLtHandle_t h, const gvl_gemm_desc* d) {
  LibPlan pl;
  // library A = gvl B (N x K as op), library B = gvl A (K x M as op), library C = C^T (N x M)
  const hipblasOperation_t opa = d->b_mn ? HIPBLAS_OP_N : HIPBLAS_OP_T;
  const hipblasOperation_t opb = d->a_mn ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  if (hipblasLtMatmulDescCreate(&pl.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
    return pl;
  int32_t ta = opa, tb = opb;
  hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof ta);
  hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof tb);
  // stored shapes (column-major rows x cols): gvl B is [K][N] row-major (b_mn) = N x K, else
  // [N][K] = K x N; gvl A is [K][M] (a_mn) = M x K, else [M][K] = K x M
  const uint64_t ar = d->b_mn ? d->n : d->k, ac = d->b_mn ? d->k : d->n;
  const uint64_t br = d->a_mn ? d->m : d->k, bc = d->a_mn ? d->k : d->m;
  if (hipblasLtMatrixLayoutCreate(&pl.la, HIP_R_16BF, ar, ac, d->ldb) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&pl.lb, HIP_R_16BF, br, bc, d->lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&pl.lc, HIP_R_16BF, d->n, d->m, d->ldc) != HIPBLAS_STATUS_SUCCESS)
    return pl;
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return pl;
  uint64_t ws = 0;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof ws);
  hipblasLtMatmulHeuristicResult_t res[8];
  int n = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, pl.op, pl.la, pl.lb, pl.lc, pl.lc, pref, 8, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS) return pl;
  for (int i = 0; i < n; ++i) {  // the heuristic's best algorithm that needs no workspace
    if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize == 0) {
      pl.algo = res[i].algo;
      pl.ok = true;
      break;
    }
  }
  return pl;
}

}  // namespace

// true when the GEMM was launched on hipBLASLt (the caller launches its own kernel otherwise)
bool gemm_lib_routed(const gvl_gemm_desc* d) {
  if (g_mode == 0 || !plain(d)) return false;
  return g_mode == 2 || measured_faster(d);
}

bool gemm_lib_try(const gvl_gemm_desc* d, hipStream_t s) {
  if (!gemm_lib_routed(d)) return false;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  const LibKey key{dev, d->m, d->n, d->k, d->lda, d->ldb, d->ldc, d->a_mn != 0, d->b_mn != 0};
  LibPlan pl;
  hipblasLtHandle_t h;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_handle[dev] && hipblasLtCreate(&g_handle[dev]) != HIPBLAS_STATUS_SUCCESS) {
      g_handle[dev] = nullptr;
      return false;
    }
    h = g_handle[dev];
    auto it = g_plans.find(key);
    if (it == g_plans.end()) it = g_plans.emplace(key, build(h, d)).first;
    pl = it->second;
  }
  if (!pl.ok) return false;
  const float alpha = d->alpha, beta = 0.f;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  const bool timed = take_launch_events(&e0, &e1);
  if (timed) (void)hipEventRecord(e0, s);
  const hipblasStatus_t st = hipblasLtMatmul(h, pl.op, &alpha, d->b, pl.la, d->a, pl.lb, &beta, d->c, pl.lc,
                                             d->c, pl.lc, &pl.algo, nullptr, 0, s);
  if (timed) (void)hipEventRecord(e1, s);
  return st == HIPBLAS_STATUS_SUCCESS;
}

}  // namespace gvl

extern "C" int gvl_gemm_lib_route(int32_t mode) {
  GVL_REQUIRE(mode >= 0 && mode <= 2, "gvl_gemm_lib_route: mode must be 0, 1 or 2");
  const int prev = gvl::g_mode;
  gvl::g_mode = mode;
  return prev;
}
