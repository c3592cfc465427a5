// Persistent ping-pong GEMM kernel (gemm_pp3_kernel) and its launch templates, shared by the
// per-layout instantiation units gemm_pp3_{ff,ft,tf,tt}.hip (compiled in parallel).
#pragma once
#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "gemm_ring.h"
#include "../../include/gvl.h"

namespace {

using namespace gvl_ring;

// Persistent variant (v5): grid = min(tiles, CUs); workgroup b walks tiles b, b+G, b+2G..
// and the LDS ring runs straight across tile boundaries (the next tile's first K-steps are
// already landing while the current tile finishes), so no tile pays a cold prologue.  A
// tile's epilogue runs at the start of the next memory cluster M(c), i.e. while the partner
// wave of the SIMD is in its compute cluster; its 16-B stores drain behind the following
// MFMAs.  (vmcnt waits stay correct: stores and loads retire in issue order, so a counted
// wait for K-step c+1 at most also waits for part of the stores issued after it.)
// DMA addresses: per-lane offsets are computed once per tile; a K-step only adds a scalar
// soffset.  The epilogue kind EPI is a template parameter so the loop carries only its ops.
// Split-K: work item w = (tile w / splits, K-slice w % splits), every slice kper deep (the
// host only splits when K divides evenly); slices store fp32 partials, gemm_splitk_reduce
// applies the epilogue.  KC = 1, bf16 output.
// Timing-only diagnostic builds (wrong results; never the shipped library): GVL_PP3_DIAG=1
// stores the plain accumulators (no epilogue operands, math or side output), 2 stores nothing.
#ifndef GVL_PP3_DIAG
#define GVL_PP3_DIAG 0
#endif
template <int BN, bool BMN>
struct SlabB {
  using type = Step<256, BMN, 8>;
};
template <bool BMN>
struct SlabB<192, BMN> {
  using type = Step192<BMN>;
};

// BN = 192 (FN = 3 fragments of 16 columns per wave): for N = 768 / 2304 outputs the 256-wide
// tiles leave CUs idle in the last round (M = 16384, N = 768: 192 tiles on 256 CUs; 192-wide:
// 256 tiles).  Its B slab is 12 DMA pieces: waves 0-3 (group 0) issue 2, waves 4-7 one, so
// the counted waits use a per-group pieces-per-step count.
// BM = 128 (FM = 4: each ping-pong group 64 rows): M = 8064, N = 768 (caption decoder) gives
// 63 x 4 = 252 tiles of 128x192, one round on 256 CUs with no K split.
template <int NS, bool AMN, bool BMN, int EPI, int BN = 256, int BM = 256>
__global__ __launch_bounds__(512, 1) void gemm_pp3_kernel(GemmP p) {
  constexpr int NW = 8, FM = BM / 32, FN = BN / 64;
  static_assert(NS >= 3 && NS <= 6, "ring geometry");
  static_assert(BN == 256 || BN == 192, "tile width");
  static_assert(BM == 256 || BM == 128, "tile height");
  using SA = Step<BM, AMN, NW>;
  using SB = typename SlabB<BN, BMN>::type;
  constexpr int SLOT = SA::BYTES + SB::BYTES;
  constexpr int IPW0 = SA::PER + SB::PER;                       // group 0 waves
  constexpr int IPW1 = SA::PER + (BN == 256 ? SB::PER : 1);     // group 1 waves
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 2, wc = wave & 3;

  const int per_batch = p.tiles_m * p.tiles_n * p.splits;
  const int total = per_batch * p.batch;
  const int G = gridDim.x, b = blockIdx.x;
  const int ntl = (total - b + G - 1) / G;  // work items of this workgroup
  const int nks = (int)(p.kper / KS);
  const int nsteps = ntl * nks;
  // work item of local item t: XCD-contiguous remap over the virtual grid of `total` items
  // (G % 8 == 0 keeps b + tG on workgroup b's XCD), then the batch (batch-major: a problem's
  // tiles stay together on an XCD) and the L2-grouped walk inside it
  auto tile_coords = [&](int t, int64_t& m0, int64_t& n0, int64_t& k0, int& split, int& bi) {
    const int vid = b + t * G;
    const int q8 = total >> 3, r8 = total & 7, xcd = vid & 7;
    int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (vid >> 3);
    bi = work / per_batch;
    work -= bi * per_batch;
    int tm, tn;
    gemm_tile_of(work, p.splits, p.tiles_m, p.tiles_n, p.group, split, tm, tn);
    m0 = (int64_t)tm * BM;
    n0 = (int64_t)tn * BN;
    k0 = (int64_t)split * p.kper;
  };

  const int64_t a_rows = AMN ? p.K : p.M, b_rows = BMN ? p.K : p.N;
  __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A, a_rows * p.lda * 2);
  __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B, b_rows * p.ldb * 2);
  const int sa_step = SA::step_bytes(p.lda), sb_step = SB::step_bytes(p.ldb);
  // issue cursor (steps are issued strictly in order)
  int is_t = 0, is_k = 0;
  int offa[SA::PER], offb[SB::PER];
  {
    int64_t m0, n0, k0;
    int sp, bi;
    tile_coords(0, m0, n0, k0, sp, bi);
    if (p.batch > 1) {
      ra = uniform_rsrc(p.Ab[bi], a_rows * p.lda * 2);
      rb = uniform_rsrc(p.Bb[bi], b_rows * p.ldb * 2);
    }
    SA::base_offsets(p.lda, m0, k0, wave, lane, offa);
    SB::base_offsets(p.ldb, n0, k0, wave, lane, offb);
  }

#define GVL_PP3_ISSUE(gstep)                                                        \
  do {                                                                              \
    if ((gstep) < nsteps) {                                                         \
      char* slot_ = smem + ((gstep) % NS) * SLOT;                                   \
      SA::issue_at(ra, offa, is_k * sa_step, slot_, wave);                          \
      SB::issue_at(rb, offb, is_k * sb_step, slot_ + SA::BYTES, wave);              \
      if (++is_k == nks) {                                                          \
        is_k = 0;                                                                   \
        if (++is_t < ntl) {                                                         \
          int64_t m0_, n0_, k0_;                                                    \
          int sp_, bi_;                                                             \
          tile_coords(is_t, m0_, n0_, k0_, sp_, bi_);                               \
          if (p.batch > 1) {                                                        \
            ra = uniform_rsrc(p.Ab[bi_], a_rows * p.lda * 2);                       \
            rb = uniform_rsrc(p.Bb[bi_], b_rows * p.ldb * 2);                       \
          }                                                                         \
          SA::base_offsets(p.lda, m0_, k0_, wave, lane, offa);                      \
          SB::base_offsets(p.ldb, n0_, k0_, wave, lane, offb);                      \
        }                                                                           \
      }                                                                             \
    }                                                                               \
  } while (0)

  float4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int arow = g * (BM / 2), bcol = wc * (BN / 4);
  // fused bias gradient (batched weight-gradient launches, GemmP::Db): the tiles of column
  // block 0 also sum their A fragments over K — MFMAs against a ones fragment, FM/4 of the
  // wave group's FM row fragments per wave — and add the row sums into Db in the epilogue
  constexpr bool DB = EPI == EPI_RES && AMN && BMN;
  constexpr int FPW = FM / 4 > 0 ? FM / 4 : 1;
  float4_t bacc[DB ? FPW : 1];
#pragma unroll
  for (int k = 0; k < (DB ? FPW : 1); ++k) bacc[k] = float4_t{0.f, 0.f, 0.f, 0.f};
  short8_t ones;
#pragma unroll
  for (int k = 0; k < 8; ++k) ones[k] = (short)0x3F80;  // bf16 1.0
  bool do_db = false;
#pragma unroll
  for (int i = 0; i < NS - 1; ++i) GVL_PP3_ISSUE(i);
  {
    const int r = nsteps - 1, n = r < 0 ? 0 : (r < NS - 2 ? r : NS - 2);
    if (g == 0) wait_vm_steps<IPW0, NS - 2>(n);
    else wait_vm_steps<IPW1, NS - 2>(n);
  }
  barrier_lds();
  if (g == 1) __builtin_amdgcn_s_barrier();

  // alpha (x *alpha_ptr, a device scalar written before this launch) read once up front: a
  // load inside the loop would make hipcc drain the DMA queue (vmcnt(0)) at every epilogue
  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;
  int cu_t = 0, cu_k = 0;  // compute cursor
  int64_t cu_m0, cu_n0, cu_k0;
  int cu_sp, cu_bi;
  tile_coords(0, cu_m0, cu_n0, cu_k0, cu_sp, cu_bi);
  EpiPre<FM, FN, EPI> pre;
  pre.load_bias(p, cu_n0 + bcol, lane);
  if constexpr (DB) do_db = p.batch > 1 && p.splits == 1 && cu_n0 == 0 && p.Db[cu_bi] != nullptr;
#define GVL_PP3_EPILOGUE()                                                                   \
  do {                                                                                       \
    bool epi_ = true;                                                                        \
    if (p.splits == 2 && p.tickets != nullptr) { /* two-way split-K combined in-launch */    \
      /* batched: problem bi's tickets follow problem bi-1's, its partials ws[bi][2][M][N] */   \
      const int tile_ = (cu_bi * p.tiles_m + (int)(cu_m0 / BM)) * p.tiles_n + (int)(cu_n0 / BN); \
      const int64_t pofs_ = (int64_t)cu_bi * 2 * p.M * p.N;                                  \
      const __amdgpu_buffer_rsrc_t rw = uniform_rsrc(p.ws + pofs_, p.ws_bytes - pofs_ * 4);   \
      epi_ = gemm_splitk_arrive<FM, FN>(p, acc, cu_sp, tile_, wave, cu_m0 + arow,            \
                                        cu_n0 + bcol, lane, rw);                             \
      if (epi_) gemm_splitk_gather<FM, FN>(p, acc, cu_sp, cu_m0 + arow, cu_n0 + bcol, lane, rw); \
    } else if (p.splits > 1) {                                                               \
      gemm_store_partial<FM, FN>(p, acc, cu_sp, cu_m0 + arow, cu_n0 + bcol, lane);           \
      epi_ = false;                                                                          \
    }                                                                                        \
    if (epi_) {                                                                              \
      void* c_ = p.batch > 1 ? p.Cb[cu_bi] : p.C;                                           \
      if constexpr (GVL_PP3_DIAG == 1) {                                                     \
        EpiPre<FM, FN, EPI_PLAIN> pp_;                                                       \
        gemm_epilogue16<FM, FN, EPI_PLAIN>(p, acc, cu_m0 + arow, cu_n0 + bcol, lane, alpha,  \
                                           pp_, c_, nullptr);                                \
      } else if constexpr (GVL_PP3_DIAG == 2) {                                              \
        _Pragma("unroll") for (int i_ = 0; i_ < FM; ++i_)                                    \
          _Pragma("unroll") for (int j_ = 0; j_ < FN; ++j_)                                  \
            asm volatile("" ::"v"(acc[i_][j_]));                                             \
      } else {                                                                               \
        gemm_epilogue16<FM, FN, EPI>(p, acc, cu_m0 + arow, cu_n0 + bcol, lane, alpha, pre, c_, \
                                     p.batch > 1 ? static_cast<const bf16_t*>(c_) : p.residual); \
      }                                                                                      \
    }                                                                                        \
    if constexpr (DB) {                                                                      \
      if (do_db && (lane >> 4) == 0) {                                                       \
        bf16_t* db_ = static_cast<bf16_t*>(p.Db[cu_bi]);                                     \
        _Pragma("unroll") for (int k = 0; k < FPW; ++k) {                                    \
          const int64_t m_ = cu_m0 + arow + 16 * (wc * FPW + k) + lane;                      \
          if (m_ < p.M) db_[m_] = f2bf(bf2f(db_[m_]) + bacc[k][0] * alpha);                  \
        }                                                                                    \
      }                                                                                      \
      _Pragma("unroll") for (int k = 0; k < FPW; ++k) bacc[k] = float4_t{0.f, 0.f, 0.f, 0.f}; \
    }                                                                                        \
  } while (0)

  short8_t af[FM], bf[FN];
  for (int c = 0; c < nsteps; ++c) {
    // ---- M(c): previous tile's epilogue, fragments of step c, DMA of step c+NS-1
    if (cu_k == 0 && c > 0) {
      GVL_PP3_EPILOGUE();
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
      ++cu_t;
      tile_coords(cu_t, cu_m0, cu_n0, cu_k0, cu_sp, cu_bi);
      pre.load_bias(p, cu_n0 + bcol, lane);
      if constexpr (DB) do_db = p.batch > 1 && p.splits == 1 && cu_n0 == 0 && p.Db[cu_bi] != nullptr;
    }
    const char* sl = smem + (c % NS) * SLOT;
#pragma unroll
    for (int j = 0; j < FN; ++j) bf[j] = SB::frag(sl + SA::BYTES, bcol + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = SA::frag(sl, arow + 16 * i, lane);
    GVL_PP3_ISSUE(c + NS - 1);
    {
      const int r = nsteps - (c + 2);  // steps issued but not needed by step c+1
      if (g == 1) wait_vm_steps<IPW1, NS - 2>(r < 0 ? 0 : (r < NS - 2 ? r : NS - 2));
    }
    barrier_lds();
    // ---- C(c)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
    if constexpr (DB) {
      if (do_db) {
#pragma unroll
        for (int k = 0; k < FPW; ++k) {  // wave-uniform branch: constant register indices
          if (wc == 0) bacc[k] = mfma16(ones, af[k], bacc[k]);
          else if (wc == 1) bacc[k] = mfma16(ones, af[(FPW + k) % FM], bacc[k]);
          else if (wc == 2) bacc[k] = mfma16(ones, af[(2 * FPW + k) % FM], bacc[k]);
          else bacc[k] = mfma16(ones, af[(3 * FPW + k) % FM], bacc[k]);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (++cu_k == nks) cu_k = 0;
    {
      const int r = nsteps - (c + 2);
      if (g == 0) wait_vm_steps<IPW0, NS - 2>(r < 0 ? 0 : (r < NS - 2 ? r : NS - 2));
    }
    barrier_lds();
  }
#undef GVL_PP3_ISSUE
  if (g == 0) __builtin_amdgcn_s_barrier();
  if (nsteps > 0) GVL_PP3_EPILOGUE();
#undef GVL_PP3_EPILOGUE
}

template <int NS, bool AMN, bool BMN, int EPI, int BN, int BM>
int launch_pp3_bn(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;  // tiles_m/n, splits, kper set by gemm_pp3_try
  constexpr int lds = NS * (BM + BN) * KS * 2;
  auto kern = gemm_pp3_kernel<NS, AMN, BMN, EPI, BN, BM>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  const int total = p.tiles_m * p.tiles_n * p.splits * p.batch;
  const int grid = total < gvl::num_cus() ? total : gvl::num_cus();
  gvl::launch_timed(kern, dim3(grid), dim3(512), lds, s, p);
  if (p.splits > 1 && !(p.splits == 2 && p.tickets)) gvl::gemm_splitk_reduce_launch(p, s);
  return 0;
}

// LDS ring depth per tile shape (slots of 32-deep K-steps; NS - 1 steps in flight):
// 4 x 32 KiB for 256x256, 4 x 28 KiB for 256x192, 4 x 20 KiB for 128x192.
#ifndef GVL_PP3_NS_256
#define GVL_PP3_NS_256 4
#endif
#ifndef GVL_PP3_NS_192
#define GVL_PP3_NS_192 4
#endif
#ifndef GVL_PP3_NS_128
#define GVL_PP3_NS_128 4
#endif
template <int NS, bool AMN, bool BMN, int EPI>
int launch_pp3(const GemmP& p, hipStream_t s) {
  if (p.bm == 128) return launch_pp3_bn<GVL_PP3_NS_128, AMN, BMN, EPI, 192, 128>(p, s);
  return p.bn == 192 ? launch_pp3_bn<GVL_PP3_NS_192, AMN, BMN, EPI, 192, 256>(p, s)
                     : launch_pp3_bn<GVL_PP3_NS_256, AMN, BMN, EPI, 256, 256>(p, s);
}

template <int NS, bool AMN, bool BMN>
int launch_pp3_epi(const GemmP& p, hipStream_t s) {
  // partials only (the reduce kernel applies the epilogue) unless combined in-launch
  if (p.splits > 1 && !(p.splits == 2 && p.tickets)) return launch_pp3<NS, AMN, BMN, EPI_PLAIN>(p, s);
  switch (gvl::gemm_epi_kind(p)) {
    case EPI_PLAIN: return launch_pp3<NS, AMN, BMN, EPI_PLAIN>(p, s);
    case EPI_BIAS: return launch_pp3<NS, AMN, BMN, EPI_BIAS>(p, s);
    case EPI_BIAS_RES: return launch_pp3<NS, AMN, BMN, EPI_BIAS_RES>(p, s);
    case EPI_BIAS_ACT: return launch_pp3<NS, AMN, BMN, EPI_BIAS_ACT>(p, s);
    case EPI_DACT: return launch_pp3<NS, AMN, BMN, EPI_DACT>(p, s);
    case EPI_RES: return launch_pp3<NS, AMN, BMN, EPI_RES>(p, s);
    case EPI_BIAS_ACT_ERF: return launch_pp3<NS, AMN, BMN, EPI_BIAS_ACT_ERF>(p, s);
    case EPI_DACT_ERF: return launch_pp3<NS, AMN, BMN, EPI_DACT_ERF>(p, s);
    case EPI_BIAS_ACT_D: return launch_pp3<NS, AMN, BMN, EPI_BIAS_ACT_D>(p, s);
    case EPI_BIAS_ACT_ERF_D: return launch_pp3<NS, AMN, BMN, EPI_BIAS_ACT_ERF_D>(p, s);
    case EPI_MUL: return launch_pp3<NS, AMN, BMN, EPI_MUL>(p, s);
    case EPI_BIAS_DROP_RES: return launch_pp3<NS, AMN, BMN, EPI_BIAS_DROP_RES>(p, s);
    default: return -1;  // EPI_GEN: gemm_pp3_plan never routes it here
  }
}

}  // namespace
