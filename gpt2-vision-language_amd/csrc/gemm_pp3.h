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
// s_waitcnt vmcnt(n * PER + X) for a runtime n in [0, MAXN]
template <int PER, int MAXN, int X>
GVL_DEV void wait_vm_steps_x(int n) {
  if (MAXN >= 4 && n >= 4) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PER + X) : "memory"); return; }
  if (MAXN >= 3 && n == 3) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER + X) : "memory"); return; }
  if (MAXN >= 2 && n == 2) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER + X) : "memory"); return; }
  if (MAXN >= 1 && n == 1) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 * PER + X) : "memory"); return; }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X) : "memory");
}

// Counted epilogue (kinds without an [M, N] epilogue operand: plain, bias, bias + GELU).  The
// epilogue's 16-B stores sit in the wave's VMEM queue between the DMA of K-steps c+2 and c+3,
// so the counted wait at the end of the next NS - 2 phases — "all but the newest two K-steps'
// pieces" — used to wait for every one of them (a store acknowledgement per tile boundary on
// the critical path), and the bias, loaded at the tile's first step by a plain load, made
// hipcc drain the whole DMA queue (vmcnt(0)) at its first use in the epilogue.  Here the
// stores are buffer stores whose out-of-range lanes get an offset past the buffer (dropped by
// the range check, no branch), so every epilogue issues exactly CNT_S stores per wave and the
// NS - 2 following waits count them; the bias row is copied to LDS at kernel start and read by
// inline asm (with its own lgkmcnt wait) in the epilogue.
constexpr uint32_t CNT_OOB = 0x7FFFFFF0u;
// cache-policy bits of the counted epilogue's stores: default, or sc1 nt (streaming) for
// outputs past the MALL (GemmP::st_nt)
constexpr int CNT_NT = 18;  // voffset past any buffer: the store is dropped
template <int EPI>
struct CntEpi {
  using KD = EpiKind<EPI>;
  static constexpr bool ON = EPI != EPI_GEN && !KD::AUX && !KD::DROP;
};
template <int FM, int FN, int EPI>
constexpr int cnt_stores() {
  return FM * (FN / 2 + FN % 2) * (EpiKind<EPI>::ACT ? 2 : 1);
}
typedef uint32_t cnt_u32x2 __attribute__((ext_vector_type(2)));
// the store offset, or the dropped-store offset for an out-of-range lane, made opaque: hipcc
// would otherwise split the store into two exec-masked branches (one per outcome), which
// issues a data-dependent number of store instructions
GVL_DEV uint32_t cnt_off(bool ok, int64_t byte_off) {
  uint32_t o = ok ? (uint32_t)byte_off : CNT_OOB;
  asm volatile("" : "+v"(o));
  return o;
}
typedef uint32_t cnt_u32x4 __attribute__((ext_vector_type(4)));

// this wave's bias quads (4 bf16 at columns nw0 + 16 j + 4 (lane >> 4)) from the LDS copy at
// byte address a (+ 32 j); one asm statement with its lgkmcnt wait (no "memory" clobber: that
// would make hipcc drain vmcnt in front of it)
template <int FN>
GVL_DEV void cnt_bias(uint32_t a, uint2 (&bv)[FN]);
template <>
GVL_DEV void cnt_bias<3>(uint32_t a, uint2 (&bv)[3]) {
  asm volatile("ds_read_b64 %0, %3\n\tds_read_b64 %1, %3 offset:32\n\tds_read_b64 %2, %3 offset:64\n\t"
               "s_waitcnt lgkmcnt(0)"
               : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2])
               : "v"(a));
}
template <>
GVL_DEV void cnt_bias<4>(uint32_t a, uint2 (&bv)[4]) {
  asm volatile("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:32\n\tds_read_b64 %2, %4 offset:64\n\t"
               "ds_read_b64 %3, %4 offset:96\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
               : "v"(a));
}

// The counted epilogue: gemm_epilogue16's math and lane pairing, buffer stores.
template <int FM, int FN, int EPI, int AUX>
GVL_DEV void gemm_epilogue_cnt(const GemmP& p, const float4_t (&acc)[FM][FN], int64_t mw0,
                               int64_t nw0, int lane, float alpha, uint32_t bias_lds,
                               __amdgpu_buffer_rsrc_t rc, __amdgpu_buffer_rsrc_t rp) {
  using KD = EpiKind<EPI>;
  const int q = lane >> 4;
  uint2 bv[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bv[j] = make_uint2(0, 0);
  if constexpr (KD::BIAS) cnt_bias<FN>(bias_lds + (uint32_t)(2 * (nw0 + 4 * q)), bv);
  const uint2 z = make_uint2(0, 0);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int64_t m = mw0 + i * 16 + (lane & 15);
    const bool mok = m < p.M;
#pragma unroll
    for (int j = 0; j + 1 < FN; j += 2) {
      const int64_t n0 = nw0 + j * 16 + 4 * q, n1 = n0 + 16;
      float v0[4], v1[4], h0[4] = {0.f, 0.f, 0.f, 0.f}, h1[4] = {0.f, 0.f, 0.f, 0.f};
      gemm_epi_vals_k<EPI>(p, acc[i][j], m, n0, alpha, 1.f, bv[j], z, v0, h0);
      gemm_epi_vals_k<EPI>(p, acc[i][j + 1], m, n1, alpha, 1.f, bv[j + 1], z, v1, h1);
      const auto sx = __builtin_amdgcn_permlane16_swap(pack2(v0[0], v0[1]), pack2(v1[0], v1[1]), false, false);
      const auto sy = __builtin_amdgcn_permlane16_swap(pack2(v0[2], v0[3]), pack2(v1[2], v1[3]), false, false);
      const int64_t n = nw0 + 16 * (j + (q & 1)) + 8 * (q >> 1);
      const bool ok = mok && n < p.N;
      __builtin_amdgcn_raw_buffer_store_b128(cnt_u32x4{sx[0], sy[0], sx[1], sy[1]}, rc,
                                             cnt_off(ok, (m * p.ldc + n) * 2), 0, AUX);
      if constexpr (KD::ACT) {
        const auto hx = __builtin_amdgcn_permlane16_swap(pack2(h0[0], h0[1]), pack2(h1[0], h1[1]), false, false);
        const auto hy = __builtin_amdgcn_permlane16_swap(pack2(h0[2], h0[3]), pack2(h1[2], h1[3]), false, false);
        __builtin_amdgcn_raw_buffer_store_b128(cnt_u32x4{hx[0], hy[0], hx[1], hy[1]}, rp,
                                               cnt_off(ok, (m * p.ldp + n) * 2), 0, AUX);
      }
    }
    if constexpr (FN % 2 == 1) {
      constexpr int j = FN - 1;
      const int64_t n0 = nw0 + j * 16 + 4 * q;
      float v0[4], h0[4] = {0.f, 0.f, 0.f, 0.f};
      gemm_epi_vals_k<EPI>(p, acc[i][j], m, n0, alpha, 1.f, bv[j], z, v0, h0);
      const bool ok = mok && n0 < p.N;
      __builtin_amdgcn_raw_buffer_store_b64(cnt_u32x2{pack2(v0[0], v0[1]), pack2(v0[2], v0[3])}, rc,
                                            cnt_off(ok, (m * p.ldc + n0) * 2), 0, AUX);
      if constexpr (KD::ACT)
        __builtin_amdgcn_raw_buffer_store_b64(cnt_u32x2{pack2(h0[0], h0[1]), pack2(h0[2], h0[3])}, rp,
                                              cnt_off(ok, (m * p.ldp + n0) * 2), 0, AUX);
    }
  }
}

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
  // counted epilogue (CntEpi): single-problem launches; the bias row in LDS after the ring
  constexpr bool CNT = CntEpi<EPI>::ON;
  constexpr int CNT_S = cnt_stores<FM, FN, EPI>();
  static_assert(!CNT || (NS - 2) * (IPW0 > IPW1 ? IPW0 : IPW1) + CNT_S <= 63, "vmcnt range");
  const bool cnt_on = CNT && p.cnt && GVL_PP3_DIAG == 0;
  const uint32_t bias_lds = (uint32_t)(NS * SLOT);
  const __amdgpu_buffer_rsrc_t rc_cnt = uniform_rsrc(p.C, CNT ? p.M * p.ldc * 2 : 0);
  const __amdgpu_buffer_rsrc_t rp_cnt =
      uniform_rsrc(EpiKind<EPI>::ACT ? p.pre_out : p.C, CNT && EpiKind<EPI>::ACT ? p.M * p.ldp * 2 : 0);
  if constexpr (CNT && EpiKind<EPI>::BIAS) {  // plain loads here, before any LDS-DMA is in flight
    if (cnt_on)
      for (int n = tid * 8; n < p.N; n += 512 * 8)
        *reinterpret_cast<uint4*>(smem + NS * SLOT + 2 * n) = *reinterpret_cast<const uint4*>(p.bias + n);
  }
  int cnt_w = 0;  // waits left that must count the last counted epilogue's stores
  // alpha (x *alpha_ptr, a device scalar written before this launch) read once up front: a
  // load inside the loop would make hipcc drain the DMA queue (vmcnt(0)) at every epilogue,
  // and here, before the first DMA, its wait drains nothing
  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;
#pragma unroll
  for (int i = 0; i < NS - 1; ++i) GVL_PP3_ISSUE(i);
  {
    const int r = nsteps - 1, n = r < 0 ? 0 : (r < NS - 2 ? r : NS - 2);
    if (g == 0) wait_vm_steps<IPW0, NS - 2>(n);
    else wait_vm_steps<IPW1, NS - 2>(n);
  }
  barrier_lds();
  if (g == 1) __builtin_amdgcn_s_barrier();

  int cu_t = 0, cu_k = 0;  // compute cursor
  int64_t cu_m0, cu_n0, cu_k0;
  int cu_sp, cu_bi;
  tile_coords(0, cu_m0, cu_n0, cu_k0, cu_sp, cu_bi);
  EpiPre<FM, FN, EPI> pre;
  if (!cnt_on) pre.load_bias(p, cu_n0 + bcol, lane);
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
      } else if (CNT && cnt_on) {                                                            \
        if (p.st_nt)                                                                         \
          gemm_epilogue_cnt<FM, FN, EPI, CNT_NT>(p, acc, cu_m0 + arow, cu_n0 + bcol, lane, alpha, \
                                                 bias_lds, rc_cnt, rp_cnt);                  \
        else                                                                                 \
          gemm_epilogue_cnt<FM, FN, EPI, 0>(p, acc, cu_m0 + arow, cu_n0 + bcol, lane, alpha,  \
                                            bias_lds, rc_cnt, rp_cnt);                       \
        cnt_w = NS - 2;                                                                      \
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
      if (!cnt_on) pre.load_bias(p, cu_n0 + bcol, lane);
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
      const int n_ = r < 0 ? 0 : (r < NS - 2 ? r : NS - 2);
      if (g == 1) {
        if (CNT && cnt_w > 0) {  // the last epilogue's CNT_S stores are younger than step c+1
          wait_vm_steps_x<IPW1, NS - 2, CNT_S>(n_);
          --cnt_w;
        } else {
          wait_vm_steps<IPW1, NS - 2>(n_);
        }
      }
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
      const int n_ = r < 0 ? 0 : (r < NS - 2 ? r : NS - 2);
      if (g == 0) {
        if (CNT && cnt_w > 0) {
          wait_vm_steps_x<IPW0, NS - 2, CNT_S>(n_);
          --cnt_w;
        } else {
          wait_vm_steps<IPW0, NS - 2>(n_);
        }
      }
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
  // counted epilogue (CntEpi): one problem, 32-bit store offsets below the dropped-store offset,
  // a 16-B aligned bias row whose LDS copy fits after the ring (GVL_PP3_CNT=0: off, A/B)
  static const bool cnt_env = [] {
    const char* e = getenv("GVL_PP3_CNT");
    return !(e && e[0] == '0');
  }();
  constexpr int ring = NS * (BM + BN) * KS * 2;
  const int64_t bias_bytes = EpiKind<EPI>::BIAS ? 2 * (int64_t)p.tiles_n * BN : 0;
  p.cnt = CntEpi<EPI>::ON && cnt_env && p.batch == 1 && ring + bias_bytes <= 160 * 1024 &&
          p.M * p.ldc * 2 <= (int64_t)CNT_OOB &&
          (!EpiKind<EPI>::ACT || (p.pre_out != nullptr && p.M * p.ldp * 2 <= (int64_t)CNT_OOB)) &&
          (!EpiKind<EPI>::BIAS || ((reinterpret_cast<uintptr_t>(p.bias) & 15) == 0 && p.N % 8 == 0));
  // outputs far beyond the 256 MiB MALL (the LM's lm_head logits, 1.65 GB) are stored streaming
  // (sc1 nt): lm_head 1316 -> 1222 us, LM step +0.5 % (921k -> 925k tokens/s, same box,
  // alternated).  The caption step's 811 MB logits stay on the default policy: part of them is
  // still in the MALL when the CE kernel reads them (Q-Former step 15.21k vs 15.10k images/s
  // with nt); outputs that fit measured far slower (c_fc + GELU 64 -> 120 us in a loop that
  // rewrites them).  profiles/r4/pp3_store_policy_r4n_r4s.txt; GVL_PP3_NT=0 off.
  static const bool nt_env = [] {
    const char* e = getenv("GVL_PP3_NT");
    return !(e && e[0] == '0');
  }();
  p.st_nt = p.cnt && nt_env && p.M * p.ldc * 2 > (int64_t)1 << 30;
  const int lds = ring + (p.cnt ? (int)bias_bytes : 0);
  auto kern = gemm_pp3_kernel<NS, AMN, BMN, EPI, BN, BM>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
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
    case EPI_BIAS_QGELU: return launch_pp3<NS, AMN, BMN, EPI_BIAS_QGELU>(p, s);
    default: return -1;  // EPI_GEN: gemm_pp3_plan never routes it here
  }
}

}  // namespace
