// Four-wave narrow-output GEMM with the A operand loaded straight into registers
// (gemm_w4d_kernel): the caption decoder's N = 768 outputs at M = 8064 / 3968 / 4096.
//
// Why: gemm_w4_kernel (gemm_w4.hip) splits its 192x128 tile 2 x 2 over the waves, so both
// operands go global -> VGPR -> LDS -> VGPR and every A and B row is read from LDS by two
// waves.  Per 32-deep K-step a CU writes 20 KiB and reads 40 KiB of LDS against 384 MFMA
// cycles: ds_write_b128 moves ~79 B/clk, ds_read_b128 256 B/clk (MICROARCH §LDS), so the LDS
// is busy ~83 % of the MFMA time and every barrier exposes it.  Here the tile is split 4 x 1:
//   * wave w owns rows [w BM/4, (w+1) BM/4) and all 128 columns (3 x 8 fragments at BM = 192),
//     so nobody else needs its A rows: they are loaded by buffer_load_dwordx4 directly in the
//     MFMA operand layout (no LDS write, no LDS read);
//   * only B (the weight: 128 columns x 64 k = 16 KiB per step) is staged in LDS, register
//     staged (2 global loads + 2 ds_write_b128 per wave per 32 k) and read by all four waves;
//   * K-steps are 64 deep (two MFMA k-chunks): a lane's two A loads of a row are the two
//     halves of one 128-B line (k is permuted consistently in A and B: chunk c of lane group g
//     holds k = 16 g + 8 c + 0..7), and there is one barrier per 48 MFMAs instead of 24.
// Per 64-deep step a CU now writes 16 KiB and reads 64 KiB of LDS (~200 + 256 cycles of the
// array against 768 MFMA cycles) — and the four waves' B reads are the only reads.
//
// Pipeline (per step c; A register sets c % 3, B staging sets c % 2, LDS slots c % 3):
//   write the staged B of step c+2 into slot (c+2) % 3, reload that staging set with c+4;
//   read chunk 1 of step c (slot c % 3) while the chunk-0 MFMAs run; read chunk 0 of
//   step c+1 (slot (c+1) % 3, published by the previous barrier) while the chunk-1 MFMAs run;
//   reload A set c % 3 with step c+3 (three steps of latency cover); one barrier.
// Persistent over tiles (grid = min(tiles, CUs)); the load cursor runs across tile boundaries
// as in gemm_w4.hip, so the next tile's first steps are in flight during the epilogue.
// A must be K-contiguous; B either layout.  K % 384 == 0 (six-step static unroll).
// Built per B layout (gemm_w4d_f.hip / gemm_w4d_t.hip) for the epilogues the four-wave
// routing uses; any other epilogue stays on gemm_w4_kernel.
#pragma once
#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "gemm_ring.h"
#include "../../include/gvl.h"

namespace {  // (anonymous: rocprofv3 and the bench timer then report the same kernel names)

using namespace gvl_ring;

constexpr int D_BN = 128, D_KS = 64, D_NW = 4;
constexpr int D_SLOT = D_BN * D_KS * 2;  // 16 KiB
constexpr int D_PB = D_SLOT / 1024 / D_NW;  // staging pieces per wave per step (4)

// B image of one 64-deep step.  Piece t of a wave covers 1 KiB of the image; global source
// offsets are per lane (computed per tile), the k progress is the scalar offset.
template <bool MN>
struct DImg;

// K-contiguous B ([N][K] weight, forward): [128 n][64 k], 128-B rows; the 16-B chunk ch of
// row n sits at ch ^ s(n), s(n) = ((n >> 1) & 5): conflict-free for the four ds_read_b128 lane
// groups of the fragment reads below (exhaustive search), and the staging stores write 8
// lanes per 128-B row (all 32 banks of a ds_write_b128 group).
template <>
struct DImg<false> {
  GVL_DEV static int sw(int n) { return (n >> 1) & 5; }
  GVL_DEV static int src(int64_t ld, int64_t n0, int piece, int lane) {  // piece = 0..15
    const int n = 8 * piece + (lane >> 3);
    return (int)(((n0 + n) * ld + (lane & 7) * 8) * 2);
  }
  GVL_DEV static int dst(int piece, int lane) {
    const int n = 8 * piece + (lane >> 3);
    return n * 128 + (((lane & 7) ^ sw(n)) << 4);
  }
  GVL_DEV static int step_bytes(int64_t) { return D_KS * 2; }
  // fragment j (cols 16 j .. +15), k-chunk c: lane holds k = 16 (lane >> 4) + 8 c + 0..7
  GVL_DEV static short8_t frag(const char* lds, int j, int c, int lane) {
    const int n = 16 * j + (lane & 15), ch = 2 * (lane >> 4) + c;
    return *reinterpret_cast<const short8_t*>(lds + n * 128 + ((ch ^ sw(n)) << 4));
  }
};

// MN-contiguous B ([K][N], the weight in dX): [64 k][128 n], 256-B rows; chunk ch of k-row kr
// at ch ^ f(kr), f(kr) = ((kr & 3) | ((kr >> 2) & 4)) << 1 (k-row bits 0, 1 and 4: the rows
// one ds_read_b64_tr_b16 half-wave touches are 16 G + 8 c + q, G = 0, 1, q = 0..3).
template <>
struct DImg<true> {
  GVL_DEV static int sw(int kr) { return ((kr & 3) | ((kr >> 2) & 4)) << 1; }
  GVL_DEV static int src(int64_t ld, int64_t n0, int piece, int lane) {
    const int kr = 4 * piece + (lane >> 4);
    return (int)((kr * ld + n0 + (lane & 15) * 8) * 2);
  }
  GVL_DEV static int dst(int piece, int lane) {
    const int kr = 4 * piece + (lane >> 4);
    return kr * 256 + (((lane & 15) ^ sw(kr)) << 4);
  }
  GVL_DEV static int step_bytes(int64_t ld) { return (int)(D_KS * ld * 2); }
  GVL_DEV static short8_t frag(const char* lds, int j, int c, int lane) {
    const int G = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int kr = 16 * G + 8 * c + q, ch = 2 * j + (pp >> 1);
    const int off = kr * 256 + ((ch ^ sw(kr)) << 4) + (pp & 1) * 8;
    short8_t r;
    r.lo = lds_read_tr(lds + off);
    r.hi = lds_read_tr(lds + off + 4 * 256);  // rows kr + 4: same swizzle (bit 2 unused)
    return r;
  }
};

#ifndef GVL_W4D_IGLP
#define GVL_W4D_IGLP 1
#endif
// Timing-only diagnostic builds (wrong results; never the shipped library): GVL_W4D_DIAG=1
// drops the in-loop A loads, 2 the in-loop B loads and LDS writes, 3 the per-step barrier.
// GVL_W4D_EPIS_MIN instantiates only the plain and bias+residual epilogues (fast A/B builds).
#ifndef GVL_W4D_DIAG
#define GVL_W4D_DIAG 0
#endif
// GVL_W4D_AUXPF=1: the epilogue's [M, N] operand (residual / pre_in) is fetched one step ahead
// of the epilogue (EpiPre FULL) instead of FM / 2 rows at a time inside it — measured slower
// (Q-Former step 15.09k vs 15.18k images/s, bias+residual GEMM 40.0-40.5 vs 39.4-39.6 us; the
// held registers make two instances spill), so off (profiles/r3/w4d_auxpf_ab_r3s2.txt)
#ifndef GVL_W4D_AUXPF
#define GVL_W4D_AUXPF 0
#endif

template <bool BMN, int EPI, int BM>
__device__ __forceinline__ void gemm_w4d_body(const GemmP& p) {
  constexpr int RW = BM / D_NW, FM = RW / 16, FN = D_BN / 16;
  using BI = DImg<BMN>;
  constexpr int NRD = BMN ? 2 * FN : FN;  // LDS read instructions per k-chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int total = p.tiles_m * p.tiles_n;
  const int G = gridDim.x, b = blockIdx.x;
  const int ntl = (total - b + G - 1) / G;
  const int nks = (int)(p.K / D_KS);
  auto tile_coords = [&](int t, int64_t& m0, int64_t& n0) {
    const int vid = b + t * G;
    const int q8 = total >> 3, r8 = total & 7, xcd = vid & 7;
    const int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (vid >> 3);
    int sp, tm, tn;
    gemm_tile_of(work, 1, p.tiles_m, p.tiles_n, p.group, sp, tm, tn);
    m0 = (int64_t)tm * BM;
    n0 = (int64_t)tn * D_BN;
  };

  const int64_t b_rows = BMN ? p.K : p.N;
  const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A, p.M * p.lda * 2);
  const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B, b_rows * p.ldb * 2);
  const int sb_step = BI::step_bytes(p.ldb);
  // Per-lane operand offsets at k = 0 of the current tile (oa/ob) and of the next one
  // (na/nb, used by the loads of the last six steps that already belong to it); the k progress
  // is the scalar offset.  No branch inside a step: the cursor crossing is at a fixed position
  // of the last unrolled block.
  int oa[FM][2], ob[D_PB], na[FM][2], nb[D_PB], dstb[D_PB];
  auto a_offs = [&](int64_t m0, int (&o)[FM][2]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        o[i][c] = (int)(((m0 + wave * RW + 16 * i + (lane & 15)) * p.lda + 16 * (lane >> 4) + 8 * c) * 2);
  };
  auto b_offs = [&](int64_t n0, int (&o)[D_PB]) {
#pragma unroll
    for (int t = 0; t < D_PB; ++t) o[t] = BI::src(p.ldb, n0, t * D_NW + wave, lane);
  };
#pragma unroll
  for (int t = 0; t < D_PB; ++t) dstb[t] = BI::dst(t * D_NW + wave, lane);

  uint4 av[3][FM][2];  // A register sets (step % 3)
  uint4 bs[2][D_PB];   // B staging sets (step % 2)
#define W4D_LOAD_A(SET, OFF, KSTEP)                                                          \
  do {                                                                                       \
    const int kb_ = (KSTEP) * (D_KS * 2);                                                    \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                           \
      _Pragma("unroll") for (int c = 0; c < 2; ++c)                                          \
        av[SET][i][c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(      \
            ra, OFF[i][c], kb_, 0));                                                         \
  } while (0)
#define W4D_LOAD_B(SET, OFF, KSTEP)                                                          \
  do {                                                                                       \
    const int kb_ = (KSTEP) * sb_step;                                                       \
    _Pragma("unroll") for (int t = 0; t < D_PB; ++t)                                         \
      bs[SET][t] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(          \
          rb, OFF[t], kb_, 0));                                                              \
  } while (0)
#define W4D_WRITE_B(SET, SLOT)                                                               \
  do {                                                                                       \
    char* sl_ = smem + (SLOT) * D_SLOT;                                                      \
    _Pragma("unroll") for (int t = 0; t < D_PB; ++t)                                         \
      *reinterpret_cast<uint4*>(sl_ + dstb[t]) = bs[SET][t];                                 \
  } while (0)

  float4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;
  int64_t cu_m0, cu_n0;
  tile_coords(0, cu_m0, cu_n0);
  a_offs(cu_m0, oa);
  b_offs(cu_n0, ob);
  EpiPre<FM, FN, EPI, GVL_W4D_AUXPF> pre;  // bias now; the residual / pre_in tile before the last step
  pre.load_bias(p, cu_n0, lane);

  // prologue: B steps 0..3 (0, 1 written to slots 0, 1; sets 0, 1 reloaded with 2, 3),
  // A steps 0..2 into sets 0..2 (nks >= 6)
  W4D_LOAD_B(0, ob, 0);
  W4D_LOAD_B(1, ob, 1);
  W4D_LOAD_A(0, oa, 0);
  W4D_LOAD_A(1, oa, 1);
  W4D_LOAD_A(2, oa, 2);
  W4D_WRITE_B(0, 0);
  W4D_LOAD_B(0, ob, 2);
  W4D_WRITE_B(1, 1);
  W4D_LOAD_B(1, ob, 3);
  barrier_lds();
  short8_t f0[FN], f1[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) f0[j] = BI::frag(smem, j, 0, lane);

#if GVL_W4D_IGLP
  // One pattern per step: chunk-0 MFMAs interleaved with the staged-B writes, the B reloads
  // and the chunk-1 fragment reads; chunk-1 MFMAs with the next step's chunk-0 reads, then
  // the A reloads (each after the last MFMA reading its registers).
#define W4D_SCHED()                                                                          \
  do {                                                                                       \
    _Pragma("unroll") for (int q_ = 0; q_ < D_PB; ++q_) {                                    \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                     \
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                                     \
    }                                                                                        \
    _Pragma("unroll") for (int q_ = 0; q_ < D_PB; ++q_) {                                    \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                     \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                     \
    }                                                                                        \
    _Pragma("unroll") for (int q_ = 0; q_ < NRD; ++q_) {                                     \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                     \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                     \
    }                                                                                        \
    if constexpr (FM * FN > 2 * D_PB + NRD)                                                  \
      __builtin_amdgcn_sched_group_barrier(0x008, FM * FN - 2 * D_PB - NRD, 0);              \
    _Pragma("unroll") for (int q_ = 0; q_ < NRD; ++q_) {                                     \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                     \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                     \
    }                                                                                        \
    _Pragma("unroll") for (int q_ = 0; q_ < 2 * FM; ++q_) {                                  \
      __builtin_amdgcn_sched_group_barrier(0x008, (FM * FN - NRD) / (2 * FM), 0);            \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                     \
    }                                                                                        \
    __builtin_amdgcn_sched_group_barrier(0x008, FM * FN, 0);                                 \
  } while (0)
#else
#define W4D_SCHED() do {} while (0)
#endif

  // step with A set SA (= step % 3), B staging set SB (= step % 2), LDS slot SL (= step % 3);
  // it reloads B set SB with (OB, KB) and A set SA with (OA, KA)
#define W4D_STEP(SA, SB, SL, OA, KA, OB, KB)                                                 \
  do {                                                                                       \
    if constexpr (GVL_W4D_DIAG != 2) {                                                       \
      W4D_WRITE_B(SB, ((SL) + 2) % 3);                                                       \
      W4D_LOAD_B(SB, OB, KB);                                                                \
    }                                                                                        \
    {                                                                                        \
      const char* sl_ = smem + (SL) * D_SLOT;                                                \
      _Pragma("unroll") for (int j = 0; j < FN; ++j) f1[j] = BI::frag(sl_, j, 1, lane);      \
    }                                                                                        \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                           \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                         \
        acc[i][j] = mfma16(f0[j], __builtin_bit_cast(short8_t, av[SA][i][0]), acc[i][j]);    \
    {                                                                                        \
      const char* sl_ = smem + (((SL) + 1) % 3) * D_SLOT;                                    \
      _Pragma("unroll") for (int j = 0; j < FN; ++j) f0[j] = BI::frag(sl_, j, 0, lane);      \
    }                                                                                        \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                           \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                         \
        acc[i][j] = mfma16(f1[j], __builtin_bit_cast(short8_t, av[SA][i][1]), acc[i][j]);    \
    if constexpr (GVL_W4D_DIAG != 1) W4D_LOAD_A(SA, OA, KA);                                 \
    W4D_SCHED();                                                                             \
    if constexpr (GVL_W4D_DIAG == 3) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      \
    else barrier_lds();                                                                      \
  } while (0)

  for (int t = 0; t < ntl; ++t) {
    // steady blocks: step k + u loads A step k + u + 3 and B step k + u + 4 of this tile
    int k = 0;
    for (; k + 6 < nks; k += 6) {
      W4D_STEP(0, 0, 0, oa, k + 3, ob, k + 4);
      W4D_STEP(1, 1, 1, oa, k + 4, ob, k + 5);
      W4D_STEP(2, 0, 2, oa, k + 5, ob, k + 6);
      W4D_STEP(0, 1, 0, oa, k + 6, ob, k + 7);
      W4D_STEP(1, 0, 1, oa, k + 7, ob, k + 8);
      W4D_STEP(2, 1, 2, oa, k + 8, ob, k + 9);
    }
    // last block: loads past this tile's end read the next tile's first steps (past the last
    // tile: this tile again, into sets / slots nobody reads)
    {
      int64_t m1 = cu_m0, n1 = cu_n0;
      if (t + 1 < ntl) tile_coords(t + 1, m1, n1);
      a_offs(m1, na);
      b_offs(n1, nb);
      W4D_STEP(0, 0, 0, oa, k + 3, ob, k + 4);
      W4D_STEP(1, 1, 1, oa, k + 4, ob, k + 5);
      W4D_STEP(2, 0, 2, oa, k + 5, nb, 0);
      W4D_STEP(0, 1, 0, na, 0, nb, 1);
      W4D_STEP(1, 0, 1, na, 1, nb, 2);
      // the epilogue's [M, N] operand (residual / pre_in) for this wave's outputs, one step
      // ahead of its use instead of FM / XH exposed fetches inside the epilogue (earlier and
      // the registers it holds make the last block spill)
      if constexpr (EpiKind<EPI>::AUX && GVL_W4D_AUXPF) pre.load_aux(p, cu_m0 + wave * RW, cu_n0, lane, 0);
      W4D_STEP(2, 1, 2, na, 2, nb, 3);
      gemm_epilogue16<FM, FN, EPI, GVL_W4D_AUXPF>(p, acc, cu_m0 + wave * RW, cu_n0, lane, alpha, pre);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
      cu_m0 = m1;
      cu_n0 = n1;
#pragma unroll
      for (int i = 0; i < FM; ++i) oa[i][0] = na[i][0], oa[i][1] = na[i][1];
#pragma unroll
      for (int q = 0; q < D_PB; ++q) ob[q] = nb[q];
      if (t + 1 < ntl) pre.load_bias(p, cu_n0, lane);
    }
  }
#undef W4D_STEP
#undef W4D_SCHED
#undef W4D_WRITE_B
#undef W4D_LOAD_B
#undef W4D_LOAD_A
}

template <bool BMN, int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4d_kernel(GemmP p) {
  gemm_w4d_body<BMN, EPI, 192>(p);
}
template <bool BMN, int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4dm_kernel(GemmP p) {
  gemm_w4d_body<BMN, EPI, 128>(p);
}

template <bool BMN, int EPI, int BM>
int launch_bm(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;
  p.tiles_m = (int)((p.M + BM - 1) / BM);
  p.tiles_n = (int)((p.N + D_BN - 1) / D_BN);
  p.splits = 1;
  p.kper = p.K;
  constexpr int lds = 3 * D_SLOT;
  auto kern = BM == 192 ? gemm_w4d_kernel<BMN, EPI> : gemm_w4dm_kernel<BMN, EPI>;
  const int total = p.tiles_m * p.tiles_n;
  const int grid = total < gvl::num_cus() ? total : gvl::num_cus();
  gvl::launch_timed(kern, dim3(grid), dim3(256), lds, s, p);
  return 0;
}

template <bool BMN, int EPI>
int launch_rows(const GemmP& p, bool rows128, hipStream_t s) {
  return rows128 ? launch_bm<BMN, EPI, 128>(p, s) : launch_bm<BMN, EPI, 192>(p, s);
}

// the epilogues the caption decoders and the Q-Former route to the four-wave kernels
inline bool epi_supported(int e) {
#ifdef GVL_W4D_EPIS_MIN
  return e == EPI_PLAIN || e == EPI_BIAS_RES;
#else
  return e == EPI_PLAIN || e == EPI_BIAS || e == EPI_BIAS_RES || e == EPI_RES || e == EPI_BIAS_DROP_RES;
#endif
}

template <bool BMN>
int launch_epi(const GemmP& p, bool rows128, hipStream_t s) {
  switch (gvl::gemm_epi_kind(p)) {
    case EPI_PLAIN: return launch_rows<BMN, EPI_PLAIN>(p, rows128, s);
    case EPI_BIAS_RES: return launch_rows<BMN, EPI_BIAS_RES>(p, rows128, s);
#ifndef GVL_W4D_EPIS_MIN
    case EPI_BIAS: return launch_rows<BMN, EPI_BIAS>(p, rows128, s);
    case EPI_RES: return launch_rows<BMN, EPI_RES>(p, rows128, s);
    case EPI_BIAS_DROP_RES: return launch_rows<BMN, EPI_BIAS_DROP_RES>(p, rows128, s);
#endif
    default: return -1;
  }
}

}  // namespace
