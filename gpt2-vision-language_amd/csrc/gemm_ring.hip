// bf16 GEMM v3: LDS-DMA ring of 32-deep K-steps, several in flight across the barriers.
//
// v2 (gemm_lds.hip) double-buffers 64-deep K-tiles and drains every DMA (vmcnt(0)) before
// each barrier, so each workgroup keeps at most one tile in flight and every K-tile starts
// with a bubble: barrier -> ds_read latency -> MFMA.  Here:
//   * the LDS holds a ring of NS slots; slot s%NS holds K-step s (A[BM][32] + B[BN][32]);
//     the DMA for K-step s+NS is issued as soon as slot s's fragments are in registers, so
//     NS-2 K-steps (2 x 16..32 KiB per step) stay in flight across every barrier;
//   * a counted `s_waitcnt vmcnt(N)` + raw `s_barrier` retires exactly the step needed next
//     (never vmcnt(0) inside the loop; __syncthreads() would drain the DMA, guide rule
//     "pipelining across barriers");
//   * fragments are double-buffered in registers: the ds_reads for the next phase are issued
//     ahead of the current phase's MFMAs.  P phases per K-step split the wave's A fragments
//     (P=2 on the 256x256 tile keeps the fragment registers at 64 VGPRs next to the 128
//     accumulator VGPRs); one barrier per K-step.
// LDS images (lane-linear per 1-KiB DMA instruction, XOR swizzle applied on the SOURCE):
//   K-contiguous operand: [R rows][32 k], 64-B rows, chunk' = chunk ^ ((row >> 1) & 2)
//     (conflict-free for the four ds_read_b128 lane groups, found by exhaustive search);
//   MN-contiguous operand: [R/128][32 k][128], 256-B rows, chunk' = chunk ^ fT(k), read with
//     ds_read_b64_tr_b16 (as gemm_lds.hip).
// Requires K % 32 == 0 and 16-byte aligned rows.  Epilogue and split-K as gemm_lds.hip.
#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "gemm_ring.h"
#include "../../include/gvl.h"

namespace {

using namespace gvl_ring;

template <int BM, int BN, int WMW, int WNW, int NS, int P, bool AMN, bool BMN>
__global__ __launch_bounds__(64 * WMW * WNW, (BM * BN > 16384 ? 1 : 2)) void gemm_ring_kernel(GemmP p) {
  constexpr int NW = WMW * WNW;
  constexpr int TM = BM / WMW, TN = BN / WNW, FM = TM / 16, FN = TN / 16, FP = FM / P;
  using SA = Step<BM, AMN, NW>;
  using SB = Step<BN, BMN, NW>;
  static_assert(SA::NINSTR % NW == 0 && SB::NINSTR % NW == 0, "DMA split must be even");
  static_assert(FM % P == 0 && NS >= 3 && NS <= 6, "bad ring geometry");
  constexpr int SLOT = SA::BYTES + SB::BYTES;
  constexpr int IPW = (SA::NINSTR + SB::NINSTR) / NW;  // DMA instructions per wave per K-step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;

  int split, tm, tn;
  gemm_work_tile(p.splits, p.tiles_m, p.tiles_n, p.group, split, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * p.kper;
  const int64_t kend = kbeg + p.kper < p.K ? kbeg + p.kper : p.K;
  const int nks = (int)((kend - kbeg) / KS);

  const int64_t a_rows = AMN ? p.K : p.M, b_rows = BMN ? p.K : p.N;
  const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A, a_rows * p.lda * 2);
  const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B, b_rows * p.ldb * 2);

  auto issue = [&](int ks) {
    if (ks < nks) {
      char* slot = smem + (ks % NS) * SLOT;
      const int64_t k0 = kbeg + (int64_t)ks * KS;
      SA::issue(ra, p.lda, m0, k0, slot, wave, lane);
      SB::issue(rb, p.ldb, n0, k0, slot + SA::BYTES, wave, lane);
    }
  };
  auto slot_of = [&](int ks) -> const char* { return smem + (ks % NS) * SLOT; };

  float4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int arow = wm * TM, bcol = wn * TN;
#pragma unroll
  for (int i = 0; i < NS; ++i) issue(i);

  if constexpr (P == 1) {
    // phase s: read step s+1 -> nxt; DMA step s+NS -> slot s; MFMA cur; retire step s+2.
    short8_t af[FM], bf[FN], an[FM], bn[FN];
    {
      const int c = nks - 2 < NS - 2 ? nks - 2 : NS - 2;
      wait_vm_steps<IPW, NS - 2>(c);
      barrier_lds();
      const char* sl = slot_of(0);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = SB::frag(sl + SA::BYTES, bcol + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = SA::frag(sl, arow + 16 * i, lane);
      barrier_lds();  // every wave's slot-0 reads retire before phase 0 refills slot 0
    }
    for (int s = 0; s < nks; ++s) {
      if (s + 1 < nks) {
        const char* sl = slot_of(s + 1);
#pragma unroll
        for (int j = 0; j < FN; ++j) bn[j] = SB::frag(sl + SA::BYTES, bcol + 16 * j, lane);
#pragma unroll
        for (int i = 0; i < FM; ++i) an[i] = SA::frag(sl, arow + 16 * i, lane);
      }
      issue(s + NS);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      const int c = nks - 3 - s < NS - 2 ? nks - 3 - s : NS - 2;
      wait_vm_steps<IPW, NS - 2>(c);
      barrier_lds();
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = bn[j];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = an[i];
    }
  } else {
    // P == 2.  phase 2s: read A(s, half 1); MFMA A(s, half 0); retire step s+1; barrier.
    //          phase 2s+1: read A(s+1, half 0), B(s+1); DMA step s+NS -> slot s; MFMA A(s, half 1).
    short8_t a0[FP], a1[FP], bf[FN], bn[FN];
    {
      const int c = nks - 1 < NS - 1 ? nks - 1 : NS - 1;
      wait_vm_steps<IPW, NS - 1>(c);
      barrier_lds();
      const char* sl = slot_of(0);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = SB::frag(sl + SA::BYTES, bcol + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < FP; ++i) a0[i] = SA::frag(sl, arow + 16 * i, lane);
    }
    for (int s = 0; s < nks; ++s) {
      {
        const char* sl = slot_of(s);
#pragma unroll
        for (int i = 0; i < FP; ++i) a1[i] = SA::frag(sl, arow + 16 * (FP + i), lane);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FP; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bf[j], a0[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      const int c = nks - 2 - s < NS - 2 ? nks - 2 - s : NS - 2;
      wait_vm_steps<IPW, NS - 2>(c);
      barrier_lds();
      if (s + 1 < nks) {
        const char* sl = slot_of(s + 1);
#pragma unroll
        for (int j = 0; j < FN; ++j) bn[j] = SB::frag(sl + SA::BYTES, bcol + 16 * j, lane);
#pragma unroll
        for (int i = 0; i < FP; ++i) a0[i] = SA::frag(sl, arow + 16 * i, lane);
      }
      issue(s + NS);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FP; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[FP + i][j] = mfma16(bf[j], a1[i], acc[FP + i][j]);
      __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = bn[j];
    }
  }

  if (p.splits > 1) {
    gemm_store_partial<FM, FN>(p, acc, split, m0 + wm * TM, n0 + wn * TN, lane);
  } else {
    gemm_epilogue<FM, FN>(p, acc, m0 + wm * TM, n0 + wn * TN, lane);
  }
}

// Ping-pong 256x256: the 8 waves form two groups of 4 (one wave per SIMD each), group g
// owning output rows [128 g, 128 g + 128).  Group 1 runs one barrier behind group 0, so on
// every SIMD one wave issues its ds_reads and DMA ("M" half) while the other runs its 16
// MFMAs ("C" half): the MFMA pipe alternates between the two waves instead of both stalling
// on the same fragment reads.  Phase p = (K-step s, row half h): M half reads the wave's A
// fragments of rows 64h.. (+ B at h = 0); C half 16 MFMAs.
//  * slot s is refilled (K-step s+NS-1) in the M half of phase (s+1, 1): by then both groups
//    have retired their last reads of it (group 1's M(2s+1), lgkmcnt(0) before barrier 4s+3);
//  * K-step s+1 is retired (counted vmcnt) by every wave before barrier 4s+3, the first
//    barrier after which a group reads it: group 1 at the end of its M half of phase 2s+1,
//    group 0 at the end of its C half of the same phase.
template <int NS, bool AMN, bool BMN>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmP p) {
  constexpr int BM = 256, BN = 256, NW = 8, FM = 8, FN = 4, FH = 4;
  using SA = Step<BM, AMN, NW>;
  using SB = Step<BN, BMN, NW>;
  constexpr int SLOT = SA::BYTES + SB::BYTES;
  constexpr int IPW = (SA::NINSTR + SB::NINSTR) / NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 2, wc = wave & 3;

  int split, tm, tn;
  gemm_work_tile(p.splits, p.tiles_m, p.tiles_n, p.group, split, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * p.kper;
  const int64_t kend = kbeg + p.kper < p.K ? kbeg + p.kper : p.K;
  const int nks = (int)((kend - kbeg) / KS);

  const int64_t a_rows = AMN ? p.K : p.M, b_rows = BMN ? p.K : p.N;
  const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A, a_rows * p.lda * 2);
  const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B, b_rows * p.ldb * 2);
  auto issue = [&](int ks) {
    if (ks < nks) {
      char* slot = smem + (ks % NS) * SLOT;
      const int64_t k0 = kbeg + (int64_t)ks * KS;
      SA::issue(ra, p.lda, m0, k0, slot, wave, lane);
      SB::issue(rb, p.ldb, n0, k0, slot + SA::BYTES, wave, lane);
    }
  };

  float4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int arow = g * 128, bcol = wc * 64;
#pragma unroll
  for (int i = 0; i < NS; ++i) issue(i);
  wait_vm_steps<IPW, NS - 1>(nks - 1 < NS - 1 ? nks - 1 : NS - 1);
  barrier_lds();
  if (g == 1) __builtin_amdgcn_s_barrier();

  short8_t af[FH], bf[FN];
  for (int s = 0; s < nks; ++s) {
    const char* sl = smem + (s % NS) * SLOT;
    const int c = nks - 2 - s < NS - 2 ? nks - 2 - s : NS - 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // M half
      if (h == 0) {
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[j] = SB::frag(sl + SA::BYTES, bcol + 16 * j, lane);
      }
#pragma unroll
      for (int i = 0; i < FH; ++i) af[i] = SA::frag(sl, arow + 64 * h + 16 * i, lane);
      if (h == 1 && s >= 1) issue(s + NS - 1);
      if (h == 1 && g == 1) wait_vm_steps<IPW, NS - 2>(c);
      barrier_lds();
      // C half
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FH; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[FH * h + i][j] = mfma16(bf[j], af[i], acc[FH * h + i][j]);
      __builtin_amdgcn_s_setprio(0);
      if (h == 1 && g == 0) wait_vm_steps<IPW, NS - 2>(c);
      barrier_lds();
    }
  }
  if (g == 0) __builtin_amdgcn_s_barrier();

  if (p.splits > 1) {
    gemm_store_partial<FM, FN>(p, acc, split, m0 + arow, n0 + bcol, lane);
  } else {
    gemm_epilogue<FM, FN>(p, acc, m0 + arow, n0 + bcol, lane);
  }
}

template <int NS, bool AMN, bool BMN>
int launch_pp(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;
  p.tiles_m = (int)((p.M + 255) / 256);
  p.tiles_n = (int)((p.N + 255) / 256);
  constexpr int lds = NS * 512 * KS * 2;
  auto kern = gemm_pp_kernel<NS, AMN, BMN>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  p.splits = 1;
  if (p.ws != nullptr) {
    const int sp = gvl::gemm_splitk_pick((int64_t)p.tiles_m * p.tiles_n, p.K);
    if (sp > 1 && (int64_t)sp * p.M * p.N * 4 <= p.ws_bytes) p.splits = sp;
  }
  p.kper = p.splits > 1 ? ((p.K / p.splits + KS - 1) / KS) * KS : p.K;
  if (p.splits > 1) p.splits = (int)((p.K + p.kper - 1) / p.kper);
  gvl::launch_timed(kern, dim3(p.tiles_m * p.tiles_n * p.splits), dim3(512), lds, s, p);
  if (p.splits > 1) gvl::gemm_splitk_reduce_launch(p, s);
  return 0;
}

template <int BM, int BN, int WMW, int WNW, int NS, int P, bool AMN, bool BMN>
int launch_cfg(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;
  p.tiles_m = (int)((p.M + BM - 1) / BM);
  p.tiles_n = (int)((p.N + BN - 1) / BN);
  constexpr int lds = NS * (BM + BN) * KS * 2;
  auto kern = gemm_ring_kernel<BM, BN, WMW, WNW, NS, P, AMN, BMN>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  p.splits = 1;
  if (p.ws != nullptr) {
    const int sp = gvl::gemm_splitk_pick((int64_t)p.tiles_m * p.tiles_n, p.K);
    if (sp > 1 && (int64_t)sp * p.M * p.N * 4 <= p.ws_bytes) p.splits = sp;
  }
  p.kper = p.splits > 1 ? ((p.K / p.splits + KS - 1) / KS) * KS : p.K;
  if (p.splits > 1) p.splits = (int)((p.K + p.kper - 1) / p.kper);
  gvl::launch_timed(kern, dim3(p.tiles_m * p.tiles_n * p.splits), dim3(64 * WMW * WNW), lds, s, p);
  if (p.splits > 1) gvl::gemm_splitk_reduce_launch(p, s);
  return 0;
}

// cfg: 0 = 256x256 (8 waves, P=2, 4 slots = 128 KiB), 1 = 256x128 (8 waves, 5 slots),
//      2 = 128x128 (4 waves, 4 slots = 64 KiB, two workgroups per CU), 3 = 256x256, 5 slots,
//      4 = 256x256 ping-pong, 4 slots, 5 = 256x256 ping-pong, 5 slots,
//      6 = 64x128 (2 waves of 64x64, 4 slots = 48 KiB, three workgroups per CU; needs a
//          K-contiguous A: the MN-contiguous LDS image is 128 rows wide).
template <bool AMN, bool BMN>
int launch_layout(const GemmP& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 6:
      if constexpr (!AMN) return launch_cfg<64, 128, 1, 2, 4, 1, AMN, BMN>(p, s);
      return launch_cfg<128, 128, 2, 2, 4, 1, AMN, BMN>(p, s);
    case 0: return launch_cfg<256, 256, 2, 4, 4, 2, AMN, BMN>(p, s);
    case 1: return launch_cfg<256, 128, 4, 2, 5, 1, AMN, BMN>(p, s);
    case 3: return launch_cfg<256, 256, 2, 4, 5, 2, AMN, BMN>(p, s);
    case 4: return launch_pp<4, AMN, BMN>(p, s);
    case 5: return launch_pp<5, AMN, BMN>(p, s);
    // 192-row tiles: M = 8064 (the caption step, 128 x 63 rows) is exactly 42 of them, so an
    // N = 768 output is 252 tiles of 192x128 (one round on 256 CUs) instead of 378 of
    // 128x128 (1.5 rounds) or 96 of 256x256.  K-contiguous A only (the MN image is 128 wide).
    case 7:
      if constexpr (!AMN) return launch_cfg<192, 128, 2, 2, 4, 2, AMN, BMN>(p, s);
      return launch_cfg<128, 128, 2, 2, 4, 1, AMN, BMN>(p, s);
    case 8:
      if constexpr (!AMN) return launch_cfg<192, 256, 2, 2, 4, 2, AMN, BMN>(p, s);
      return launch_cfg<128, 128, 2, 2, 4, 1, AMN, BMN>(p, s);
    case 9:  // 128x192 (K-contiguous operands only)
      if constexpr (!AMN && !BMN) return launch_cfg<128, 192, 2, 2, 4, 1, AMN, BMN>(p, s);
      return launch_cfg<128, 128, 2, 2, 4, 1, AMN, BMN>(p, s);
    default: return launch_cfg<128, 128, 2, 2, 4, 1, AMN, BMN>(p, s);
  }
}

}  // namespace

namespace gvl {
const char* gemm_ring_name(int cfg) {
  switch (cfg) {
    case 0: return "gemm_ring_kernel<256, 256, 2, 4, 4, 2";
    case 1: return "gemm_ring_kernel<256, 128, 4, 2, 5, 1";
    case 3: return "gemm_ring_kernel<256, 256, 2, 4, 5, 2";
    case 4: return "gemm_pp_kernel<4";
    case 5: return "gemm_pp_kernel<5";
    case 6: return "gemm_ring_kernel<64, 128, 1, 2, 4, 1";
    case 7: return "gemm_ring_kernel<192, 128, 2, 2, 4, 2";
    case 8: return "gemm_ring_kernel<192, 256, 2, 2, 4, 2";
    case 9: return "gemm_ring_kernel<128, 192, 2, 2, 4, 1";
    default: return "gemm_ring_kernel<128, 128, 2, 2, 4, 1";
  }
}

bool gemm_ring_ok(const gvl_gemm_desc* d) {
  return d->k % KS == 0 && d->k > 0 && d->lda % 8 == 0 && d->ldb % 8 == 0 &&
         aligned16(d->a) && aligned16(d->b) &&
         (d->a_mn ? d->k * d->lda : d->m * d->lda) * 2 < 0x7fffffffLL &&
         (d->b_mn ? d->k * d->ldb : d->n * d->ldb) * 2 < 0x7fffffffLL;
}

int gemm_ring_launch(const GemmP& p, int a_mn, int b_mn, int cfg, hipStream_t s) {
  if (!a_mn && !b_mn) return launch_layout<false, false>(p, cfg, s);
  if (!a_mn && b_mn) return launch_layout<false, true>(p, cfg, s);
  if (a_mn && !b_mn) return launch_layout<true, false>(p, cfg, s);
  return launch_layout<true, true>(p, cfg, s);
}
}  // namespace gvl

namespace gvl {
// Tile choice (measured, tools/gemm_sweep.sh on MI355X): the ping-pong 256x256 kernel once the
// output has >= 192 of its tiles, except between 1 and 1.25 rounds of 256 CUs (a nearly empty
// second round); else the 128x128 ring kernel at two workgroups per CU.
// GVL_RING_SMALL=<cfg> (1 = 256x128, 6 = 64x128) overrides that choice for outputs of
// 256..512 tiles of 128x128 (A/B measurement; tools/gpu_ab.sh).  64x128 measured on the
// Q-Former caption step (its N = 768 GEMMs at M = 8064): dominant GEMM 0.198 -> 0.200 of
// peak but the step 13.0k -> 12.8k img/s, so it is not the default.
static int ring_band_cfg() {
  static const int cfg = [] {
    const char* e = getenv("GVL_RING_SMALL");
    return (e && (e[0] == '1' || e[0] == '6') && e[1] == 0) ? e[0] - '0' : 2;
  }();
  return cfg;
}
int gemm_ring_pick(int64_t M, int64_t N, int64_t K, int forced, int a_mn) {
  if (forced >= 0) return forced;
  const int64_t t256 = ((M + 255) / 256) * ((N + 255) / 256);
  if (t256 < 192 || (t256 > 256 && t256 <= 320)) {
    const int64_t t128 = ((M + 127) / 128) * ((N + 127) / 128);
    if (!a_mn && t128 > 256 && t128 < 512) return ring_band_cfg();
    return 2;
  }
  return 4;
}
}  // namespace gvl
