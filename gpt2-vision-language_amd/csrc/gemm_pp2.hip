// bf16 GEMM v4: ping-pong 256x256 with whole-tile clusters.
//
// The v3 ping-pong (gemm_ring.hip, gemm_pp_kernel) splits every 32-deep K-step into two
// row halves, so each barrier-delimited cluster holds 16 MFMAs (256 cycles of the SIMD's
// matrix pipe) while the partner wave's memory cluster (8 ds_read_b128, or 4 reads + the
// step's 4 LDS-DMA issues) often runs longer: the matrix pipe idles at every other barrier.
// Here a cluster is KC whole K-steps of the wave's 128x64 output: 32*KC MFMAs against a
// memory cluster of 12*KC fragment reads + 4*KC DMA issues, and one barrier pair per
// cluster instead of per half step.
//
// Waves: group g = wave / 4 (output rows 128 g ..), column block wc = wave % 4 (64 cols);
// group 1 runs one barrier behind group 0, so on every SIMD one wave computes while the
// other loads.  Phase 2c: group 0 M(c), group 1 C(c-1); phase 2c+1: group 0 C(c), group 1
// M(c).  LDS ring of NS slots of 32-deep K-steps (A[256][32] + B[256][32] = 32 KiB each).
//  * M(c) reads cluster c's fragments and issues the DMA of steps [cKC+NS-KC, cKC+NS) into
//    cluster c-1's slots: their last readers (group 1's M(c-1), phase 2c-1) retired their
//    reads (lgkmcnt(0)) before the barrier closing phase 2c-1;
//  * cluster c+1's steps are retired (counted vmcnt) by every wave before the barrier that
//    closes phase 2c+1: group 1 at the end of M(c), group 0 at the end of C(c).
#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "gemm_ring.h"
#include "gemm_pp3.h"
#include "../../include/gvl.h"

namespace {

using namespace gvl_ring;

template <int NS, int KC, bool AMN, bool BMN>
__global__ __launch_bounds__(512, 1) void gemm_pp2_kernel(GemmP p) {
  constexpr int BM = 256, BN = 256, NW = 8, FM = 8, FN = 4;
  static_assert(NS >= 2 * KC && NS <= 5, "ring geometry");
  using SA = Step<BM, AMN, NW>;
  using SB = Step<BN, BMN, NW>;
  constexpr int SLOT = SA::BYTES + SB::BYTES;
  constexpr int IPW = (SA::NINSTR + SB::NINSTR) / NW;
  constexpr int INFL = NS - 2 * KC;  // steps left in flight across the cluster barrier
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
  const int ncl = (nks + KC - 1) / KC;

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
  // steps issued but not needed by cluster c+1, after M(c)'s issue: min(INFL, nks - (c+2)KC)
  auto inflight_after = [&](int c) {
    const int r = nks - (c + 2) * KC;
    return r < 0 ? 0 : (r < INFL ? r : INFL);
  };

  float4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int arow = g * 128, bcol = wc * 64;
#pragma unroll
  for (int i = 0; i < NS - KC; ++i) issue(i);
  {  // cluster 0 retired: of steps [0, NS-KC) leave min(NS-2KC, nks-KC) in flight
    const int r = nks - KC;
    wait_vm_steps<IPW, (INFL > 0 ? INFL : 0)>(r < 0 ? 0 : (r < INFL ? r : INFL));
  }
  barrier_lds();
  if (g == 1) __builtin_amdgcn_s_barrier();

  short8_t af[KC][FM], bf[KC][FN];
  for (int c = 0; c < ncl; ++c) {
    // ---- M(c): fragments of cluster c, DMA of the steps refilling cluster c-1's slots
#pragma unroll
    for (int q = 0; q < KC; ++q) {
      const int s = c * KC + q;
      const char* sl = smem + (s % NS) * SLOT;
      if (s < nks) {
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[q][j] = SB::frag(sl + SA::BYTES, bcol + 16 * j, lane);
#pragma unroll
        for (int i = 0; i < FM; ++i) af[q][i] = SA::frag(sl, arow + 16 * i, lane);
      }
    }
#pragma unroll
    for (int q = 0; q < KC; ++q) issue(c * KC + NS - KC + q);
    if (g == 1) wait_vm_steps<IPW, (INFL > 0 ? INFL : 0)>(inflight_after(c));
    barrier_lds();
    // ---- C(c)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < KC; ++q) {
      if (c * KC + q < nks) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bf[q][j], af[q][i], acc[i][j]);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (g == 0) wait_vm_steps<IPW, (INFL > 0 ? INFL : 0)>(inflight_after(c));
    barrier_lds();
  }
  if (g == 0) __builtin_amdgcn_s_barrier();

  if (p.splits > 1) {
    gemm_store_partial<FM, FN>(p, acc, split, m0 + arow, n0 + bcol, lane);
  } else {
    gemm_epilogue<FM, FN>(p, acc, m0 + arow, n0 + bcol, lane);
  }
}

template <int NS, int KC, bool AMN, bool BMN>
int launch_pp2(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;
  p.tiles_m = (int)((p.M + 255) / 256);
  p.tiles_n = (int)((p.N + 255) / 256);
  constexpr int lds = NS * 512 * KS * 2;
  auto kern = gemm_pp2_kernel<NS, KC, AMN, BMN>;
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

// cfg 0: NS=4, KC=1 (3 steps in flight, 32-MFMA clusters); 1: NS=4, KC=2 (64-MFMA clusters,
// ring drained per cluster); 2: NS=5, KC=2 (one step in flight across the cluster barrier).
template <bool AMN, bool BMN>
int launch_layout(const GemmP& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 3: {
      GemmP q = p;
      if (gvl::gemm_pp3_plan(q, true) && gvl::gemm_pp3_launch(q, AMN, BMN, s) == 0) return 0;
      return launch_pp2<4, 1, AMN, BMN>(p, s);
    }
    case 1: return launch_pp2<4, 2, AMN, BMN>(p, s);
    case 2: return launch_pp2<5, 2, AMN, BMN>(p, s);
    default: return launch_pp2<4, 1, AMN, BMN>(p, s);
  }
}

}  // namespace

namespace gvl {
const char* gemm_pp2_name(int cfg) {
  switch (cfg) {
    case 3: return "gemm_pp3_kernel<4";
    case 1: return "gemm_pp2_kernel<4, 2";
    case 2: return "gemm_pp2_kernel<5, 2";
    default: return "gemm_pp2_kernel<4, 1";
  }
}

int gemm_epi_kind(const GemmP& p) {
  if (p.has_drop && !p.gate && !p.c_f32 && !p.act && !p.dact && p.bias && p.residual)
    return EPI_BIAS_DROP_RES;
  if (p.has_drop || p.gate || p.c_f32) return EPI_GEN;
  const bool b = p.bias != nullptr, r = p.residual != nullptr;
  if (!p.act && !p.dact) {
    if (!b && !r) return EPI_PLAIN;
    if (b && !r) return EPI_BIAS;
    if (b && r) return EPI_BIAS_RES;
    return EPI_RES;
  }
  if (p.act && !p.dact && b && !r) {
    const int k[5] = {EPI_GEN, EPI_BIAS_ACT, EPI_BIAS_ACT_ERF, EPI_BIAS_ACT_D, EPI_BIAS_ACT_ERF_D};
    return k[p.act];
  }
  if (p.dact && !p.act && !b && !r) {
    const int k[4] = {EPI_GEN, EPI_DACT, EPI_DACT_ERF, EPI_MUL};
    return k[p.dact];
  }
  return EPI_GEN;
}

// Split-K factor for the persistent kernel: minimise the estimated time in units of one
// 256x256 tile's 32-deep K-step, T(s) = rounds(tiles*s) * (K/32s + 6) + slab round trip
// (s fp32 partials written + read, at ~6 TB/s, ~1.1 PF/s of MFMA per 256 CUs); slices must
// be equal and at least 16 K-steps deep.
int gemm_pp3_splits(int64_t M, int64_t N, int64_t K, int gran) {
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int cus = num_cus();
  const double step_s = 2.0 * 256 * 256 * 32 / (1.1e15 / cus);
  double best = 1e30;
  int best_s = 1;
  for (int s = 1; s <= 16; ++s) {
    if (K % ((int64_t)gran * s) != 0 || (s > 1 && K / s < 512)) continue;
    const int64_t rounds = (tiles * s + cus - 1) / cus;
    double t = (double)rounds * ((double)K / (32.0 * s) + 6.0);
    if (s > 1) t += (double)s * M * N * 8.0 / 6e12 / step_s;
    if (t < best * 0.97) { best = t; best_s = s; }
  }
  return best_s;
}

// Persistent-kernel plan: bf16 output with 16-B stores; tiles, split-K factor and K-slice
// depth filled into p.  Without `force`, only when the work items fill the chip well enough
// to beat the 128x128 ring (measured, tools/gemm_shapes.py): >= 160 items.
// Work-item floor for the persistent kernel (GVL_PP3_MIN overrides it for A/B measurement).
static int64_t pp3_min_items() {
  static const int64_t v = [] {
    const char* e = getenv("GVL_PP3_MIN");
    const long x = e ? atol(e) : 0;
    return (int64_t)(x > 0 ? x : 160);
  }();
  return v;
}

// Output tile width: 192 when its tiles fill the last round of CUs better than 256-wide ones
// (per-tile efficiency of the narrower tile counted at 0.9); GVL_PP3_BN=256|192 forces one.
static int pp3_tile_width(int64_t M, int64_t N) {
  static const int forced = [] {
    const char* e = getenv("GVL_PP3_BN");
    return e ? atoi(e) : 0;
  }();
  if (N % 64 != 0 || N < 384) return 256;
  if (forced == 256 || forced == 192) return forced;
  const int64_t cus = num_cus(), tm = (M + 255) / 256;
  auto fill = [&](int64_t tiles) {
    const int64_t rounds = (tiles + cus - 1) / cus;
    return (double)tiles / (double)(rounds * cus);
  };
  const double e256 = fill(tm * ((N + 255) / 256)), e192 = 0.9 * fill(tm * ((N + 191) / 192));
  return e192 > e256 ? 192 : 256;
}

// Tile width and K split for shapes whose slab split-K choice is at most two-way, when the
// two halves can meet inside the launch: estimated time in units of one 256x256 32-deep
// K-step, rounds(items) * (steps per item + 6) * tile cost + ~4 for the combine (the last
// arriver's write-through partial store and the other half's read).  A 192-wide step counts
// 0.75 / 0.9 of a 256-wide one (pp3_tile_width).  M = 8064, N = 768 (caption decoder):
// 128 tiles of 256x192 split in two = 256 items, one per CU.
static void pp3_choose_combined(GemmP& p, int gran) {
  const int64_t cus = num_cus(), tm = (p.M + 255) / 256;
  double best = 1e30;
  for (int bn : {256, 192}) {
    if (bn == 192 && (p.N % 64 != 0 || p.N < 384 || gran != KS)) continue;
    const double w = bn == 256 ? 1.0 : 0.75 / 0.9;
    const int64_t tiles = tm * ((p.N + bn - 1) / bn);
    for (int s = 1; s <= 2; ++s) {
      if (s == 2 && (p.K % (2 * gran) != 0 || p.K / 2 < 256 || tiles * 8 > p.nticket ||
                     2 * p.M * p.N * 4 > p.ws_bytes))
        continue;
      const int64_t rounds = (tiles * s + cus - 1) / cus;
      const double t = (double)rounds * ((double)p.K / (32.0 * s) + 6.0) * w + (s == 2 ? 4.0 : 0.0);
      if (t < best * 0.97) {
        best = t;
        p.bn = bn;
        p.splits = s;
      }
    }
  }
  p.tiles_n = (int)((p.N + p.bn - 1) / p.bn);
  p.kper = p.K / p.splits;
}

// Tile height 128 (with 192-wide tiles) when its tiles fill the CUs in fewer rounds than the
// 256-row tiles: estimated per-tile cost 0.375 / E128 of a 256x256 tile (E128 = per-FLOP
// efficiency of the half-height tile, GVL_PP3_E128 x 100, default 70: measured equal to the
// 128x128 ring at N = 768, 8 % slower than 256x192 at N = 2304); GVL_PP3_BM=128|256
// forces the height (A/B).
static int pp3_tile_height(int64_t M, int64_t N, int bn) {
  static const int forced = [] {
    const char* e = getenv("GVL_PP3_BM");
    return e ? atoi(e) : 0;
  }();
  static const double e128 = [] {
    const char* e = getenv("GVL_PP3_E128");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v / 100.0 : 0.70;
  }();
  if (N % 64 != 0 || N < 384) return 256;
  if (forced == 256 || forced == 128) return forced;
  const int64_t cus = num_cus();
  auto rounds = [&](int64_t t) { return (double)((t + cus - 1) / cus); };
  const double w_bn = bn == 256 ? 1.0 : 0.75 / 0.9;
  const double t256 = rounds(((M + 255) / 256) * ((N + bn - 1) / bn)) * w_bn;
  const double t128 = rounds(((M + 127) / 128) * ((N + 191) / 192)) * 0.375 / e128;
  return t128 < 0.95 * t256 ? 128 : 256;
}

bool gemm_pp3_plan(GemmP& p, bool force, int gran) {
  if (p.c_f32 || p.N % 8 != 0 || p.ldc % 8 != 0) return false;
  if (p.pre_out && (p.ldp % 8 != 0 || (reinterpret_cast<uintptr_t>(p.pre_out) & 15))) return false;
  p.tiles_m = (int)((p.M + 255) / 256);
  p.tiles_n = (int)((p.N + 255) / 256);
  p.splits = 1;
  p.bm = 256;
  int sp = 1;
  if (p.ws != nullptr) sp = gemm_pp3_splits(p.M, p.N, p.K, gran);
  if (sp <= 2 && p.ws != nullptr && p.tickets != nullptr && gemm_epi_kind(p) != EPI_GEN) {
    p.bn = 256;
    pp3_choose_combined(p, gran);
    if (force) return true;
    return (int64_t)p.tiles_m * p.tiles_n * p.splits >= pp3_min_items();
  }
  p.tickets = nullptr;  // slab split-K (gemm_splitk_reduce) or no split
  if (sp > 1 && (int64_t)sp * p.M * p.N * 4 <= p.ws_bytes) p.splits = sp;
  p.kper = p.K / p.splits;
  if (p.splits == 1 && gemm_epi_kind(p) == EPI_GEN) return false;
  p.bn = 256;
  if (p.splits == 1 && gran == KS) p.bn = pp3_tile_width(p.M, p.N);
  if (p.splits == 1 && gran == KS && pp3_tile_height(p.M, p.N, p.bn) == 128) {
    p.bm = 128;
    p.bn = 192;
    p.tiles_m = (int)((p.M + 127) / 128);
  }
  if (p.bn != 256) p.tiles_n = (int)((p.N + p.bn - 1) / p.bn);
  if (force) return true;
  const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
  // split-K slabs only pay off for really few tiles (dW, the caption lm_head dX); with
  // >= 64 tiles the 128x128 ring at two workgroups per CU is faster
  if (p.splits > 1 && tiles >= 64) return false;
  return tiles * p.splits >= pp3_min_items();
}

int gemm_pp3_launch(const GemmP& p, int a_mn, int b_mn, hipStream_t s) {
  if (!a_mn && !b_mn) return gemm_pp3_launch_ff(p, s);
  if (!a_mn && b_mn) return gemm_pp3_launch_ft(p, s);
  if (a_mn && !b_mn) return gemm_pp3_launch_tf(p, s);
  return gemm_pp3_launch_tt(p, s);
}

bool gemm_pp3_try(const GemmP& p0, int a_mn, int b_mn, hipStream_t s) {
  GemmP p = p0;
  if (!gemm_pp3_plan(p, false)) return false;
  return gemm_pp3_launch(p, a_mn, b_mn, s) == 0;
}

int gemm_pp2_launch(const GemmP& p, int a_mn, int b_mn, int cfg, hipStream_t s) {
  if (!a_mn && !b_mn) return launch_layout<false, false>(p, cfg, s);
  if (!a_mn && b_mn) return launch_layout<false, true>(p, cfg, s);
  if (a_mn && !b_mn) return launch_layout<true, false>(p, cfg, s);
  return launch_layout<true, true>(p, cfg, s);
}
}  // namespace gvl
