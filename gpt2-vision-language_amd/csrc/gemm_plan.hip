// Host-side planning of the persistent GEMM (gemm_pp3_kernel, gemm_pp3.h): epilogue kind,
// tile shape (256 / 192 wide, 256 / 128 high), split-K and the in-launch two-way combine,
// and the per-layout launch (gemm_pp3_{ff,ft,tf,tt}.hip are the instantiation units).
#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "gemm_ring.h"
#include "../../include/gvl.h"

namespace gvl {

using gvl_ring::KS;

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
  if (p.act == 5) return (!p.dact && b && !r && !p.pre_out) ? EPI_BIAS_QGELU : EPI_GEN;
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
  // the persistent kernel's in-launch two-way combine for single GEMMs: measured slower than
  // whole-K tiles, so only with GVL_PP3_COMBINE=1, whatever tickets the caller passes
  // (since round 5 gvl.kernels always passes them, for the AGPR kernel's split, gemm_w4x.hip)
  static const bool combine_env = [] {
    const char* e = getenv("GVL_PP3_COMBINE");
    return e && e[0] == '1';
  }();
  const bool combine_on = combine_env || pp3_combine_forced();  // (gvl_gemm_tune(3, 13): tests)
  if (sp <= 2 && combine_on && p.ws != nullptr && p.tickets != nullptr && gemm_epi_kind(p) != EPI_GEN) {
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
}  // namespace gvl
