// bf16 GEMM v2: LDS-DMA staged (buffer_load_dwordx4 ... lds), 8-wave 256-wide tiles.
//
// Differences from the register-staged kernel (gemm.hip):
//   * operand tiles move HBM/L2 -> LDS by LDS-DMA (no VGPR round trip, no ds_write pass);
//     the LDS image is lane-linear per 1-KiB wave instruction, so the bank swizzle is
//     applied on the SOURCE address (logical chunk = physical chunk ^ f(row)) and the
//     same XOR on the fragment read (guide rule 21);
//   * buffer resource descriptors bound every load: rows past the matrix read as zero;
//   * tiles BMxBN in {256x256, 256x128, 128x128} with 8 / 8 / 4 waves; the next K-tile's
//     DMA is issued before the current tile's MFMAs, one vmcnt(0)+barrier per K-tile.
// Requires K % 64 == 0 (no K tail inside a row) and 16-byte aligned rows; the host falls
// back to gemm.hip otherwise.  Epilogue identical to gemm.hip.
#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "../../include/gvl.h"

namespace {

constexpr int BK = 64;
typedef __attribute__((address_space(3))) void lds_void_t;

GVL_DEV int fK(int row) { return (row >> 1) & 7; }                          // 128-B rows
GVL_DEV int fT(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }           // 256-B rows

GVL_DEV __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffff ? bytes : 0x7fffffff));
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

// One operand tile in LDS.
//  K-contiguous: [R rows][64 k], 128-B rows; one DMA instruction = 8 rows.
//  MN-contiguous: [R/128 halves][64 k][128 cols], 256-B rows; one DMA = 4 k-rows of a half.
template <int R, bool MN>
struct Tile {
  static constexpr int BYTES = R * BK * 2;
  static constexpr int NINSTR = BYTES / 1024;

  // Issue this wave's share of DMA instructions for the tile at (r0, k0).
  GVL_DEV static void issue(__amdgpu_buffer_rsrc_t rs, int64_t ld, int64_t r0, int64_t k0,
                            char* lds, int wave, int nwaves, int lane) {
#pragma unroll
    for (int j = 0; j < NINSTR; ++j) {
      if ((j % nwaves) != wave) continue;
      int64_t off_elems;
      if (!MN) {
        const int row = 8 * j + (lane >> 3);
        const int lc = (lane & 7) ^ fK(row);
        off_elems = (r0 + row) * ld + k0 + lc * 8;
      } else {
        const int half = j / 16, kr = 4 * (j % 16) + (lane >> 4);
        const int lc = (lane & 15) ^ fT(kr);
        off_elems = (k0 + kr) * ld + r0 + half * 128 + lc * 8;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + j * 1024), 16,
                                               (int)(off_elems * 2), 0, 0, 0);
    }
  }

  // 16x32 operand fragment: rows/cols [c0, c0+16), k-step s.
  GVL_DEV static short8_t frag(const char* lds, int c0, int s, int lane) {
    if (!MN) {
      const int row = c0 + (lane & 15), ch = 4 * s + (lane >> 4);
      return *reinterpret_cast<const short8_t*>(lds + row * 128 + ((ch ^ fK(row)) << 4));
    } else {
      const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
      const int half = c0 >> 7, cl = c0 & 127;
      const int kr = 32 * s + 8 * G + q;
      const int ch = (cl >> 3) + (p >> 1);
      const char* base = lds + half * 16384;
      const int off1 = kr * 256 + ((ch ^ fT(kr)) << 4) + (p & 1) * 8;
      short8_t r;
      r.lo = lds_read_tr(base + off1);
      r.hi = lds_read_tr(base + off1 + 4 * 256);
      return r;
    }
  }
};

template <int BM, int BN, int WMW, int WNW, bool AMN, bool BMN>
__global__ __launch_bounds__(64 * WMW * WNW, (BM * BN > 16384 ? 1 : 2)) void gemm_lds_kernel(GemmP p) {
  constexpr int NW = WMW * WNW;
  constexpr int TM = BM / WMW, TN = BN / WNW, FM = TM / 16, FN = TN / 16;
  using TA = Tile<BM, AMN>;
  using TB = Tile<BN, BMN>;
  constexpr int STAGE = TA::BYTES + TB::BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;

  int split, tm, tn;
  gemm_work_tile(p.splits, p.tiles_m, p.tiles_n, p.group, split, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * p.kper;
  const int64_t kend = kbeg + p.kper < p.K ? kbeg + p.kper : p.K;

  // buffer descriptors over the whole operand extents (reads past the end return 0);
  // inputs readfirstlane'd so hipcc can prove them wave-uniform (no waterfall loops, T20)
  const int64_t a_rows = AMN ? p.K : p.M, b_rows = BMN ? p.K : p.N;
  const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A, a_rows * p.lda * 2);
  const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B, b_rows * p.ldb * 2);

  float4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((kend - kbeg) / BK);
  TA::issue(ra, p.lda, m0, kbeg, smem, wave, NW, lane);
  TB::issue(rb, p.ldb, n0, kbeg, smem + TA::BYTES, wave, NW, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * STAGE;
      const int64_t k1 = kbeg + (int64_t)(kt + 1) * BK;
      TA::issue(ra, p.lda, m0, k1, nxt, wave, NW, lane);
      TB::issue(rb, p.ldb, n0, k1, nxt + TA::BYTES, wave, NW, lane);
    }
    const char* sa = cur;
    const char* sb = cur + TA::BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      short8_t bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = TB::frag(sb, wn * TN + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const short8_t af = TA::frag(sa, wm * TM + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bfr[j], af, acc[i][j]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if (p.splits > 1) {
    gemm_store_partial<FM, FN>(p, acc, split, m0 + wm * TM, n0 + wn * TN, lane);
  } else {
    gemm_epilogue<FM, FN>(p, acc, m0 + wm * TM, n0 + wn * TN, lane);
  }
}

// Sum the split-K partials and apply the epilogue: one thread per 4 output columns.
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemmP p) {
  const int64_t nq = p.N >> 2;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= p.M * nq) return;
  const int64_t m = idx / nq, n = (idx - m * nq) * 4;
  float4_t s = {0.f, 0.f, 0.f, 0.f};
  const int64_t stride = p.M * p.N;
  const float* src = p.ws + m * p.N + n;
  for (int k = 0; k < p.splits; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(src + k * stride);
    s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
  }
  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;
  const float gatev = p.gate ? tanhf(bf2f(*p.gate)) : 1.f;
  gemm_epi_quad(p, s, m, n, alpha, gatev);
}

template <int BM, int BN, int WMW, int WNW, bool AMN, bool BMN>
int launch_cfg(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;
  p.tiles_m = (int)((p.M + BM - 1) / BM);
  p.tiles_n = (int)((p.N + BN - 1) / BN);
  constexpr int lds = 2 * (BM + BN) * BK * 2;
  auto kern = gemm_lds_kernel<BM, BN, WMW, WNW, AMN, BMN>;
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
  p.kper = p.splits > 1 ? ((p.K / p.splits + BK - 1) / BK) * BK : p.K;
  if (p.splits > 1) p.splits = (int)((p.K + p.kper - 1) / p.kper);
  gvl::launch_timed(kern, dim3(p.tiles_m * p.tiles_n * p.splits), dim3(64 * WMW * WNW), lds, s, p);
  if (p.splits > 1) gvl::gemm_splitk_reduce_launch(p, s);
  return 0;
}

template <bool AMN, bool BMN>
int launch_layout(const GemmP& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_cfg<256, 256, 2, 4, AMN, BMN>(p, s);
    case 1: return launch_cfg<256, 128, 4, 2, AMN, BMN>(p, s);
    default: return launch_cfg<128, 128, 2, 2, AMN, BMN>(p, s);
  }
}

}  // namespace

namespace gvl {
void gemm_splitk_reduce_launch(const GemmP& p, hipStream_t s) {
  const int64_t quads = p.M * (p.N >> 2);
  hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)((quads + 255) / 256)), dim3(256), 0, s, p);
}

// Tile choice: estimated time = waves-of-tiles x tile work / relative per-CU efficiency.
// Measured on MI355X (tools/gpu_probe_gemm.py, profiles/r1): 128x128 (2 WGs/CU) wins for the
// caption-step shapes (M ~ 8k, N 768-3072); 256x256 only once there are >= 2 tiles per CU.
// Split K only when the output has fewer tiles than CUs and each slice keeps >= 8 K-tiles.
int gemm_splitk_pick(int64_t tiles, int64_t K) {
  if (tiles >= 256 || K < 1024) return 1;
  int64_t sp = 512 / tiles;
  const int64_t kmax = K / 512;
  if (sp > kmax) sp = kmax;
  if (sp > 16) sp = 16;
  return sp < 2 ? 1 : (int)sp;
}

int gemm_lds_pick(int64_t M, int64_t N, int64_t K, int forced) {
  if (forced >= 0) return forced;
  const int64_t t256 = ((M + 255) / 256) * ((N + 255) / 256);
  return t256 >= 512 ? 0 : 2;
}

bool gemm_lds_ok(const gvl_gemm_desc* d) {
  return d->k % BK == 0 && d->k > 0 && d->lda % 8 == 0 && d->ldb % 8 == 0 &&
         aligned16(d->a) && aligned16(d->b) &&
         (d->a_mn ? d->k * d->lda : d->m * d->lda) * 2 < 0x7fffffffLL &&
         (d->b_mn ? d->k * d->ldb : d->n * d->ldb) * 2 < 0x7fffffffLL;
}

int gemm_lds_launch(const GemmP& p, int a_mn, int b_mn, int cfg, hipStream_t s) {
  if (!a_mn && !b_mn) return launch_layout<false, false>(p, cfg, s);
  if (!a_mn && b_mn) return launch_layout<false, true>(p, cfg, s);
  if (a_mn && !b_mn) return launch_layout<true, false>(p, cfg, s);
  return launch_layout<true, true>(p, cfg, s);
}
}  // namespace gvl
