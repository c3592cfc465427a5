// bf16 GEMM v6: persistent 256x256 tiles over 64-deep K-tiles in quadrant phases (gfx950).
//
// Where v5 (gemm_pp2.hip, gemm_pp3_kernel) stages 32-deep K-steps — 64-B row pieces, two
// requests per 128-B line — and runs one 32-MFMA cluster per barrier pair, this kernel
// stages 64-deep K-tiles in four half-tiles (A rows 0-127 / 128-255, B cols 0-127 /
// 128-255; 128 x 64 bf16 = 16 KiB = 2 LDS-DMA pieces per wave) and splits every K-tile into
// four phases of 16 MFMAs, one output quadrant each.  Two LDS buffers (128 KiB).
//
// Waves: g = wave / 4 (stagger group), wr = g, wc = wave % 4.  A wave owns output rows
// {wr*64 + 128 i + [0, 64)} and cols {wc*32 + 128 j + [0, 32)}, i, j in {0, 1}: quadrant
// (i, j) reads only A half i and B half j, so every half-tile has one first use:
//   phase r=0: quadrant (0,0), reads A0 (8 frags) + B0 (4)     A0 = A rows 0-127 ...
//   phase r=1: quadrant (0,1), reads B1 (4)                    (A0 frags held)
//   phase r=2: quadrant (1,1), reads A1 (8)                    (B1 held)
//   phase r=3: quadrant (1,0), no reads                        (A1, B0 held)
// Staging, over the WG's stream of K-tiles g = 0, 1, ... (all its tiles back to back):
// {A0,B0}(g) at phase 4g-6, B1(g) at 4g-5, A1(g) at 4g-4 — each exactly 2 phases after the
// last read of the same region by K-tile g-2 (same buffer): WAR safe for both stagger
// groups.  A half-tile used in phase p is retired by a counted vmcnt in phase p-1 before
// its first barrier (RAW); the counts leave 8-10 pieces (4-5 half-tiles) in flight.
// Group 1 runs one barrier behind group 0, so on each SIMD one wave's MFMA cluster overlaps
// the other's LDS reads + DMA issue.
// LDS images: K-contiguous operand: [128 rows][64 k], 128-B rows, 16-B chunk c of row r at
// c ^ ((r >> 1) & 7) (conflict-free ds_read_b128 lane groups); MN-contiguous operand:
// [64 k][128 cols], 256-B rows, read with ds_read_b64_tr_b16 (gemm_ring.h fT swizzle).
#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "gemm_ring.h"
#include "../../include/gvl.h"

namespace {

using namespace gvl_ring;

constexpr int BK = 64;
constexpr int HALF = 128 * BK * 2;  // 16 KiB half-tile
constexpr int KT_BYTES = 4 * HALF;  // one K-tile: A0 A1 B0 B1
constexpr int LDS_BYTES = 2 * KT_BYTES;

GVL_DEV int f128(int row) { return (row >> 1) & 7; }  // 128-B rows

template <bool MN>
struct Half {
  // this wave's two DMA pieces (j = wave, wave + 8) of the half-tile at slab r0, K-tile k0
  GVL_DEV static void offsets(int64_t ld, int64_t r0, int64_t k0, int wave, int lane, int (&off)[2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = wave + 8 * t;
      int64_t e;
      if (!MN) {
        const int row = 8 * j + (lane >> 3);
        e = (r0 + row) * ld + k0 + ((lane & 7) ^ f128(row)) * 8;
      } else {
        const int kr = 4 * j + (lane >> 4);
        e = (k0 + kr) * ld + r0 + ((lane & 15) ^ fT(kr)) * 8;
      }
      off[t] = (int)(e * 2);
    }
  }
  GVL_DEV static int kt_bytes(int64_t ld) { return MN ? (int)(BK * ld * 2) : BK * 2; }
  GVL_DEV static int half_bytes(int64_t ld) { return MN ? 256 : (int)(128 * ld * 2); }
  GVL_DEV static void issue(__amdgpu_buffer_rsrc_t rs, const int (&off)[2], int soff, char* lds,
                            int wave) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + (wave + 8 * t) * 1024), 16,
                                               off[t], soff, 0, 0);
  }
  // 16 rows/cols [c0, c0 + 16) of the half (c0 < 128) x k-sub s (32 deep)
  GVL_DEV static short8_t frag(const char* lds, int c0, int s, int lane) {
    if (!MN) {
      const int row = c0 + (lane & 15), ch = 4 * s + (lane >> 4);
      return *reinterpret_cast<const short8_t*>(lds + row * 128 + ((ch ^ f128(row)) << 4));
    } else {
      const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
      const int kr = 32 * s + 8 * G + q;
      const int ch = (c0 >> 3) + (p >> 1);
      const int off1 = kr * 256 + ((ch ^ fT(kr)) << 4) + (p & 1) * 8;
      short8_t r;
      r.lo = lds_read_tr(lds + off1);
      r.hi = lds_read_tr(lds + off1 + 4 * 256);
      return r;
    }
  }
};

// s_waitcnt vmcnt(n) for a runtime even n in [0, 10]
GVL_DEV void wait_vm(int n) {
  if (n >= 10) { asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); return; }
  if (n >= 8) { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); return; }
  if (n >= 6) { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); return; }
  if (n >= 4) { asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); return; }
  if (n >= 2) { asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); return; }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool AMN, bool BMN, int EPI>
__global__ __launch_bounds__(512, 1) void gemm_8p_kernel(GemmP p) {
  using HA = Half<AMN>;
  using HB = Half<BMN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 2, wc = wave & 3;

  const int total = p.tiles_m * p.tiles_n * p.splits;
  const int G = gridDim.x, b = blockIdx.x;
  const int ntl = (total - b + G - 1) / G;
  const int nkt = (int)(p.kper / BK);
  const int n = ntl * nkt;  // K-tiles of this workgroup
  auto tile_coords = [&](int t, int64_t& m0, int64_t& n0, int64_t& k0, int& split) {
    const int vid = b + t * G;
    const int q8 = total >> 3, r8 = total & 7, xcd = vid & 7;
    const int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (vid >> 3);
    int tm, tn;
    gemm_tile_of(work, p.splits, p.tiles_m, p.tiles_n, p.group, split, tm, tn);
    m0 = (int64_t)tm * 256;
    n0 = (int64_t)tn * 256;
    k0 = (int64_t)split * p.kper;
  };

  const int64_t a_rows = AMN ? p.K : p.M, b_rows = BMN ? p.K : p.N;
  const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A, a_rows * p.lda * 2);
  const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B, b_rows * p.ldb * 2);
  const int a_kt = HA::kt_bytes(p.lda), b_kt = HB::kt_bytes(p.ldb);
  const int a_h1 = HA::half_bytes(p.lda), b_h1 = HB::half_bytes(p.ldb);

  // issue cursor: K-tile is_g (tile is_t, K-tile is_k within it), half-group is_h:
  // 0 = {A0, B0}, 1 = B1, 2 = A1
  int is_t = 0, is_k = 0, is_g = 0, is_h = 0;
  int offa[2], offb[2];
  {
    int64_t m0, n0, k0;
    int sp;
    tile_coords(0, m0, n0, k0, sp);
    HA::offsets(p.lda, m0, k0, wave, lane, offa);
    HB::offsets(p.ldb, n0, k0, wave, lane, offb);
  }
  auto issue_next = [&]() {
    if (is_g >= n) return;
    char* buf = smem + (is_g & 1) * KT_BYTES;  // A0 | A1 | B0 | B1
    if (is_h == 0) {
      HA::issue(ra, offa, is_k * a_kt, buf, wave);
      HB::issue(rb, offb, is_k * b_kt, buf + 2 * HALF, wave);
      is_h = 1;
    } else if (is_h == 1) {
      HB::issue(rb, offb, is_k * b_kt + b_h1, buf + 3 * HALF, wave);
      is_h = 2;
    } else {
      HA::issue(ra, offa, is_k * a_kt + a_h1, buf + HALF, wave);
      is_h = 0;
      ++is_g;
      if (++is_k == nkt) {
        is_k = 0;
        if (++is_t < ntl) {
          int64_t m0, n0, k0;
          int sp;
          tile_coords(is_t, m0, n0, k0, sp);
          HA::offsets(p.lda, m0, k0, wave, lane, offa);
          HB::offsets(p.ldb, n0, k0, wave, lane, offb);
        }
      }
    }
  };

  float4_t acc[2][2][4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[i][j][x][y] = float4_t{0.f, 0.f, 0.f, 0.f};

  // prologue: {A0,B0}(0), B1(0), A1(0), {A0,B0}(1), B1(1); retire {A0,B0}(0)
#pragma unroll
  for (int i = 0; i < 5; ++i) issue_next();
  wait_vm((0 < n ? 4 : 0) + (1 < n ? 6 : 0));
  barrier_lds();
  if (g == 1) __builtin_amdgcn_s_barrier();

  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;
  int cu_k = 0, cu_t = 0;
  int64_t cu_m0, cu_n0, cu_k0;
  int cu_sp;
  tile_coords(0, cu_m0, cu_n0, cu_k0, cu_sp);
  const int arow = g * 64, bcol = wc * 32;
  EpiPre<4, 2, EPI> pre[2];
  pre[0].load_bias(p, cu_n0 + bcol, lane);
  pre[1].load_bias(p, cu_n0 + 128 + bcol, lane);
  auto epilogue = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t mw = cu_m0 + 128 * i + arow, nw = cu_n0 + 128 * j + bcol;
        if (p.splits > 1)
          gemm_store_partial<4, 2>(p, acc[i][j], cu_sp, mw, nw, lane);
        else
          gemm_epilogue16<4, 2, EPI>(p, acc[i][j], mw, nw, lane, alpha, pre[j]);
      }
  };

  short8_t a0[4][2], a1[4][2], b0[2][2], b1[2][2];
  auto mma = [&](float4_t (&c)[4][2], const short8_t (&af)[4][2], const short8_t (&bf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) c[x][y] = mfma16(bf[y][s], af[x][s], c[x][y]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto mid = [&]() {  // first barrier of a phase, then this phase's fragments are in VGPRs
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  for (int u = 0; u < n; ++u) {
    const char* buf = smem + (u & 1) * KT_BYTES;
    // ---- phase 0: (new tile: previous tile's epilogue) reads A0, B0; issues A1(u+1);
    //      retires B1(u)
    if (cu_k == 0 && u > 0) {
      epilogue();
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) acc[i][j][x][y] = float4_t{0.f, 0.f, 0.f, 0.f};
      ++cu_t;
      tile_coords(cu_t, cu_m0, cu_n0, cu_k0, cu_sp);
      pre[0].load_bias(p, cu_n0 + bcol, lane);
      pre[1].load_bias(p, cu_n0 + 128 + bcol, lane);
    }
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int s = 0; s < 2; ++s) b0[y][s] = HB::frag(buf + 2 * HALF, bcol + 16 * y, s, lane);
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int s = 0; s < 2; ++s) a0[x][s] = HA::frag(buf, arow + 16 * x, s, lane);
    issue_next();
    wait_vm(2 + (u + 1 < n ? 8 : 0));
    mid();
    mma(acc[0][0], a0, b0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 1: reads B1; retires A1(u)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int s = 0; s < 2; ++s) b1[y][s] = HB::frag(buf + 3 * HALF, bcol + 16 * y, s, lane);
    wait_vm(u + 1 < n ? 8 : 0);
    mid();
    mma(acc[0][1], a0, b1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: reads A1; issues {A0,B0}(u+2)
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int s = 0; s < 2; ++s) a1[x][s] = HA::frag(buf + HALF, arow + 16 * x, s, lane);
    issue_next();
    mid();
    mma(acc[1][1], a1, b1);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: no reads; issues B1(u+2); retires {A0,B0}(u+1)
    issue_next();
    wait_vm((u + 1 < n ? 4 : 0) + (u + 2 < n ? 6 : 0));
    mid();
    mma(acc[1][0], a1, b0);
    if (++cu_k == nkt) cu_k = 0;
    __builtin_amdgcn_s_barrier();
  }
  if (g == 0) __builtin_amdgcn_s_barrier();
  if (n > 0) epilogue();
}

template <bool AMN, bool BMN, int EPI>
void launch_8p(const GemmP& p, hipStream_t s) {
  auto kern = gemm_8p_kernel<AMN, BMN, EPI>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    attr_set = true;
  }
  const int total = p.tiles_m * p.tiles_n * p.splits;
  const int grid = total < gvl::num_cus() ? total : gvl::num_cus();
  gvl::launch_timed(kern, dim3(grid), dim3(512), LDS_BYTES, s, p);
  if (p.splits > 1) gvl::gemm_splitk_reduce_launch(p, s);
}

// EPI_GEN (dropout / gate / fp32 output) is left to the older kernels: the plan rejects it.
template <bool AMN, bool BMN>
void launch_8p_epi(const GemmP& p, hipStream_t s) {
  if (p.splits > 1) return launch_8p<AMN, BMN, EPI_PLAIN>(p, s);  // partials only
  switch (gvl::gemm_epi_kind(p)) {
    case EPI_PLAIN: return launch_8p<AMN, BMN, EPI_PLAIN>(p, s);
    case EPI_BIAS: return launch_8p<AMN, BMN, EPI_BIAS>(p, s);
    case EPI_BIAS_RES: return launch_8p<AMN, BMN, EPI_BIAS_RES>(p, s);
    case EPI_BIAS_ACT: return launch_8p<AMN, BMN, EPI_BIAS_ACT>(p, s);
    case EPI_DACT: return launch_8p<AMN, BMN, EPI_DACT>(p, s);
    case EPI_RES: return launch_8p<AMN, BMN, EPI_RES>(p, s);
    case EPI_BIAS_ACT_ERF: return launch_8p<AMN, BMN, EPI_BIAS_ACT_ERF>(p, s);
    case EPI_DACT_ERF: return launch_8p<AMN, BMN, EPI_DACT_ERF>(p, s);
    case EPI_BIAS_ACT_D: return launch_8p<AMN, BMN, EPI_BIAS_ACT_D>(p, s);
    case EPI_BIAS_ACT_ERF_D: return launch_8p<AMN, BMN, EPI_BIAS_ACT_ERF_D>(p, s);
    case EPI_MUL: return launch_8p<AMN, BMN, EPI_MUL>(p, s);
    default: return;  // unreachable (gemm_8p_plan)
  }
}

}  // namespace

namespace gvl {
// Same plan as the v5 kernel (tiles, split-K slices, >= 160 work items) with 64-deep
// K-tiles: K (and every split-K slice) a multiple of 64.
bool gemm_8p_plan(GemmP& p, bool force) {
  if (p.K % BK != 0) return false;
  if (!gemm_pp3_plan(p, force, BK)) return false;
  return gemm_epi_kind(p) != EPI_GEN && gemm_epi_kind(p) != EPI_BIAS_DROP_RES;
}

bool gemm_8p_try(const GemmP& p0, int a_mn, int b_mn, bool force, hipStream_t s) {
  GemmP p = p0;
  if (!gemm_8p_plan(p, force)) return false;
  if (!a_mn && !b_mn) launch_8p_epi<false, false>(p, s);
  else if (!a_mn && b_mn) launch_8p_epi<false, true>(p, s);
  else if (a_mn && !b_mn) launch_8p_epi<true, false>(p, s);
  else launch_8p_epi<true, true>(p, s);
  return true;
}
}  // namespace gvl
