// Four-wave deep-ring GEMM for narrow outputs (N = 768 at M = 8064: the caption decoder's
// attn.c_proj / mlp.c_proj forward and c_attn / c_fc / c_proj dX).
//
// Why a fourth kernel: those outputs are 96 tiles of 256x256 (a third of the chip) or 378 of
// 128x128 (1.5 rounds), and the 192x128 tile that fills the chip in one round (42 x 6 = 252
// tiles at M = 8064) ran no faster than 128x128 in the ring kernel (gemm_ring.hip cfg 7): with
// one workgroup of 4 waves per CU there is one wave per SIMD, so every stall is an MFMA bubble,
// and its 4-slot ring keeps only two 32-deep K-steps (~0.35 us of MFMA work) in flight — less
// than an L2/MALL miss.  Here:
//   * tile 192x128, 4 waves of 96x64 (6 x 4 fragments, 24 MFMA 16x16x32 per K-step);
//   * an NS-slot LDS-DMA ring (7 x 20 KiB = 140 KiB): NS - 2 K-steps stay in flight past
//     every barrier (~1 us of MFMA work), one barrier per K-step, counted vmcnt waits;
//   * fragments double-buffered in registers: the 10 ds_reads of step c+1 are issued before
//     the 24 MFMAs of step c, so the LDS latency hides behind them;
//   * persistent over tiles (grid = min(tiles, CUs)) with the ring running across tile
//     boundaries, XCD-contiguous + L2-grouped tile walk, compile-time fused epilogues with
//     16-B stores (gemm_epilogue16, as gemm_pp3_kernel).
// A must be K-contiguous (activations / output gradients); B either layout (nn.Linear weight
// in the forward, the same weight MN-contiguous in dX).  K % 64 == 0.
#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "gemm_ring.h"
#include "../../include/gvl.h"

namespace {

using namespace gvl_ring;

constexpr int W4_BM = 192, W4_BN = 128;

// Register-staged operand copy of one K-step: this wave's PER 1-KiB pieces (the Step images,
// swizzle on the global source address) loaded to VGPRs, later written lane-linear to LDS.
// (LDS-DMA would need no VGPRs, but each buffer_load...lds costs ~60-185 issue cycles at one
// wave per SIMD, MICROARCH cycle constants: 5 pieces per K-step ~ the whole MFMA budget.)
template <int PER>
GVL_DEV void w4_load(__amdgpu_buffer_rsrc_t rs, const int* off, int kbytes, uint4* v) {
#pragma unroll
  for (int t = 0; t < PER; ++t)
    v[t] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off[t], kbytes, 0));
}
template <int PER, int NWV>
GVL_DEV void w4_store(char* lds, const uint4* v, int wave, int lane) {
#pragma unroll
  for (int t = 0; t < PER; ++t)
    *reinterpret_cast<uint4*>(lds + (t * NWV + wave) * 1024 + lane * 16) = v[t];
}

// 96-wide B slab of a 32-deep K-step (gemm_w4n_kernel: 128 x 96 tiles).
// 6 KiB of operand in 1-KiB pieces over 4 waves: pieces j = 4t + wave, j < 6 real; waves 2-3's
// second piece (j = 6, 7) is a dummy whose buffer offset is out of range (the load returns
// zeros without touching memory) and whose LDS write lands in a 2 KiB pad no fragment reads,
// so every wave runs the same branch-free staging code.
//  * K-contiguous (the weight in forward GEMMs): [96 rows][32] 64-B rows, the Step image;
//  * MN-contiguous (the weight in dX): cols 0-63 as [32][64] 128-B rows (Step192's tail image,
//    f2 swizzle), cols 64-95 as [32][32] 64-B rows at +4 KiB, chunk c of k-row kr at
//    c ^ f3(kr): the ds_read_b64_tr_b16 lane groups of the fragment pattern below hit 32
//    distinct 8-B bank pairs (checked exhaustively, like attn_swizzle_check.py).
constexpr uint32_t W4_OOB = 0x7FFFFFF0u;
GVL_DEV int f3(int k) { return (k >> 2) & 2; }  // 64-B rows
template <bool MN, int NWV = 4>
struct Step96 {
  static constexpr int R = 96;
  static constexpr int REAL = 6;
  static constexpr int BYTES = 8 * 1024;  // 6 KiB image + 2 KiB pad for the dummy pieces
  static constexpr int PER = 2;
  static_assert(NWV == 4, "four waves");
  GVL_DEV static int64_t elem(int64_t ld, int64_t r0, int64_t k0, int j, int lane) {
    if (!MN) {
      const int row = 16 * j + (lane >> 2);
      return (r0 + row) * ld + k0 + ((lane & 3) ^ f64b(row)) * 8;
    }
    if (j < 4) {
      const int kr = 8 * j + (lane >> 3);
      return (k0 + kr) * ld + r0 + ((lane & 7) ^ f2(kr)) * 8;
    }
    const int kr = 16 * (j - 4) + (lane >> 2);
    return (k0 + kr) * ld + r0 + 64 + ((lane & 3) ^ f3(kr)) * 8;
  }
  GVL_DEV static void base_offsets(int64_t ld, int64_t r0, int64_t k0, int wave, int lane,
                                   int (&off)[PER]) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int j = t * NWV + wave;
      off[t] = j < REAL ? (int)(elem(ld, r0, k0, j, lane) * 2) : (int)W4_OOB;
    }
  }
  GVL_DEV static int step_bytes(int64_t ld) { return MN ? (int)(KS * ld * 2) : KS * 2; }
  GVL_DEV static short8_t frag(const char* lds, int c0, int lane) {
    if (!MN) {
      const int row = c0 + (lane & 15), ch = lane >> 4;
      return *reinterpret_cast<const short8_t*>(lds + row * 64 + ((ch ^ f64b(row)) << 4));
    }
    const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int kr = 8 * G + q;
    short8_t r;
    if (c0 < 64) {
      const int ch = (c0 >> 3) + (p >> 1);
      const int off1 = kr * 128 + ((ch ^ f2(kr)) << 4) + (p & 1) * 8;
      r.lo = lds_read_tr(lds + off1);
      r.hi = lds_read_tr(lds + off1 + 4 * 128);
    } else {
      const int ch = ((c0 - 64) >> 3) + (p >> 1);
      const int off1 = kr * 64 + ((ch ^ f3(kr)) << 4) + (p & 1) * 8;
      r.lo = lds_read_tr(lds + 4096 + off1);
      r.hi = lds_read_tr(lds + 4096 + off1 + 4 * 64);
    }
    return r;
  }
};
template <int BN, bool MN>
struct W4SlabB {
  using type = Step<BN, MN, 4>;
};
template <bool MN>
struct W4SlabB<96, MN> {
  using type = Step96<MN>;
};
// A slab (K-contiguous): the Step image, or Step96's [96 rows][32] one for 96-row tiles
template <int BM>
struct W4SlabA {
  using type = Step<BM, false, 4>;
};
template <>
struct W4SlabA<96> {
  using type = Step96<false>;
};

// K-steps are 32 deep; the register staging runs P = 3 steps ahead of the LDS writes, the LDS
// ring holds NS = 3 steps (the one being read, the next, the one being written).  Step c:
//   read the fragments of step c+1 (written and published by the previous barrier);
//   write step c+2 from its register set to LDS slot (c+2)%3 (slot of step c-1, whose reads
//   retired before the previous barrier), then reload that set with step c+5;
//   MFMAs of step c; barrier (retires this step's fragment reads and LDS writes).
// The loop body is unrolled 6 times (register set = step % 3, fragment buffer = step % 2, both
// static), so K must be a multiple of 6 steps (K % 192 == 0).
// GVL_W4_IGLP (default 3, measured best of 0-3 on the caption shapes; 0 = off): ask the scheduler to spread the step's LDS reads, LDS writes and global
// loads between its 24 MFMAs (one wave per SIMD: whatever is not issued in an MFMA's shadow
// is an MFMA bubble) instead of issuing them as one block ahead of the MFMAs.
#ifndef GVL_W4_IGLP
#define GVL_W4_IGLP 3
#endif
#if GVL_W4_IGLP == 1  // reads, then writes, then global loads, one per MFMA
#define W4_INTERLEAVE()                                                           \
  do {                                                                            \
    _Pragma("unroll") for (int q_ = 0; q_ < 10; ++q_) {                           \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                          \
    }                                                                             \
    _Pragma("unroll") for (int q_ = 0; q_ < 5; ++q_) {                            \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                          \
    }                                                                             \
    _Pragma("unroll") for (int q_ = 0; q_ < 5; ++q_) {                            \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                          \
    }                                                                             \
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                            \
  } while (0)
#elif GVL_W4_IGLP == 2  // global loads first, then reads, then writes
#define W4_INTERLEAVE()                                                           \
  do {                                                                            \
    _Pragma("unroll") for (int q_ = 0; q_ < 5; ++q_) {                            \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                          \
    }                                                                             \
    _Pragma("unroll") for (int q_ = 0; q_ < 10; ++q_) {                           \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                          \
    }                                                                             \
    _Pragma("unroll") for (int q_ = 0; q_ < 5; ++q_) {                            \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                          \
    }                                                                             \
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                            \
  } while (0)
#elif GVL_W4_IGLP == 3  // PA+PB rounds of {MFMA, read, MFMA, read, MFMA, load, MFMA, write}
// (at most FM * FN / 4 rounds: the 128 x 96 tile has 12 MFMAs per step for 4 loads)
#define W4_INTERLEAVE()                                                           \
  do {                                                                            \
    _Pragma("unroll") for (int q_ = 0; q_ < (PA + PB < FM * FN / 4 ? PA + PB : FM * FN / 4); ++q_) { \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                          \
    }                                                                             \
    if constexpr (FM * FN > 4 * (PA + PB))                                        \
      __builtin_amdgcn_sched_group_barrier(0x008, FM * FN - 4 * (PA + PB), 0);    \
  } while (0)
#endif
#if GVL_W4_IGLP
#define W4_PRIO(x) do {} while (0)  // s_setprio would split the scheduling region
#else
#define W4_INTERLEAVE() do {} while (0)
#define W4_PRIO(x) __builtin_amdgcn_s_setprio(x)
#endif

// Timing-only diagnostic builds (wrong results; never the shipped library):
// GVL_W4_DIAG=1 drops the per-step barrier, 2 drops the per-step LDS writes and global loads.
#ifndef GVL_W4_DIAG
#define GVL_W4_DIAG 0
#endif
#if GVL_W4_DIAG == 1
#define W4_DIAG_BAR() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#else
#define W4_DIAG_BAR() barrier_lds()
#endif
#if GVL_W4_DIAG == 2
#define W4_DIAG_MEM(...) do {} while (0)
#else
#define W4_DIAG_MEM(...) do { __VA_ARGS__; } while (0)
#endif

// BM = 192 (6 x 4 fragments per wave) or 128 (4 x 4): the 128-row tile fills the chip when
// 192-row tiles would leave over a quarter of the CUs idle (3968 / 4096-row caption GEMMs).
template <int NS, bool BMN, int EPI, int BM, int BN = W4_BN>
__device__ __forceinline__ void gemm_w4_body(const GemmP& p) {
  constexpr int NW = 4, FM = BM / 32, FN = BN / 32, P = 3;
  static_assert(NS == 3, "ring geometry");
  static_assert(BM == 192 || BM == 128 || (BM == 96 && BN == 128), "tile rows");
  static_assert(BN == 128 || (BN == 96 && BM == 128), "tile columns");
  using SA = typename W4SlabA<BM>::type;
  using SB = typename W4SlabB<BN, BMN>::type;
  constexpr int SLOT = SA::BYTES + SB::BYTES;
  constexpr int PA = SA::PER, PB = SB::PER;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int arow = (wave >> 1) * (BM / 2), bcol = (wave & 1) * (BN / 2);

  const int total = p.tiles_m * p.tiles_n;
  const int G = gridDim.x, b = blockIdx.x;
  const int ntl = (total - b + G - 1) / G;
  const int nks = (int)(p.K / KS);
  auto tile_coords = [&](int t, int64_t& m0, int64_t& n0) {
    const int vid = b + t * G;
    const int q8 = total >> 3, r8 = total & 7, xcd = vid & 7;
    const int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (vid >> 3);
    int sp, tm, tn;
    gemm_tile_of(work, 1, p.tiles_m, p.tiles_n, p.group, sp, tm, tn);
    m0 = (int64_t)tm * BM;
    n0 = (int64_t)tn * BN;
  };

  const int64_t b_rows = BMN ? p.K : p.N;
  const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A, p.M * p.lda * 2);
  const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B, b_rows * p.ldb * 2);
  const int sa_step = SA::step_bytes(p.lda), sb_step = SB::step_bytes(p.ldb);
  int is_t = 0, is_k = 0;  // load cursor (steps are loaded strictly in order)
  int offa[PA], offb[PB];
  {
    int64_t m0, n0;
    tile_coords(0, m0, n0);
    SA::base_offsets(p.lda, m0, 0, wave, lane, offa);
    SB::base_offsets(p.ldb, n0, 0, wave, lane, offb);
  }
  uint4 st[P][PA + PB];
// Loads and LDS writes past the last step are issued anyway (they re-read the last tile's
// first steps into a slot nobody reads again): a branch around them would make hipcc's
// vmcnt bookkeeping assume the newest loads belong to the set being written and wait for
// all of them (no loads left in flight).
#define GVL_W4_LOAD(SET)                                                        \
  do {                                                                          \
    w4_load<PA>(ra, offa, is_k * sa_step, st[SET]);                             \
    w4_load<PB>(rb, offb, is_k * sb_step, st[SET] + PA);                        \
    if (++is_k == nks) {                                                        \
      is_k = 0;                                                                 \
      if (++is_t < ntl) {                                                       \
        int64_t m0_, n0_;                                                       \
        tile_coords(is_t, m0_, n0_);                                            \
        SA::base_offsets(p.lda, m0_, 0, wave, lane, offa);                      \
        SB::base_offsets(p.ldb, n0_, 0, wave, lane, offb);                      \
      }                                                                         \
    }                                                                           \
  } while (0)
#define GVL_W4_WRITE(C, SET)  /* step C lives in LDS slot C % 3 == SET */     \
  do {                                                                          \
    char* slot_ = smem + (SET) * SLOT;                                          \
    w4_store<PA, NW>(slot_, st[SET], wave, lane);                               \
    w4_store<PB, NW>(slot_ + SA::BYTES, st[SET] + PA, wave, lane);              \
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
  EpiPre<FM, FN, EPI> pre;
  pre.load_bias(p, cu_n0 + bcol, lane);

  // prologue: steps 0..2 into sets 0..2; steps 0, 1 written; sets 0, 1 reloaded with 3, 4
  GVL_W4_LOAD(0);
  GVL_W4_LOAD(1);
  GVL_W4_LOAD(2);
  GVL_W4_WRITE(0, 0);
  GVL_W4_LOAD(0);
  GVL_W4_WRITE(1, 1);
  GVL_W4_LOAD(1);
  barrier_lds();
  short8_t af[FM], bf[FN], an[FM], bn[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bf[j] = SB::frag(smem + SA::BYTES, bcol + 16 * j, lane);
#pragma unroll
  for (int i = 0; i < FM; ++i) af[i] = SA::frag(smem, arow + 16 * i, lane);

#ifndef GVL_W4_ORDER
#define GVL_W4_ORDER 0
#endif
#if GVL_W4_ORDER == 3
// Variant: the step is cut into MFMA chunks pinned in source order by sched_barrier(0), with
// the step's memory operations placed between them by hand: the LDS writes of step C+2 lead
// (chunk 0), the global reloads of that register set follow, and the fragment reads of step
// C+1 are spread over the remaining chunks, so every MFMA gap carries at most a few issues.
#define W4_SB() __builtin_amdgcn_sched_barrier(0)
#define GVL_W4_STEP(C, SET, CA, CB, NA, NB)                                                 \
  do {                                                                                      \
    const char* sl_ = smem + (((SET) + 2) % 3) * SLOT; /* step C+1's slot */                \
    static_assert(FN == 4, "chunking assumes 4 B fragments");                                \
    /* chunk 0: writes of step C+2 + MFMA row 0 */                                          \
    W4_DIAG_MEM(GVL_W4_WRITE((C) + 2, SET));                                                \
    _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[0][j] = mfma16(CB[j], CA[0], acc[0][j]); \
    W4_SB();                                                                                \
    W4_DIAG_MEM(GVL_W4_LOAD(SET));                                                          \
    _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[1][j] = mfma16(CB[j], CA[1], acc[1][j]); \
    W4_SB();                                                                                \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                           \
        NB[j] = SB::frag(sl_ + SA::BYTES, bcol + 16 * j, lane);                             \
    _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[2][j] = mfma16(CB[j], CA[2], acc[2][j]); \
    W4_SB();                                                                                \
    _Pragma("unroll") for (int j = 2; j < 4; ++j)                                           \
        NB[j] = SB::frag(sl_ + SA::BYTES, bcol + 16 * j, lane);                             \
    _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[3][j] = mfma16(CB[j], CA[3], acc[3][j]); \
    W4_SB();                                                                                \
    _Pragma("unroll") for (int i = 0; i < FM / 2; ++i) NA[i] = SA::frag(sl_, arow + 16 * i, lane); \
    _Pragma("unroll") for (int i = 4; i < FM; ++i)                                          \
        _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(CB[j], CA[i], acc[i][j]); \
    W4_SB();                                                                                \
    _Pragma("unroll") for (int i = FM / 2; i < FM; ++i) NA[i] = SA::frag(sl_, arow + 16 * i, lane); \
    W4_DIAG_BAR();                                                                          \
  } while (0)
#elif GVL_W4_ORDER == 2
// Variant: the LDS writes of step C+2 are pinned at the head of the step (sched_barrier), the
// register set is reloaded after them (no AGPR parking of the staged data), and the step's
// fragment reads and global loads are spread between its MFMAs.
constexpr int W4_NR = FM + (BMN ? 2 * FN : FN);  // DS reads per step (tr reads: 2 per B frag)
#define W4_INTERLEAVE2()                                                          \
  do {                                                                            \
    _Pragma("unroll") for (int q_ = 0; q_ < W4_NR; ++q_) {                        \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                          \
    }                                                                             \
    _Pragma("unroll") for (int q_ = 0; q_ < PA + PB; ++q_) {                      \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                          \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                          \
    }                                                                             \
    if constexpr (FM * FN > W4_NR + PA + PB)                                      \
      __builtin_amdgcn_sched_group_barrier(0x008, FM * FN - W4_NR - PA - PB, 0);  \
  } while (0)
#define GVL_W4_STEP(C, SET, CA, CB, NA, NB)                                                 \
  do {                                                                                      \
    W4_DIAG_MEM(GVL_W4_WRITE((C) + 2, SET));                                                \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    { /* step C+1 in slot (SET + 2) % 3 */                                                  \
      const char* sl_ = smem + (((SET) + 2) % 3) * SLOT;                                    \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                        \
          NB[j] = SB::frag(sl_ + SA::BYTES, bcol + 16 * j, lane);                           \
      _Pragma("unroll") for (int i = 0; i < FM; ++i) NA[i] = SA::frag(sl_, arow + 16 * i, lane); \
    }                                                                                       \
    W4_DIAG_MEM(GVL_W4_LOAD(SET));                                                          \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                          \
        _Pragma("unroll") for (int j = 0; j < FN; ++j)                                      \
            acc[i][j] = mfma16(CB[j], CA[i], acc[i][j]);                                    \
    W4_INTERLEAVE2();                                                                       \
    W4_DIAG_BAR();                                                                          \
  } while (0)
#elif GVL_W4_ORDER == 1
// Variant: the LDS writes of step C+2 lead the step (right after the barrier that retired
// slot (C+2)%3's reads), so their VGPR->LDS transfer overlaps the MFMAs instead of queueing
// behind them before the barrier; the register set is reloaded after the fragment reads.
#define GVL_W4_STEP(C, SET, CA, CB, NA, NB)                                                 \
  do {                                                                                      \
    W4_DIAG_MEM(GVL_W4_WRITE((C) + 2, SET));                                                \
    { /* step C+1 in slot (SET + 2) % 3 */                                                  \
      const char* sl_ = smem + (((SET) + 2) % 3) * SLOT;                                    \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                        \
          NB[j] = SB::frag(sl_ + SA::BYTES, bcol + 16 * j, lane);                           \
      _Pragma("unroll") for (int i = 0; i < FM; ++i) NA[i] = SA::frag(sl_, arow + 16 * i, lane); \
    }                                                                                       \
    W4_DIAG_MEM(GVL_W4_LOAD(SET));                                                          \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                          \
        _Pragma("unroll") for (int j = 0; j < FN; ++j)                                      \
            acc[i][j] = mfma16(CB[j], CA[i], acc[i][j]);                                    \
    W4_INTERLEAVE();                                                                        \
    W4_DIAG_BAR();                                                                          \
  } while (0)
#else
#define GVL_W4_STEP(C, SET, CA, CB, NA, NB)                                                 \
  do {                                                                                      \
    { /* step C+1 in slot (SET + 2) % 3 */                                                  \
      const char* sl_ = smem + (((SET) + 2) % 3) * SLOT;                                    \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                        \
          NB[j] = SB::frag(sl_ + SA::BYTES, bcol + 16 * j, lane);                           \
      _Pragma("unroll") for (int i = 0; i < FM; ++i) NA[i] = SA::frag(sl_, arow + 16 * i, lane); \
    }                                                                                       \
    W4_DIAG_MEM(GVL_W4_WRITE((C) + 2, SET); GVL_W4_LOAD(SET));                              \
    W4_PRIO(1);                                                                             \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                          \
        _Pragma("unroll") for (int j = 0; j < FN; ++j)                                      \
            acc[i][j] = mfma16(CB[j], CA[i], acc[i][j]);                                    \
    W4_PRIO(0);                                                                             \
    W4_INTERLEAVE();                                                                        \
    W4_DIAG_BAR();                                                                          \
  } while (0)
#endif

  int c = 0;
  for (int t = 0; t < ntl; ++t) {
    for (int k = 0; k < nks; k += 6, c += 6) {
      GVL_W4_STEP(c, 2, af, bf, an, bn);
      GVL_W4_STEP(c + 1, 0, an, bn, af, bf);
      GVL_W4_STEP(c + 2, 1, af, bf, an, bn);
      GVL_W4_STEP(c + 3, 2, an, bn, af, bf);
      GVL_W4_STEP(c + 4, 0, af, bf, an, bn);
      GVL_W4_STEP(c + 5, 1, an, bn, af, bf);
    }
    gemm_epilogue16<FM, FN, EPI>(p, acc, cu_m0 + arow, cu_n0 + bcol, lane, alpha, pre);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
    if (t + 1 < ntl) {
      tile_coords(t + 1, cu_m0, cu_n0);
      pre.load_bias(p, cu_n0 + bcol, lane);
    }
  }
#undef GVL_W4_STEP
#undef GVL_W4_WRITE
#undef GVL_W4_LOAD
}

// Two kernel names (rocprofv3 / the bench timer tell them apart): 192-row and 128-row tiles.
template <int NS, bool BMN, int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(GemmP p) {
  gemm_w4_body<NS, BMN, EPI, 192>(p);
}
template <int NS, bool BMN, int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4m_kernel(GemmP p) {
  gemm_w4_body<NS, BMN, EPI, 128>(p);
}
template <int NS, bool BMN, int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4n_kernel(GemmP p) {
  gemm_w4_body<NS, BMN, EPI, 128, 96>(p);
}
template <int NS, bool BMN, int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4r_kernel(GemmP p) {
  gemm_w4_body<NS, BMN, EPI, 96, 128>(p);
}

#ifndef GVL_W4_NS
#define GVL_W4_NS 3
#endif

// Tile walk: XCD-contiguous work items, then groups of `group` tile rows walked row-fastest.
// GVL_W4_GROUP=1 walks all column tiles of a row block before the next one, so an XCD reads
// each A row block once (and every column block of B); default: the GEMM-wide group.
int w4_group(int dflt) {
  static const int g = [] {
    const char* e = getenv("GVL_W4_GROUP");
    return e ? atoi(e) : 0;
  }();
  return g > 0 ? g : dflt;
}

// the kernel of a tile shape (if constexpr: only the chosen one is instantiated)
template <int BM, int BN, bool BMN, int EPI>
constexpr auto w4_kernel_of() {
  if constexpr (BN == 96) return gemm_w4n_kernel<GVL_W4_NS, BMN, EPI>;
  else if constexpr (BM == 96) return gemm_w4r_kernel<GVL_W4_NS, BMN, EPI>;
  else if constexpr (BM == 192) return gemm_w4_kernel<GVL_W4_NS, BMN, EPI>;
  else return gemm_w4m_kernel<GVL_W4_NS, BMN, EPI>;
}

template <bool BMN, int EPI, int BM, int BN = W4_BN>
int launch_w4_bm(const GemmP& p0, hipStream_t s) {
  constexpr int NS = GVL_W4_NS;
  GemmP p = p0;
  p.tiles_m = (int)((p.M + BM - 1) / BM);
  p.tiles_n = (int)((p.N + BN - 1) / BN);
  p.splits = 1;
  p.kper = p.K;
  p.group = w4_group(p.group);
  constexpr int slot = W4SlabA<BM>::type::BYTES + W4SlabB<BN, BMN>::type::BYTES;
  constexpr int lds = NS * slot;
  auto kern = w4_kernel_of<BM, BN, BMN, EPI>();
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  const int total = p.tiles_m * p.tiles_n;
  const int grid = total < gvl::num_cus() ? total : gvl::num_cus();
  gvl::launch_timed(kern, dim3(grid), dim3(256), lds, s, p);
  return 0;
}

// 128-row tiles where 192-row ones fill under 3/4 of the CUs and 128-row ones fill more
// (GVL_W4_BM128=0: always 192, A/B)
bool w4_use128(const GemmP& p) {
  static const bool on = [] {
    const char* e = getenv("GVL_W4_BM128");
    return !(e && e[0] == '0');
  }();
  const int64_t cus = gvl::num_cus(), tn = (p.N + W4_BN - 1) / W4_BN;
  const int64_t t192 = (p.M + 191) / 192 * tn, t128 = (p.M + 127) / 128 * tn;
  return on && t192 * 4 < cus * 3 && t128 > t192 && t128 <= cus;
}

// 128 x 96 tiles (gemm_w4n_kernel) where 128-row tiles are used and 96-column ones fill more
// of the chip in one round: the cross-att decoder's 3968 text rows (186 -> 248 tiles at
// N = 768) and the Q-Former bridge's 4096 query rows (192 -> 256).  A CU streams 224 operand
// rows per K-step instead of 256 for its (smaller) tile, so a one-round launch of these shapes,
// paced by the per-CU operand stream, ends ~1/8 sooner.  Measured
// (profiles/r6/w4n_bn96_r6c.txt, 3968 / 4096 rows): the forward products (K-contiguous weight)
// gain 8-10 % (attn.c_proj + bias + residual 16.3 -> 14.5 us, mlp.c_proj 39.1 -> 35.3), the dX
// ones (MN-contiguous weight, whose 32-column image is fetched as 64-B row segments) lose 6-8 %
// (c_fc.dX 35.8 -> 38.5), so only K-contiguous B takes them (GVL_W4_BN96=2: both, A/B).
// GVL_W4_BN96=0: 128 x 128 as before (A/B).
bool w4_use96(const GemmP& p, bool b_mn) {
  static const int mode = [] {
    const char* e = getenv("GVL_W4_BN96");
    return e ? atoi(e) : 1;
  }();
  if (mode == 0 || (b_mn && mode < 2) || !w4_use128(p)) return false;
  const int64_t cus = gvl::num_cus(), tm = (p.M + 127) / 128;
  const int64_t t128 = tm * ((p.N + 127) / 128), t96 = tm * ((p.N + 95) / 96);
  return t96 > t128 && t96 <= cus;
}

// 96 x 128 tiles (gemm_w4r_kernel) for the dX products (MN-contiguous weight, plain epilogue)
// where 128-row tiles are used and 96-row ones fill more of the chip in one round: the cross-att
// decoder's 3968 text rows, 186 -> 252 tiles at N = 768.  The 128-column B image keeps its full
// 256-B rows (the 96-column one of gemm_w4n_kernel lost on dX: 64-B row segments); the A slab is
// Step96's [96][32] image (two dummy pieces).  GVL_W4_BM96=0: off (A/B).
bool w4_use96r(const GemmP& p, bool b_mn) {
  static const bool on = [] {
    const char* e = getenv("GVL_W4_BM96");
    return !(e && e[0] == '0');
  }();
  if (!on || !b_mn || !w4_use128(p)) return false;
  const int64_t cus = gvl::num_cus(), tn = (p.N + 127) / 128;
  const int64_t t128 = (p.M + 127) / 128 * tn, t96 = (p.M + 95) / 96 * tn;
  return t96 > t128 && t96 <= cus;
}

template <bool BMN, int EPI>
int launch_w4(const GemmP& p, hipStream_t s) {
  if constexpr (BMN && EPI == EPI_PLAIN) {
    if (w4_use96r(p, BMN)) return launch_w4_bm<BMN, EPI, 96, 128>(p, s);
  }
  if (w4_use96(p, BMN)) return launch_w4_bm<BMN, EPI, 128, 96>(p, s);
  return w4_use128(p) ? launch_w4_bm<BMN, EPI, 128>(p, s) : launch_w4_bm<BMN, EPI, 192>(p, s);
}

template <bool BMN>
int launch_w4_epi(const GemmP& p, hipStream_t s) {
  switch (gvl::gemm_w4_epi_kind(p)) {
    case EPI_PLAIN: return launch_w4<BMN, EPI_PLAIN>(p, s);
    case EPI_BIAS: return launch_w4<BMN, EPI_BIAS>(p, s);
    case EPI_BIAS_RES: return launch_w4<BMN, EPI_BIAS_RES>(p, s);
    case EPI_BIAS_ACT: return launch_w4<BMN, EPI_BIAS_ACT>(p, s);
    case EPI_DACT: return launch_w4<BMN, EPI_DACT>(p, s);
    case EPI_RES: return launch_w4<BMN, EPI_RES>(p, s);
    case EPI_BIAS_ACT_ERF: return launch_w4<BMN, EPI_BIAS_ACT_ERF>(p, s);
    case EPI_DACT_ERF: return launch_w4<BMN, EPI_DACT_ERF>(p, s);
    case EPI_BIAS_ACT_D: return launch_w4<BMN, EPI_BIAS_ACT_D>(p, s);
    case EPI_BIAS_ACT_ERF_D: return launch_w4<BMN, EPI_BIAS_ACT_ERF_D>(p, s);
    case EPI_MUL: return launch_w4<BMN, EPI_MUL>(p, s);
    case EPI_BIAS_DROP_RES: return launch_w4<BMN, EPI_BIAS_DROP_RES>(p, s);
    case EPI_GATE_RES: return launch_w4<BMN, EPI_GATE_RES>(p, s);
    default: return -1;
  }
}

// Routing: GVL_W4=0 disables, =2 forces it for every shape it supports (tests / A/B).
int w4_mode() {
  static const int v = [] {
    const char* e = getenv("GVL_W4");
    return e ? atoi(e) : 1;
  }();
  return v;
}

}  // namespace

namespace gvl {

// The four-wave kernels' epilogue kind: gemm_epi_kind, plus the gated residual (EPI_GATE_RES:
// bias, residual, gate and the un-gated branch stored to pre_out; no dropout / activation) that
// every other family runs on the generic epilogue.  Before round 5 the cross-att decoder's 12
// gated xattn.c_proj GEMMs per step (3968 x 768 x 768) fell to the 128 x 128 ring kernel's
// runtime-flag epilogue for that reason: 32 us each, 0.058 of peak.
int gemm_w4_epi_kind(const GemmP& p) {
  static const bool gate_on = [] {  // GVL_W4_GATE=0: the generic path as before (A/B)
    const char* e = getenv("GVL_W4_GATE");
    return !(e && e[0] == '0');
  }();
  if (gate_on && p.gate && p.bias && p.residual && p.pre_out && !p.has_drop && !p.c_f32 && !p.act &&
      !p.dact)
    return EPI_GATE_RES;
  return gemm_epi_kind(p);
}

// Shapes it takes by default: narrow outputs (N <= 1024) whose 256x256 tiling leaves most CUs
// idle and whose 192x128 tiling fills at least half the chip.
bool gemm_w4_plan(const GemmP& p, int a_mn, bool force) {
  if (a_mn || p.c_f32 || p.K % (6 * KS) != 0 || p.N % 8 != 0 || p.ldc % 8 != 0) return false;
  if (p.pre_out && (p.ldp % 8 != 0 || (reinterpret_cast<uintptr_t>(p.pre_out) & 15))) return false;
  if (gemm_w4_epi_kind(p) == EPI_GEN || gemm_w4_epi_kind(p) == EPI_BIAS_QGELU) return false;
  if (force || w4_mode() == 2) return true;
  if (w4_mode() == 0) return false;
  // GVL_W4=3 (A/B): also the short-K wide outputs (K <= 1024, N <= 4096: c_attn / c_fc
  // forward, mlp.c_proj dX), whose 192x256 ping-pong tiles run only 24 K-steps each —
  // measured slower (profiles/r2/r2i/w4s_shapes.txt: 575 vs 790 TF/s at M = 16384).
  if (w4_mode() == 3 && p.K <= 1024 && p.N <= 4096) return true;
  const int64_t cus = num_cus();
  const int64_t t256 = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  const int64_t tw4 = ((p.M + W4_BM - 1) / W4_BM) * ((p.N + W4_BN - 1) / W4_BN);
  if (p.N > 1024 || t256 >= 160 || tw4 > cus) return false;
  if (w4_mode() == 4) return tw4 * 2 >= cus;  // GVL_W4=4: the round-2 half-chip rule (A/B)
  if (tw4 * 4 >= cus * 3) return true;
  // 40-75 % of the CUs (the cross-att decoder's 3968 text rows: 126 tiles) only with a K short
  // enough that one tile per CU beats splitting K (the caption lm_head dX, K = 50304, and the
  // cross-att batched kv_proj dX, K = 18432, do not)
  return tw4 * 5 >= cus * 2 && p.K <= 4096;
}

bool gemm_w4_rows128(const GemmP& p) { return w4_use128(p); }
bool gemm_w4_cols96(const GemmP& p, bool b_mn) { return w4_use96(p, b_mn); }
bool gemm_w4_rows96(const GemmP& p, bool b_mn) {
  return gemm_w4_epi_kind(p) == EPI_PLAIN && w4_use96r(p, b_mn);
}

int gemm_w4_launch(const GemmP& p, int b_mn, hipStream_t s) {
  if (gemm_w4d_ok(p)) {
    // direct-A tiles walk all column tiles of a row block before the next one, so an XCD reads
    // each A row block once: HBM bytes per Q-Former dX launch 104 -> 80 MB at equal time
    // (profiles/r3/w4d_group_ab_r3s2.txt); GVL_W4_GROUP overrides
    GemmP q = p;
    q.group = w4_group(1);
    return gemm_w4d_launch(q, b_mn, w4_use128(q), s);
  }
  return b_mn ? launch_w4_epi<true>(p, s) : launch_w4_epi<false>(p, s);
}

bool gemm_w4_try(const GemmP& p, int a_mn, int b_mn, hipStream_t s) {
  if (!gemm_w4_plan(p, a_mn, false)) return false;
  return gemm_w4_launch(p, b_mn, s) == 0;
}

}  // namespace gvl
