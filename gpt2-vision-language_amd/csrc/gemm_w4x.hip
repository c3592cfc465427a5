// Four-wave GEMM with the accumulators in AGPRs (gemm_w4x_kernel): 256 x 192 output tiles, one
// wave per SIMD, each wave a 128 x 96 block = 8 x 6 fragments, i.e. 48 MFMA 16x16x32 per
// 32-deep K-step against 14 fragment reads from LDS (0.29 reads per MFMA; the persistent
// kernel's 128 x 48 per-wave block of eight waves reads 0.46 per MFMA, and its LDS is busy for
// most of the MFMA time: DESIGN §3).  This is the structure of hipBLASLt's MT192x256x64 kernel
// that runs the N = 768 products 17-28 % faster than gemm_pp3_kernel
// (profiles/r4/hipblaslt_n768_r4i.txt): M = 16384, N = 768 is exactly 256 tiles, one per CU.
//
// 192 accumulators per lane do not fit next to the operands in 256 VGPRs; hipcc's own MFMA
// builtin then keeps them in AGPRs but permutes them through v_accvgpr_mov chains on every
// loop iteration (round 2's failed attempt; checked again in round 4 on a probe kernel).  The
// MFMAs are therefore inline asm whose accumulator operand is pinned to AGPRs ("+a"): no copy
// in the loop.  hipcc's hazard recognizer does not look into the asm, so the two hazards it
// would cover are handled here: an accumulator is read or rewritten only after w4x_fence (24
// wait states after the last MFMA) and the zeroed accumulators pass one before the first MFMA.
// Within a K-step the same accumulator is written once and 47 MFMAs apart between steps.
//
// Operands move global -> LDS by LDS-DMA (buffer_load ... lds) into a 5-slot ring of 32-deep
// K-steps (A 256 rows, B 192 columns: the Step / Step192 images and swizzles of the persistent
// kernel, 7 pieces per wave per step), three steps ahead of the step whose fragments are being
// read; fragments are double-buffered in VGPRs one step ahead, so a step's 48 MFMAs run while
// the next step's 14 fragment reads and 7 DMA pieces are issued between them.  One barrier per
// K-step.  Tiles are walked like the persistent kernel's (XCD-contiguous, L2-grouped); each
// tile has its own prologue (the shapes routed here run one or few tiles per CU).
#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "gemm_ring.h"
#include "../../include/gvl.h"

namespace {

using namespace gvl_ring;

// ring slots by tile: 5 x 28 KiB (256 x 192), 7 x 20 KiB (128 x 192), 5 x 32 KiB (256 x 256)
template <int BM>
constexpr int x_ns() { return BM == 256 ? 5 : 7; }

// acc += (B fragment) x (A fragment) with the accumulator pinned to AGPRs.  The "a"
// constraint means a register of the host ISA in the host pass, where it cannot hold a
// float4 and clang then drops the kernel's host stub silently, so the asm exists only in the
// device pass (the host pass compiles the launch stub, never the body).
#if defined(__HIP_DEVICE_COMPILE__)
#define W4X_MFMA(acc, bfr, afr) \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(bfr), "v"(afr))
#define W4X_PIN(acc) asm volatile("" : "+a"(acc))
#else
#define W4X_MFMA(acc, bfr, afr) (void)0
#define W4X_PIN(acc) (void)0
#endif

// Ordering point with wait states for the accumulators: every asm MFMA above it has written
// its result (24 wait states >= the XDL write -> VALU read / write requirement of a 16x16x32
// MFMA) before any instruction below it reads or rewrites an accumulator, and a zeroing write
// above it lands before an MFMA below reads it as srcC.
template <int FM, int FN>
GVL_DEV void w4x_fence(float4_t (&acc)[FM][FN]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) W4X_PIN(acc[i][j]);
}

// one 1-KiB LDS-DMA piece (a device function: target builtins in a __global__ body are host
// errors that make clang drop the kernel's host stub)
GVL_DEV void w4x_piece(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds, 16, voff, soff, 0, 0);
}

// B fragment of an MN-contiguous 192-wide slab (the Step192<true> image: columns 0-127 as
// [32][128] 256-B rows with the fT swizzle, 128-191 as [32][64] 128-B rows at +8 KiB with f2)
// by inline asm: hipcc treats the ds_read_b64_tr_b16 builtin as possibly aliasing any LDS-DMA
// in flight and drains vmcnt(0) in front of every one (measured: 2x slower dX GEMMs).  The
// half is chosen by selects (c0 is wave-uniform but not constant), not a branch.  No wait:
// w4x_wait threads the fragments through the step's lgkmcnt(0).  Early-clobber outputs: the
// second read must not take its address from a register the first one is filling
// (attention.hip frag_tr_asm, round 3's wrong dQ).
GVL_DEV short8_t w4x_frag_bmn(const char* slab, int c0, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int kr = 8 * G + q;
  const int h = c0 >> 7;  // 0: columns 0-127, 1: 128-191 (arithmetic, so hipcc cannot branch)
  const int ch = ((c0 - 128 * h) >> 3) + (pp >> 1);
  const int pitch = 256 >> h;
  const int sw = fT(kr) + (f2(kr) - fT(kr)) * h;
  const uint32_t o1 = (uint32_t)reinterpret_cast<uintptr_t>(slab) + 8192 * h + kr * pitch +
                      ((ch ^ sw) << 4) + (pp & 1) * 8;
  const uint32_t o2 = o1 + 4 * pitch;
  short4_t lo, hv;
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3"
               : "=&v"(lo), "=&v"(hv) : "v"(o1), "v"(o2) : "memory");
  short8_t r;
  r.lo = lo;
  r.hi = hv;
  return r;
}
// Fragment of an MN-contiguous Step<R, true> slab ([32][128] 256-B rows per 128-row / column
// half, fT swizzle) by inline asm: the A operand of the weight gradients (dY^T) and a 256-wide
// MN-contiguous B; as w4x_frag_bmn.
GVL_DEV short8_t w4x_frag_amn(const char* slab, int c0, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int kr = 8 * G + q;
  const int ch = ((c0 & 127) >> 3) + (pp >> 1);
  const uint32_t o1 = (uint32_t)reinterpret_cast<uintptr_t>(slab) + (c0 >> 7) * (KS * 256) + kr * 256 +
                      ((ch ^ fT(kr)) << 4) + (pp & 1) * 8;
  const uint32_t o2 = o1 + 4 * 256;
  short4_t lo, hv;
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3"
               : "=&v"(lo), "=&v"(hv) : "v"(o1), "v"(o2) : "memory");
  short8_t r;
  r.lo = lo;
  r.hi = hv;
  return r;
}

// lgkmcnt(0) with a step's fragments threaded through: hipcc sees them redefined here, so it
// adds no waits of its own for them further down the step (its count of LDS operations in
// flight also misses the asm reads)
template <int FM, int FN>
GVL_DEV void w4x_wait(short8_t (&a)[FM], short8_t (&b)[FN]);
template <>
GVL_DEV void w4x_wait<8, 8>(short8_t (&a)[8], short8_t (&b)[8]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                 "+v"(a[7]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]),
                 "+v"(b[6]), "+v"(b[7])
               :
               : "memory");
}
template <>
GVL_DEV void w4x_wait<8, 6>(short8_t (&a)[8], short8_t (&b)[6]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                 "+v"(a[7]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5])
               :
               : "memory");
}
template <>
GVL_DEV void w4x_wait<4, 6>(short8_t (&a)[4], short8_t (&b)[6]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]),
                 "+v"(b[3]), "+v"(b[4]), "+v"(b[5])
               :
               : "memory");
}

// B slab of a BN-wide tile: the persistent kernel's 192-wide image, or the standard 256 one
template <int BN, bool MN>
struct XSlabB {
  using type = Step192<MN, 4>;
};
template <bool MN>
struct XSlabB<256, MN> {
  using type = Step<256, MN, 4>;
};

// BM x BN = 256 x 192: waves 2 x 2 of 128 x 96 (8 x 6 fragments); 128 x 192 (the caption
// decoder's 8064 rows: 252 tiles at N = 768): waves of 64 x 96 (0.42 reads per MFMA); 256 x 256:
// waves of 128 x 128 (8 x 8 fragments = all 256 AGPRs, 0.25 reads per MFMA).
// GR: a grouped launch (gvl_gemm_grouped): the problems differ in M, N, K and strides
// (GemmP::Mb.. / gtile), read per tile.
// Residual folded into the accumulators (GVL_W4X_FOLD, default 1; build-time A/B): for the
// bias + residual epilogue (the LM's attn.c_proj / mlp.c_proj forward, x + yW^T + b with one
// 256 x 192 tile per CU) the residual tile is read at the tile's start, before the prologue's
// DMA and while no fragment registers are live (the K-loop has no registers to spare), and
// becomes the accumulators' initial value (acc = residual + AB), so the epilogue stores
// acc + bias with no operand read.  Round 4's form (half of the residual two K-steps ahead,
// half in the epilogue) cost ~9.5 us per GEMM over the plain product at M = 16384; this one
// takes 1.4 / 3.4 us of that back (attn.c_proj / mlp.c_proj forward: 33.1 vs 34.5, 79.7 vs
// 83.1 us; profiles/r5/w4x_fold_r5q_r5r.txt) — the residual's 25 MB read, wherever it sits in
// a one-tile-per-CU launch, is most of the rest.  Needs alpha == 1 (the planner sends no other
// bias + residual GEMM here).
#ifndef GVL_W4X_FOLD
#define GVL_W4X_FOLD 1
#endif

template <int BM, int BN, bool AMN, bool BMN, int EPI, bool GR>
GVL_DEV void gemm_w4x_body(const GemmP& p) {
  constexpr int NS = x_ns<BM>(), FM = BM / 32, FN = BN / 32;
  using SA = Step<BM, AMN, 4>;                // 16 / 8 pieces: 4 / 2 per wave
  using SB = typename XSlabB<BN, BMN>::type;  // 12 / 16 pieces: 3 / 4 per wave
  constexpr int SLOT = SA::BYTES + SB::BYTES;
  constexpr int PER = SA::PER + SB::PER;
  static_assert(SA::PER * 4 == SA::NINSTR && SB::PER * 4 == SB::NINSTR, "piece split");
  static_assert(NS * SLOT <= 160 * 1024, "LDS");
  static_assert((NS - 2) * PER <= 63, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int arow = (wave >> 1) * (BM / 2), bcol = (wave & 1) * (BN / 2);
  const int per_batch = p.tiles_m * p.tiles_n;
  const int total = GR ? p.gtile[p.batch] : per_batch * p.batch;
  const int G = gridDim.x;
  __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A, (AMN ? p.K : p.M) * p.lda * 2);
  __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B, (BMN ? p.K : p.N) * p.ldb * 2);
  // fused bias gradients of a batched weight-gradient launch (GemmP::Db, as gemm_pp3_kernel):
  // the tiles of column block 0 also sum their A fragments over K by MFMAs against a ones
  // fragment, each wave of a row half 4 of its 8 row fragments.  These accumulators are left
  // to hipcc (builtin MFMAs): a first version with asm MFMAs got garbage sums, since the copies
  // hipcc makes of them at the do_db branch joins ran without the MFMA's wait states
  constexpr bool DB = EPI == EPI_RES && AMN && BMN && BM == 256;
  float4_t bacc[4];
  short8_t ones;
#pragma unroll
  for (int k = 0; k < 8; ++k) ones[k] = (short)0x3F80;  // bf16 1.0
  const uint32_t db_hi = (wave & 1) ? 0xFFFFFFFFu : 0u;  // odd waves sum fragments 4..7
  // alpha x *alpha_ptr read once, before any DMA is in flight (grouped: the problems of
  // GemmP::alpha_mask take the device scale, the others alpha alone)
  const float alpha_dev = p.alpha_ptr ? *p.alpha_ptr : 1.f;
  const float alpha_all = GR ? p.alpha : p.alpha * alpha_dev;

  float4_t acc[FM][FN];
  short8_t fa[2][FM], fb[2][FN];
  int offa[SA::PER], offb[SB::PER];

  for (int vid = blockIdx.x; vid < total; vid += G) {
    // XCD-contiguous remap of the virtual grid, then the L2-grouped walk (gemm_tile_of)
    const int q8 = total >> 3, r8 = total & 7, xcd = vid & 7;
    const int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (vid >> 3);
    // this tile's problem (batch-major: a problem's tiles stay together) and its sizes
    int bi, local, tiles_m = p.tiles_m, tiles_n = p.tiles_n;
    int64_t M_ = p.M, N_ = p.N, K_ = p.K, lda_ = p.lda, ldb_ = p.ldb, ldc_ = p.ldc;
    if constexpr (GR) {
      bi = 0;
      while (bi + 1 < p.batch && work >= p.gtile[bi + 1]) ++bi;
      local = work - p.gtile[bi];
      M_ = p.Mb[bi], N_ = p.Nb[bi], K_ = p.Kb[bi], lda_ = p.ldab[bi], ldb_ = p.ldbb[bi], ldc_ = p.ldcb[bi];
      tiles_m = (int)((M_ + BM - 1) / BM);
      tiles_n = (int)((N_ + BN - 1) / BN);
    } else {
      bi = work / per_batch;
      local = work - bi * per_batch;
    }
    const int nks = (int)(K_ / KS);
    const int64_t a_rows = AMN ? K_ : M_, b_rows = BMN ? K_ : N_;
    const int sa_step = SA::step_bytes(lda_), sb_step = SB::step_bytes(ldb_);
    int split, tm, tn;
    gemm_tile_of(local, 1, tiles_m, tiles_n, p.group, split, tm, tn);
    const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
    // per-problem operands: a batched launch of several problems, or a grouped one of any count
    // (a grouped launch of ONE problem still carries its bias sum in Db[0])
    const bool multi = GR || p.batch > 1;
    void* const cout = multi ? p.Cb[bi] : p.C;
    const bf16_t* const res = multi ? static_cast<const bf16_t*>(p.Cb[bi]) : p.residual;
    if (multi) {
      ra = uniform_rsrc(p.Ab[bi], a_rows * lda_ * 2);
      rb = uniform_rsrc(p.Bb[bi], b_rows * ldb_ * 2);
    }
    const float alpha = GR && ((p.alpha_mask >> bi) & 1) ? alpha_all * alpha_dev : alpha_all;
    bool do_db = false;
    if constexpr (DB) do_db = multi && n0 == 0 && p.Db[bi] != nullptr;
    SA::base_offsets(lda_, m0, 0, wave, lane, offa);
    SB::base_offsets(ldb_, n0, 0, wave, lane, offb);
    // the first half of the epilogue operand (residual) is fetched two K-steps before the tile
    // ends (at the epilogue its latency is exposed: one tile per CU on the routed shapes); the
    // whole of it would spill
    EpiPre<FM, FN, EPI> pre;
    pre.load_bias(p, n0 + bcol, lane);
    const int aux_at = nks >= 2 ? nks - 2 : 0;
    // (the planner sends only alpha == 1, >= 12 K-step bias + residual GEMMs here: gemm_w4x_plan)
    constexpr bool FOLD = GVL_W4X_FOLD && EPI == EPI_BIAS_RES && !GR && !AMN;
    // the residual tile, read before the prologue's DMA (no fragment registers live yet)
    uint2 rx[FOLD ? FM : 1][FOLD ? FN : 1];
    if constexpr (FOLD) {
      // 8-B loads in the accumulator layout (the epilogue's 16-B store pattern + lane swaps
      // measured no better here: profiles/r5/w4x_fold_r5q_r5r.txt)
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int64_t m = m0 + arow + 16 * i + (lane & 15);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int64_t n = n0 + bcol + 16 * j + 4 * (lane >> 4);
          rx[i][j] = (m < p.M && n < p.N) ? *reinterpret_cast<const uint2*>(res + m * p.ldr + n)
                                          : make_uint2(0, 0);
        }
      }
    }

#define W4X_PIECE_A(t, step) \
  w4x_piece(ra, smem + ((step) % NS) * SLOT + ((t) * 4 + wave) * 1024, offa[t], (step) * sa_step)
#define W4X_PIECE_B(t, step)                                                                  \
  w4x_piece(rb, smem + ((step) % NS) * SLOT + SA::BYTES + ((t) * 4 + wave) * 1024, offb[t],    \
            (step) * sb_step)

#pragma unroll
    for (int s = 0; s < NS - 1; ++s) {
      if (s < nks) {
#pragma unroll
        for (int t = 0; t < SA::PER; ++t) W4X_PIECE_A(t, s);
#pragma unroll
        for (int t = 0; t < SB::PER; ++t) W4X_PIECE_B(t, s);
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (FOLD) {
          const uint2 v = rx[i][j];
          acc[i][j] = float4_t{lo_bf(v.x), hi_bf(v.x), lo_bf(v.y), hi_bf(v.y)};
        } else {
          acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
        }
      }
    if constexpr (DB) {
#pragma unroll
      for (int k = 0; k < 4; ++k) bacc[k] = float4_t{0.f, 0.f, 0.f, 0.f};
    }
    w4x_fence(acc);
    {
      const int r = nks - 1, n = r < NS - 2 ? r : NS - 2;  // steps issued after step 0
      wait_vm_steps<PER, NS - 2>(n);
      barrier_lds();
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
      fa[0][i] = AMN ? w4x_frag_amn(smem, arow + 16 * i, lane) : SA::frag(smem, arow + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j)
      fb[0][j] = BMN ? (BN == 192 ? w4x_frag_bmn(smem + SA::BYTES, bcol + 16 * j, lane)
                                  : w4x_frag_amn(smem + SA::BYTES, bcol + 16 * j, lane))
                     : SB::frag(smem + SA::BYTES, bcol + 16 * j, lane);

    // One K-step: its fragments (buffer CUR) landed, step c+1's slot published by the barrier,
    // then 48 MFMAs with step c+1's 14 fragment reads (buffer NXT) and step c+NS-1's 7 DMA
    // pieces issued between them.  FULL: a step with both (every step but the last NS - 1), no
    // branches; otherwise each is conditional.
#define W4X_STEP(c, CUR, NXT, FULL, DBS)                                                       \
  do {                                                                                         \
    w4x_wait(fa[CUR], fb[CUR]);                                                                \
    if (FULL) {                                                                                \
      wait_vm_steps<PER, NS - 3>(NS - 3);                                                      \
    } else {                                                                                   \
      const int r_ = nks - 2 - (c);                                                            \
      wait_vm_steps<PER, NS - 3>(r_ < 0 ? 0 : (r_ < NS - 3 ? r_ : NS - 3));                    \
    }                                                                                          \
    __builtin_amdgcn_s_barrier();                                                              \
    if (!(FULL) && !BMN && EpiKind<EPI>::AUX && !FOLD && (c) == aux_at)  /* BMN: it would spill */ \
      pre.load_aux(p, m0 + arow, n0 + bcol, lane, 0, res), pre.pre0 = true;                   \
    const bool nx_ = FULL || (c) + 1 < nks, dm_ = FULL || (c) + NS - 1 < nks;                  \
    const char* sl_ = smem + (((c) + 1) % NS) * SLOT;                                          \
    _Pragma("unroll") for (int i = 0; i < FM; ++i) {                                           \
      _Pragma("unroll") for (int j = 0; j < FN; ++j) W4X_MFMA(acc[i][j], fb[CUR][j], fa[CUR][i]); \
      if (nx_) {                                                                               \
        fa[NXT][i] = AMN ? w4x_frag_amn(sl_, arow + 16 * i, lane)                             \
                         : SA::frag(sl_, arow + 16 * i, lane);                                 \
        /* B fragments i, i + FM, ..: FN > FM for 128-row tiles */                             \
        _Pragma("unroll") for (int j_ = i; j_ < FN; j_ += FM)                                  \
          fb[NXT][j_] = BMN ? (BN == 192 ? w4x_frag_bmn(sl_ + SA::BYTES, bcol + 16 * j_, lane) \
                                         : w4x_frag_amn(sl_ + SA::BYTES, bcol + 16 * j_, lane)) \
                            : SB::frag(sl_ + SA::BYTES, bcol + 16 * j_, lane);                 \
      }                                                                                        \
      if (dm_) {                                                                               \
        _Pragma("unroll") for (int q_ = i; q_ < PER; q_ += FM) {                               \
          if (q_ < SA::PER) W4X_PIECE_A(q_, (c) + NS - 1);                                     \
          else W4X_PIECE_B(q_ - SA::PER, (c) + NS - 1);                                         \
        }                                                                                      \
      }                                                                                        \
    }                                                                                          \
    /* builtin MFMAs: hipcc may copy bacc at the branch joins, and must see the MFMA to */    \
    /* put the wait states in front of such a copy */                                          \
    /* bias sums: the wave's row half picked by bit masks (a branch on the parity made hipcc */ \
    /* copy the sums at its join after waiting for the MFMAs; a ?: on the fragments went */      \
    /* through scratch) */                                                                     \
    if (DBS && do_db) {                                                                        \
      _Pragma("unroll") for (int k = 0; k < 4; ++k) {                                          \
        const u32x4_t lo_ = __builtin_bit_cast(u32x4_t, fa[CUR][k]);                           \
        const u32x4_t hi_ = __builtin_bit_cast(u32x4_t, fa[CUR][4 + k]);                       \
        const short8_t x_ = __builtin_bit_cast(short8_t, (hi_ & db_hi) | (lo_ & ~db_hi));       \
        bacc[k] = mfma16(ones, x_, bacc[k]);                                                   \
      }                                                                                        \
    }                                                                                          \
  } while (0)

    const int nfull = nks - (NS - 1);  // steps c < nfull issue both their reads and a DMA
    int c = 0;
    for (; c + 1 < nfull; c += 2) {
      W4X_STEP(c, 0, 1, true, DB);
      W4X_STEP(c + 1, 1, 0, true, DB);
    }
    for (; c < nks; c += 2) {  // c even: fragments in buffer 0
      W4X_STEP(c, 0, 1, false, DB);
      if (c + 1 < nks) W4X_STEP(c + 1, 1, 0, false, DB);
    }
#undef W4X_STEP
#undef W4X_PIECE_A
#undef W4X_PIECE_B
    w4x_fence(acc);
    // every wave is past its last fragment read of this tile before anyone's next prologue DMA
    __builtin_amdgcn_s_barrier();
    if constexpr (GR) {  // this problem's sizes for the epilogue (only the scalars used survive)
      GemmP q = p;
      q.M = M_, q.N = N_, q.ldc = ldc_, q.ldr = ldc_;
      gemm_epilogue16<FM, FN, EPI>(q, acc, m0 + arow, n0 + bcol, lane, alpha, pre, cout, res);
    } else if constexpr (FOLD) {  // the residual is in acc: bias only
      EpiPre<FM, FN, EPI_BIAS> pb;
#pragma unroll
      for (int j = 0; j < FN; ++j) pb.b[j] = pre.b[j];
      gemm_epilogue16<FM, FN, EPI_BIAS>(p, acc, m0 + arow, n0 + bcol, lane, alpha, pb, cout, nullptr);
    } else {
      gemm_epilogue16<FM, FN, EPI>(p, acc, m0 + arow, n0 + bcol, lane, alpha, pre, cout, res);
    }
    if constexpr (DB) {
      if (do_db && (lane >> 4) == 0) {
        bf16_t* db_ = static_cast<bf16_t*>(p.Db[bi]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t m_ = m0 + arow + 16 * ((wave & 1) * 4 + k) + lane;
          if (m_ < M_) db_[m_] = f2bf(bf2f(db_[m_]) + bacc[k][0] * alpha);
        }
      }
    }
  }
}

// (a device body under a thin __global__: target builtins and "a"-constrained asm in a
// __global__ body make clang drop the kernel's host stub)
template <int BM, int BN, bool AMN, bool BMN, int EPI, bool GR = false>
__global__ __launch_bounds__(256, 1) void gemm_w4x_kernel(GemmP p) {
  gemm_w4x_body<BM, BN, AMN, BMN, EPI, GR>(p);
}

// Weight-gradient launches (AMN && BMN: the LM's batched / grouped dW over 16384 tokens, 3-7
// rounds of whole-K tiles) and their grid (the grouped launch reads 2.16x its
// operand bytes).  The three 256-column tiles that share a dY slab sit next to each other in an
// XCD's work range, but in a persistent grid (one workgroup per CU walking vid += G) each starts
// when ITS CU finished its previous tile, so after a few rounds the siblings are far apart and
// the slab is fetched again by the late one.  GVL_W4X_NP=1: one workgroup per tile instead
// (grid = tiles); the XCD's dispatcher hands the next tile of its contiguous range to the first
// CU that frees up, so siblings start within one tile-retire of each other in every round.
// GVL_W4X_DW_GROUP=n: tile rows per L2 group of the dW tile walk (default: the GEMM's).
int w4x_np_mode() {
  static const int v = [] {
    const char* e = getenv("GVL_W4X_NP");
    return e ? atoi(e) : 0;
  }();
  return v;
}
int w4x_dw_group(int dflt) {
  static const int v = [] {
    const char* e = getenv("GVL_W4X_DW_GROUP");
    return e ? atoi(e) : 0;
  }();
  return v > 0 ? v : dflt;
}

template <int BM, int BN, bool AMN, bool BMN, int EPI, bool GR = false>
void launch_w4x(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;
  constexpr bool DW = AMN && BMN;
  if constexpr (DW) p.group = w4x_dw_group(p.group);
  auto kern = gemm_w4x_kernel<BM, BN, AMN, BMN, EPI, GR>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const int total = GR ? p.gtile[p.batch] : p.tiles_m * p.tiles_n * p.batch;
  const bool np = DW ? w4x_np_mode() >= 1 : w4x_np_mode() >= 2;
  const int grid = (np || total < gvl::num_cus()) ? total : gvl::num_cus();
  constexpr int lds = x_ns<BM>() * (BM + BN) * KS * 2;
  gvl::launch_timed(kern, dim3(grid), dim3(256), lds, s, p);
}

template <int BM, bool BMN>
bool launch_w4x_epi(const GemmP& p, hipStream_t s) {
  switch (gvl::gemm_epi_kind(p)) {
    case EPI_PLAIN: launch_w4x<BM, 192, false, BMN, EPI_PLAIN>(p, s); return true;
    case EPI_BIAS_RES: launch_w4x<BM, 192, false, BMN, EPI_BIAS_RES>(p, s); return true;
    default: return false;
  }
}
}  // namespace

namespace gvl {

// GVL_W4X: 0 never, 1 the shapes below (default), 2 every shape the kernel takes (tests);
// gvl_gemm_tune(3, 12) forces it too.  LM step 885k -> 900k tokens/s, same box, alternated
// (profiles/r4/w4x_lm_ab_r4p.txt)
int w4x_mode() {
  static const int m = [] {
    const char* e = getenv("GVL_W4X");
    return e ? atoi(e) : 1;
  }();
  return m;
}

// The kernel takes K-contiguous A (activations / dY), either B layout, bf16 out, K % 32 == 0,
// plain or bias + residual epilogues, one problem, no split.  Routed: outputs whose 256 x 192
// tiling fills the chip in whole rounds (M = 16384, N = 768: 256 tiles).
bool w4x_dw_plan(GemmP& p);

bool gemm_w4x_plan(GemmP& p, int a_mn, int b_mn, bool force) {
  const int epi = gemm_epi_kind(p);
  if (a_mn) return p.batch == 1 && w4x_dw_plan(p) && p.K >= 4096;  // the lm_head's dW (b_mn)
  if ( p.c_f32 || p.K % KS != 0 || p.K < 2 * KS || p.N % 8 != 0 || p.ldc % 8 != 0 ||
      p.lda % 8 != 0 || p.ldb % 8 != 0 || (epi != EPI_PLAIN && epi != EPI_BIAS_RES))
    return false;
  // the folded residual (GVL_W4X_FOLD) needs alpha == 1
  if (GVL_W4X_FOLD && epi == EPI_BIAS_RES && (p.alpha != 1.f || p.alpha_ptr)) return false;
  (void)b_mn;
  // 256-row tiles where they (nearly) fill the chip, else 128-row tiles
  const int64_t cus = num_cus(), tn = (p.N + 192 - 1) / 192;
  p.bm = ((p.M + 255) / 256) * tn * 10 >= cus * 9 ? 256 : 128;
  p.tiles_m = (int)((p.M + p.bm - 1) / p.bm);
  p.tiles_n = (int)tn;
  p.splits = 1;
  p.kper = p.K;
  if (force || w4x_mode() == 2) return true;
  if (w4x_mode() == 0) return false;
  const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
  if (p.bm == 256) return p.N == 768 && tiles >= cus && tiles % cus == 0;
  // 128-row tiles (GVL_W4X_128: 0 never, 1 wherever they fill one round, 2 = default: only where
  // the direct-A kernel's 192 x 128 tiles overflow one round).  At the Q-Former / cross decoders'
  // 8064 rows the direct-A kernel fills one round (252 tiles) and is faster in the step (round 4
  // r4r and round 5 r5a: 15.45k vs 15.63k images/s with 128-row AGPR tiles); the linear caption
  // decoder's 8192 rows are 258 of its tiles (a second round for 2 tiles), which sent those
  // GEMMs to the 128 x 128 ring kernel (59-71 us, 30 % of the linear step in r5g) — here they
  // are exactly 256 tiles of 128 x 192
  static const int rows128 = [] {
    const char* e = getenv("GVL_W4X_128");
    return e ? atoi(e) : 2;
  }();
  const int64_t t_direct = ((p.M + 191) / 192) * ((p.N + 127) / 128);
  const bool want = rows128 == 1 || (rows128 == 2 && t_direct > cus);
  return want && p.N == 768 && tiles * 10 >= cus * 9 && tiles <= cus;
}

bool gemm_w4x_dw_try(const GemmP& p0, hipStream_t s);

bool gemm_w4x_try(const GemmP& p0, int a_mn, int b_mn, bool force, hipStream_t s) {
  GemmP p = p0;
  if (!gemm_w4x_plan(p, a_mn, b_mn, force)) return false;
  if (a_mn) return b_mn && gemm_w4x_dw_try(p0, s);
  if (p.bm == 256) return b_mn ? launch_w4x_epi<256, true>(p, s) : launch_w4x_epi<256, false>(p, s);
  return b_mn ? launch_w4x_epi<128, true>(p, s) : launch_w4x_epi<128, false>(p, s);
}

// Weight gradients (dW = dY^T X, both operands MN-contiguous, C += AB): the 12 blocks' of one
// shape in one batched launch (gvl_gemm_batched[_dbias], bias gradients fused) or the tied
// lm_head's alone (gvl_gemm), whole-K tiles of 256 x 192 or 256 x 256, whichever fills the last
// round of CUs better (192 counted at 0.95: its per-wave block reads 0.29 vs 0.25 fragments per
// MFMA), when that round is >= 65 % full: whole rounds matter more than the per-tile gain (12
// c_attn problems, 432 tiles of 256 x 192 = two rounds, the last 69 % full: 785 vs 906 us on
// the persistent kernel; 12 c_fc / mlp.c_proj ones as 576 such tiles, a third round 25 % full:
// 1109 / 1014 vs 989 / 964, profiles/r4/w4x_r4r.txt — 256 x 256 gives them 432).  The 12
// attn.c_proj problems (144 / 108 tiles) keep the persistent kernel's in-launch K split.
// GVL_W4X_DW=0 turns it off (A/B).
bool w4x_dw_plan(GemmP& p) {
  static const bool on = [] {
    const char* e = getenv("GVL_W4X_DW");
    return !(e && e[0] == '0');
  }();
  if (!on || w4x_mode() == 0) return false;
  if (gemm_epi_kind(p) != EPI_RES || p.c_f32 || p.K % KS != 0 || p.K < 2 * KS || p.M % 8 != 0 ||
      p.N % 8 != 0 || p.ldc % 8 != 0 || p.lda % 8 != 0 || p.ldb % 8 != 0)
    return false;
  const int64_t cus = num_cus(), tm = (p.M + 255) / 256;
  auto fill = [&](int64_t tiles) { return (double)tiles / (double)(((tiles + cus - 1) / cus) * cus); };
  const int64_t t192 = tm * ((p.N + 191) / 192) * p.batch, t256 = tm * ((p.N + 255) / 256) * p.batch;
  const double f192 = 0.95 * fill(t192), f256 = fill(t256);
  p.bm = 256;
  p.bn = f256 >= f192 ? 256 : 192;
  p.tiles_m = (int)tm;
  p.tiles_n = (int)((p.N + p.bn - 1) / p.bn);
  p.splits = 1;
  p.kper = p.K;
  const int64_t tiles = (p.bn == 256 ? t256 : t192);
  return tiles * 10 >= cus * 9 && (p.bn == 256 ? f256 : f192 / 0.95) >= 0.65;
}

bool gemm_w4x_dw_try(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;
  if (!w4x_dw_plan(p)) return false;
  if (p.bn == 256) launch_w4x<256, 256, true, true, EPI_RES>(p, s);
  else launch_w4x<256, 192, true, true, EPI_RES>(p, s);
  return true;
}
bool gemm_w4x_batched_try(const GemmP& p, hipStream_t s) { return gemm_w4x_dw_try(p, s); }

// Weight gradients of different shapes in one launch (gvl_gemm_grouped: the Q-Former bridge's
// deferred dW of one backward, 2-16 problems of 768 x 768 .. 3072 x 768 at K = 4096 tokens,
// bias sums fused): whole-K 256 x 256 tiles, the problems' tile lists concatenated (GemmP::gtile);
// each problem alone would be 9-36 tiles and a split-K launch + reduce + a column-sum pair.
// Tiles of 256 x 256 or 256 x 192, whichever fills the last round better.
// p: batch, Ab / Bb / Cb / Db and the per-problem sizes set by the caller.  GVL_W4X_GR=0 off.
bool gemm_w4x_grouped_try(GemmP& p, hipStream_t s) {
  static const bool on = [] {
    const char* e = getenv("GVL_W4X_GR");
    return !(e && e[0] == '0');
  }();
  if (!on || w4x_mode() == 0 || p.batch < 1 || p.batch > GVL_MAX_GROUP) return false;
  int64_t t192 = 0, t256 = 0;
  for (int i = 0; i < p.batch; ++i) {
    if (p.Kb[i] % KS != 0 || p.Kb[i] < 2 * KS || p.Mb[i] % 8 != 0 || p.Nb[i] % 8 != 0 ||
        p.ldab[i] % 8 != 0 || p.ldbb[i] % 8 != 0 || p.ldcb[i] % 8 != 0)
      return false;
    t192 += ((p.Mb[i] + 255) / 256) * ((p.Nb[i] + 191) / 192);
    t256 += ((p.Mb[i] + 255) / 256) * ((p.Nb[i] + 255) / 256);
  }
  // tile width by last-round fill as for the batched weight gradients (w4x_dw_plan)
  const int64_t cus = num_cus();
  auto fill = [&](int64_t tiles) { return (double)tiles / (double)(((tiles + cus - 1) / cus) * cus); };
  p.bn = fill(t256) >= 0.95 * fill(t192) ? 256 : 192;
  // GVL_W4X_GR_BN=192|256 forces the tile width (A/B; read per call)
  if (const char* e = getenv("GVL_W4X_GR_BN")) {
    if (atoi(e) == 192 || atoi(e) == 256) p.bn = atoi(e);
  }
  int t = 0;
  for (int i = 0; i < p.batch; ++i) {
    p.gtile[i] = t;
    t += (int)(((p.Mb[i] + 255) / 256) * ((p.Nb[i] + p.bn - 1) / p.bn));
  }
  p.gtile[p.batch] = t;
  p.grouped = 1;
  p.bm = 256;
  p.splits = 1;
  if (p.bn == 256) launch_w4x<256, 256, true, true, EPI_RES, true>(p, s);
  else launch_w4x<256, 192, true, true, EPI_RES, true>(p, s);
  return true;
}

}  // namespace gvl
