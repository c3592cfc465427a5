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

// Deferred epilogue (DEFER instances; gemm_pp3_kernel below).  A tile's epilogue used to run
// whole in the memory phase M(c) of the next tile's first K-step: ~100 fragments x GELU per
// lane while the SIMD partner wave (compute phase) finished its 24-32 MFMAs and then waited
// at the barrier, and the epilogue's operand loads and stores made the counted waits drain
// the DMA queue.  Instead the tile's accumulators become the layer's bf16 output values at
// the tile boundary ("stage": acc * alpha + bias, rounded to bf16 exactly as the reference's
// autocast nn.Linear output is) and are kept packed in 48 VGPRs; each following M phase
// finishes ONE fragment (GELU + gelu'(x) for the MLP's c_fc, nothing else for a plain bias
// output) and stores it with buffer stores whose out-of-range lanes get an offset past the
// buffer (dropped by the range check: no branch, so every M phase issues exactly ES stores and
// the counted vmcnt waits stay exact; phases with nothing pending issue ES dropped stores).
// The bias comes from an LDS copy made at kernel start (a global load would make hipcc wait
// vmcnt(0) behind the LDS-DMA).
constexpr uint32_t DEF_OOB = 0x7FFFFFF0u;  // voffset past any buffer: the access is dropped

template <int EPI, int FM, int FN>
struct DefEpi {
  using KD = EpiKind<EPI>;
  static constexpr bool ON = EPI == EPI_BIAS || EPI == EPI_BIAS_ACT_D || EPI == EPI_BIAS_ACT_ERF_D ||
                             EPI == EPI_MUL;
  static constexpr int NCH = FM * FN;         // one fragment per chunk
  static constexpr int ES = KD::ACT ? 2 : 1;  // stores per chunk: output (+ gelu'(x))
  static constexpr int EL = KD::MUL ? 2 : 0;  // the next chunk's gelu'(x) operand (MUL): 2 DMA
  static constexpr int EOPS = ES + EL;        // VMEM ops every M phase issues
  typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

  // fragment (I, J) of the pending tile (wave origin pm0, pn0); aux = its gelu'(x) (MUL)
  template <int I, int J>
  GVL_DEV static void chunk(const GemmP& p, const uint32_t (&pend)[FM][FN][2], int64_t pm0,
                            int64_t pn0, int lane, __amdgpu_buffer_rsrc_t rc,
                            __amdgpu_buffer_rsrc_t rp, u32x2_t aux) {
    const int64_t m = pm0 + 16 * I + (lane & 15), n = pn0 + 16 * J + 4 * (lane >> 4);
    const bool ok = m < p.M && n < p.N;
    const uint32_t oc = ok ? (uint32_t)((m * p.ldc + n) * 2) : DEF_OOB;
    const uint32_t w0 = pend[I][J][0], w1 = pend[I][J][1];
    if constexpr (KD::ACT) {
      const uint32_t op = ok ? (uint32_t)((m * p.ldp + n) * 2) : DEF_OOB;
      const float x[4] = {lo_bf(w0), hi_bf(w0), lo_bf(w1), hi_bf(w1)};
      float gv[4], dv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (KD::ERF) gelu_dgelu_erf(x[r], gv[r], dv[r]);
        else gelu_dgelu_tanh(x[r], gv[r], dv[r]);
      }
      __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pack2(gv[0], gv[1]), pack2(gv[2], gv[3])}, rc,
                                            oc, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pack2(dv[0], dv[1]), pack2(dv[2], dv[3])}, rp,
                                            op, 0, 0);
    } else if constexpr (KD::MUL) {  // dH = bf16(dY W^T) * gelu'(x), as autograd's GELU backward
      __builtin_amdgcn_raw_buffer_store_b64(
          u32x2_t{pack2(lo_bf(w0) * lo_bf(aux[0]), hi_bf(w0) * hi_bf(aux[0])),
                  pack2(lo_bf(w1) * lo_bf(aux[1]), hi_bf(w1) * hi_bf(aux[1]))},
          rc, oc, 0, 0);
    } else {
      __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{w0, w1}, rc, oc, 0, 0);
    }
  }
  // chunk q (runtime) -> its compile-time fragment; q >= NCH: ES dropped stores
  template <int Q = 0>
  GVL_DEV static void run(int q, const GemmP& p, const uint32_t (&pend)[FM][FN][2], int64_t pm0,
                          int64_t pn0, int lane, __amdgpu_buffer_rsrc_t rc,
                          __amdgpu_buffer_rsrc_t rp, u32x2_t aux) {
    if constexpr (Q < NCH) {
      if (q == Q) {
        chunk<Q / FN, Q % FN>(p, pend, pm0, pn0, lane, rc, rp, aux);
        return;
      }
      run<Q + 1>(q, p, pend, pm0, pn0, lane, rc, rp, aux);
    } else {
#pragma unroll
      for (int s = 0; s < ES; ++s)
        __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pend[0][0][0], pend[0][0][1]}, rc, DEF_OOB, 0, 0);
    }
  }
  // MUL: the gelu'(x) operand of chunk q of the tile at wave origin (m0, n0) (q >= NCH or
  // !valid: dropped loads) into this wave's 512-B LDS slot by two 4-B-per-lane LDS-DMA pieces
  // (no VGPR destination: nothing hipcc could copy before the data lands; counted by the
  // ring's waits like the K-step pieces); aux_read() retires and reads it.
  GVL_DEV static void aux_dma(const GemmP& p, int64_t m0, int64_t n0, int q, bool valid,
                              int lane, __amdgpu_buffer_rsrc_t ra, const char* aux_lds) {
    const int i = q / FN, j = q - (q / FN) * FN;
    const int64_t m = m0 + 16 * i + (lane & 15), n = n0 + 16 * j + 4 * (lane >> 4);
    const bool ok = valid && q < NCH && m < p.M && n < p.N;
    const int off = (int)(ok ? (uint32_t)((m * p.ldp + n) * 2) : DEF_OOB);
    dma4_lds(ra, off, 0, aux_lds);
    dma4_lds(ra, off + 4, 0, aux_lds + 256);
  }
  // wait until at most VM VMEM ops are outstanding (the slot's pieces retired), then read it
  template <int VM>
  GVL_DEV static u32x2_t aux_read(const char* aux_lds, int lane) {
    typedef __attribute__((address_space(3))) const char lds_c;
    const uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>((lds_c*)(aux_lds + 4 * lane));
    uint32_t lo, hi;
    asm volatile("s_waitcnt vmcnt(%2)\n\tds_read_b32 %0, %3\n\tds_read_b32 %1, %3 offset:256\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(lo), "=&v"(hi)
                 : "n"(VM), "v"(a));
    return u32x2_t{lo, hi};
  }
  // acc -> pending bf16 (acc * alpha [+ bias]); bias row of the tile's columns from LDS, read
  // by inline asm with its own lgkmcnt wait: as a C++ LDS load hipcc would order it behind
  // every LDS-DMA in flight (s_waitcnt vmcnt(0)), as it cannot tell the bias copy from the ring
  GVL_DEV static void stage(const float4_t (&acc)[FM][FN], uint32_t (&pend)[FM][FN][2],
                            const char* bias_lds, int64_t nw0, int lane, float alpha) {
    static_assert(FN == 3, "bias read below");
    uint2 bv[3] = {make_uint2(0, 0), make_uint2(0, 0), make_uint2(0, 0)};
    if constexpr (KD::BIAS) {
      typedef __attribute__((address_space(3))) const char lds_c;
      const uint32_t a0 = (uint32_t)reinterpret_cast<uintptr_t>(
          (lds_c*)(bias_lds + 2 * (nw0 + 4 * (lane >> 4))));
      asm volatile("ds_read_b64 %0, %3\n\tds_read_b64 %1, %3 offset:32\n\tds_read_b64 %2, %3 offset:64\n\t"
                   "s_waitcnt lgkmcnt(0)"
                   : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2])
                   : "v"(a0));  // no "memory": that would make hipcc drain vmcnt first
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const uint2 bb = bv[j];
      const float b4[4] = {lo_bf(bb.x), hi_bf(bb.x), lo_bf(bb.y), hi_bf(bb.y)};
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        pend[i][j][0] = pack2(fmaf(acc[i][j][0], alpha, b4[0]), fmaf(acc[i][j][1], alpha, b4[1]));
        pend[i][j][1] = pack2(fmaf(acc[i][j][2], alpha, b4[2]), fmaf(acc[i][j][3], alpha, b4[3]));
      }
    }
  }
};

// s_waitcnt vmcnt(n * PER + X) for a runtime n in [0, MAXN]
template <int PER, int MAXN, int X>
GVL_DEV void wait_vm_steps_x(int n) {
  if (MAXN >= 4 && n >= 4) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PER + X) : "memory"); return; }
  if (MAXN >= 3 && n == 3) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER + X) : "memory"); return; }
  if (MAXN >= 2 && n == 2) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER + X) : "memory"); return; }
  if (MAXN >= 1 && n == 1) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 * PER + X) : "memory"); return; }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X) : "memory");
}

// BN = 192 (FN = 3 fragments of 16 columns per wave): for N = 768 / 2304 outputs the 256-wide
// tiles leave CUs idle in the last round (M = 16384, N = 768: 192 tiles on 256 CUs; 192-wide:
// 256 tiles).  Its B slab is 12 DMA pieces: waves 0-3 (group 0) issue 2, waves 4-7 one, so
// the counted waits use a per-group pieces-per-step count.
// BM = 128 (FM = 4: each ping-pong group 64 rows): M = 8064, N = 768 (caption decoder) gives
// 63 x 4 = 252 tiles of 128x192, one round on 256 CUs with no K split.
template <int NS, bool AMN, bool BMN, int EPI, int BN = 256, int BM = 256, bool DEFER = false>
__global__ __launch_bounds__(512, 1) void gemm_pp3_kernel(GemmP p) {
  constexpr int NW = 8, FM = BM / 32, FN = BN / 64;
  static_assert(NS >= 3 && NS <= 6, "ring geometry");
  using DE = DefEpi<EPI, FM, FN>;
  // deferred epilogue: host routes only single-problem, unsplit launches with K / 32 >= NCH
  constexpr bool DEF = DEFER;
  static_assert(!DEF || (DE::ON && BN == 192 && BM == 256), "deferred epilogue instance");
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
  // deferred-epilogue state: pending tile (bf16 outputs), its wave origin, next chunk
  uint32_t pend[DEF ? FM : 1][DEF ? FN : 1][2];
  int64_t pm0 = 0, pn0 = 0;
  int pq = DE::NCH;
  typename DE::u32x2_t paux = {0u, 0u};  // MUL: gelu'(x) of chunk pq
  const char* bias_lds = smem + NS * SLOT;
  // MUL: per-wave 512-B slot for the next chunk's gelu'(x), after the bias row
  const char* aux_lds = smem + NS * SLOT + 2 * p.tiles_n * BN + wave * 512;
  // (DEF) output / gelu' buffers; non-DEF instances never read them
  const __amdgpu_buffer_rsrc_t rc_def = uniform_rsrc(p.C, DEF ? p.M * p.ldc * 2 : 0);
  const __amdgpu_buffer_rsrc_t rp_def = uniform_rsrc(
      EpiKind<EPI>::ACT ? p.pre_out : EpiKind<EPI>::MUL ? p.pre_in : p.C,
      DEF ? p.M * (EpiKind<EPI>::ACT || EpiKind<EPI>::MUL ? p.ldp : p.ldc) * 2 : 0);
  if constexpr (DEF) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) pend[i][j][0] = pend[i][j][1] = 0u;
    // the bias row in LDS (plain loads here, before any LDS-DMA is in flight)
    if constexpr (EpiKind<EPI>::BIAS)
      for (int n = tid * 8; n < p.N; n += 512 * 8)
        *reinterpret_cast<uint4*>(smem + NS * SLOT + 2 * n) = *reinterpret_cast<const uint4*>(p.bias + n);
  }
#pragma unroll
  for (int i = 0; i < NS - 1; ++i) GVL_PP3_ISSUE(i);
  {
    const int r = nsteps - 1, n = r < 0 ? 0 : (r < NS - 2 ? r : NS - 2);
    if (g == 0) wait_vm_steps<IPW0, NS - 2>(n);
    else wait_vm_steps<IPW1, NS - 2>(n);
  }
  // the counted waits of a DEFER instance count ES stores in each of the last two M phases:
  // one phase's worth (dropped) before the first
  if constexpr (DEF) {
    DE::run(DE::NCH, p, pend, pm0, pn0, lane, rc_def, rp_def, paux);
    if constexpr (DE::EL) DE::aux_dma(p, 0, 0, 0, false, lane, rp_def, aux_lds);
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
  if constexpr (!DEF) pre.load_bias(p, cu_n0 + bcol, lane);
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
      if constexpr (DEF) {
        DE::stage(acc, pend, bias_lds, cu_n0 + bcol, lane, alpha);
        pm0 = cu_m0 + arow;
        pn0 = cu_n0 + bcol;
        pq = 0;
      } else {
        GVL_PP3_EPILOGUE();
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
      ++cu_t;
      tile_coords(cu_t, cu_m0, cu_n0, cu_k0, cu_sp, cu_bi);
      if constexpr (!DEF) pre.load_bias(p, cu_n0 + bcol, lane);
      if constexpr (DB) do_db = p.batch > 1 && p.splits == 1 && cu_n0 == 0 && p.Db[cu_bi] != nullptr;
    }
    if constexpr (DEF && DE::EL) {
      // this chunk's operand, fetched in the previous M phase before D(c+2): only D(c+2)'s
      // pieces are younger (none past the last step; none at c = 0, whose fetch followed the
      // prologue's DMA)
      const bool d2 = c > 0 && c + 2 < nsteps;
      if (g == 0) paux = d2 ? DE::template aux_read<IPW0>(aux_lds, lane) : DE::template aux_read<0>(aux_lds, lane);
      else paux = d2 ? DE::template aux_read<IPW1>(aux_lds, lane) : DE::template aux_read<0>(aux_lds, lane);
    }
    const char* sl = smem + (c % NS) * SLOT;
#pragma unroll
    for (int j = 0; j < FN; ++j) bf[j] = SB::frag(sl + SA::BYTES, bcol + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = SA::frag(sl, arow + 16 * i, lane);
    if constexpr (DEF) {  // one fragment of the pending tile: EOPS VMEM ops, always issued
      DE::run(pq, p, pend, pm0, pn0, lane, rc_def, rp_def, paux);
      if (pq < DE::NCH) ++pq;
      if constexpr (DE::EL) {  // the next chunk's operand; the last step of a tile fetches the
        //                        first chunk of the tile it finishes (pending from the next step)
        const bool nxt = pq < DE::NCH;
        DE::aux_dma(p, nxt ? pm0 : cu_m0 + arow, nxt ? pn0 : cu_n0 + bcol, nxt ? pq : 0,
                    nxt || cu_k == nks - 1, lane, rp_def, aux_lds);
      }
    }
    GVL_PP3_ISSUE(c + NS - 1);
    {
      const int r = nsteps - (c + 2);  // steps issued but not needed by step c+1
      const int n_ = r < 0 ? 0 : (r < NS - 2 ? r : NS - 2);
      if constexpr (DEF) {
        if (g == 1) wait_vm_steps_x<IPW1, NS - 2, 2 * DE::EOPS>(n_);
      } else {
        if (g == 1) wait_vm_steps<IPW1, NS - 2>(n_);
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
      if constexpr (DEF) {
        if (g == 0) wait_vm_steps_x<IPW0, NS - 2, 2 * DE::EOPS>(n_);
      } else {
        if (g == 0) wait_vm_steps<IPW0, NS - 2>(n_);
      }
    }
    barrier_lds();
  }
#undef GVL_PP3_ISSUE
  if (g == 0) __builtin_amdgcn_s_barrier();
  if constexpr (DEF) {
    if (nsteps > 0) {
      DE::stage(acc, pend, bias_lds, cu_n0 + bcol, lane, alpha);
      typename DE::u32x2_t ax[DE::EL ? DE::NCH : 1];
      if constexpr (DE::EL) {  // every operand of the last tile at once, then the chunks
        ax[0] = DE::template aux_read<0>(aux_lds, lane);  // fetched in the last M phase
#pragma unroll
        for (int q = 1; q < DE::NCH; ++q) {
          const int64_t m = cu_m0 + arow + 16 * (q / FN) + (lane & 15);
          const int64_t n = cu_n0 + bcol + 16 * (q % FN) + 4 * (lane >> 4);
          const uint32_t off = (m < p.M && n < p.N) ? (uint32_t)((m * p.ldp + n) * 2) : DEF_OOB;
          ax[q] = __builtin_bit_cast(typename DE::u32x2_t,
                                     __builtin_amdgcn_raw_buffer_load_b64(rp_def, off, 0, 0));
        }
      }
#pragma unroll
      for (int q = 0; q < DE::NCH; ++q)
        DE::run(q, p, pend, cu_m0 + arow, cu_n0 + bcol, lane, rc_def, rp_def, ax[DE::EL ? q : 0]);
    }
  } else {
    if (nsteps > 0) GVL_PP3_EPILOGUE();
  }
#undef GVL_PP3_EPILOGUE
}

template <int NS, bool AMN, bool BMN, int EPI, int BN, int BM, bool DEFER = false>
int launch_pp3_bn(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;  // tiles_m/n, splits, kper set by gemm_pp3_try
  // DEFER: the bias row's LDS copy follows the ring
  const int lds = NS * (BM + BN) * KS * 2 + (DEFER ? 2 * p.tiles_n * BN + 8 * 512 : 0);
  auto kern = gemm_pp3_kernel<NS, AMN, BMN, EPI, BN, BM, DEFER>;
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
  // deferred-epilogue instances: forward outputs (B = the [N, K] weight) and the MLP's dX x gelu'
  if constexpr (!AMN && DefEpi<EPI, 8, 3>::ON && (BMN == (EPI == EPI_MUL))) {
    if (gvl::gemm_pp3_defer(p, AMN, BMN)) return launch_pp3_bn<GVL_PP3_NS_192, AMN, BMN, EPI, 192, 256, true>(p, s);
  }
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
