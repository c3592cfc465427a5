// Persistent AGPR four-wave GEMM (gemm_w4p_kernel) for the short-K wide outputs of the
// forward / dX products (K = 768: c_attn + bias, c_fc + bias + GELU with gelu' stored, the
// lm_head) — the shapes with many 256 x 192 tiles per CU, where gemm_w4x_kernel's per-tile
// prologue would be exposed every 24 K-steps.  The tile is gemm_w4x_kernel's (4 waves, one per
// SIMD, 128 x 96 per wave, accumulators pinned to AGPRs by asm MFMAs, the same LDS images, 5-slot
// LDS-DMA ring, fragments one step ahead in registers), but the ring runs straight across tile
// boundaries like gemm_pp3_kernel's: an issue cursor walks the CU's tiles three K-steps ahead of
// the compute cursor, so the next tile's first steps are landing while the current one ends,
// and its first fragments are read during its predecessor's last MFMAs.
//
// The epilogue is the persistent kernel's counted one (gemm_pp3.h gemm_epilogue_cnt): the bias
// row staged in LDS after the ring and read by asm, buffer stores whose out-of-range lanes are
// dropped by an offset past the buffer, so every epilogue issues exactly S stores per wave and
// the next NS - 2 counted waits allow for them (the in-order vmcnt would otherwise make the next
// tile's operand waits wait for the stores' acknowledgement).  Outputs past 1 GiB (the LM's
// logits) are stored streaming (sc1 nt), as in gemm_pp3_kernel.
#include "gemm_pp3.h"

namespace {

using namespace gvl_ring;

#if defined(__HIP_DEVICE_COMPILE__)
#define W4P_MFMA(acc, bfr, afr) \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(bfr), "v"(afr))
#define W4P_PIN(acc) asm volatile("" : "+a"(acc))
#else
#define W4P_MFMA(acc, bfr, afr) (void)0
#define W4P_PIN(acc) (void)0
#endif

constexpr int P_BM = 256, P_BN = 192, P_FM = 8, P_FN = 6, P_NS = 5;

// 24 wait states after the last asm MFMA before the accumulators are read or rewritten, and
// after the zeroing before the next MFMA reads them (gemm_w4x.hip w4x_fence)
GVL_DEV void w4p_fence(float4_t (&acc)[P_FM][P_FN]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < P_FM; ++i)
#pragma unroll
    for (int j = 0; j < P_FN; ++j) W4P_PIN(acc[i][j]);
}

GVL_DEV void w4p_piece(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds, 16, voff, soff, 0, 0);
}

// gemm_w4x.hip's MN-contiguous 192-wide B fragment by asm (no vmcnt(0) in front of it)
GVL_DEV short8_t w4p_frag_bmn(const char* slab, int c0, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int kr = 8 * G + q;
  const int h = c0 >> 7;
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

GVL_DEV void w4p_wait(short8_t (&a)[P_FM], short8_t (&b)[P_FN]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                 "+v"(a[7]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5])
               :
               : "memory");
}

template <bool BMN, int EPI>
__global__ __launch_bounds__(256, 1) void gemm_w4p_kernel(GemmP p) {
  constexpr int NS = P_NS, FM = P_FM, FN = P_FN;
  using SA = Step<P_BM, false, 4>;
  using SB = Step192<BMN, 4>;
  constexpr int SLOT = SA::BYTES + SB::BYTES;
  constexpr int PER = SA::PER + SB::PER;  // 4 + 3 pieces per wave per step
  using KD = EpiKind<EPI>;
  static_assert(CntEpi<EPI>::ON, "counted epilogue kinds only");
  constexpr int S = cnt_stores<FM, FN, EPI>();  // stores per wave per epilogue
  static_assert((NS - 3) * PER + S <= 63, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int arow = (wave >> 1) * 128, bcol = (wave & 1) * 96;
  const int total = p.tiles_m * p.tiles_n;
  const int G = gridDim.x, b = blockIdx.x;
  const int ntl = (total - b + G - 1) / G;  // this workgroup's tiles: b, b + G, ..
  const int nks = (int)(p.K / KS);
  const int nsteps = ntl * nks;
  auto tile_of = [&](int t, int64_t& m0, int64_t& n0) {
    const int vid = b + t * G;
    const int q8 = total >> 3, r8 = total & 7, xcd = vid & 7;
    const int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (vid >> 3);
    int split, tm, tn;
    gemm_tile_of(work, 1, p.tiles_m, p.tiles_n, p.group, split, tm, tn);
    m0 = (int64_t)tm * P_BM;
    n0 = (int64_t)tn * P_BN;
  };
  const int64_t b_rows = BMN ? p.K : p.N;
  const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(p.A, p.M * p.lda * 2);
  const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(p.B, b_rows * p.ldb * 2);
  const int sa_step = SA::step_bytes(p.lda), sb_step = SB::step_bytes(p.ldb);
  const __amdgpu_buffer_rsrc_t rc = uniform_rsrc(p.C, p.M * p.ldc * 2);
  const __amdgpu_buffer_rsrc_t rp = uniform_rsrc(KD::ACT ? p.pre_out : p.C, KD::ACT ? p.M * p.ldp * 2 : 0);
  const uint32_t bias_lds = (uint32_t)(NS * SLOT);
  if constexpr (KD::BIAS) {  // plain loads here, before any LDS-DMA is in flight
    for (int n = tid * 8; n < p.N; n += 256 * 8)
      *reinterpret_cast<uint4*>(smem + NS * SLOT + 2 * n) = *reinterpret_cast<const uint4*>(p.bias + n);
  }
  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;

  // issue cursor: tile is_t, step is_k, this wave's DMA offsets for that tile
  int is_t = 0, is_k = 0;
  int offa[SA::PER], offb[SB::PER];
  {
    int64_t m0, n0;
    tile_of(0, m0, n0);
    SA::base_offsets(p.lda, m0, 0, wave, lane, offa);
    SB::base_offsets(p.ldb, n0, 0, wave, lane, offb);
  }
  // piece q (0..PER-1) of the issue cursor's step into the slot of global step g; the cursor
  // moves on (and into the next tile) after its last piece
#define W4P_PIECE(q, g)                                                                          \
  do {                                                                                           \
    char* sl_ = smem + ((g) % NS) * SLOT;                                                        \
    if ((q) < SA::PER) w4p_piece(ra, sl_ + ((q) * 4 + wave) * 1024, offa[(q) < SA::PER ? (q) : 0], \
                                 is_k * sa_step);                                                \
    else w4p_piece(rb, sl_ + SA::BYTES + (((q) - SA::PER) * 4 + wave) * 1024,                    \
                   offb[(q) >= SA::PER ? (q) - SA::PER : 0], is_k * sb_step);                    \
    if ((q) == PER - 1 && ++is_k == nks) {                                                       \
      is_k = 0;                                                                                  \
      if (++is_t < ntl) {                                                                        \
        int64_t m0_, n0_;                                                                        \
        tile_of(is_t, m0_, n0_);                                                                 \
        SA::base_offsets(p.lda, m0_, 0, wave, lane, offa);                                       \
        SB::base_offsets(p.ldb, n0_, 0, wave, lane, offb);                                       \
      }                                                                                          \
    }                                                                                            \
  } while (0)

#pragma unroll
  for (int g = 0; g < NS - 1; ++g)
    if (g < nsteps) {
#pragma unroll
      for (int q = 0; q < PER; ++q) W4P_PIECE(q, g);
    }

  float4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
  w4p_fence(acc);
  {
    const int r = nsteps - 1, n = r < 0 ? 0 : (r < NS - 2 ? r : NS - 2);
    wait_vm_steps<PER, NS - 2>(n);
    barrier_lds();
  }
  short8_t fa[2][FM], fb[2][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i) fa[0][i] = SA::frag(smem, arow + 16 * i, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j)
    fb[0][j] = BMN ? w4p_frag_bmn(smem + SA::BYTES, bcol + 16 * j, lane) : SB::frag(smem + SA::BYTES, bcol + 16 * j, lane);

  int cnt_w = 0;  // waits left that must allow for the last epilogue's S stores

  // Global step c: fragments (buffer CUR) landed, step c+1 published by the barrier; 48 MFMAs
  // with step c+1's fragment reads and step c+NS-1's DMA pieces between them.
#define W4P_STEP(c, CUR, NXT)                                                                    \
  do {                                                                                           \
    w4p_wait(fa[CUR], fb[CUR]);                                                                  \
    {                                                                                            \
      const int r_ = nsteps - 2 - (c);                                                           \
      const int n_ = r_ < 0 ? 0 : (r_ < NS - 3 ? r_ : NS - 3);                                   \
      if (cnt_w > 0) {                                                                           \
        wait_vm_steps_x<PER, NS - 3, S>(n_);                                                     \
        --cnt_w;                                                                                 \
      } else {                                                                                   \
        wait_vm_steps<PER, NS - 3>(n_);                                                          \
      }                                                                                          \
    }                                                                                            \
    __builtin_amdgcn_s_barrier();                                                                \
    const bool nx_ = (c) + 1 < nsteps, dm_ = (c) + NS - 1 < nsteps;                              \
    const char* sl_ = smem + (((c) + 1) % NS) * SLOT;                                            \
    _Pragma("unroll") for (int i = 0; i < FM; ++i) {                                             \
      _Pragma("unroll") for (int j = 0; j < FN; ++j) W4P_MFMA(acc[i][j], fb[CUR][j], fa[CUR][i]); \
      if (nx_) {                                                                                 \
        fa[NXT][i] = SA::frag(sl_, arow + 16 * i, lane);                                         \
        if (i < FN)                                                                              \
          fb[NXT][i] = BMN ? w4p_frag_bmn(sl_ + SA::BYTES, bcol + 16 * i, lane)                 \
                           : SB::frag(sl_ + SA::BYTES, bcol + 16 * i, lane);                     \
      }                                                                                          \
      if (dm_ && i < PER) W4P_PIECE(i, (c) + NS - 1);                                            \
    }                                                                                            \
  } while (0)

  // K % 64 == 0 (planner): every tile starts at an even global step, fragments in buffer 0
  for (int cu_t = 0, c = 0; cu_t < ntl; ++cu_t) {
    int64_t cm0, cn0;
    tile_of(cu_t, cm0, cn0);
    for (int k = 0; k < nks; k += 2, c += 2) {
      W4P_STEP(c, 0, 1);
      W4P_STEP(c + 1, 1, 0);
    }
    w4p_fence(acc);
    if (p.st_nt)
      gemm_epilogue_cnt<FM, FN, EPI, CNT_NT>(p, acc, cm0 + arow, cn0 + bcol, lane, alpha, bias_lds, rc, rp);
    else
      gemm_epilogue_cnt<FM, FN, EPI, 0>(p, acc, cm0 + arow, cn0 + bcol, lane, alpha, bias_lds, rc, rp);
    cnt_w = NS - 2;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
    w4p_fence(acc);
  }
#undef W4P_STEP
#undef W4P_PIECE
}

template <bool BMN, int EPI>
void launch_w4p(const GemmP& p, hipStream_t s) {
  auto kern = gemm_w4p_kernel<BMN, EPI>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const int total = p.tiles_m * p.tiles_n;
  const int grid = total < gvl::num_cus() ? total : gvl::num_cus();
  const int lds = P_NS * (P_BM + P_BN) * KS * 2 + (EpiKind<EPI>::BIAS ? (int)(2 * p.N) : 0);
  gvl::launch_timed(kern, dim3(grid), dim3(256), lds, s, p);
}

template <bool BMN>
bool launch_w4p_epi(const GemmP& p, hipStream_t s) {
  switch (gvl::gemm_epi_kind(p)) {
    case EPI_PLAIN: launch_w4p<BMN, EPI_PLAIN>(p, s); return true;
    case EPI_BIAS: launch_w4p<BMN, EPI_BIAS>(p, s); return true;
    case EPI_BIAS_ACT_D: launch_w4p<BMN, EPI_BIAS_ACT_D>(p, s); return true;
    case EPI_BIAS_ACT_ERF_D: launch_w4p<BMN, EPI_BIAS_ACT_ERF_D>(p, s); return true;
    default: return false;
  }
}

}  // namespace

namespace gvl {

// GVL_W4P: 0 never (default until measured), 1 the shapes below, 2 every shape it takes (tests);
// gvl_gemm_tune(3, 13) forces it too.
static int w4p_mode() {
  static const int m = [] {
    const char* e = getenv("GVL_W4P");
    return e ? atoi(e) : 0;
  }();
  return m;
}

// K-contiguous A, either B layout, bf16 out, K % 64 == 0 (every tile starts at an even global
// step: fragment buffer 0), the counted epilogue kinds (plain,
// bias, bias + GELU with gelu' stored), 32-bit store offsets, a 16-B aligned bias whose LDS copy
// fits after the ring.  Routed: at least two 256 x 192 tiles per CU.
bool gemm_w4p_plan(GemmP& p, int a_mn, bool force) {
  const int epi = gemm_epi_kind(p);
  if (a_mn || p.c_f32 || p.K % (2 * KS) != 0 || p.N % 8 != 0 || p.ldc % 8 != 0 || p.lda % 8 != 0 ||
      p.ldb % 8 != 0 || p.batch != 1)
    return false;
  if (epi != EPI_PLAIN && epi != EPI_BIAS && epi != EPI_BIAS_ACT_D && epi != EPI_BIAS_ACT_ERF_D) return false;
  if (p.M * p.ldc * 2 > (int64_t)CNT_OOB) return false;
  if (EpiKind<EPI_BIAS>::BIAS && p.bias &&
      ((reinterpret_cast<uintptr_t>(p.bias) & 15) || P_NS * (P_BM + P_BN) * KS * 2 + 2 * p.N > 160 * 1024))
    return false;
  if ((epi == EPI_BIAS_ACT_D || epi == EPI_BIAS_ACT_ERF_D) &&
      (!p.pre_out || p.ldp % 8 || (reinterpret_cast<uintptr_t>(p.pre_out) & 15) ||
       p.M * p.ldp * 2 > (int64_t)CNT_OOB))
    return false;
  p.bm = 256;
  p.bn = 192;
  p.tiles_m = (int)((p.M + 255) / 256);
  p.tiles_n = (int)((p.N + 191) / 192);
  p.splits = 1;
  p.kper = p.K;
  p.st_nt = p.M * p.ldc * 2 > (int64_t)1 << 30;
  if (force || w4p_mode() == 2) return true;
  if (w4p_mode() == 0) return false;
  return (int64_t)p.tiles_m * p.tiles_n >= 2 * num_cus();
}

bool gemm_w4p_try(const GemmP& p0, int a_mn, int b_mn, bool force, hipStream_t s) {
  GemmP p = p0;
  if (!gemm_w4p_plan(p, a_mn, force)) return false;
  return b_mn ? launch_w4p_epi<true>(p, s) : launch_w4p_epi<false>(p, s);
}

}  // namespace gvl
