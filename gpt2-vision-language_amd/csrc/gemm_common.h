// Shared GEMM parameter block and fused epilogue (gemm.hip, gemm_lds.hip).
#pragma once
#include "common.h"
#include "../../include/gvl.h"

#define GVL_MAX_BATCH 16
// problems of one grouped launch: every LM weight gradient of a backward flush (12 blocks x 4)
#define GVL_MAX_GROUP 48

struct GemmP {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  int64_t M, N, K, lda, ldb, ldc;
  float alpha;
  const float* alpha_ptr;
  const bf16_t* bias;
  bf16_t* pre_out;
  const bf16_t* pre_in;
  int64_t ldp;
  const bf16_t* residual;
  int64_t ldr;
  const bf16_t* gate;
  uint64_t seed;
  const uint64_t* seed_ptr;
  float drop_scale;
  uint32_t drop_thresh;
  int tiles_m, tiles_n;
  int bn;     // output tile width of the persistent kernel (256 or 192; gemm_pp3_plan)
  int bm;     // output tile height of the persistent kernel (256, or 128 with bn 192)
  int group;  // tile rows per L2 group (gemm_work_tile)
  int act, dact, c_f32, has_drop;
  int cnt;  // gemm_pp3_kernel: counted epilogue (set by its launcher, gemm_pp3.h CntEpi)
  int st_nt;  // gemm_pp3_kernel counted epilogue: streaming (sc1 nt) stores for outputs past the MALL
  // split-K: `splits` workgroups per output tile, each over K range [s*kper, (s+1)*kper),
  // writing fp32 partials to ws[s][M][N]; gemm_splitk_reduce applies the epilogue.
  int splits;
  int64_t kper;
  float* ws;
  int64_t ws_bytes;
  // in-launch two-way split-K combine (gemm_pp3_kernel): per-(tile, wave) arrival tickets,
  // zero between calls; null -> partials go to gemm_splitk_reduce
  uint32_t* tickets;
  int64_t nticket;
  // batched launch (gvl_gemm_batched, gemm_pp3_kernel): `batch` problems of one shape, work
  // items batch-major, per-problem operands below (batch == 1: A, B, C, residual above)
  int batch;
  const bf16_t* Ab[GVL_MAX_GROUP];
  const bf16_t* Bb[GVL_MAX_GROUP];
  void* Cb[GVL_MAX_GROUP];
  // optional per-problem bf16 [M] bias gradients, Db[i] += row sums of op(A_i) over K (the
  // nn.Linear bias grad next to its weight grad dW = dY^T X: A = dY^T), computed by the
  // weight-gradient tiles of the first column block with MFMAs against a ones fragment
  void* Db[GVL_MAX_GROUP];
  // grouped launch (gvl_gemm_grouped, gemm_w4x_kernel GR): problems of different sizes, the
  // per-problem sizes / strides here (32-bit: the kernel argument block stays ~3.2 KB with 48
  // problems), gtile[i] = problem i's first work item (gtile[batch] = all)
  int grouped;
  uint64_t alpha_mask;  // grouped: problems (bit i) whose alpha is alpha * *alpha_ptr (others: alpha)
  int32_t Mb[GVL_MAX_GROUP], Nb[GVL_MAX_GROUP], Kb[GVL_MAX_GROUP];
  int32_t ldab[GVL_MAX_GROUP], ldbb[GVL_MAX_GROUP], ldcb[GVL_MAX_GROUP];
  int gtile[GVL_MAX_GROUP + 1];
};
// 3160 B with 48 problems.  A kernel reads its arguments by scalar loads of the fields it uses,
// so the per-problem tables cost the launches that never touch them only the host-side copy of
// the block (graph replays re-use the captured copy); the bound keeps it clear of the 4 KiB limit.
static_assert(sizeof(GemmP) <= 3584, "GemmP must stay well inside the 4 KiB kernel-argument limit");

// Work item -> (split, tile row, tile col).  Workgroups are first remapped so that each
// XCD (blockIdx % 8) owns a contiguous range of work items, then that range is walked in
// groups of `group` tile rows, column by column: the ~32-64 tiles an XCD runs at once form a
// group x (32-64 / group) block and share A and B panels in that XCD's L2 (a row-major walk
// shares only the A panel and streams every B panel from HBM/MALL).
GVL_DEV int gemm_xcd_work() {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}
GVL_DEV void gemm_tile_of(int work, int splits, int tiles_m, int tiles_n, int group, int& split,
                          int& tm, int& tn) {
  split = work % splits;
  const int tile = work / splits;
  const int per_group = group * tiles_n;
  const int grp = tile / per_group, first_m = grp * group;
  const int gsz = tiles_m - first_m < group ? tiles_m - first_m : group;
  const int in = tile - grp * per_group;
  tm = first_m + in % gsz;
  tn = in / gsz;
}
GVL_DEV void gemm_work_tile(int splits, int tiles_m, int tiles_n, int group, int& split, int& tm,
                            int& tn) {
  gemm_tile_of(gemm_xcd_work(), splits, tiles_m, tiles_n, group, split, tm, tn);
}

// Epilogue for accumulators produced with swapped operands: acc[i][j] holds, for this lane,
// row m = mw0 + 16 i + (lane & 15) and columns n = nw0 + 16 j + 4 (lane >> 4) + r, r = 0..3.
// Order: *alpha(*alpha_ptr), +bias, *dgelu(pre_in), {pre_out; gelu}, dropout,
// {pre_out if gate && !act; *tanh(gate)}, +residual, store bf16|fp32.
// One 4-column group of one row.  The tile loops around it must unroll completely or the
// accumulator array is demoted to scratch: the Makefile raises -pragma-unroll-threshold.
static __device__ __forceinline__ void gemm_epi_quad(const GemmP& p, float4_t a, int64_t m,
                                                        int64_t n, float alpha, float gatev);

template <int FM, int FN>
GVL_DEV void gemm_epilogue(const GemmP& p, const float4_t (&acc)[FM][FN], int64_t mw0,
                           int64_t nw0, int lane) {
  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;
  const float gatev = p.gate ? tanhf(bf2f(*p.gate)) : 1.f;
  const bool plain = !p.bias && !p.dact && !p.act && !p.has_drop && !p.gate && !p.residual &&
                     !p.c_f32;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int64_t m = mw0 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t n = nw0 + j * 16 + 4 * (lane >> 4);
      if (m < p.M && n < p.N) {
        if (plain) {
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.C) + m * p.ldc + n) =
              make_uint2(pack2(acc[i][j][0] * alpha, acc[i][j][1] * alpha),
                         pack2(acc[i][j][2] * alpha, acc[i][j][3] * alpha));
        } else {
          gemm_epi_quad(p, acc[i][j], m, n, alpha, gatev);
        }
      }
    }
  }
}

// Fused epilogue math for one 4-column group (row m, cols n..n+3) -> the 4 output values
// in fp32 (side outputs — pre-activation / un-gated branch — are stored here).
static __device__ __forceinline__ void gemm_epi_vals(const GemmP& p, float4_t a, int64_t m,
                                                        int64_t n, float alpha, float gatev,
                                                        float (&v)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = a[r] * alpha;
  if (p.bias) {
    const uint2 bb = *reinterpret_cast<const uint2*>(p.bias + n);
    v[0] += lo_bf(bb.x); v[1] += hi_bf(bb.x); v[2] += lo_bf(bb.y); v[3] += hi_bf(bb.y);
  }
  if (p.dact) {
    const uint2 hh = *reinterpret_cast<const uint2*>(p.pre_in + m * p.ldp + n);
    const float h[4] = {lo_bf(hh.x), hi_bf(hh.x), lo_bf(hh.y), hi_bf(hh.y)};
    if (p.dact == 1) {
      for (int r = 0; r < 4; ++r) v[r] *= dgelu_tanh(h[r]);
    } else if (p.dact == 2) {
      for (int r = 0; r < 4; ++r) v[r] *= dgelu_erf(h[r]);
    } else {  // 3: pre_in already holds gelu'(x)
      for (int r = 0; r < 4; ++r) v[r] *= h[r];
    }
  }
  if (p.act == 5) {  // quick-GELU (no pre-activation output)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = quick_gelu(v[r]);
  } else if (p.act) {
    float d[4];
    if (p.act == 1 || p.act == 2) {
      for (int r = 0; r < 4; ++r) d[r] = v[r];
      if (p.act == 1) {
        for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
      } else {
        for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
      }
    } else if (p.act == 3) {
      for (int r = 0; r < 4; ++r) gelu_dgelu_tanh(v[r], v[r], d[r]);
    } else {
      for (int r = 0; r < 4; ++r) gelu_dgelu_erf(v[r], v[r], d[r]);
    }
    if (p.pre_out) {
      *reinterpret_cast<uint2*>(p.pre_out + m * p.ldp + n) =
          make_uint2(pack2(d[0], d[1]), pack2(d[2], d[3]));
    }
  }
  if (p.has_drop) {
    const uint64_t seed = seed_eff(p.seed, p.seed_ptr);
    const uint64_t base = (uint64_t)m * (uint64_t)p.N + (uint64_t)n;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      v[r] = rng_keep(seed, base + r, p.drop_thresh) ? v[r] * p.drop_scale : 0.f;
  }
  if (p.gate) {
    if (p.pre_out && !p.act) {  // save the un-gated branch for the gate gradient
      *reinterpret_cast<uint2*>(p.pre_out + m * p.ldp + n) =
          make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= gatev;
  }
  if (p.residual) {
    const uint2 rr = *reinterpret_cast<const uint2*>(p.residual + m * p.ldr + n);
    v[0] += lo_bf(rr.x); v[1] += hi_bf(rr.x); v[2] += lo_bf(rr.y); v[3] += hi_bf(rr.y);
  }
}

// Compile-time epilogue kinds for the persistent kernels (gemm_pp3.h): each instance
// carries only its own ops; EPI_GEN runs the runtime-flag path above.
enum {
  EPI_PLAIN = 0, EPI_BIAS = 1, EPI_BIAS_RES = 2, EPI_BIAS_ACT = 3, EPI_DACT = 4, EPI_GEN = 5,
  EPI_RES = 6,  // C = AB + residual (in-place gradient accumulation: residual == C)
  EPI_BIAS_ACT_ERF = 7, EPI_DACT_ERF = 8,  // 3 / 4 are the tanh-GELU forms
  // GELU forward storing gelu'(x) (act 3 / 4) and the backward multiply by it (dact 3)
  EPI_BIAS_ACT_D = 9, EPI_BIAS_ACT_ERF_D = 10, EPI_MUL = 11,
  // C = residual + dropout(AB + bias): the Q-Former out_proj / MLP output branches
  // (gpt2_q_former/model.py:139-145, q += drop(...)), mask = the counter hash of (m, n)
  EPI_BIAS_DROP_RES = 12,
  // C = residual + tanh(gate) * (AB + bias), the un-gated branch AB + bias stored to pre_out for
  // the gate gradient: the cross-att decoder's xattn.c_proj (gpt2_cross-att/model.py:57,99-101).
  // Only the four-wave kernels take it (gemm_w4.hip, gemm_w4_epi_kind); gemm_epi_kind still
  // answers EPI_GEN for a gated GEMM, so no other kernel family sees this kind
  EPI_GATE_RES = 13,
  // C = quick_gelu(AB + bias) (act 5, no side output): the frozen CLIP ViT-L/14 MLP's fc1
  // (transformers CLIPMLP, QuickGELUActivation) on the gvl-native feature stage (gvl/clip.py)
  EPI_BIAS_QGELU = 14
};
constexpr int EPI_KINDS = 15;

template <int EPI>
struct EpiKind {
  static constexpr bool DERIV = EPI == EPI_BIAS_ACT_D || EPI == EPI_BIAS_ACT_ERF_D;
  static constexpr bool ACT = EPI == EPI_BIAS_ACT || EPI == EPI_BIAS_ACT_ERF || DERIV;
  static constexpr bool MUL = EPI == EPI_MUL;
  static constexpr bool DACT = EPI == EPI_DACT || EPI == EPI_DACT_ERF || MUL;
  static constexpr bool ERF = EPI == EPI_BIAS_ACT_ERF || EPI == EPI_DACT_ERF || EPI == EPI_BIAS_ACT_ERF_D;
  static constexpr bool DROP = EPI == EPI_BIAS_DROP_RES;
  static constexpr bool GATE = EPI == EPI_GATE_RES;
  static constexpr bool QGELU = EPI == EPI_BIAS_QGELU;
  static constexpr bool BIAS = EPI == EPI_BIAS || EPI == EPI_BIAS_RES || ACT || DROP || GATE || QGELU;
  static constexpr bool RES = EPI == EPI_BIAS_RES || EPI == EPI_RES || DROP || GATE;
  static constexpr bool PRE_OUT = ACT || GATE;  // stores a bf16 [M, N] side output (pre_out)
  static constexpr bool AUX = DACT || RES;  // reads a bf16 [M, N] operand (pre_in / residual)
};

// Epilogue operands of the persistent kernel, fetched in batches: the bias at the tile's
// first K-step (its wait then hides behind the whole tile), the [M, N] operand (pre_in /
// residual, 64 VGPRs per tile: too many to hold across the MFMA cluster) in two half-tile
// batches inside the epilogue, so the epilogue pays two memory latencies — not one per
// fragment pair, each of which would also wait behind the LDS-DMA of later K-steps.
// Lane (row l&15, column quad q) holds, per fragment (i, j), the 4 bf16 at row
// mw0 + 16 i + (l & 15), cols nw0 + 16 j + 4 q.
// FULL: the whole wave tile's [M, N] operand is fetched at once, by the kernel, ahead of the
// epilogue (gemm_w4d.h: one tile per CU, so a fetch inside the epilogue is exposed latency).
template <int FM, int FN, int EPI, bool FULL = false>
struct EpiPre {
  using KD = EpiKind<EPI>;
  uint2 b[KD::BIAS ? FN : 1];
  static constexpr int XH = FULL ? FM : FM / 2;  // else half a tile at a time, in the epilogue
  uint2 x[KD::AUX ? XH : 1][KD::AUX ? FN : 1];
  uint64_t seed = 0;  // effective dropout seed (DROP), read with the bias, not per element
  float gatev = 1.f;  // tanh(gate) (GATE), read with the bias
  bool pre0 = false;  // the first half (fragment rows 0 .. XH-1) was fetched ahead of the epilogue
  GVL_DEV void load_bias(const GemmP& p, int64_t nw0, int lane) {
    if constexpr (KD::DROP) seed = seed_eff(p.seed, p.seed_ptr);
    if constexpr (KD::GATE) gatev = tanhf(bf2f(*p.gate));
    if constexpr (KD::BIAS) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t n = nw0 + 16 * j + 4 * (lane >> 4);
        b[j] = n < p.N ? *reinterpret_cast<const uint2*>(p.bias + n) : make_uint2(0, 0);
      }
    }
  }
  // rows of fragments i0 .. i0 + XH - 1
  GVL_DEV void load_aux(const GemmP& p, int64_t mw0, int64_t nw0, int lane, int i0,
                        const bf16_t* res = nullptr) {
    if constexpr (KD::AUX) {
      const bf16_t* base = KD::DACT ? p.pre_in : (res ? res : p.residual);
      const int64_t ld = KD::DACT ? p.ldp : p.ldr;
#pragma unroll
      for (int i = 0; i < XH; ++i) {
        const int64_t m = mw0 + 16 * (i0 + i) + (lane & 15);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int64_t n = nw0 + 16 * j + 4 * (lane >> 4);
          x[i][j] = (m < p.M && n < p.N) ? *reinterpret_cast<const uint2*>(base + m * ld + n)
                                         : make_uint2(0, 0);
        }
      }
    }
  }
};

template <int EPI>
static __device__ __forceinline__ void gemm_epi_vals_k(const GemmP& p, float4_t a, int64_t m,
                                                          int64_t n, float alpha, float gatev,
                                                          const uint2& bb, const uint2& ax,
                                                          float (&v)[4], float (&pre)[4],
                                                          uint64_t seed = 0) {
  if constexpr (EPI == EPI_GEN) {
    gemm_epi_vals(p, a, m, n, alpha, gatev, v);
  } else {
    using KD = EpiKind<EPI>;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = a[r] * alpha;
    if constexpr (KD::BIAS) {
      v[0] += lo_bf(bb.x); v[1] += hi_bf(bb.x); v[2] += lo_bf(bb.y); v[3] += hi_bf(bb.y);
    }
    if constexpr (KD::QGELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = quick_gelu(v[r]);
    }
    if constexpr (KD::DACT) {
      const float h[4] = {lo_bf(ax.x), hi_bf(ax.x), lo_bf(ax.y), hi_bf(ax.y)};
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] *= KD::MUL ? h[r] : KD::ERF ? dgelu_erf(h[r]) : dgelu_tanh(h[r]);
    }
    if constexpr (KD::ACT) {  // the caller stores pre (x, or gelu'(x)) with 16-B stores
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (KD::DERIV) {
          if constexpr (KD::ERF) gelu_dgelu_erf(v[r], v[r], pre[r]);
          else gelu_dgelu_tanh(v[r], v[r], pre[r]);
        } else {
          pre[r] = v[r];
          v[r] = KD::ERF ? gelu_erf(v[r]) : gelu_tanh(v[r]);
        }
      }
    }
    if constexpr (KD::DROP) {
      const uint64_t base = (uint64_t)m * (uint64_t)p.N + (uint64_t)n;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] = rng_keep(seed, base + r, p.drop_thresh) ? v[r] * p.drop_scale : 0.f;
    }
    if constexpr (KD::GATE) {  // the caller stores pre (the un-gated branch) with 16-B stores
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pre[r] = v[r];
        v[r] *= gatev;
      }
    }
    if constexpr (KD::RES) {
      v[0] += lo_bf(ax.x); v[1] += hi_bf(ax.x); v[2] += lo_bf(ax.y); v[3] += hi_bf(ax.y);
    }
  }
}

static __device__ __forceinline__ void gemm_epi_quad(const GemmP& p, float4_t a, int64_t m,
                                                        int64_t n, float alpha, float gatev) {
  float v[4];
  gemm_epi_vals(p, a, m, n, alpha, gatev, v);
  if (p.c_f32) {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.C) + m * p.ldc + n) =
        make_float4(v[0], v[1], v[2], v[3]);
  } else {
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.C) + m * p.ldc + n) =
        make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
  }
}

// bf16-output epilogue with 16-byte stores (needs N % 8 == 0, ldc % 8 == 0, FN even).
// For fragment pair (j, j+1) a lane of column quad q holds 4 columns of each; two
// v_permlane16_swap_b32 (lanes l <-> l^16 across the pair) leave every lane 8 consecutive
// columns: quad q stores cols 16 (j + (q & 1)) + 8 (q >> 1) .. + 7, so one store
// instruction writes 16 rows x 64 B instead of 16 rows x 32 B.
// Odd FN: the last fragment is stored unpaired (8-B stores).
template <int FM, int FN, int EPI = EPI_GEN, bool FULL = false>
GVL_DEV void gemm_epilogue16(const GemmP& p, const float4_t (&acc)[FM][FN], int64_t mw0,
                             int64_t nw0, int lane, float alpha, EpiPre<FM, FN, EPI, FULL>& pre,
                             void* cout = nullptr, const bf16_t* res = nullptr) {
  // cout / res: this problem's C and residual in a batched launch (default p.C / p.residual)
  bf16_t* const cbase = reinterpret_cast<bf16_t*>(cout ? cout : p.C);
  float gatev = 1.f;
  if constexpr (EPI == EPI_GEN) gatev = p.gate ? tanhf(bf2f(*p.gate)) : 1.f;
  if constexpr (EpiKind<EPI>::GATE) gatev = pre.gatev;
  const bool plain = EPI == EPI_PLAIN ||
                     (EPI == EPI_GEN && !p.bias && !p.dact && !p.act && !p.has_drop && !p.gate &&
                      !p.residual);
  const int q = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int64_t m = mw0 + i * 16 + (lane & 15);
    const bool mok = m < p.M;
    if (EpiKind<EPI>::AUX && !FULL && i % EpiPre<FM, FN, EPI>::XH == 0 && !(i == 0 && pre.pre0))
      pre.load_aux(p, mw0, nw0, lane, i, res);
#pragma unroll
    for (int j = 0; j + 1 < FN; j += 2) {
      const int64_t n0 = nw0 + j * 16 + 4 * q, n1 = n0 + 16;
      uint32_t x0, y0, x1, y1;  // packed bf16 pairs: frag j (x0: cols 0-1, y0: 2-3), frag j+1
      if (plain) {
        x0 = pack2(acc[i][j][0] * alpha, acc[i][j][1] * alpha);
        y0 = pack2(acc[i][j][2] * alpha, acc[i][j][3] * alpha);
        x1 = pack2(acc[i][j + 1][0] * alpha, acc[i][j + 1][1] * alpha);
        y1 = pack2(acc[i][j + 1][2] * alpha, acc[i][j + 1][3] * alpha);
      } else {
        float v0[4] = {0.f, 0.f, 0.f, 0.f}, v1[4] = {0.f, 0.f, 0.f, 0.f};
        float h0[4] = {0.f, 0.f, 0.f, 0.f}, h1[4] = {0.f, 0.f, 0.f, 0.f};
        using KD = EpiKind<EPI>;
        const uint2 b0 = KD::BIAS ? pre.b[KD::BIAS ? j : 0] : make_uint2(0, 0);
        const uint2 b1 = KD::BIAS ? pre.b[KD::BIAS ? j + 1 : 0] : make_uint2(0, 0);
        constexpr int XH = EpiPre<FM, FN, EPI, FULL>::XH;
        const uint2 a0 = KD::AUX ? pre.x[KD::AUX ? i % XH : 0][KD::AUX ? j : 0] : make_uint2(0, 0);
        const uint2 a1 = KD::AUX ? pre.x[KD::AUX ? i % XH : 0][KD::AUX ? j + 1 : 0] : make_uint2(0, 0);
        if (mok && n0 < p.N) gemm_epi_vals_k<EPI>(p, acc[i][j], m, n0, alpha, gatev, b0, a0, v0, h0, pre.seed);
        if (mok && n1 < p.N) gemm_epi_vals_k<EPI>(p, acc[i][j + 1], m, n1, alpha, gatev, b1, a1, v1, h1, pre.seed);
        x0 = pack2(v0[0], v0[1]); y0 = pack2(v0[2], v0[3]);
        x1 = pack2(v1[0], v1[1]); y1 = pack2(v1[2], v1[3]);
        if (KD::PRE_OUT && p.pre_out) {  // pre-activation / un-gated branch: same lane swap, 16-B stores
          const auto hx = __builtin_amdgcn_permlane16_swap(pack2(h0[0], h0[1]), pack2(h1[0], h1[1]),
                                                           false, false);
          const auto hy = __builtin_amdgcn_permlane16_swap(pack2(h0[2], h0[3]), pack2(h1[2], h1[3]),
                                                           false, false);
          const int64_t n = nw0 + 16 * (j + (q & 1)) + 8 * (q >> 1);
          if (mok && n < p.N)
            *reinterpret_cast<uint4*>(p.pre_out + m * p.ldp + n) = make_uint4(hx[0], hy[0], hx[1], hy[1]);
        }
      }
      const auto sx = __builtin_amdgcn_permlane16_swap(x0, x1, false, false);
      const auto sy = __builtin_amdgcn_permlane16_swap(y0, y1, false, false);
      const int64_t n = nw0 + 16 * (j + (q & 1)) + 8 * (q >> 1);
      if (mok && n < p.N)
        *reinterpret_cast<uint4*>(cbase + m * p.ldc + n) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
    }
    if constexpr (FN % 2 == 1) {
      constexpr int j = FN - 1;
      const int64_t n0 = nw0 + j * 16 + 4 * q;
      uint32_t x0, y0;
      if (plain) {
        x0 = pack2(acc[i][j][0] * alpha, acc[i][j][1] * alpha);
        y0 = pack2(acc[i][j][2] * alpha, acc[i][j][3] * alpha);
      } else {
        float v0[4] = {0.f, 0.f, 0.f, 0.f}, h0[4] = {0.f, 0.f, 0.f, 0.f};
        using KD = EpiKind<EPI>;
        const uint2 b0 = KD::BIAS ? pre.b[KD::BIAS ? j : 0] : make_uint2(0, 0);
        constexpr int XH = EpiPre<FM, FN, EPI, FULL>::XH;
        const uint2 a0 = KD::AUX ? pre.x[KD::AUX ? i % XH : 0][KD::AUX ? j : 0] : make_uint2(0, 0);
        if (mok && n0 < p.N) gemm_epi_vals_k<EPI>(p, acc[i][j], m, n0, alpha, gatev, b0, a0, v0, h0, pre.seed);
        x0 = pack2(v0[0], v0[1]); y0 = pack2(v0[2], v0[3]);
        if (KD::PRE_OUT && p.pre_out && mok && n0 < p.N)
          *reinterpret_cast<uint2*>(p.pre_out + m * p.ldp + n0) =
              make_uint2(pack2(h0[0], h0[1]), pack2(h0[2], h0[3]));
      }
      if (mok && n0 < p.N)
        *reinterpret_cast<uint2*>(cbase + m * p.ldc + n0) = make_uint2(x0, y0);
    }
  }
}

// Store raw fp32 accumulators of a split-K slice.
template <int FM, int FN>
GVL_DEV void gemm_store_partial(const GemmP& p, const float4_t (&acc)[FM][FN], int split,
                                int64_t mw0, int64_t nw0, int lane) {
  float* base = p.ws + (int64_t)split * p.M * p.N;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int64_t m = mw0 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t n = nw0 + j * 16 + 4 * (lane >> 4);
      if (m < p.M && n < p.N)
        *reinterpret_cast<float4*>(base + m * p.N + n) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
}

// In-launch combine of a tile's two K-halves (splits == 2), per wave, lock-free: each wave
// publishes its 128 x BN/4 fp32 partial with write-through (sc1) 16-B stores, drains them
// (vmcnt(0)), then lane 0 takes an agent-scope ticket for (tile, wave).  The wave drawing
// ticket 1 arrived last: it reads the other half's partial with sc1 loads, adds it and runs
// the epilogue; it also returns the ticket to 0 for the next call.  Nobody waits, so no
// residency assumption; two-term fp32 addition is commutative, so the result does not
// depend on which half arrives last (cdna_hip_programming.md §6 Guideline 16, counter form).
typedef __attribute__((address_space(1))) uint32_t gvl_gu32_t;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// Addressing: the lane part of the offset is one VGPR ((lane & 15) rows, 4 (lane >> 4) cols);
// the fragment / tile part is uniform and goes to soffset (tile-dependent, so the compiler
// does not hoist 32 offsets out of the persistent loop and spill them).
template <int FM, int FN>
GVL_DEV bool gemm_splitk_arrive(const GemmP& p, const float4_t (&acc)[FM][FN], int split,
                                int tile, int wave, int64_t mw0, int64_t nw0, int lane,
                                __amdgpu_buffer_rsrc_t rw) {
  const int voff = (int)(((int64_t)(lane & 15) * p.N + 4 * (lane >> 4)) * 4);
  const int64_t base = (int64_t)split * p.M * p.N + mw0 * p.N + nw0;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const bool mok = mw0 + i * 16 + (lane & 15) < p.M;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int soff = __builtin_amdgcn_readfirstlane((int)((base + (int64_t)i * 16 * p.N + j * 16) * 4));
      if (mok && nw0 + j * 16 < p.N)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[i][j]), rw, voff,
                                               soff, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  gvl_gu32_t* t = (gvl_gu32_t*)(p.tickets + (int64_t)tile * 8 + wave);
  uint32_t got = 0;
  if (lane == 0) got = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  got = __builtin_amdgcn_readfirstlane(got);
  if (got == 0) return false;
  if (lane == 0) __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// Last arriver: acc += the other half's partial (sc1 loads, 2 x FN 16-B loads in flight;
// rows past M are read unguarded inside the workspace and never stored).
template <int FM, int FN>
GVL_DEV void gemm_splitk_gather(const GemmP& p, float4_t (&acc)[FM][FN], int split,
                                int64_t mw0, int64_t nw0, int lane, __amdgpu_buffer_rsrc_t rw) {
  const int voff = (int)(((int64_t)(lane & 15) * p.N + 4 * (lane >> 4)) * 4);
  const int64_t base = (int64_t)(1 - split) * p.M * p.N + mw0 * p.N + nw0;
  constexpr int H = 2;  // fragment rows per batch of loads (register budget: acc is live)
#pragma unroll
  for (int h = 0; h < FM / H; ++h) {
    u32x4_t t[H][FN];
#pragma unroll
    for (int i = 0; i < H; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int soff = __builtin_amdgcn_readfirstlane(
            (int)((base + (int64_t)(h * H + i) * 16 * p.N + j * 16) * 4));
        t[i][j] = __builtin_amdgcn_raw_buffer_load_b128(rw, voff, soff, 16);
      }
#pragma unroll
    for (int i = 0; i < H; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[h * H + i][j] += __builtin_bit_cast(float4_t, t[i][j]);
  }
}

namespace gvl {
int gemm_lds_pick(int64_t M, int64_t N, int64_t K, int forced);
int gemm_splitk_pick(int64_t tiles, int64_t K);
bool gemm_lds_ok(const gvl_gemm_desc* d);
int gemm_lds_launch(const GemmP& p, int a_mn, int b_mn, int cfg, hipStream_t s);
void gemm_splitk_reduce_launch(const GemmP& p, hipStream_t s);
const char* gemm_ring_name(int cfg);
bool gemm_ring_ok(const gvl_gemm_desc* d);
int gemm_ring_launch(const GemmP& p, int a_mn, int b_mn, int cfg, hipStream_t s);
int gemm_ring_pick(int64_t M, int64_t N, int64_t K, int forced, int a_mn);
int gemm_epi_kind(const GemmP& p);  // EPI_* for the persistent kernels (gemm_plan.hip)
bool gemm_pp3_plan(GemmP& p, bool force, int gran = 32);  // gran: K-step depth
bool gemm_pp3_try(const GemmP& p, int a_mn, int b_mn, hipStream_t s);
bool pp3_combine_forced();  // gemm.hip: gvl_gemm_tune(3, 13) (the persistent kernel's combine, tests)
int gemm_pp3_launch(const GemmP& p, int a_mn, int b_mn, hipStream_t s);  // planned p
int gemm_pp3_launch_ff(const GemmP& p, hipStream_t s);  // gemm_pp3_{ff,ft,tf,tt}.hip
int gemm_pp3_launch_ft(const GemmP& p, hipStream_t s);
int gemm_pp3_launch_tf(const GemmP& p, hipStream_t s);
int gemm_pp3_launch_tt(const GemmP& p, hipStream_t s);
int gemm_pp3_splits(int64_t M, int64_t N, int64_t K, int gran = 32);
bool gemm_w4_plan(const GemmP& p, int a_mn, bool force);  // gemm_w4.hip
int gemm_w4_launch(const GemmP& p, int b_mn, hipStream_t s);
bool gemm_w4_rows128(const GemmP& p);  // the launch uses 128-row tiles (gemm_w4m_kernel)
bool gemm_w4_cols96(const GemmP& p, bool b_mn);  // ... and 96-column ones (gemm_w4n_kernel)
bool gemm_w4_rows96(const GemmP& p, bool b_mn);  // 96 x 128 dX tiles (gemm_w4r_kernel)
int gemm_w4_epi_kind(const GemmP& p);  // gemm_epi_kind + EPI_GATE_RES (four-wave kernels only)
bool gemm_w4_try(const GemmP& p, int a_mn, int b_mn, hipStream_t s);
bool gemm_w4d_ok(const GemmP& p);  // gemm_w4d.hip: direct-A variant for a w4-planned shape
int gemm_w4d_launch(const GemmP& p, int b_mn, bool rows128, hipStream_t s);
bool gemm_w4x_plan(GemmP& p, int a_mn, int b_mn, bool force);  // gemm_w4x.hip: AGPR four-wave kernel
bool gemm_w4x_try(const GemmP& p, int a_mn, int b_mn, bool force, hipStream_t s);
bool gemm_w4x_batched_try(const GemmP& p, hipStream_t s);  // batched dW (a_mn, b_mn, C += AB)
bool w4x_dw_plan(GemmP& p);  // its tile choice (bm / bn / tiles), false when not routed
bool gemm_w4x_grouped_try(GemmP& p, hipStream_t s);  // grouped dW of different shapes
}  // namespace gvl
