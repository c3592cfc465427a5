// Fused attention for head dim 64 on gfx950 MFMA (16x16x32 bf16), forward + backward.
//
// Forward (flash-style, online softmax in fp32): block = (64*G-query tile, head, batch),
// 4 waves x G groups of 16 query rows.  K and V tiles of 64 keys are register-staged into
// a double-buffered LDS ring.  S is computed "swapped" (K fragment as the MFMA A operand),
// which leaves one query row per lane (lane&15) and 16 keys in registers, so the row
// max/sum need only two cross-lane steps, and the P fragment of the following P.V MFMA is
// lane-local (the MFMA k-slots are permuted to match; V is read with ds_read_b64_tr_b16).
// The output accumulator keeps the same query on the lane, so rescales are lane-local.
// With G = 2 every K/V fragment read from LDS feeds two MFMAs (two query groups).
//
// Backward (FA2 recompute, no atomics, deterministic): dQ by a query-tile kernel looping over
// key tiles, which also writes D = rowsum(dO*O); dK/dV by a key-tile kernel (16 keys per wave)
// looping over query tiles; both stage their streamed tiles by LDS-DMA (so does the no-dropout
// forward, attn_fwd_dma_kernel).  Sequences of <= 64 rows take one fused kernel.  P is recomputed from the saved
// log-sum-exp.  Dropout (Q-Former MHA) is a counter-hash mask on (b,h,q,k), identical in
// every kernel.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "capi_util.h"
#include "gemm_ring.h"
#include "../../include/gvl.h"

namespace {

constexpr int D = 64;        // head dim
constexpr int KT = 64;       // key tile (forward / dq) and query tile (dkdv)
constexpr int NT = 256;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

struct AttnP {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; bf16_t* o; float* lse;
  int64_t B, H, Tq, Tk;
  int64_t q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_st, o_sh;
  int causal;
  float scale;       // softmax scale (1/sqrt(64))
  float c2;          // scale * log2(e)
  int has_drop;
  uint32_t drop_thresh;
  float drop_scale;
  uint64_t seed;
  const uint64_t* seed_ptr;
};

struct AttnG {
  const bf16_t* dout; int64_t do_sb, do_st, do_sh;
  bf16_t* dq; int64_t dq_sb, dq_st, dq_sh;
  bf16_t* dk; int64_t dk_sb, dk_st, dk_sh;
  bf16_t* dv; int64_t dv_sb, dv_st, dv_sh;
  float* Dws;  // D = rowsum(dO * O) per query row, written by the dQ kernel
  float* Lws;  // lse * log2(e) per query row (ditto): the dK/dV kernel's exp2 argument as is
};

// 1-D grid, heavy tiles first: the block id's slowest digit is the tile index, so every
// (head, batch) pair's longest causal tile is dispatched in the first wave of blocks and the
// short ones fill the tail.  LATE_HEAVY: the last query tiles see the most keys (forward,
// dQ); otherwise the first key tiles see the most queries (dK/dV).
template <bool LATE_HEAVY>
GVL_DEV void tile_of_block(const AttnP& p, int64_t ntile, int64_t& t, int64_t& h, int64_t& b) {
  const int64_t hb = p.H * p.B, bid = blockIdx.x;
  const int64_t r = bid / hb, rem = bid - r * hb;
  t = (LATE_HEAVY && p.causal) ? ntile - 1 - r : r;
  b = rem / p.H;
  h = rem - b * p.H;
}

// [64 rows][64 d] bf16 tile, 128-B rows, 16-B chunk c of row r at c ^ (((r >> 1) & 3) << 1).
// This one XOR is conflict-free for both fragment reads the kernels issue on a tile: the
// ds_read_b128 row fragments (frag_row) and the ds_read_b64_tr_b16 transposed ones (frag_tr),
// checked lane group by lane group (tools/attn_swizzle_check.py).  Round 1 used
// c ^ ((r >> 1) & 7) for row-read tiles, which is 2-way conflicted on the transposed reads the
// backward issues on Q, dO and K (PMC: 20-25 % of the dK/dV and dQ kernels' LDS cycles).
GVL_DEV int swz_tr(int row, int chunk) { return row * 128 + ((chunk ^ (((row >> 1) & 3) << 1)) << 4); }
GVL_DEV int swz_row(int row, int chunk) { return swz_tr(row, chunk); }

// Register-stage a (2 * NTH / 8) x 64 tile (rows r0.., valid rows < R) from a strided tensor.
template <int NTH = NT, int NC = 2>  // NTH threads, NC 16-B chunks each: NC * NTH / 8 rows
GVL_DEV void load_rows(uint4 (&r)[NC], const bf16_t* base, int64_t st, int64_t r0, int64_t R, int tid) {
#pragma unroll
  for (int it = 0; it < NC; ++it) {
    const int row = (tid >> 3) + (NTH / 8) * it, ch = tid & 7;
    if (r0 + row < R) r[it] = *reinterpret_cast<const uint4*>(base + (r0 + row) * st + ch * 8);
    else r[it] = make_uint4(0, 0, 0, 0);
  }
}
template <bool TR, int NTH = NT, int NC = 2>  // NTH threads store NC * NTH / 8 rows
GVL_DEV void store_rows(const uint4 (&r)[NC], char* lds, int tid) {
#pragma unroll
  for (int it = 0; it < NC; ++it) {
    const int row = (tid >> 3) + (NTH / 8) * it, ch = tid & 7;
    const int off = TR ? swz_tr(row, ch) : swz_row(row, ch);
    *reinterpret_cast<uint4*>(lds + off) = r[it];
  }
}

// Row fragment (16 rows from row0, k-step s over d): lane holds tile[row0+(l&15)][32s+8G..+7].
GVL_DEV short8_t frag_row(const char* lds, int row0, int s, int lane) {
  const int row = row0 + (lane & 15), ch = 4 * s + (lane >> 4);
  return *reinterpret_cast<const short8_t*>(lds + swz_row(row, ch));
}
// Transposed fragment for the permuted k-slot order used by P.V-type products:
// lane (G, i) gets column 16t+i of rows {32s+4G+0..3} (elements 0..3) and
// {32s+16+4G+0..3} (elements 4..7).
template <bool TR>
GVL_DEV short8_t frag_tr(const char* lds, int t, int s, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ch = 2 * t + (p >> 1);
  const int ra = 32 * s + 4 * G + q, rb = ra + 16;
  const int oa = (TR ? swz_tr(ra, ch) : swz_row(ra, ch)) + (p & 1) * 8;
  const int ob = (TR ? swz_tr(rb, ch) : swz_row(rb, ch)) + (p & 1) * 8;
  short8_t r;
  r.lo = lds_read_tr(lds + oa);
  r.hi = lds_read_tr(lds + ob);
  return r;
}

// Branch-free forms: rows past the end read row 0 (finite data) instead of being zero-filled.
// Every use of such a row in attn_bwd_short_kernel is multiplied by a masked (exactly zero)
// probability or score gradient, or not stored, so the results are unchanged; with no branch or
// select on the loaded data hipcc issues the block's loads back to back and waits once, instead
// of one round trip per conditional load (the prologue was six).
template <int NTH = NT, int NC = 2>
GVL_DEV void load_rows_nb(uint4 (&r)[NC], const bf16_t* base, int64_t st, int64_t R, int tid) {
#pragma unroll
  for (int it = 0; it < NC; ++it) {
    const int row = (tid >> 3) + (NTH / 8) * it, ch = tid & 7;
    r[it] = *reinterpret_cast<const uint4*>(base + (row < R ? row : 0) * st + ch * 8);
  }
}
GVL_DEV short8_t load_frag_global_nb(const bf16_t* rowptr0, int64_t st, int row, int s, int lane,
                                     bool ok) {
  return __builtin_bit_cast(
      short8_t, *reinterpret_cast<const uint4*>(rowptr0 + (ok ? row : 0) * st + 32 * s + 8 * (lane >> 4)));
}

GVL_DEV short8_t load_frag_global(const bf16_t* rowptr, int s, int lane, bool ok) {
  if (!ok) return short8_t{0, 0, 0, 0, 0, 0, 0, 0};
  const uint4 u = *reinterpret_cast<const uint4*>(rowptr + 32 * s + 8 * (lane >> 4));
  return __builtin_bit_cast(short8_t, u);
}

// Max over the four lanes l, l^16, l^32, l^48 that hold one query row (the S fragment's row is
// spread over the lane groups): two VALU lane swaps (v_permlane16_swap / v_permlane32_swap, no
// LDS crossbar).  __shfl_xor lowered to ds_bpermute_b32 with an lgkmcnt(0) wait each, i.e. two
// LDS round trips per query group and key tile on the softmax's critical path.
#ifndef GVL_ATTN_LDS_SHFL  // 1: the round-4 __shfl_xor form (A/B variant builds only)
#define GVL_ATTN_LDS_SHFL 0
#endif
GVL_DEV float rowmax4(float x) {
  if (GVL_ATTN_LDS_SHFL) {
    x = fmaxf(x, __shfl_xor(x, 16, 64));
    return fmaxf(x, __shfl_xor(x, 32, 64));
  }
  const uint32_t u = __float_as_uint(x);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const float y = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const uint32_t v = __float_as_uint(y);
  const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

GVL_DEV short8_t pack_frag(const float4_t& a, const float4_t& b) {
  uint4 u = make_uint4(pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(b[0], b[1]), pack2(b[2], b[3]));
  return __builtin_bit_cast(short8_t, u);
}

// ------------------------------------------------------------------------------------
// Short sequences (G = 1, no dropout) compile for 4 waves per SIMD (<= 128 VGPRs, no spill):
// 4 blocks per CU instead of 3, so the caption decoder's 1536 (b, h) blocks take 1.5 rounds.
// Timing-only diagnostic builds of the forward (wrong results; never the shipped library):
// GVL_ATTN_FWD_DIAG=1 replaces the softmax exponentials by a multiply, 2 drops the in-loop K/V
// loads and LDS stores, 3 drops the per-tile __syncthreads.
#ifndef GVL_ATTN_FWD_DIAG
#define GVL_ATTN_FWD_DIAG 0
#endif
#ifndef GVL_ATTN_ONE_BPC  // blocks per CU the one-tile forward is compiled for
#define GVL_ATTN_ONE_BPC 6
#endif
// ONE (Tk <= 64: one key tile, G = 1): a single LDS stage (16 KiB) and a 6-blocks-per-CU register
// budget, so the caption decoders' 1536 (b, h) blocks of T = 63 are one round of 256 CUs (4 blocks
// per CU by registers and 5 by LDS made it 1.5 rounds).
// R = 32 (ONE, Tq, Tk <= 32: the cross-att decoder's 31-token self-attention, the Q-Former
// bridge's 32 queries): 2 waves over 32-row Q / K / V tiles instead of 4 waves over 64-row ones
// half of which were padding.
template <int G, bool DROP, bool ONE = false, int R = 64, int RK = R>  // R: query rows, RK: key rows
__global__ __launch_bounds__(R * 4, ONE ? (RK > R ? 5 : GVL_ATTN_ONE_BPC) : ((G == 1 && !DROP) ? 4 : 2)) void attn_fwd_kernel(AttnP p) {
  static_assert(!ONE || G == 1, "one-tile forward: G = 1");
  static_assert((R == 64 && RK == 64) || (R == 32 && ONE && (RK == 32 || RK == 64)), "tile rows");
  constexpr int NG = RK / 16, NKS = RK / 32;  // key groups of 16, 32-deep k-steps per key tile
  constexpr int NC = 2 * RK / R;             // 16-B chunks per thread of a K / V tile
  const uint64_t seed_ = DROP ? seed_eff(p.seed, p.seed_ptr) : 0;
  constexpr int QT = R == 32 ? 32 : 64 * G;
  __shared__ __attribute__((aligned(16))) char smem[ONE ? 1 : 2][2][RK * D * 2];  // [stage][K,V]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Gl = lane >> 4;
  int64_t qt, h, b;
  tile_of_block<true>(p, (p.Tq + QT - 1) / QT, qt, h, b);
  const int64_t qblk0 = qt * QT;
  const bf16_t* qbase = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kbase = p.k + b * p.k_sb + h * p.k_sh;
  const bf16_t* vbase = p.v + b * p.v_sb + h * p.v_sh;

  int64_t q[G];
  bool qok[G];
  short8_t qf[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    q[g] = qblk0 + wave * 16 * G + g * 16 + (lane & 15);
    qok[g] = q[g] < p.Tq;
    qf[g][0] = load_frag_global(qbase + q[g] * p.q_st, 0, lane, qok[g]);
    qf[g][1] = load_frag_global(qbase + q[g] * p.q_st, 1, lane, qok[g]);
  }

  int64_t kend = p.Tk;
  if (p.causal) {
    const int64_t lim = qblk0 + QT;
    if (lim < kend) kend = lim;
  }
  const int nkt0 = (int)((kend + KT - 1) / KT);
  const int nkt = ONE ? (nkt0 > 0 ? 1 : 0) : nkt0;

#ifndef GVL_ATTN_FWD_V2
#define GVL_ATTN_FWD_V2 1
#endif
#if GVL_ATTN_FWD_V2
  // o[g][4] = row sum of the bf16 P (an MFMA against a ones fragment: the softmax
  // denominator of exactly the P values that enter P.V, and 16 fewer VALU adds per tile)
  constexpr int NO = 5;
#else
  constexpr int NO = 4;
#endif
  float4_t o[G][NO];
  float m[G], l[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int t = 0; t < NO; ++t) o[g][t] = float4_t{0.f, 0.f, 0.f, 0.f};
    m[g] = -INFINITY;
    l[g] = 0.f;
  }
  short8_t ones;
#pragma unroll
  for (int k = 0; k < 8; ++k) ones[k] = (short)0x3F80;  // bf16 1.0

  uint4 rk[NC], rv[NC];
  load_rows<R * 4, NC>(rk, kbase, p.k_st, 0, p.Tk, tid);
  load_rows<R * 4, NC>(rv, vbase, p.v_st, 0, p.Tk, tid);
  store_rows<false, R * 4, NC>(rk, smem[0][0], tid);
  store_rows<true, R * 4, NC>(rv, smem[0][1], tid);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const bool more = !ONE && GVL_ATTN_FWD_DIAG != 2 && kt + 1 < nkt;
    if (more) {
      load_rows<R * 4, NC>(rk, kbase, p.k_st, (int64_t)(kt + 1) * KT, p.Tk, tid);
      load_rows<R * 4, NC>(rv, vbase, p.v_st, (int64_t)(kt + 1) * KT, p.Tk, tid);
    }
    const char* ks = smem[ONE ? 0 : (kt & 1)][0];
    const char* vs = smem[ONE ? 0 : (kt & 1)][1];
    const int64_t k0 = (int64_t)kt * KT;
    float4_t sc[G][NG];
#pragma unroll
    for (int n = 0; n < NG; ++n) {
#pragma unroll
      for (int g = 0; g < G; ++g) sc[g][n] = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const short8_t kf = frag_row(ks, 16 * n, s, lane);
#pragma unroll
        for (int g = 0; g < G; ++g) sc[g][n] = mfma16(kf, qf[g][s], sc[g][n]);
      }
    }
    short8_t pf[G][2];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      // lane holds raw S[q][key = k0 + 16n + 4Gl + r]; masks only on boundary / diagonal
      // tiles (wave-uniform test), the softmax scale folded into the exp2 argument
      const int64_t qg0 = qblk0 + wave * 16 * G + g * 16;
      if (k0 + RK > p.Tk || (p.causal && k0 + RK - 1 > qg0)) {
        const int kl = (int)(p.Tk - k0), ql = (int)(q[g] - k0);
#pragma unroll
        for (int n = 0; n < NG; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int kk = 16 * n + 4 * Gl + r;
            if (kk >= kl || (p.causal && kk > ql)) sc[g][n][r] = -INFINITY;
          }
      }
      float mx = fmaxf(fmaxf(sc[g][0][0], sc[g][0][1]), sc[g][0][2]);
      mx = fmaxf(fmaxf(mx, sc[g][0][3]), sc[g][1][0]);
      mx = fmaxf(fmaxf(mx, sc[g][1][1]), sc[g][1][2]);
      mx = fmaxf(mx, sc[g][1][3]);
      if constexpr (NG == 4) {
        mx = fmaxf(fmaxf(mx, sc[g][NG - 2][0]), sc[g][NG - 2][1]);
        mx = fmaxf(fmaxf(mx, sc[g][NG - 2][2]), sc[g][NG - 2][3]);
        mx = fmaxf(fmaxf(mx, sc[g][NG - 1][0]), sc[g][NG - 1][1]);
        mx = fmaxf(fmaxf(mx, sc[g][NG - 1][2]), sc[g][NG - 1][3]);
      }
      mx = rowmax4(mx);
#if GVL_ATTN_FWD_V2
      // deferred rescale (T13): keep the running max while no row's max grew by more than
      // RESCALE_LOG2 (P then stays <= 2^4 before normalisation); rescale O and the row sum
      // only when some row of the wave needs it — every P of this tile is exponentiated
      // against the max the decision leaves, after the previous tile's P.V completed
      constexpr float RESCALE_LOG2 = 4.f;
      const float cand = mx * p.c2;
      if (!__all(cand - m[g] <= RESCALE_LOG2)) {
        const float mnew = fmaxf(m[g], cand);
        const float msub0 = (mnew == -INFINITY) ? 0.f : mnew;
        const float alpha = __builtin_amdgcn_exp2f(m[g] - msub0);
        m[g] = mnew;
#pragma unroll
        for (int t = 0; t < NO; ++t) o[g][t] *= alpha;
        l[g] *= alpha;
      }
      const float msub = (m[g] == -INFINITY) ? 0.f : m[g];
      float ls = 0.f;  // (dropout: the denominator counts the un-dropped probabilities)
#else
      const float mnew = fmaxf(m[g], mx * p.c2);
      const float msub = (mnew == -INFINITY) ? 0.f : mnew;
      const float alpha = __builtin_amdgcn_exp2f(m[g] - msub);
      m[g] = mnew;
      float ls = 0.f;
#endif
      const uint64_t drow = (((uint64_t)b * p.H + h) * p.Tq + (uint64_t)q[g]) * (uint64_t)p.Tk;
#pragma unroll
      for (int n = 0; n < NG; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#if GVL_ATTN_FWD_DIAG == 1
          const float e = fmaf(sc[g][n][r], p.c2, -msub) * 1e-3f;
#else
          const float e = __builtin_amdgcn_exp2f(fmaf(sc[g][n][r], p.c2, -msub));
#endif
          if (!GVL_ATTN_FWD_V2 || DROP) ls += e;
          float pe = e;
          if constexpr (DROP) {
            const int64_t key = k0 + 16 * n + 4 * Gl + r;
            pe = rng_keep(seed_, drow + (uint64_t)key, p.drop_thresh) ? e * p.drop_scale : 0.f;
          }
          sc[g][n][r] = pe;
        }
#if !GVL_ATTN_FWD_V2
      l[g] = l[g] * alpha + ls;
#pragma unroll
      for (int t = 0; t < 4; ++t) o[g][t] *= alpha;
#endif
      pf[g][0] = pack_frag(sc[g][0], sc[g][1]);
      if constexpr (NKS == 2) pf[g][1] = pack_frag(sc[g][NG - 2], sc[g][NG - 1]);
#if GVL_ATTN_FWD_V2
      if constexpr (DROP) l[g] += ls;
#endif
    }
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const short8_t vf = frag_tr<true>(vs, t, s, lane);
#pragma unroll
        for (int g = 0; g < G; ++g) o[g][t] = mfma16(vf, pf[g][s], o[g][t]);
      }
#if GVL_ATTN_FWD_V2
      if constexpr (!DROP) {
#pragma unroll
        for (int g = 0; g < G; ++g) o[g][4] = mfma16(ones, pf[g][s], o[g][4]);
      }
#endif
    }
    if (more) {
      store_rows<false, R * 4, NC>(rk, smem[ONE ? 0 : ((kt + 1) & 1)][0], tid);
      store_rows<true, R * 4, NC>(rv, smem[ONE ? 0 : ((kt + 1) & 1)][1], tid);
    }
#if GVL_ATTN_FWD_DIAG == 3
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
    __syncthreads();
#endif
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float lt = l[g];
    lt = swap32_reduce<false>(swap16_reduce<false>(lt));  // lanes l, l^16, l^32, l^48 (VALU swaps)
#if GVL_ATTN_FWD_V2
    if constexpr (!DROP) lt = o[g][4][0];
#endif
    if (!qok[g]) continue;
    const float inv = 1.f / lt;
    bf16_t* orow = p.o + b * p.o_sb + h * p.o_sh + q[g] * p.o_st;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int d = 16 * t + 4 * Gl;
      *reinterpret_cast<uint2*>(orow + d) = make_uint2(pack2(o[g][t][0] * inv, o[g][t][1] * inv),
                                                       pack2(o[g][t][2] * inv, o[g][t][3] * inv));
    }
    if (Gl == 0 && p.lse) p.lse[(b * p.H + h) * p.Tq + q[g]] = (m[g] + log2f(lt)) * LN2;
  }
  (void)l;
}


// dK/dV, LDS-DMA pipelined (Tk > 64): block = (64-key tile, head, batch); the Q / dO tiles
// and their lse / D rows move global -> LDS by buffer_load ... lds (no staging registers)
// into a 3-slot ring, two query tiles ahead of the one being computed, with counted
// vmcnt waits (PMC of the round-2 register-staged kernel: waves waiting 48 % of their cycles, LDS 5 %:
// the one-tile-ahead register prefetch did not cover the load latency).  The DMA writes each
// 64x64 tile lane-linearly in 1-KiB pieces (8 rows of 128 B); the swz_tr XOR is applied to
// the source chunk, so the image is the same as store_rows'.  Rows past Tq read zero (buffer
// bounds).  All LDS in one array (a second __shared__ object makes hipcc drain vmcnt before
// the fragment reads).
constexpr int DK_SLOT = 2 * KT * D * 2 + 2 * KT * 4;  // Q, dO tiles + lse2, D rows

// frag_tr<false> by inline asm, without a wait: hipcc treats a ds_read_b64_tr_b16 builtin as
// possibly aliasing any in-flight LDS DMA and drains vmcnt(0) in front of it.  The caller
// waits (lds_wait8) before the MFMAs use the fragments.
GVL_DEV short8_t frag_tr_asm(const char* lds, int t, int s, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ch = 2 * t + (p >> 1);
  const int ra = 32 * s + 4 * G + q, rb = ra + 16;
  const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(lds);
  const uint32_t oa = base + swz_tr(ra, ch) + (p & 1) * 8, ob = base + swz_tr(rb, ch) + (p & 1) * 8;
  short4_t lo, hi;
  // early-clobber outputs: without "&" the register allocator may put lo over ob (it did, in
  // the dQ and dK/dV kernels), and the second read then takes its address from a register the
  // first read is filling; when that read returns before the second issues (LDS queue backed
  // up), the second read fetches from a wrong LDS address — round 3's intermittent wrong dQ
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3"
               : "=&v"(lo), "=&v"(hi) : "v"(oa), "v"(ob) : "memory");
  short8_t r;
  r.lo = lo;
  r.hi = hi;
  return r;
}
// The same fragment from a per-lane address register and instruction offsets.  In frag_tr's
// layout only the lane picks the swizzled chunk ((row >> 1) & 3 is the same for rows ra,
// ra + 16 and ra + 32 s), so a tile's transposed reads need one address register per column
// block t (tr_lane) and the k-half / second row group are offsets (+4096 s, +2048).
// frag_tr_asm took two fully computed addresses per read: hipcc spent a v_add_u32 on each, 64 per
// dK/dV query tile (a quarter of that loop's vector issue cycles) and 16-32 per forward / dQ key tile.
GVL_DEV uint32_t tr_lane(const char* lds, int t, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  return (uint32_t)reinterpret_cast<uintptr_t>(lds) + swz_tr(4 * G + q, 2 * t + (p >> 1)) + (p & 1) * 8;
}
template <int OFF>  // tile offset + 4096 s (< 65536 - 2048: the ds offset field)
GVL_DEV short8_t frag_tr_imm(uint32_t a) {
  static_assert(OFF >= 0 && OFF + 2048 < 65536, "ds offset");
  short4_t lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4"
               : "=&v"(lo), "=&v"(hi) : "v"(a), "n"(OFF), "n"(OFF + 2048) : "memory");
  short8_t r;
  r.lo = lo;
  r.hi = hi;
  return r;
}
// lgkmcnt(N) with the fragments threaded through: all but this wave's N newest LDS operations
// done (LDS operations complete in order, so the fragments read before the N newest are in)
template <int N>
GVL_DEV void lds_wait_n(short8_t (&a)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]) : "n"(N) : "memory");
}
// lgkmcnt(0), with the fragments threaded through so no use is scheduled above the wait
GVL_DEV void lds_wait4(short8_t (&a)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]) : : "memory");
}
GVL_DEV void lds_wait8(short8_t (&a)[4], short8_t (&b)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]),
                 "+v"(b[3])
               :
               : "memory");
}

// Mark register fragments loaded at kernel entry as landed HERE, after the ring's first DMA
// instructions are issued: the asm takes them as inputs, so hipcc waits for their loads right
// before it (counting the younger DMAs), and its outputs are what the loop uses, so no wait is
// placed at their first use inside the loop (hipcc's count there drained the whole ring).  The
// fragment loads and the first tiles' DMAs are then one round trip, not two in a row.
template <int G>
GVL_DEV void frags_landed(short8_t (&a)[G][2], short8_t (&b)[G][2]) {
#pragma unroll
  for (int g = 0; g < G; ++g) asm volatile("" : "+v"(a[g][0]), "+v"(a[g][1]), "+v"(b[g][0]), "+v"(b[g][1]));
}

// Issue the lse and D float4 of one fragment row (ds_read_b128 at a and a + 256) without waiting;
// lds_wait_pair<N> waits until at most N of this wave's LDS operations are in flight, with the
// pair threaded through so no use is scheduled above the wait.  Early-clobber: a result must not
// land on the address register of the second read.
template <int OFF>  // byte offset of the fragment row from a (one address register per tile)
GVL_DEV void lds_pair(float4_t& l4, float4_t& d4, uint32_t a) {
  asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4"
               : "=&v"(l4), "=&v"(d4)
               : "v"(a), "n"(OFF), "n"(OFF + 256)
               : "memory");
}
template <int N>
GVL_DEV void lds_wait_pair(float4_t& l4, float4_t& d4) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(l4), "+v"(d4) : "n"(N) : "memory");
}

// G key groups of 16 per wave (64 G keys per block): every Q / dO fragment read from LDS
// (row and transposed) feeds G MFMAs.  With G = 1 a CU reads 128 KiB of fragments per block
// and query tile against 4 x 32 MFMAs per SIMD (3 blocks: LDS and MFMA pipe both ~100 %
// busy, PMC-free count from the MICROARCH LDS rates); G = 2 halves the LDS bytes per MFMA.
template <int G, bool DROP>
__global__ __launch_bounds__(NT, G == 1 ? 3 : 2) void attn_bwd_dkdv_dma_kernel(AttnP p, AttnG gg) {
  using gvl_ring::lds_void_t;
  const uint64_t seed_ = DROP ? seed_eff(p.seed, p.seed_ptr) : 0;
  __shared__ __attribute__((aligned(16))) char smem[3 * DK_SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Gl = lane >> 4;
  int64_t kt, h, b;
  tile_of_block<false>(p, (p.Tk + KT * G - 1) / (KT * G), kt, h, b);
  const int64_t kblk0 = kt * KT * G;
  const bf16_t* qbase = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* dobase = gg.dout + b * gg.do_sb + h * gg.do_sh;
  const bf16_t* kbase = p.k + b * p.k_sb + h * p.k_sh;
  const bf16_t* vbase = p.v + b * p.v_sb + h * p.v_sh;
  const int64_t rbase = (b * p.H + h) * p.Tq;
  int64_t key[G];
  bool kok[G];
  short8_t kf[G][2], vf[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    key[g] = kblk0 + wave * 16 * G + g * 16 + (lane & 15);
    kok[g] = key[g] < p.Tk;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      kf[g][s2] = load_frag_global(kbase + key[g] * p.k_st, s2, lane, kok[g]);
      vf[g][s2] = load_frag_global(vbase + key[g] * p.v_st, s2, lane, kok[g]);
    }
  }
  const int qt_first = p.causal ? (int)(kblk0 / KT) : 0;
  const int nqt = (int)((p.Tq + KT - 1) / KT);
  const int nq = nqt - qt_first;
  float4_t dk[G][4], dv[G][4];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dk[g][t] = float4_t{0.f, 0.f, 0.f, 0.f};
      dv[g][t] = float4_t{0.f, 0.f, 0.f, 0.f};
    }
  // buffer resources (bounds = the last valid row's end: rows >= Tq read zero)
  const __amdgpu_buffer_rsrc_t rq = gvl_ring::uniform_rsrc(qbase, ((p.Tq - 1) * p.q_st + D) * 2);
  const __amdgpu_buffer_rsrc_t rd = gvl_ring::uniform_rsrc(dobase, ((p.Tq - 1) * gg.do_st + D) * 2);
  const __amdgpu_buffer_rsrc_t rl = gvl_ring::uniform_rsrc(gg.Lws + rbase, p.Tq * 4);
  const __amdgpu_buffer_rsrc_t rD = gvl_ring::uniform_rsrc(gg.Dws + rbase, p.Tq * 4);
  // DMA instructions per wave per tile: 4 (+1 for waves 0 / 1: the lse / D row).  Wave w
  // issues pieces 2w, 2w+1 (rows 8j .. 8j+7) of each tile; the lane offsets include the tile
  // row q0 so they are recomputed per tile (not hoisted out of the loop and spilled).
  auto issue = [&](int qt, int slot) {
    char* sb = smem + slot * DK_SLOT;
    const int64_t q0 = (int64_t)qt * KT;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = 2 * wave + t;
      const int row = 8 * j + (lane >> 3);
      const int chunk = (lane & 7) ^ (((row >> 1) & 3) << 1);
      const int voq = (int)(((q0 + row) * p.q_st + chunk * 8) * 2);
      const int vod = (int)(((q0 + row) * gg.do_st + chunk * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, (lds_void_t*)(sb + j * 1024), 16, voq, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (lds_void_t*)(sb + KT * D * 2 + j * 1024), 16,
                                               vod, 0, 0, 0);
    }
    if (wave == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rl, (lds_void_t*)(sb + 2 * KT * D * 2), 4, lane * 4,
                                               (int)(q0 * 4), 0, 0);
    if (wave == 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rD, (lds_void_t*)(sb + 2 * KT * D * 2 + KT * 4), 4,
                                               lane * 4, (int)(q0 * 4), 0, 0);
  };
  // wait until all but the newest tile's DMA of this wave have landed (n = 1) or all (n = 0)
  auto wait_tiles = [&](int n) {
    if (n == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (wave < 2) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  };
  // the K / V fragments' loads and the first DMAs in flight together (the dropout instance
  // keeps them apart: the extra live range spills it)
  if constexpr (DROP) frags_landed<G>(kf, vf);
  if (nq > 0) {
    issue(qt_first, 0);
    if (nq > 1) issue(qt_first + 1, 1);
  }
  if constexpr (!DROP) frags_landed<G>(kf, vf);
  if (nq > 0) {
    wait_tiles(nq > 1 ? 1 : 0);
    gvl_ring::barrier_lds();
  }
  // query tiles with no mask for any of this wave's keys (all its keys < Tk and, causal, at or
  // below the tile's first query; the tile inside Tq) run a body without the mask code: with
  // causal masking only the first (diagonal) tile and a ragged last one need it
  const int64_t kw_max = kblk0 + wave * 16 * G + 16 * G - 1;  // this wave's last key
  const bool keys_in = kw_max < p.Tk;
  auto masked = [&](int i) {
    const int64_t q0 = (int64_t)(qt_first + i) * KT;
    return !keys_in || q0 + KT > p.Tq || (p.causal && kw_max > q0);
  };
  auto tile = [&](int i, auto mtag) __attribute__((always_inline)) {
    constexpr bool MASK = decltype(mtag)::value;
    const int qt = qt_first + i, st = i % 3;
    if (i + 2 < nq) issue(qt + 2, (i + 2) % 3);
    // the slot offset opaque to hipcc: otherwise it strength-reduces the slot addresses into an
    // induction pointer past the slot and every row read needs its own v_add (negative offsets)
    int soff = __builtin_amdgcn_readfirstlane(st * DK_SLOT);
    asm volatile("" : "+s"(soff));
    const char* qs = smem + soff;
    const char* ds = qs + KT * D * 2;
    const float* sl = reinterpret_cast<const float*>(qs + 2 * KT * D * 2);
    const int64_t q0 = (int64_t)qt * KT;
    float4_t sc[G][4], dp[G][4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        sc[g][n] = float4_t{0.f, 0.f, 0.f, 0.f};
        dp[g][n] = float4_t{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const short8_t qrf = frag_row(qs, 16 * n, s2, lane), drf = frag_row(ds, 16 * n, s2, lane);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          sc[g][n] = mfma16(qrf, kf[g][s2], sc[g][n]);
          dp[g][n] = mfma16(drf, vf[g][s2], dp[g][n]);
        }
      }
    }
    const int qlim = (int)(p.Tq - q0);
    short8_t pf[G][2], sf[G][2];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t kg_max = kblk0 + wave * 16 * G + g * 16 + 15;
      const bool msk = MASK && (q0 + KT > p.Tq || kg_max >= p.Tk || (p.causal && kg_max > q0));
      const int kq = (int)(key[g] - q0);
      float4_t pd[4];
      // lse / D of this lane's 4 queries per fragment row n: read by inline asm, because hipcc
      // cannot tell these bytes apart from the in-flight lse / D DMA of another slot and would
      // drain vmcnt(0) (the whole two-ahead prefetch) before a plain read; they landed before the
      // barrier.  Row n + 1's pair is issued before row n is processed, and the counted wait
      // leaves it in flight (round 4 waited for each pair with lgkmcnt(0): four exposed LDS round
      // trips per query tile; PMC r5d: waves parked 37 % of their cycles)
      float4_t lv[2], dv2[2];
      const uint32_t sla = (uint32_t)reinterpret_cast<uintptr_t>(sl + 4 * Gl);
      lds_pair<0>(lv[0], dv2[0], sla);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        if (n == 0) lds_pair<64>(lv[1], dv2[1], sla);
        if (n == 1) lds_pair<128>(lv[0], dv2[0], sla);
        if (n == 2) lds_pair<192>(lv[1], dv2[1], sla);
        if (n < 3) {
          lds_wait_pair<2>(lv[n & 1], dv2[n & 1]);
        } else {
          lds_wait_pair<0>(lv[n & 1], dv2[n & 1]);
        }
        const float4_t l4 = lv[n & 1], d4 = dv2[n & 1];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = 16 * n + 4 * Gl + r;
          const float lr = l4[r];  // lse * log2(e) (Lws)
          const float dr = d4[r];
          float pv = __builtin_amdgcn_exp2f(fmaf(sc[g][n][r], p.c2, -lr));
          if (msk && (!kok[g] || qi >= qlim || (p.causal && kq > qi))) pv = 0.f;
          float pdrop = pv, dpv = dp[g][n][r];
          if constexpr (DROP) {
            const bool keep = rng_keep(
                seed_, (uint64_t)(rbase + q0 + qi) * (uint64_t)p.Tk + (uint64_t)key[g], p.drop_thresh);
            pdrop = keep ? pv * p.drop_scale : 0.f;
            dpv = keep ? dpv * p.drop_scale : 0.f;
          }
          pd[n][r] = pdrop;
          sc[g][n][r] = pv * (dpv - dr);  // dS
        }
      }
      pf[g][0] = pack_frag(pd[0], pd[1]);
      pf[g][1] = pack_frag(pd[2], pd[3]);
      sf[g][0] = pack_frag(sc[g][0], sc[g][1]);
      sf[g][1] = pack_frag(sc[g][2], sc[g][3]);
    }
    uint32_t ta[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) ta[t] = tr_lane(qs, t, lane);
    auto half = [&](auto s2c) __attribute__((always_inline)) {
      constexpr int s2 = decltype(s2c)::value;
      short8_t dof[4], qtf[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        dof[t] = frag_tr_imm<KT * D * 2 + 4096 * s2>(ta[t]);
        qtf[t] = frag_tr_imm<4096 * s2>(ta[t]);
      }
      lds_wait8(dof, qtf);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) {
          dv[g][t] = mfma16(dof[t], pf[g][s2], dv[g][t]);
          dk[g][t] = mfma16(qtf[t], sf[g][s2], dk[g][t]);
        }
    };
    half(std::integral_constant<int, 0>{});
    half(std::integral_constant<int, 1>{});
    if (i + 1 < nq) wait_tiles(i + 2 < nq ? 1 : 0);
    gvl_ring::barrier_lds();  // slot st is refilled by iteration i+1's issue
    };
  for (int i = 0; i < nq; ++i) {
    if (masked(i)) tile(i, std::true_type{});
    else tile(i, std::false_type{});
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (!kok[g]) continue;
    bf16_t* dkr = gg.dk + b * gg.dk_sb + h * gg.dk_sh + key[g] * gg.dk_st;
    bf16_t* dvr = gg.dv + b * gg.dv_sb + h * gg.dv_sh + key[g] * gg.dv_st;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int d = 16 * t + 4 * Gl;
      *reinterpret_cast<uint2*>(dkr + d) =
          make_uint2(pack2(dk[g][t][0] * p.scale, dk[g][t][1] * p.scale),
                     pack2(dk[g][t][2] * p.scale, dk[g][t][3] * p.scale));
      *reinterpret_cast<uint2*>(dvr + d) =
          make_uint2(pack2(dv[g][t][0], dv[g][t][1]), pack2(dv[g][t][2], dv[g][t][3]));
    }
  }
}

// dQ, LDS-DMA pipelined (Tq > 64): block = (64*G-query tile, head, batch), each wave G groups
// of 16 query rows; the K / V tiles move global -> LDS by buffer_load ... lds into a 3-slot ring two key tiles ahead (as
// attn_bwd_dkdv_dma_kernel; transposed K reads by inline asm for the same reason).
// It also computes D = rowsum(dO * O) (no separate pre-pass launch): each lane holds 16 of
// its row's 64 dO values as MFMA fragments, loads the matching O values, and the row's four
// lanes reduce by two shuffles; D goes to the workspace for the dK/dV kernel that runs next.
// (Round 3's first version of this gave intermittently wrong dQ; the cause was frag_tr_asm's
// missing early-clobber — see there — which the fused variant's timing exposed.)
template <int G, bool DROP>
__global__ __launch_bounds__(NT, 2) void attn_bwd_dq_dma_kernel(AttnP p, AttnG gg) {
  using gvl_ring::lds_void_t;
  const uint64_t seed_ = DROP ? seed_eff(p.seed, p.seed_ptr) : 0;
  constexpr int QT = 64 * G, SLOT = 2 * KT * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[3 * SLOT];  // [slot][K, V]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Gl = lane >> 4;
  int64_t qt, h, b;
  tile_of_block<true>(p, (p.Tq + QT - 1) / QT, qt, h, b);
  const int64_t qblk0 = qt * QT;
  const bf16_t* qbase = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* dobase = gg.dout + b * gg.do_sb + h * gg.do_sh;
  const bf16_t* kbase = p.k + b * p.k_sb + h * p.k_sh;
  const bf16_t* vbase = p.v + b * p.v_sb + h * p.v_sh;
  int64_t q[G];
  bool qok[G];
  short8_t qf[G][2], df[G][2];
  float lse2[G], Dq[G];
  uint64_t drow[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    q[g] = qblk0 + wave * 16 * G + g * 16 + (lane & 15);
    qok[g] = q[g] < p.Tq;
    // branch-free (rows past Tq read row 0; their dQ is never stored and a query row's dQ
    // depends on that row alone), so hipcc issues every prologue load back to back: the
    // conditional forms cost four dependent round trips before the first DMA
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      qf[g][s2] = load_frag_global_nb(qbase, p.q_st, (int)q[g], s2, lane, qok[g]);
      df[g][s2] = load_frag_global_nb(dobase, gg.do_st, (int)q[g], s2, lane, qok[g]);
    }
    const int64_t ridx = (b * p.H + h) * p.Tq + q[g];
    const float lraw = p.lse[qok[g] ? ridx : (b * p.H + h) * p.Tq];
    lse2[g] = qok[g] ? lraw * LOG2E : 0.f;
    drow[g] = (uint64_t)ridx * (uint64_t)p.Tk;
  }
  int64_t kend = p.Tk;
  if (p.causal) {
    const int64_t lim = qblk0 + QT;
    if (lim < kend) kend = lim;
  }
  const int nkt = (int)((kend + KT - 1) / KT);
  float4_t acc[G][4];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[g][t] = float4_t{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rk = gvl_ring::uniform_rsrc(kbase, ((p.Tk - 1) * p.k_st + D) * 2);
  const __amdgpu_buffer_rsrc_t rv = gvl_ring::uniform_rsrc(vbase, ((p.Tk - 1) * p.v_st + D) * 2);
  auto issue = [&](int kt, int slot) {  // 4 DMA instructions per wave
    char* sb = smem + slot * SLOT;
    const int64_t k0 = (int64_t)kt * KT;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = 2 * wave + t;
      const int row = 8 * j + (lane >> 3);
      const int chunk = (lane & 7) ^ (((row >> 1) & 3) << 1);
      const int vok = (int)(((k0 + row) * p.k_st + chunk * 8) * 2);
      const int vov = (int)(((k0 + row) * p.v_st + chunk * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_void_t*)(sb + j * 1024), 16, vok, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_void_t*)(sb + KT * D * 2 + j * 1024), 16,
                                               vov, 0, 0, 0);
    }
  };
  if (nkt > 0) {
    issue(0, 0);
    if (nkt > 1) issue(1, 1);
  }
  // D = rowsum(dO * O), after the first DMAs are issued (O / dO land under them): this lane's
  // 16 dims (8 at 32 s2 + 8 Gl, s2 = 0, 1), then the row's 4 lanes
  {
    const bf16_t* obase = p.o + b * p.o_sb + h * p.o_sh;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float sd = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const short8_t of = load_frag_global_nb(obase, p.o_st, (int)q[g], s2, lane, qok[g]);
        const uint4 ou = __builtin_bit_cast(uint4, of), du = __builtin_bit_cast(uint4, df[g][s2]);
        const uint32_t ow[4] = {ou.x, ou.y, ou.z, ou.w}, dw[4] = {du.x, du.y, du.z, du.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) sd += lo_bf(ow[k]) * lo_bf(dw[k]) + hi_bf(ow[k]) * hi_bf(dw[k]);
      }
      sd = swap32_reduce<false>(swap16_reduce<false>(sd));  // the row's 4 lanes (VALU swaps)
      Dq[g] = qok[g] ? sd : 0.f;
    }
  }
  frags_landed<G>(qf, df);
#pragma unroll
  for (int g = 0; g < G; ++g) asm volatile("" : "+v"(lse2[g]));
  if (nkt > 0) {
    if (nkt > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    gvl_ring::barrier_lds();
  }
  // key tiles with no mask for any of this wave's query groups run a body without the mask
  // code (as attn_fwd_dma_kernel)
  const int64_t qw0 = qblk0 + wave * 16 * G;
  int nfull = (int)(p.Tk / KT);
  if (p.causal) nfull = (int)((qw0 + 1) / KT) < nfull ? (int)((qw0 + 1) / KT) : nfull;
  nfull = nfull < nkt ? nfull : nkt;
  auto tile = [&](int kt, auto mtag) __attribute__((always_inline)) {
    constexpr bool MASK = decltype(mtag)::value;
    if (kt + 2 < nkt) issue(kt + 2, (kt + 2) % 3);
    const char* ks = smem + (kt % 3) * SLOT;
    const char* vs = ks + KT * D * 2;
    const int64_t k0 = (int64_t)kt * KT;
    float4_t sc[G][4], dp[G][4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        sc[g][n] = float4_t{0.f, 0.f, 0.f, 0.f};
        dp[g][n] = float4_t{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const short8_t kf = frag_row(ks, 16 * n, s2, lane);
        const short8_t vf = frag_row(vs, 16 * n, s2, lane);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          sc[g][n] = mfma16(kf, qf[g][s2], sc[g][n]);
          dp[g][n] = mfma16(vf, df[g][s2], dp[g][n]);
        }
      }
    }
    short8_t sf[G][2];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t qg0 = qblk0 + wave * 16 * G + g * 16;
      const bool msk = MASK && (k0 + KT > p.Tk || (p.causal && k0 + KT - 1 > qg0));
      const int kl = (int)(p.Tk - k0), ql = (int)(q[g] - k0);
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kk = 16 * n + 4 * Gl + r;
          float pv = __builtin_amdgcn_exp2f(fmaf(sc[g][n][r], p.c2, -lse2[g]));
          if (msk && (kk >= kl || (p.causal && kk > ql))) pv = 0.f;
          float dpv = dp[g][n][r];
          if constexpr (DROP)
            dpv = rng_keep(seed_, drow[g] + (uint64_t)(k0 + kk), p.drop_thresh) ? dpv * p.drop_scale : 0.f;
          sc[g][n][r] = pv * (dpv - Dq[g]);  // dS
        }
      sf[g][0] = pack_frag(sc[g][0], sc[g][1]);
      sf[g][1] = pack_frag(sc[g][2], sc[g][3]);
    }
    // K^T fragments of both k-halves issued before the first half's MFMAs (+16 VGPRs; the
    // kernel is at 2 waves per SIMD either way)
    // (issue order: the k-half 0 reads first — lds_wait_n<8> below counts on it)
    short8_t kta[2][4];
    uint32_t ta[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) ta[t] = tr_lane(ks, t, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) kta[0][t] = frag_tr_imm<0>(ta[t]);
#pragma unroll
    for (int t = 0; t < 4; ++t) kta[1][t] = frag_tr_imm<4096>(ta[t]);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      short8_t (&kt4)[4] = kta[s2];
      if (s2 == 0) lds_wait_n<8>(kt4); else lds_wait4(kt4);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g][t] = mfma16(kt4[t], sf[g][s2], acc[g][t]);
    }
    if (kt + 1 < nkt) {
      if (kt + 2 < nkt) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    gvl_ring::barrier_lds();
    };
  int kt = 0;
  for (; kt < nfull; ++kt) tile(kt, std::false_type{});
  for (; kt < nkt; ++kt) tile(kt, std::true_type{});
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (!qok[g]) continue;
    if (Gl == 0) {  // read by the dK/dV kernel
      gg.Dws[(b * p.H + h) * p.Tq + q[g]] = Dq[g];
      gg.Lws[(b * p.H + h) * p.Tq + q[g]] = lse2[g];
    }
    bf16_t* dst = gg.dq + b * gg.dq_sb + h * gg.dq_sh + q[g] * gg.dq_st;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int d = 16 * t + 4 * Gl;
      *reinterpret_cast<uint2*>(dst + d) =
          make_uint2(pack2(acc[g][t][0] * p.scale, acc[g][t][1] * p.scale),
                     pack2(acc[g][t][2] * p.scale, acc[g][t][3] * p.scale));
    }
  }
}

// Forward, LDS-DMA pipelined (no dropout, more than one key tile: the LM's T = 1024): the
// query tile stays in registers while the K / V tiles stream global -> LDS by buffer_load ...
// lds into a 3-slot ring two key tiles ahead (attn_bwd_dq_dma_kernel's ring: same 1-KiB
// pieces, source-side swizzle, counted vmcnt), instead of attn_fwd_kernel's register staging
// one tile ahead (its timing-only build without the staging ran 18 % faster).  V is read
// transposed by frag_tr_asm (a builtin transposed read would make hipcc drain the DMA queue).
// Math as attn_fwd_kernel<G, false> (deferred rescale, the row sum from a ones MFMA).
template <int G>
__global__ __launch_bounds__(NT, 2) void attn_fwd_dma_kernel(AttnP p) {
  using gvl_ring::lds_void_t;
  constexpr int QT = 64 * G, SLOT = 2 * KT * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[3 * SLOT];  // [slot][K, V]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Gl = lane >> 4;
  int64_t qt, h, b;
  tile_of_block<true>(p, (p.Tq + QT - 1) / QT, qt, h, b);
  const int64_t qblk0 = qt * QT;
  const bf16_t* qbase = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kbase = p.k + b * p.k_sb + h * p.k_sh;
  const bf16_t* vbase = p.v + b * p.v_sb + h * p.v_sh;
  int64_t q[G];
  bool qok[G];
  short8_t qf[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    q[g] = qblk0 + wave * 16 * G + g * 16 + (lane & 15);
    qok[g] = q[g] < p.Tq;
    qf[g][0] = load_frag_global(qbase + q[g] * p.q_st, 0, lane, qok[g]);
    qf[g][1] = load_frag_global(qbase + q[g] * p.q_st, 1, lane, qok[g]);
  }
  int64_t kend = p.Tk;
  if (p.causal) {
    const int64_t lim = qblk0 + QT;
    if (lim < kend) kend = lim;
  }
  const int nkt = (int)((kend + KT - 1) / KT);
  constexpr int NO = 5;  // o[g][4]: row sum of the bf16 P (ones MFMA)
  float4_t o[G][NO];
  float m[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int t = 0; t < NO; ++t) o[g][t] = float4_t{0.f, 0.f, 0.f, 0.f};
    m[g] = -INFINITY;
  }
  short8_t ones;
#pragma unroll
  for (int k = 0; k < 8; ++k) ones[k] = (short)0x3F80;  // bf16 1.0
  const __amdgpu_buffer_rsrc_t rk = gvl_ring::uniform_rsrc(kbase, ((p.Tk - 1) * p.k_st + D) * 2);
  const __amdgpu_buffer_rsrc_t rv = gvl_ring::uniform_rsrc(vbase, ((p.Tk - 1) * p.v_st + D) * 2);
  auto issue = [&](int kt, int slot) {  // 4 DMA instructions per wave
    char* sb = smem + slot * SLOT;
    const int64_t k0 = (int64_t)kt * KT;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = 2 * wave + t;
      const int row = 8 * j + (lane >> 3);
      const int chunk = (lane & 7) ^ (((row >> 1) & 3) << 1);
      const int vok = (int)(((k0 + row) * p.k_st + chunk * 8) * 2);
      const int vov = (int)(((k0 + row) * p.v_st + chunk * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_void_t*)(sb + j * 1024), 16, vok, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_void_t*)(sb + KT * D * 2 + j * 1024), 16,
                                               vov, 0, 0, 0);
    }
  };
  if (nkt > 0) {
    issue(0, 0);
    if (nkt > 1) issue(1, 1);
  }
#pragma unroll
  for (int g = 0; g < G; ++g) asm volatile("" : "+v"(qf[g][0]), "+v"(qf[g][1]));  // (frags_landed)
  if (nkt > 0) {
    if (nkt > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    gvl_ring::barrier_lds();
  }
  // Key tiles that need no mask for any of this wave's query groups (inside Tk, and at or below
  // the wave's first query) run a body compiled without the mask code: hipcc hoisted the
  // boundary compares of the masked branch above it, 16 v_cmp per group on EVERY tile (PMC r5d:
  // ~230 VALU instructions per wave and tile, the softmax's VALU half the SIMD's cycles)
  const int64_t qw0 = qblk0 + wave * 16 * G;
  int nfull = (int)(p.Tk / KT);
  if (p.causal) nfull = (int)((qw0 + 1) / KT) < nfull ? (int)((qw0 + 1) / KT) : nfull;
  nfull = nfull < nkt ? nfull : nkt;
  auto tile = [&](int kt, auto mtag) __attribute__((always_inline)) {
    constexpr bool MASK = decltype(mtag)::value;
    if (kt + 2 < nkt) issue(kt + 2, (kt + 2) % 3);
    const char* ks = smem + (kt % 3) * SLOT;  // V: the tile at + KT * D * 2
    const int64_t k0 = (int64_t)kt * KT;
    float4_t sc[G][4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int g = 0; g < G; ++g) sc[g][n] = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const short8_t kf = frag_row(ks, 16 * n, s2, lane);
#pragma unroll
        for (int g = 0; g < G; ++g) sc[g][n] = mfma16(kf, qf[g][s2], sc[g][n]);
      }
    }
    short8_t pf[G][2];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t qg0 = qblk0 + wave * 16 * G + g * 16;
      if (MASK && (k0 + KT > p.Tk || (p.causal && k0 + KT - 1 > qg0))) {
        const int kl = (int)(p.Tk - k0), ql = (int)(q[g] - k0);
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int kk = 16 * n + 4 * Gl + r;
            if (kk >= kl || (p.causal && kk > ql)) sc[g][n][r] = -INFINITY;
          }
      }
      float mx = fmaxf(fmaxf(sc[g][0][0], sc[g][0][1]), sc[g][0][2]);
      mx = fmaxf(fmaxf(mx, sc[g][0][3]), sc[g][1][0]);
      mx = fmaxf(fmaxf(mx, sc[g][1][1]), sc[g][1][2]);
      mx = fmaxf(fmaxf(mx, sc[g][1][3]), sc[g][2][0]);
      mx = fmaxf(fmaxf(mx, sc[g][2][1]), sc[g][2][2]);
      mx = fmaxf(fmaxf(mx, sc[g][2][3]), sc[g][3][0]);
      mx = fmaxf(fmaxf(mx, sc[g][3][1]), sc[g][3][2]);
      mx = fmaxf(mx, sc[g][3][3]);
      mx = rowmax4(mx);
      constexpr float RESCALE_LOG2 = 4.f;  // deferred rescale, as attn_fwd_kernel
      const float cand = mx * p.c2;
      if (!__all(cand - m[g] <= RESCALE_LOG2)) {
        const float mnew = fmaxf(m[g], cand);
        const float msub0 = (mnew == -INFINITY) ? 0.f : mnew;
        const float alpha = __builtin_amdgcn_exp2f(m[g] - msub0);
        m[g] = mnew;
#pragma unroll
        for (int t = 0; t < NO; ++t) o[g][t] *= alpha;
      }
      const float msub = (m[g] == -INFINITY) ? 0.f : m[g];
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[g][n][r] = __builtin_amdgcn_exp2f(fmaf(sc[g][n][r], p.c2, -msub));
      pf[g][0] = pack_frag(sc[g][0], sc[g][1]);
      pf[g][1] = pack_frag(sc[g][2], sc[g][3]);
    }
    // V fragments of both k-halves issued before the first half's MFMAs (the second half's
    // LDS latency hides behind them; +16 VGPRs, still 3 waves per SIMD)
    // (issue order: the k-half 0 reads first — lds_wait_n<8> below counts on it)
    short8_t vfa[2][4];
    uint32_t ta[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) ta[t] = tr_lane(ks, t, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) vfa[0][t] = frag_tr_imm<KT * D * 2>(ta[t]);
#pragma unroll
    for (int t = 0; t < 4; ++t) vfa[1][t] = frag_tr_imm<KT * D * 2 + 4096>(ta[t]);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      short8_t (&vf)[4] = vfa[s2];
      if (s2 == 0) lds_wait_n<8>(vf); else lds_wait4(vf);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) o[g][t] = mfma16(vf[t], pf[g][s2], o[g][t]);
#pragma unroll
      for (int g = 0; g < G; ++g) o[g][4] = mfma16(ones, pf[g][s2], o[g][4]);
    }
    if (kt + 1 < nkt) {
      if (kt + 2 < nkt) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    gvl_ring::barrier_lds();
    };
  int kt = 0;
  for (; kt < nfull; ++kt) tile(kt, std::false_type{});
  for (; kt < nkt; ++kt) tile(kt, std::true_type{});
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float lt = o[g][4][0];
    if (!qok[g]) continue;
    const float inv = 1.f / lt;
    bf16_t* orow = p.o + b * p.o_sb + h * p.o_sh + q[g] * p.o_st;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int d = 16 * t + 4 * Gl;
      *reinterpret_cast<uint2*>(orow + d) = make_uint2(pack2(o[g][t][0] * inv, o[g][t][1] * inv),
                                                       pack2(o[g][t][2] * inv, o[g][t][3] * inv));
    }
    if (Gl == 0 && p.lse) p.lse[(b * p.H + h) * p.Tq + q[g]] = (m[g] + log2f(lt)) * LN2;
  }
}

// Short sequences (Tq, Tk <= 64: the caption decoder's 63 tokens, the Q-Former's 32 queries
// over 32 / 33 tokens): the whole backward of one (b, h) in one block, no recompute.
// Q, K, V, dO land in LDS once; phase 1 (wave w = queries 16w..16w+15) computes D = rowsum(dO O),
// S, P, dP, dS exactly as the dQ kernel, writes dQ, and leaves P (dropped) and dS in LDS as
// [query][key] tiles; phase 2 (wave w = keys 16w..16w+15) reads them transposed
// (ds_read_b64_tr_b16 gives the same permuted k-slot order as the dK/dV kernel's registers) for
// dV = P^T dO and dK = dS^T Q.  One launch instead of three, and S / dP computed once.
// GVL_ATTN_SHORT_LDS32 (default 1): P and dS are written over the V and K tiles once every wave
// is past its last K / V read (one more barrier), so a block needs 32 KiB of LDS instead of
// 48: five blocks per CU instead of three (1536 (b, h) blocks: 1.2 rounds instead of 2).
#ifndef GVL_ATTN_SHORT_LDS32
#define GVL_ATTN_SHORT_LDS32 1
#endif
// GVL_ATTN_SHORT_DIAG=1: timing-only build of the short backward (wrong results; never the shipped
// library): every load, then dQ / dK / dV stores of the loaded bytes — the kernel's memory floor.
#ifndef GVL_ATTN_SHORT_DIAG
#define GVL_ATTN_SHORT_DIAG 0
#endif
template <int NCK>
struct ShortIn {  // one (b, h)'s operands of the short backward, loaded ahead of its math
  uint4 rq[2], rk[NCK], rv[NCK], rd[2], oa[2];
  float lse_raw;
};
template <bool DROP, int R, int RK>
GVL_DEV void bwd_short_load(const AttnP& p, const AttnG& gg, int64_t bh, ShortIn<2 * RK / R>& in) {
  constexpr int NCK = 2 * RK / R;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Gl = lane >> 4;
  const int64_t b = bh / p.H, h = bh - b * p.H;
  const bf16_t* qbase = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kbase = p.k + b * p.k_sb + h * p.k_sh;
  const bf16_t* vbase = p.v + b * p.v_sb + h * p.v_sh;
  const bf16_t* obase = p.o + b * p.o_sb + h * p.o_sh;
  const bf16_t* dobase = gg.dout + b * gg.do_sb + h * gg.do_sh;
  // every global operand of the (b, h) issued before the first wait (branch-free loads)
  const int ql = wave * 16 + (lane & 15);
  const bool qok = ql < p.Tq;
  const int qlc = qok ? ql : 0;
  load_rows_nb<R * 4>(in.rq, qbase, p.q_st, p.Tq, tid);
  load_rows_nb<R * 4, NCK>(in.rk, kbase, p.k_st, p.Tk, tid);
  load_rows_nb<R * 4, NCK>(in.rv, vbase, p.v_st, p.Tk, tid);
  load_rows_nb<R * 4>(in.rd, dobase, gg.do_st, p.Tq, tid);
#pragma unroll
  for (int c = 0; c < 2; ++c) in.oa[c] = reinterpret_cast<const uint4*>(obase + qlc * p.o_st + 16 * Gl)[c];
  in.lse_raw = p.lse[bh * p.Tq + qlc];
}

// One (b, h) of the short backward from its loaded operands (bwd_short_load); smem: the Q / dO
// tiles of R rows, the K / V tiles of RK rows, and P / dS ([query][key], R rows) over V / K (L32)
// or after them.  R = RK = 64: 4 waves (16 queries / keys each); R = 32 (Tq <= 32): 2 waves over
// 32-row query tiles, each wave taking RK / 32 key groups of 16 in phase 2; RK = 32 (Tk <= 32):
// one 32-deep k-step over the keys where 64 take two.
template <bool DROP, int R, int RK>
GVL_DEV void bwd_short_item(const AttnP& p, const AttnG& gg, int64_t bh, const ShortIn<2 * RK / R>& in,
                            char* smem0, uint64_t seed_) {
  static_assert((R == 64 && RK == 64) || (R == 32 && (RK == 32 || RK == 64)), "short tile rows");
  constexpr bool L32 = GVL_ATTN_SHORT_LDS32;
  constexpr int TQ = R * D * 2, TK = RK * D * 2;
  constexpr int NG = RK / 16, NKS = RK / 32;  // key groups of 16, 32-deep k-steps over the keys
  constexpr int NQS = R / 32, KPW = RK / R;   // k-steps over the queries; key groups per wave
  constexpr int NCK = 2 * RK / R;
  char* const qs = smem0;
  char* const ks = smem0 + TQ;
  char* const vs = smem0 + TQ + TK;
  char* const ds = smem0 + TQ + 2 * TK;
  char* const ps = L32 ? vs : smem0 + 2 * TQ + 2 * TK;       // (L32: over V)
  char* const ss = L32 ? ks : smem0 + 3 * TQ + 2 * TK;       // (L32: over K)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Gl = lane >> 4;
  const int64_t b = bh / p.H, h = bh - b * p.H;
  const int ql = wave * 16 + (lane & 15);
  const bool qok = ql < p.Tq;
  const int64_t ridx = bh * p.Tq + ql;
  const uint4 (&rq)[2] = in.rq, (&rk)[NCK] = in.rk, (&rv)[NCK] = in.rv, (&rd)[2] = in.rd;
  const uint4 (&oa)[2] = in.oa;
  const float lse_raw = in.lse_raw;
  if constexpr (GVL_ATTN_SHORT_DIAG == 1 && R == RK) {  // timing-only: the loads, then stores of the same bytes
    uint32_t x = in.oa[0].x ^ in.oa[1].y ^ __float_as_uint(lse_raw);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int row = (tid >> 3) + (R / 2) * it, ch = tid & 7;
      if (row < p.Tq) {
        *reinterpret_cast<uint4*>(gg.dq + b * gg.dq_sb + h * gg.dq_sh + row * gg.dq_st + ch * 8) = rq[it] ^ make_uint4(x, x, x, x);
        *reinterpret_cast<uint4*>(gg.dk + b * gg.dk_sb + h * gg.dk_sh + row * gg.dk_st + ch * 8) = rk[it] ^ rd[it];
        *reinterpret_cast<uint4*>(gg.dv + b * gg.dv_sb + h * gg.dv_sh + row * gg.dv_st + ch * 8) = rv[it];
      }
    }
    return;
  }
  store_rows<false, R * 4>(rq, qs, tid);
  store_rows<false, R * 4, NCK>(rk, ks, tid);
  store_rows<false, R * 4, NCK>(rv, vs, tid);
  store_rows<false, R * 4>(rd, ds, tid);
  __syncthreads();
  // this lane's Q / dO fragments and dO row piece from the LDS tiles (rows past Tq hold row 0,
  // as load_rows_nb staged them: the data the global fragment loads used to fetch)
  short8_t qf[2], df[2];
  uint4 da[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    qf[s2] = frag_row(qs, 16 * wave, s2, lane);
    df[s2] = frag_row(ds, 16 * wave, s2, lane);
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) da[c] = *reinterpret_cast<const uint4*>(ds + swz_row(ql, 2 * Gl + c));
  // phase 1: this lane's query, its D (4 lanes x 16 dims of dO . O) and log-sum-exp
  float Dq = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const uint4 a = oa[c], d = da[c];
    Dq += lo_bf(a.x) * lo_bf(d.x) + hi_bf(a.x) * hi_bf(d.x) + lo_bf(a.y) * lo_bf(d.y) +
          hi_bf(a.y) * hi_bf(d.y) + lo_bf(a.z) * lo_bf(d.z) + hi_bf(a.z) * hi_bf(d.z) +
          lo_bf(a.w) * lo_bf(d.w) + hi_bf(a.w) * hi_bf(d.w);
  }
  if (!qok) Dq = 0.f;
  const float lse2 = qok ? lse_raw * LOG2E : 0.f;
  Dq = swap32_reduce<false>(swap16_reduce<false>(Dq));  // the row's 4 lanes (VALU swaps)
  float4_t sc[NG], dp[NG];
#pragma unroll
  for (int n = 0; n < NG; ++n) {
    sc[n] = float4_t{0.f, 0.f, 0.f, 0.f};
    dp[n] = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      sc[n] = mfma16(frag_row(ks, 16 * n, s2, lane), qf[s2], sc[n]);
      dp[n] = mfma16(frag_row(vs, 16 * n, s2, lane), df[s2], dp[n]);
    }
  }
  const uint64_t drow0 = (uint64_t)ridx * (uint64_t)p.Tk;
  float4_t pd[NG];
#pragma unroll
  for (int n = 0; n < NG; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kk = 16 * n + 4 * Gl + r;
      float pv = __builtin_amdgcn_exp2f(fmaf(sc[n][r], p.c2, -lse2));
      if (!qok || kk >= p.Tk || (p.causal && kk > ql)) pv = 0.f;
      float pdrop = pv, dpv = dp[n][r];
      if constexpr (DROP) {
        const bool keep = rng_keep(seed_, drow0 + (uint64_t)kk, p.drop_thresh);
        pdrop = keep ? pv * p.drop_scale : 0.f;
        dpv = keep ? dpv * p.drop_scale : 0.f;
      }
      pd[n][r] = pdrop;
      sc[n][r] = pv * (dpv - Dq);  // dS
    }
  // P and dS to LDS as [query][key]: lane (query ql) owns keys 16n + 4Gl .. +3 (8 bytes)
  uint2 pw[NG], sw[NG];
#pragma unroll
  for (int n = 0; n < NG; ++n) {
    pw[n] = make_uint2(pack2(pd[n][0], pd[n][1]), pack2(pd[n][2], pd[n][3]));
    sw[n] = make_uint2(pack2(sc[n][0], sc[n][1]), pack2(sc[n][2], sc[n][3]));
  }
  auto store_p_ds = [&]() {
#pragma unroll
    for (int n = 0; n < NG; ++n) {
      const int off = swz_tr(ql, 2 * n + (Gl >> 1)) + (Gl & 1) * 8;
      *reinterpret_cast<uint2*>(ps + off) = pw[n];
      *reinterpret_cast<uint2*>(ss + off) = sw[n];
    }
  };
  if constexpr (!L32) store_p_ds();
  {  // dQ = dS K (lane-local dS fragments, K read transposed)
    const short8_t sf0 = pack_frag(sc[0], sc[1]);
    const short8_t sf1 = NKS == 2 ? pack_frag(sc[NG - 2], sc[NG - 1]) : sf0;
    float4_t acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t] = mfma16(frag_tr<false>(ks, t, 0, lane), sf0, float4_t{0.f, 0.f, 0.f, 0.f});
      if constexpr (NKS == 2) acc[t] = mfma16(frag_tr<false>(ks, t, 1, lane), sf1, acc[t]);
    }
    if (qok) {
      bf16_t* dst = gg.dq + b * gg.dq_sb + h * gg.dq_sh + ql * gg.dq_st;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        *reinterpret_cast<uint2*>(dst + 16 * t + 4 * Gl) =
            make_uint2(pack2(acc[t][0] * p.scale, acc[t][1] * p.scale),
                       pack2(acc[t][2] * p.scale, acc[t][3] * p.scale));
    }
  }
  if constexpr (L32) {  // every wave past its K / V reads, then P / dS over them
    __syncthreads();
    store_p_ds();
  }
  __syncthreads();
  // phase 2: this lane's key (key groups wave, wave + R / 16 when RK > R); P^T / dS^T fragments
  // in the dK/dV kernel's k-slot order
#pragma unroll
  for (int j = 0; j < KPW; ++j) {
    const int kg = wave + (R / 16) * j, kl = kg * 16 + (lane & 15);
    float4_t dk[4], dv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dk[t] = float4_t{0.f, 0.f, 0.f, 0.f};
      dv[t] = float4_t{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s2 = 0; s2 < NQS; ++s2) {
      const short8_t pf = frag_tr<false>(ps, kg, s2, lane);
      const short8_t sf = frag_tr<false>(ss, kg, s2, lane);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        dv[t] = mfma16(frag_tr<false>(ds, t, s2, lane), pf, dv[t]);
        dk[t] = mfma16(frag_tr<false>(qs, t, s2, lane), sf, dk[t]);
      }
    }
    if (kl < p.Tk) {
      bf16_t* dkr = gg.dk + b * gg.dk_sb + h * gg.dk_sh + kl * gg.dk_st;
      bf16_t* dvr = gg.dv + b * gg.dv_sb + h * gg.dv_sh + kl * gg.dv_st;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int d = 16 * t + 4 * Gl;
        *reinterpret_cast<uint2*>(dkr + d) =
            make_uint2(pack2(dk[t][0] * p.scale, dk[t][1] * p.scale),
                       pack2(dk[t][2] * p.scale, dk[t][3] * p.scale));
        *reinterpret_cast<uint2*>(dvr + d) =
            make_uint2(pack2(dv[t][0], dv[t][1]), pack2(dv[t][2], dv[t][3]));
      }
    }
  }
}

// (Round 6 measured two (b, h) per block, the second one's loads issued before the first one's
// math, at 3 waves per SIMD: no faster — T = 63 0.023-0.024 vs 0.023 ms, T = 32 with dropout
// 0.020 vs 0.018 ms; Q-Former / cross / linear steps 0.1-0.9 % slower; profiles/r6/
// attn_short_pair_r6d.txt — and was removed.)
// R = 32 (Tq, Tk <= 32: the cross-att decoder's 31-token self-attention, the Q-Former bridge's
// 32 queries): 2 waves and 16 KiB of LDS per (b, h) instead of 4 waves over 64-row tiles half of
// whose rows and waves were padding (5 blocks per CU by LDS -> 10).
template <bool DROP, int R = 64, int RK = R>
__global__ __launch_bounds__(R * 4, R == 64 ? 2 : (RK > R ? 3 : 5)) void attn_bwd_short_kernel(AttnP p, AttnG gg) {
  const uint64_t seed_ = DROP ? seed_eff(p.seed, p.seed_ptr) : 0;
  constexpr bool L32 = GVL_ATTN_SHORT_LDS32;
  __shared__ __attribute__((aligned(16))) char smem[(L32 ? 2 : 4) * R * D * 2 + 2 * RK * D * 2];
  ShortIn<2 * RK / R> in;
  bwd_short_load<DROP, R, RK>(p, gg, blockIdx.x, in);
  bwd_short_item<DROP, R, RK>(p, gg, blockIdx.x, in, smem, seed_);
}

int fill(const gvl_attn_desc* d, AttnP& p) {
  GVL_REQUIRE(d && d->q && d->k && d->v && d->o, "gvl_attn: null tensor");
  GVL_REQUIRE(d->B > 0 && d->H > 0 && d->Tq > 0 && d->Tk > 0, "gvl_attn: empty shape");
  GVL_REQUIRE(d->B * d->H * ((std::max(d->Tq, d->Tk) + 63) / 64) < ((int64_t)1 << 31),
              "gvl_attn: B*H*tiles too large for one grid");
  const int64_t st[] = {d->q_sb, d->q_st, d->q_sh, d->k_sb, d->k_st, d->k_sh,
                        d->v_sb, d->v_st, d->v_sh, d->o_sb, d->o_st, d->o_sh};
  for (int64_t s : st) GVL_REQUIRE(s % 8 == 0, "gvl_attn: strides must be multiples of 8 elements");
  GVL_REQUIRE(gvl::aligned16(d->q) && gvl::aligned16(d->k) && gvl::aligned16(d->v) &&
                  gvl::aligned16(d->o),
              "gvl_attn: tensors must be 16-byte aligned");
  GVL_REQUIRE(d->drop_p >= 0.f && d->drop_p < 1.f, "gvl_attn: drop_p out of range");
  p.q = static_cast<const bf16_t*>(d->q);
  p.k = static_cast<const bf16_t*>(d->k);
  p.v = static_cast<const bf16_t*>(d->v);
  p.o = static_cast<bf16_t*>(d->o);
  p.lse = d->lse;
  p.B = d->B; p.H = d->H; p.Tq = d->Tq; p.Tk = d->Tk;
  p.q_sb = d->q_sb; p.q_st = d->q_st; p.q_sh = d->q_sh;
  p.k_sb = d->k_sb; p.k_st = d->k_st; p.k_sh = d->k_sh;
  p.v_sb = d->v_sb; p.v_st = d->v_st; p.v_sh = d->v_sh;
  p.o_sb = d->o_sb; p.o_st = d->o_st; p.o_sh = d->o_sh;
  p.causal = d->causal;
  p.scale = d->scale;
  p.c2 = d->scale * LOG2E;
  p.has_drop = d->drop_p > 0.f;
  p.drop_thresh = (uint32_t)((double)d->drop_p * 4294967296.0);
  p.drop_scale = p.has_drop ? 1.f / (1.f - d->drop_p) : 1.f;
  p.seed = d->seed;
  p.seed_ptr = static_cast<const uint64_t*>(d->seed_ptr);
  return 0;
}

// Two query groups per wave (128-row blocks) only pay off once a block has enough rows;
// the short caption sequences (31-64 rows) keep 64-row blocks.
// GVL_ATTN_G=1 keeps 64-row blocks everywhere (A/B of occupancy against rows per block).
int pick_groups(int64_t T) {
  static const int forced = [] {
    const char* e = getenv("GVL_ATTN_G");
    return e ? atoi(e) : 0;
  }();
  if (forced == 1) return 1;
  return T > 64 ? 2 : 1;
}

// Single-launch backward for Tq, Tk <= 64 (attn_bwd_short_kernel); GVL_ATTN_SHORT=0 restores the
// three-kernel path (A/B measurement).
bool short_bwd_enabled() {
  static const bool on = [] {
    const char* e = getenv("GVL_ATTN_SHORT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// LDS-DMA forward (attn_fwd_dma_kernel) for multi-tile key ranges without dropout;
// GVL_ATTN_FWD_DMA=0: the register-staged attn_fwd_kernel (A/B).
bool fwd_dma_enabled() {
  static const bool on = [] {
    const char* e = getenv("GVL_ATTN_FWD_DMA");
    return !(e && e[0] == '0');
  }();
  return on;
}

// 32-row short backward (attn_bwd_short_kernel<*, 32>) for Tq, Tk <= 32; GVL_ATTN_SHORT32=0: the
// 64-row kernel (A/B).
bool short32_enabled() {
  static const bool on = [] {
    const char* e = getenv("GVL_ATTN_SHORT32");
    return !(e && e[0] == '0');
  }();
  return on;
}

// 32-query tiles over a 64-key tile (attn_fwd_kernel<1, *, true, 32, 64>, attn_bwd_short_kernel<*, 32,
// 64>) for Tq <= 32 < Tk <= 64 (the cross-attention over 33 image tokens); GVL_ATTN_SHORT3264=0:
// the 64-row kernels (A/B).
bool short3264_enabled() {
  static const bool on = [] {
    const char* e = getenv("GVL_ATTN_SHORT3264");
    return !(e && e[0] == '0');
  }();
  return on;
}

// One-tile forward (attn_fwd_kernel<1, *, true>) for Tk <= 64; GVL_ATTN_FWD_ONE=0: the two-stage
// kernel (A/B).
bool fwd_one_enabled() {
  static const bool on = [] {
    const char* e = getenv("GVL_ATTN_FWD_ONE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Block count of the 1-D heavy-first grid (see tile_of_block); fill() bounds it.
unsigned grid_1d(const gvl_attn_desc* d, int64_t ntile) { return (unsigned)(ntile * d->H * d->B); }

}  // namespace

extern "C" int gvl_attn_fwd(const gvl_attn_desc* d, gvl_stream_t stream) {
  AttnP p;
  if (fill(d, p)) return -1;
  const int G = pick_groups(d->Tq);
  dim3 grid(grid_1d(d, (d->Tq + 64 * G - 1) / (64 * G)));
  hipStream_t s = gvl::as_stream(stream);
  if (!p.has_drop && d->Tk > KT && fwd_dma_enabled()) {
    if (G == 2) gvl::launch_timed(attn_fwd_dma_kernel<2>, grid, dim3(NT), 0, s, p);
    else gvl::launch_timed(attn_fwd_dma_kernel<1>, grid, dim3(NT), 0, s, p);
  } else if (G == 2) {
    if (p.has_drop) gvl::launch_timed(attn_fwd_kernel<2, true>, grid, dim3(NT), 0, s, p);
    else gvl::launch_timed(attn_fwd_kernel<2, false>, grid, dim3(NT), 0, s, p);
  } else if (d->Tq <= 32 && d->Tk <= 32 && fwd_one_enabled() && short32_enabled()) {
    dim3 g32(grid_1d(d, 1));
    if (p.has_drop) gvl::launch_timed(attn_fwd_kernel<1, true, true, 32>, g32, dim3(128), 0, s, p);
    else gvl::launch_timed(attn_fwd_kernel<1, false, true, 32>, g32, dim3(128), 0, s, p);
  } else if (d->Tq <= 32 && d->Tk <= KT && fwd_one_enabled() && short32_enabled() && short3264_enabled()) {
    dim3 g32(grid_1d(d, 1));
    if (p.has_drop) gvl::launch_timed(attn_fwd_kernel<1, true, true, 32, 64>, g32, dim3(128), 0, s, p);
    else gvl::launch_timed(attn_fwd_kernel<1, false, true, 32, 64>, g32, dim3(128), 0, s, p);
  } else if (d->Tk <= KT && fwd_one_enabled()) {
    if (p.has_drop) gvl::launch_timed(attn_fwd_kernel<1, true, true>, grid, dim3(NT), 0, s, p);
    else gvl::launch_timed(attn_fwd_kernel<1, false, true>, grid, dim3(NT), 0, s, p);
  } else {
    if (p.has_drop) gvl::launch_timed(attn_fwd_kernel<1, true>, grid, dim3(NT), 0, s, p);
    else gvl::launch_timed(attn_fwd_kernel<1, false>, grid, dim3(NT), 0, s, p);
  }
  GVL_LAUNCH_CHECK("gvl_attn_fwd");
  return 0;
}

extern "C" int64_t gvl_attn_bwd_workspace_size(const gvl_attn_desc* d) {
  return 2 * d->B * d->H * d->Tq * (int64_t)sizeof(float);  // Dws, Lws
}

extern "C" int gvl_attn_bwd(const gvl_attn_desc* d, const gvl_attn_bwd_desc* gd,
                            gvl_stream_t stream) {
  AttnP p;
  if (fill(d, p)) return -1;
  GVL_REQUIRE(gd && gd->dout && gd->dq && gd->dk && gd->dv && gd->workspace && d->lse,
              "gvl_attn_bwd: null tensor");
  const int64_t st[] = {gd->do_sb, gd->do_st, gd->do_sh, gd->dq_sb, gd->dq_st, gd->dq_sh,
                        gd->dk_sb, gd->dk_st, gd->dk_sh, gd->dv_sb, gd->dv_st, gd->dv_sh};
  for (int64_t s : st) GVL_REQUIRE(s % 8 == 0, "gvl_attn_bwd: strides must be multiples of 8");
  AttnG g;
  g.dout = static_cast<const bf16_t*>(gd->dout);
  g.do_sb = gd->do_sb; g.do_st = gd->do_st; g.do_sh = gd->do_sh;
  g.dq = static_cast<bf16_t*>(gd->dq);
  g.dq_sb = gd->dq_sb; g.dq_st = gd->dq_st; g.dq_sh = gd->dq_sh;
  g.dk = static_cast<bf16_t*>(gd->dk);
  g.dk_sb = gd->dk_sb; g.dk_st = gd->dk_st; g.dk_sh = gd->dk_sh;
  g.dv = static_cast<bf16_t*>(gd->dv);
  g.dv_sb = gd->dv_sb; g.dv_st = gd->dv_st; g.dv_sh = gd->dv_sh;
  g.Dws = static_cast<float*>(gd->workspace);
  g.Lws = g.Dws + d->B * d->H * d->Tq;
  hipStream_t s = gvl::as_stream(stream);
  if (d->Tq <= 64 && d->Tk <= 64 && short_bwd_enabled()) {
    dim3 grid((unsigned)(d->B * d->H));
    if (d->Tq <= 32 && d->Tk <= 32 && short32_enabled()) {
      if (p.has_drop) gvl::launch_timed(attn_bwd_short_kernel<true, 32>, grid, dim3(128), 0, s, p, g);
      else gvl::launch_timed(attn_bwd_short_kernel<false, 32>, grid, dim3(128), 0, s, p, g);
    } else if (d->Tq <= 32 && short32_enabled() && short3264_enabled()) {
      if (p.has_drop) gvl::launch_timed(attn_bwd_short_kernel<true, 32, 64>, grid, dim3(128), 0, s, p, g);
      else gvl::launch_timed(attn_bwd_short_kernel<false, 32, 64>, grid, dim3(128), 0, s, p, g);
    } else {
      if (p.has_drop) gvl::launch_timed(attn_bwd_short_kernel<true>, grid, dim3(NT), 0, s, p, g);
      else gvl::launch_timed(attn_bwd_short_kernel<false>, grid, dim3(NT), 0, s, p, g);
    }
    GVL_LAUNCH_CHECK("gvl_attn_bwd(short)");
    return 0;
  }
  // dQ (which also writes D = rowsum(dO * O) into the workspace), then dK/dV
  const int Gq = pick_groups(d->Tq);
  dim3 gq(grid_1d(d, (d->Tq + 64 * Gq - 1) / (64 * Gq)));
  if (Gq == 2) {
    if (p.has_drop) gvl::launch_timed(attn_bwd_dq_dma_kernel<2, true>, gq, dim3(NT), 0, s, p, g);
    else gvl::launch_timed(attn_bwd_dq_dma_kernel<2, false>, gq, dim3(NT), 0, s, p, g);
  } else {
    if (p.has_drop) gvl::launch_timed(attn_bwd_dq_dma_kernel<1, true>, gq, dim3(NT), 0, s, p, g);
    else gvl::launch_timed(attn_bwd_dq_dma_kernel<1, false>, gq, dim3(NT), 0, s, p, g);
  }
  GVL_LAUNCH_CHECK("gvl_attn_bwd(dq)");
  // dK/dV: 16 keys per wave (32 measured no faster at T = 1024: 2 instead of 3 blocks per CU,
  // profiles/r3/attn_g_ab_r3s2.txt)
  dim3 gk(grid_1d(d, (d->Tk + 63) / 64));
  if (p.has_drop) gvl::launch_timed(attn_bwd_dkdv_dma_kernel<1, true>, gk, dim3(NT), 0, s, p, g);
  else gvl::launch_timed(attn_bwd_dkdv_dma_kernel<1, false>, gk, dim3(NT), 0, s, p, g);
  GVL_LAUNCH_CHECK("gvl_attn_bwd(dkdv)");
  return 0;
}
