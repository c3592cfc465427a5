// LayerNorm forward/backward (nn.LayerNorm, eps 1e-5 in the reference), HBM-bound.
// Forward layout: one HALF-wave (32 lanes) per row, 16-B accesses: lane l of the half holds
// chunks l, l+32, l+64, ... of 8 columns (C = 768 -> 3 chunks, 24 values in registers), so a
// load instruction moves 2 rows x 512 B.  Statistics in fp32 (two-pass variance on the
// register copy), row reductions over the 32 lanes of the half.
// Bytes per row: forward 2C read + 2C written (+8 B stats); backward reads x, dy (and dx when
// accumulating) and writes dx: 4C..6C, plus the dw/db partials.
#include "common.h"
#include "capi_util.h"
#include "../../include/gvl.h"

namespace {

constexpr int LN_FWD_NT = 256;   // 8 rows per block
constexpr int LN_BWD_NT = 256;   // 4 waves, one row each (+1 prefetched)
// backward blocks (rows per wave = rows / (4 x blocks)): 512 measured best of 256 / 384 / 512 /
// 1024 / 2048 (16384 x 768 22.2-22.5 vs 23.1-23.4 us at 1024, 8064 x 768 15.0 vs 16.5, 4224 x 1024
// 14.3 vs 15.3, incl. the finalize, back to back; no measurable change inside the steps;
// profiles/r4/ln_bwd_blocks_r4lnb.txt)
#ifndef GVL_LN_BWD_MAXB
#define GVL_LN_BWD_MAXB 512
#endif
constexpr int LN_BWD_MAXB = GVL_LN_BWD_MAXB;

// Row sums by DPP + lane swaps (common.h wave_sum_v / half_sum_v: no ds_bpermute round trips,
// six per row sum in the __shfl_xor butterflies).
#ifndef GVL_LN_DPP  // 0: the __shfl_xor butterflies (A/B builds)
#define GVL_LN_DPP 1
#endif
GVL_DEV float half_sum(float v) {  // over the 32 lanes of this half-wave
  if (GVL_LN_DPP) return half_sum_v(v);
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
GVL_DEV float row_sum64(float v) {  // over the wave
  if (GVL_LN_DPP) return wave_sum_v(v);
  return warp_sum(v);
}

template <int IT>
__global__ __launch_bounds__(LN_FWD_NT) void ln_fwd_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                           const bf16_t* __restrict__ w,
                                                           const bf16_t* __restrict__ b,
                                                           bf16_t* __restrict__ y, int64_t ldy,
                                                           float* __restrict__ mean_out,
                                                           float* __restrict__ rstd_out,
                                                           int64_t rows, int C, float eps) {
  const int hl = threadIdx.x & 31;
  const int64_t row = (int64_t)blockIdx.x * (LN_FWD_NT / 32) + (threadIdx.x >> 5);
  const bool live = row < rows;  // (no early exit: the half-wave shuffles need both halves)
  const bf16_t* xr = x + (live ? row : 0) * ldx;
  float v[IT][8];
  float s = 0.f;
  uint4 wq[IT], bq[IT];  // gamma / beta issued with the row loads (their latency overlaps)
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (hl + 32 * it) * 8;
    if (c < C) {
      wq[it] = *reinterpret_cast<const uint4*>(w + c);
      bq[it] = *reinterpret_cast<const uint4*>(b + c);
    }
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (hl + 32 * it) * 8;
    if (live && c < C) {
      unpack8(*reinterpret_cast<const uint4*>(xr + c), v[it]);
#pragma unroll
      for (int r = 0; r < 8; ++r) s += v[it][r];
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) v[it][r] = 0.f;
    }
  }
  const float mean = half_sum(s) / (float)C;
  float ss = 0.f;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (hl + 32 * it) * 8;
    if (c < C) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float d = v[it][r] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(half_sum(ss) / (float)C + eps);
  if (!live) return;
  bf16_t* yr = y + row * ldy;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (hl + 32 * it) * 8;
    if (c < C) {
      float wf[8], bf[8], o[8];
      unpack8(wq[it], wf);
      unpack8(bq[it], bf);
#pragma unroll
      for (int r = 0; r < 8; ++r) o[r] = (v[it][r] - mean) * rstd * wf[r] + bf[r];
      *reinterpret_cast<uint4*>(yr + c) = pack8(o);
    }
  }
  if (hl == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// Persistent form (default; GVL_LN_FWD_PERSIST=0 builds the one-shot grid above for A/B): at most
// GVL_LN_FWD_MAXB blocks, each half-wave walks rows r, r + stride, ... and issues the next row's
// loads before it normalises and stores the current one, so every half-wave keeps a read and a
// write in flight instead of the whole grid reading first and writing afterwards.  4-7 % faster
// at 4096-16384 rows (1024 blocks = 2048 the same; 512 slower at 16384 rows), same arithmetic
// (profiles/r5/ln_fwd_persist_r5ln.txt).
#ifndef GVL_LN_FWD_PERSIST
#define GVL_LN_FWD_PERSIST 1
#endif
#ifndef GVL_LN_FWD_MAXB
#define GVL_LN_FWD_MAXB 1024
#endif
template <int IT>
__global__ __launch_bounds__(LN_FWD_NT) void ln_fwd_persist_kernel(
    const bf16_t* __restrict__ x, int64_t ldx, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ b, bf16_t* __restrict__ y, int64_t ldy, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int64_t rows, int C, float eps) {
  const int hl = threadIdx.x & 31;
  const int64_t stride = (int64_t)gridDim.x * (LN_FWD_NT / 32);
  int64_t row = (int64_t)blockIdx.x * (LN_FWD_NT / 32) + (threadIdx.x >> 5);
  uint4 wq[IT], bq[IT], nx[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (hl + 32 * it) * 8;
    if (c < C) {
      wq[it] = *reinterpret_cast<const uint4*>(w + c);
      bq[it] = *reinterpret_cast<const uint4*>(b + c);
    }
  }
  // rows past the end read row 0 (their results are never stored); every half-wave of the grid
  // runs the same number of iterations, so the half-wave shuffles always see both halves live
  const int64_t iters = (rows + stride - 1) / stride;
  auto fetch = [&](int64_t r) {
    const bf16_t* xr = x + (r < rows ? r : 0) * ldx;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int c = (hl + 32 * it) * 8;
      if (c < C) nx[it] = *reinterpret_cast<const uint4*>(xr + c);
    }
  };
  fetch(row);
  for (int64_t i = 0; i < iters; ++i, row += stride) {
    float v[IT][8];
    float s = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int c = (hl + 32 * it) * 8;
      if (c < C) {
        unpack8(nx[it], v[it]);
#pragma unroll
        for (int r = 0; r < 8; ++r) s += v[it][r];
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r) v[it][r] = 0.f;
      }
    }
    if (i + 1 < iters) fetch(row + stride);
    const float mean = half_sum(s) / (float)C;
    float ss = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int c = (hl + 32 * it) * 8;
      if (c < C) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float d = v[it][r] - mean;
          ss += d * d;
        }
      }
    }
    const float rstd = rsqrtf(half_sum(ss) / (float)C + eps);
    if (row < rows) {
      bf16_t* yr = y + row * ldy;
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int c = (hl + 32 * it) * 8;
        if (c < C) {
          float wf[8], bf[8], o[8];
          unpack8(wq[it], wf);
          unpack8(bq[it], bf);
#pragma unroll
          for (int r = 0; r < 8; ++r) o[r] = (v[it][r] - mean) * rstd * wf[r] + bf[r];
          *reinterpret_cast<uint4*>(yr + c) = pack8(o);
        }
      }
      if (hl == 0) {
        if (mean_out) mean_out[row] = mean;
        if (rstd_out) rstd_out[row] = rstd;
      }
    }
  }
}

// Backward: one wave per row (lane l holds 4-column chunks l, l+64, l+128: 8-B accesses keep
// the per-lane state small — dw/db partials, w, the row in hand and the prefetched next row
// fit ~100 VGPRs, 4 blocks per CU).  Wave w of block k walks rows k*4 + w, stepping
// gridDim.x*4; the next row's x / dy / dx(prev) / stats loads are issued before the current
// row is computed, so each wave keeps two rows of loads in flight.  dw/db column partials
// accumulate in registers and are reduced once per block into ws[block][2C].
template <int IT>
__global__ __launch_bounds__(LN_BWD_NT) void ln_bwd_kernel(
    const bf16_t* __restrict__ dy, int64_t lddy, const bf16_t* __restrict__ x, int64_t ldx,
    const bf16_t* __restrict__ w, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const bf16_t* res, int64_t ldr, bf16_t* dx, int64_t lddx,
    int acc_dx, float* __restrict__ ws, int64_t rows, int C) {
  __shared__ float red[LN_BWD_NT / 64][2 * 64 * 4 * IT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pw[IT][4], pb[IT][4];
  uint2 wu[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (lane + 64 * it) * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) pw[it][r] = pb[it][r] = 0.f;
    wu[it] = c < C ? *reinterpret_cast<const uint2*>(w + c) : make_uint2(0, 0);
  }
  const int64_t stride = (int64_t)gridDim.x * (LN_BWD_NT / 64);
  int64_t row = (int64_t)blockIdx.x * (LN_BWD_NT / 64) + wave;
  uint2 xu[IT], du[IT], pu[IT];
  float mean = 0.f, rstd = 0.f;
  auto fetch = [&](int64_t r) {
    mean = mean_in[r];
    rstd = rstd_in[r];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int c = (lane + 64 * it) * 4;
      if (c < C) {
        xu[it] = *reinterpret_cast<const uint2*>(x + r * ldx + c);
        du[it] = *reinterpret_cast<const uint2*>(dy + r * lddy + c);
        if (acc_dx) pu[it] = *reinterpret_cast<const uint2*>(res + r * ldr + c);
      }
    }
  };
  if (row < rows) fetch(row);
  for (; row < rows; row += stride) {
    uint2 cx[IT], cd[IT], cp[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      cx[it] = xu[it];
      cd[it] = du[it];
      cp[it] = pu[it];
    }
    const float mu = mean, rs = rstd;
    if (row + stride < rows) fetch(row + stride);
    float xh[IT][4], g[IT][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int c = (lane + 64 * it) * 4;
      if (c < C) {
        const float xs[4] = {lo_bf(cx[it].x), hi_bf(cx[it].x), lo_bf(cx[it].y), hi_bf(cx[it].y)};
        const float ds[4] = {lo_bf(cd[it].x), hi_bf(cd[it].x), lo_bf(cd[it].y), hi_bf(cd[it].y)};
        const float ws4[4] = {lo_bf(wu[it].x), hi_bf(wu[it].x), lo_bf(wu[it].y), hi_bf(wu[it].y)};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xh[it][r] = (xs[r] - mu) * rs;
          g[it][r] = ds[r] * ws4[r];
          s1 += g[it][r];
          s2 += g[it][r] * xh[it][r];
          pw[it][r] += ds[r] * xh[it][r];
          pb[it][r] += ds[r];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) xh[it][r] = g[it][r] = 0.f;
      }
    }
    const float m1 = row_sum64(s1) / (float)C, m2 = row_sum64(s2) / (float)C;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int c = (lane + 64 * it) * 4;
      if (c < C) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = rs * (g[it][r] - m1 - xh[it][r] * m2);
        if (acc_dx) {
          o[0] += lo_bf(cp[it].x); o[1] += hi_bf(cp[it].x);
          o[2] += lo_bf(cp[it].y); o[3] += hi_bf(cp[it].y);
        }
        *reinterpret_cast<uint2*>(dx + row * lddx + c) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  }
  if (ws == nullptr) return;
  constexpr int CM = 64 * 4 * IT;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (lane + 64 * it) * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[wave][c + r] = pw[it][r];
      red[wave][CM + c + r] = pb[it][r];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += LN_BWD_NT) {
    float a = 0.f, bsum = 0.f;
#pragma unroll
    for (int k = 0; k < LN_BWD_NT / 64; ++k) {
      a += red[k][c];
      bsum += red[k][CM + c];
    }
    ws[(int64_t)blockIdx.x * 2 * C + c] = a;
    ws[(int64_t)blockIdx.x * 2 * C + C + c] = bsum;
  }
}

// Column reduction of the per-block partials: block = 64 columns x 16 partial groups; each
// thread sums <= LN_BWD_MAXB/16 partials (all loads in flight), a wave reading 256 contiguous
// bytes of one partial row per load (16 columns x 64 groups read 64-B pieces of four rows:
// 30 us for the LM's 25 deferred LayerNorms), then the groups reduce in LDS.  Both finalize
// forms share it, so the deferred one stays bit-identical to the in-place one.
constexpr int LN_FIN_COLS = 64, LN_FIN_GROUPS = 16;
GVL_DEV void ln_fin_block(const float* __restrict__ ws, int nblk, int C, bf16_t* dw, bf16_t* db,
                          int acc, float (&red)[LN_FIN_GROUPS][LN_FIN_COLS + 1]) {
  const int cl = threadIdx.x & (LN_FIN_COLS - 1), g = threadIdx.x / LN_FIN_COLS;
  const int c = blockIdx.x * LN_FIN_COLS + cl;
  float s = 0.f;
  if (c < 2 * C) {
    float v[LN_BWD_MAXB / LN_FIN_GROUPS];
#pragma unroll
    for (int j = 0; j < LN_BWD_MAXB / LN_FIN_GROUPS; ++j) {
      const int k = g + LN_FIN_GROUPS * j;
      v[j] = k < nblk ? ws[(int64_t)k * 2 * C + c] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < LN_BWD_MAXB / LN_FIN_GROUPS; ++j) s += v[j];
  }
  red[g][cl] = s;
  __syncthreads();
  if (threadIdx.x >= LN_FIN_COLS || c >= 2 * C) return;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < LN_FIN_GROUPS; ++k) t += red[k][cl];
  bf16_t* dst = (c < C) ? (dw ? dw + c : nullptr) : (db ? db + (c - C) : nullptr);
  if (!dst) return;
  if (acc) t += bf2f(*dst);
  *dst = f2bf(t);
}

__global__ __launch_bounds__(1024) void ln_bwd_finalize(const float* __restrict__ ws, int nblk,
                                                        int C, bf16_t* __restrict__ dw,
                                                        bf16_t* __restrict__ db, int acc) {
  __shared__ float red[LN_FIN_GROUPS][LN_FIN_COLS + 1];
  ln_fin_block(ws, nblk, C, dw, db, acc, red);
}

// Batched form (gvl_layernorm_bwd_finalize_batched): blockIdx.y = item, each item as above.
constexpr int LN_FIN_MAX = 64;
struct LnFinBatch {
  const float* ws[LN_FIN_MAX];
  bf16_t* dw[LN_FIN_MAX];
  bf16_t* db[LN_FIN_MAX];
  int nblk[LN_FIN_MAX];
};
__global__ __launch_bounds__(1024) void ln_bwd_finalize_batched(LnFinBatch b, int C, int acc) {
  __shared__ float red[LN_FIN_GROUPS][LN_FIN_COLS + 1];
  const int it = blockIdx.y;
  ln_fin_block(b.ws[it], b.nblk[it], C, b.dw[it], b.db[it], acc, red);
}

// >= 2 rows per wave, <= LN_BWD_MAXB blocks (512: 2 per CU, 8 waves, ~16 rows in flight per CU).
int ln_bwd_blocks(int64_t rows) {
  int64_t nb = (rows + 7) / 8;
  if (nb > LN_BWD_MAXB) nb = LN_BWD_MAXB;
  if (nb < 1) nb = 1;
  return (int)nb;
}

bool ln_shape_ok(int64_t cols, int64_t ld1, int64_t ld2, const void* p1, const void* p2) {
  return cols > 0 && cols <= 1024 && cols % 8 == 0 && ld1 % 8 == 0 && ld2 % 8 == 0 &&
         gvl::aligned16(p1) && gvl::aligned16(p2);
}

}  // namespace

extern "C" int gvl_layernorm_fwd(const void* x, int64_t ldx, const void* w, const void* b, void* y,
                                 int64_t ldy, float* mean, float* rstd, int64_t rows, int64_t cols,
                                 float eps, gvl_stream_t stream) {
  GVL_REQUIRE(ln_shape_ok(cols, ldx, ldy, x, y) && gvl::aligned16(w) && gvl::aligned16(b),
              "gvl_layernorm_fwd: cols=%lld unsupported (need cols %% 8 == 0, <= 1024, ld %% 8 "
              "== 0, 16-byte aligned rows)", (long long)cols);
  if (rows == 0) return 0;
  const int grid = (int)((rows + 7) / 8);
  hipStream_t s = gvl::as_stream(stream);
  const auto xp = static_cast<const bf16_t*>(x);
  const auto wp = static_cast<const bf16_t*>(w);
  const auto bp = static_cast<const bf16_t*>(b);
  auto yp = static_cast<bf16_t*>(y);
  if (GVL_LN_FWD_PERSIST) {
    const int pg = grid < GVL_LN_FWD_MAXB ? grid : GVL_LN_FWD_MAXB;
    if (cols <= 768)
      hipLaunchKernelGGL(ln_fwd_persist_kernel<3>, dim3(pg), dim3(LN_FWD_NT), 0, s, xp, ldx, wp, bp,
                         yp, ldy, mean, rstd, rows, (int)cols, eps);
    else
      hipLaunchKernelGGL(ln_fwd_persist_kernel<4>, dim3(pg), dim3(LN_FWD_NT), 0, s, xp, ldx, wp, bp,
                         yp, ldy, mean, rstd, rows, (int)cols, eps);
    GVL_LAUNCH_CHECK("gvl_layernorm_fwd");
    return 0;
  }
  if (cols <= 768)
    hipLaunchKernelGGL(ln_fwd_kernel<3>, dim3(grid), dim3(LN_FWD_NT), 0, s, xp, ldx, wp, bp, yp,
                       ldy, mean, rstd, rows, (int)cols, eps);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<4>, dim3(grid), dim3(LN_FWD_NT), 0, s, xp, ldx, wp, bp, yp,
                       ldy, mean, rstd, rows, (int)cols, eps);
  GVL_LAUNCH_CHECK("gvl_layernorm_fwd");
  return 0;
}

extern "C" int64_t gvl_layernorm_bwd_workspace_size(int64_t rows, int64_t cols) {
  return (int64_t)ln_bwd_blocks(rows) * 2 * cols * (int64_t)sizeof(float);
}

// dx = [res +] LN backward; res may alias dx (in-place accumulation, gvl_layernorm_bwd)
static int ln_bwd_launch(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w,
                         const float* mean, const float* rstd, const void* res, int64_t ldr,
                         void* dx, int64_t lddx, int32_t accumulate_dx, void* dw, void* db,
                         int32_t accumulate_wb, void* workspace, int64_t rows, int64_t cols,
                         gvl_stream_t stream) {
  GVL_REQUIRE(ln_shape_ok(cols, lddy, ldx, dy, x) && lddx % 8 == 0 && gvl::aligned16(dx) &&
                  gvl::aligned16(w) && (!accumulate_dx || (ldr % 8 == 0 && gvl::aligned16(res))),
              "gvl_layernorm_bwd: cols unsupported (need cols %% 8 == 0, <= 1024, ld %% 8 == 0, "
              "16-byte aligned rows)");
  // accumulate_wb bit 1 (ABI v12): leave the column partials in the workspace for a later
  // gvl_layernorm_bwd_finalize_batched (dw / db are not touched here)
  const bool defer = (accumulate_wb & 2) != 0;
  GVL_REQUIRE(!(dw || db || defer) || workspace, "gvl_layernorm_bwd: dw/db need a workspace");
  if (rows == 0) return 0;
  const int nb = ln_bwd_blocks(rows);
  hipStream_t s = gvl::as_stream(stream);
  float* ws = (dw || db || defer) ? static_cast<float*>(workspace) : nullptr;
  const auto dyp = static_cast<const bf16_t*>(dy);
  const auto xp = static_cast<const bf16_t*>(x);
  const auto wp = static_cast<const bf16_t*>(w);
  const auto rp = static_cast<const bf16_t*>(res);
  auto dxp = static_cast<bf16_t*>(dx);
  if (cols <= 768)
    hipLaunchKernelGGL(ln_bwd_kernel<3>, dim3(nb), dim3(LN_BWD_NT), 0, s, dyp, lddy, xp, ldx, wp,
                       mean, rstd, rp, ldr, dxp, lddx, (int)accumulate_dx, ws, rows, (int)cols);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<4>, dim3(nb), dim3(LN_BWD_NT), 0, s, dyp, lddy, xp, ldx, wp,
                       mean, rstd, rp, ldr, dxp, lddx, (int)accumulate_dx, ws, rows, (int)cols);
  GVL_LAUNCH_CHECK("gvl_layernorm_bwd");
  if (ws && !defer) {
    const int g2 = (int)((2 * cols + LN_FIN_COLS - 1) / LN_FIN_COLS);
    hipLaunchKernelGGL(ln_bwd_finalize, dim3(g2), dim3(1024), 0, s, ws, nb, (int)cols,
                       static_cast<bf16_t*>(dw), static_cast<bf16_t*>(db), (int)accumulate_wb);
    GVL_LAUNCH_CHECK("gvl_layernorm_bwd(finalize)");
  }
  return 0;
}

extern "C" int gvl_layernorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx,
                                 const void* w, const float* mean, const float* rstd, void* dx,
                                 int64_t lddx, int32_t accumulate_dx, void* dw, void* db,
                                 int32_t accumulate_wb, void* workspace, int64_t rows, int64_t cols,
                                 gvl_stream_t stream) {
  return ln_bwd_launch(dy, lddy, x, ldx, w, mean, rstd, dx, lddx, dx, lddx, accumulate_dx, dw, db,
                       accumulate_wb, workspace, rows, cols, stream);
}

extern "C" int gvl_layernorm_bwd_res(const void* dy, int64_t lddy, const void* x, int64_t ldx,
                                     const void* w, const float* mean, const float* rstd,
                                     const void* res, int64_t ldr, void* dx, int64_t lddx, void* dw,
                                     void* db, int32_t accumulate_wb, void* workspace, int64_t rows,
                                     int64_t cols, gvl_stream_t stream) {
  GVL_REQUIRE(res != nullptr, "gvl_layernorm_bwd_res: null residual");
  return ln_bwd_launch(dy, lddy, x, ldx, w, mean, rstd, res, ldr, dx, lddx, 1, dw, db,
                       accumulate_wb, workspace, rows, cols, stream);
}

extern "C" int32_t gvl_layernorm_bwd_blocks(int64_t rows) { return rows > 0 ? ln_bwd_blocks(rows) : 0; }

extern "C" int gvl_layernorm_bwd_finalize_batched(const float* const* ws, const int32_t* nblk,
                                                  int32_t count, int64_t cols, void* const* dw,
                                                  void* const* db, int32_t accumulate_wb,
                                                  gvl_stream_t stream) {
  GVL_REQUIRE(ws && nblk && count >= 0 && count <= LN_FIN_MAX && cols > 0 && cols <= 1024,
              "gvl_layernorm_bwd_finalize_batched: bad arguments (count <= %d, cols <= 1024)",
              LN_FIN_MAX);
  if (count == 0) return 0;
  LnFinBatch b{};
  for (int i = 0; i < count; ++i) {
    GVL_REQUIRE(ws[i] != nullptr && nblk[i] >= 0 && nblk[i] <= LN_BWD_MAXB,
                "gvl_layernorm_bwd_finalize_batched: item %d: null workspace or bad block count", i);
    b.ws[i] = ws[i];
    b.nblk[i] = nblk[i];
    b.dw[i] = dw ? static_cast<bf16_t*>(dw[i]) : nullptr;
    b.db[i] = db ? static_cast<bf16_t*>(db[i]) : nullptr;
  }
  const int g2 = (int)((2 * cols + LN_FIN_COLS - 1) / LN_FIN_COLS);
  hipLaunchKernelGGL(ln_bwd_finalize_batched, dim3(g2, count), dim3(1024), 0, gvl::as_stream(stream), b,
                     (int)cols, (int)(accumulate_wb & 1));
  GVL_LAUNCH_CHECK("gvl_layernorm_bwd_finalize_batched");
  return 0;
}
