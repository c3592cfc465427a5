// LayerNorm forward/backward (nn.LayerNorm, eps 1e-5 in the reference), one wave per row.
// Row values stay in registers (C <= 1024, 4 bf16 per 8-byte load per lane), statistics
// in fp32 (two-pass variance on the register copy), output bf16.
// HBM-bound: fwd reads C*2 B and writes C*2 B (+8 B stats) per row.
#include "common.h"
#include "capi_util.h"
#include "../../include/gvl.h"

namespace {

constexpr int LN_NT = 256;       // 4 rows (waves) per block
constexpr int LN_MAXIT = 4;      // 4 * 64 lanes * 4 elems = 1024 columns max

__global__ __launch_bounds__(LN_NT) void ln_fwd_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                       const bf16_t* __restrict__ w,
                                                       const bf16_t* __restrict__ b,
                                                       bf16_t* __restrict__ y, int64_t ldy,
                                                       float* __restrict__ mean_out,
                                                       float* __restrict__ rstd_out, int64_t rows,
                                                       int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (LN_NT / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16_t* xr = x + row * ldx;
  float v[LN_MAXIT][4];
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < LN_MAXIT; ++it) {
    const int c = (lane + 64 * it) * 4;
    if (c < C) {
      const uint2 u = *reinterpret_cast<const uint2*>(xr + c);
      v[it][0] = lo_bf(u.x); v[it][1] = hi_bf(u.x); v[it][2] = lo_bf(u.y); v[it][3] = hi_bf(u.y);
      s += v[it][0] + v[it][1] + v[it][2] + v[it][3];
    } else {
      v[it][0] = v[it][1] = v[it][2] = v[it][3] = 0.f;
    }
  }
  const float mean = warp_sum(s) / (float)C;
  float ss = 0.f;
#pragma unroll
  for (int it = 0; it < LN_MAXIT; ++it) {
    const int c = (lane + 64 * it) * 4;
    if (c < C) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = v[it][r] - mean;
        ss += d * d;
      }
    }
  }
  const float var = warp_sum(ss) / (float)C;
  const float rstd = rsqrtf(var + eps);
  bf16_t* yr = y + row * ldy;
#pragma unroll
  for (int it = 0; it < LN_MAXIT; ++it) {
    const int c = (lane + 64 * it) * 4;
    if (c < C) {
      const uint2 wu = *reinterpret_cast<const uint2*>(w + c);
      const uint2 bu = *reinterpret_cast<const uint2*>(b + c);
      const float o0 = (v[it][0] - mean) * rstd * lo_bf(wu.x) + lo_bf(bu.x);
      const float o1 = (v[it][1] - mean) * rstd * hi_bf(wu.x) + hi_bf(bu.x);
      const float o2 = (v[it][2] - mean) * rstd * lo_bf(wu.y) + lo_bf(bu.y);
      const float o3 = (v[it][3] - mean) * rstd * hi_bf(wu.y) + hi_bf(bu.y);
      *reinterpret_cast<uint2*>(yr + c) = make_uint2(pack2(o0, o1), pack2(o2, o3));
    }
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// Backward. Each block walks rows blockIdx.x*4+wave, stepping gridDim.x*4; dw/db column
// partials accumulate in registers and are reduced once per block into ws[block][2C].
__global__ __launch_bounds__(LN_NT) void ln_bwd_kernel(
    const bf16_t* __restrict__ dy, int64_t lddy, const bf16_t* __restrict__ x, int64_t ldx,
    const bf16_t* __restrict__ w, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, bf16_t* __restrict__ dx, int64_t lddx, int acc_dx,
    float* __restrict__ ws, int64_t rows, int C) {
  __shared__ float red[LN_NT / 64][1024 * 2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pw[LN_MAXIT][4], pb[LN_MAXIT][4];
#pragma unroll
  for (int it = 0; it < LN_MAXIT; ++it)
#pragma unroll
    for (int r = 0; r < 4; ++r) pw[it][r] = pb[it][r] = 0.f;
  float wv[LN_MAXIT][4];
#pragma unroll
  for (int it = 0; it < LN_MAXIT; ++it) {
    const int c = (lane + 64 * it) * 4;
    if (c < C) {
      const uint2 wu = *reinterpret_cast<const uint2*>(w + c);
      wv[it][0] = lo_bf(wu.x); wv[it][1] = hi_bf(wu.x); wv[it][2] = lo_bf(wu.y); wv[it][3] = hi_bf(wu.y);
    } else {
      wv[it][0] = wv[it][1] = wv[it][2] = wv[it][3] = 0.f;
    }
  }
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < rows; row += (int64_t)gridDim.x * 4) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[LN_MAXIT][4], g[LN_MAXIT][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int it = 0; it < LN_MAXIT; ++it) {
      const int c = (lane + 64 * it) * 4;
      if (c < C) {
        const uint2 xu = *reinterpret_cast<const uint2*>(x + row * ldx + c);
        const uint2 du = *reinterpret_cast<const uint2*>(dy + row * lddy + c);
        const float xs[4] = {lo_bf(xu.x), hi_bf(xu.x), lo_bf(xu.y), hi_bf(xu.y)};
        const float ds[4] = {lo_bf(du.x), hi_bf(du.x), lo_bf(du.y), hi_bf(du.y)};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xh[it][r] = (xs[r] - mean) * rstd;
          g[it][r] = ds[r] * wv[it][r];
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
    const float m1 = warp_sum(s1) / (float)C, m2 = warp_sum(s2) / (float)C;
#pragma unroll
    for (int it = 0; it < LN_MAXIT; ++it) {
      const int c = (lane + 64 * it) * 4;
      if (c < C) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = rstd * (g[it][r] - m1 - xh[it][r] * m2);
        bf16_t* dst = dx + row * lddx + c;
        if (acc_dx) {
          const uint2 pu = *reinterpret_cast<const uint2*>(dst);
          o[0] += lo_bf(pu.x); o[1] += hi_bf(pu.x); o[2] += lo_bf(pu.y); o[3] += hi_bf(pu.y);
        }
        *reinterpret_cast<uint2*>(dst) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  }
  if (ws == nullptr) return;
#pragma unroll
  for (int it = 0; it < LN_MAXIT; ++it) {
    const int c = (lane + 64 * it) * 4;
    if (c < C) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[wave][c + r] = pw[it][r];
        red[wave][1024 + c + r] = pb[it][r];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += LN_NT) {
    float a = 0.f, bsum = 0.f;
#pragma unroll
    for (int k = 0; k < LN_NT / 64; ++k) {
      a += red[k][c];
      bsum += red[k][1024 + c];
    }
    ws[(int64_t)blockIdx.x * 2 * C + c] = a;
    ws[(int64_t)blockIdx.x * 2 * C + C + c] = bsum;
  }
}

// Column reduction of the per-block partials: block = 64 columns x 4 partial-groups, each
// thread summing nblk/4 partials with 8 independent loads in flight (the partials were
// previously summed by one serial dependent-load chain per column: ~120 us).
__global__ __launch_bounds__(256) void ln_bwd_finalize(const float* __restrict__ ws, int nblk,
                                                       int C, bf16_t* __restrict__ dw,
                                                       bf16_t* __restrict__ db, int acc) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < 2 * C) {
    int k = g;
    for (; k + 28 < nblk; k += 32) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += ws[(int64_t)(k + 4 * j) * 2 * C + c];
    }
    for (; k < nblk; k += 4) s[0] += ws[(int64_t)k * 2 * C + c];
  }
  red[g][cl] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (g != 0 || c >= 2 * C) return;
  float t = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
  bf16_t* dst = (c < C) ? (dw ? dw + c : nullptr) : (db ? db + (c - C) : nullptr);
  if (!dst) return;
  if (acc) t += bf2f(*dst);
  *dst = f2bf(t);
}

// Up to 1024 blocks (4 per CU resident beside the 32 KiB reduction array): at 512 the
// 16k-row LM backward kept 8 waves per CU, each walking its rows one dependent load round
// trip at a time (~2.3 TB/s); 1024 doubles the rows in flight.
int ln_bwd_blocks(int64_t rows) {
  int64_t nb = (rows + 3) / 4;
  if (nb > 1024) nb = 1024;
  if (nb < 1) nb = 1;
  return (int)nb;
}

}  // namespace

extern "C" int gvl_layernorm_fwd(const void* x, int64_t ldx, const void* w, const void* b, void* y,
                                 int64_t ldy, float* mean, float* rstd, int64_t rows, int64_t cols,
                                 float eps, gvl_stream_t stream) {
  GVL_REQUIRE(cols > 0 && cols <= 1024 && cols % 4 == 0, "gvl_layernorm_fwd: cols=%lld unsupported",
              (long long)cols);
  GVL_REQUIRE(ldx % 4 == 0 && ldy % 4 == 0, "gvl_layernorm_fwd: ld must be multiple of 4");
  if (rows == 0) return 0;
  const int grid = (int)((rows + 3) / 4);
  hipLaunchKernelGGL(ln_fwd_kernel, dim3(grid), dim3(LN_NT), 0, gvl::as_stream(stream),
                     static_cast<const bf16_t*>(x), ldx, static_cast<const bf16_t*>(w),
                     static_cast<const bf16_t*>(b), static_cast<bf16_t*>(y), ldy, mean, rstd, rows,
                     (int)cols, eps);
  GVL_LAUNCH_CHECK("gvl_layernorm_fwd");
  return 0;
}

extern "C" int64_t gvl_layernorm_bwd_workspace_size(int64_t rows, int64_t cols) {
  return (int64_t)ln_bwd_blocks(rows) * 2 * cols * (int64_t)sizeof(float);
}

extern "C" int gvl_layernorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx,
                                 const void* w, const float* mean, const float* rstd, void* dx,
                                 int64_t lddx, int32_t accumulate_dx, void* dw, void* db,
                                 int32_t accumulate_wb, void* workspace, int64_t rows, int64_t cols,
                                 gvl_stream_t stream) {
  GVL_REQUIRE(cols > 0 && cols <= 1024 && cols % 4 == 0, "gvl_layernorm_bwd: cols unsupported");
  GVL_REQUIRE(!(dw || db) || workspace, "gvl_layernorm_bwd: dw/db need a workspace");
  if (rows == 0) return 0;
  const int nb = ln_bwd_blocks(rows);
  hipStream_t s = gvl::as_stream(stream);
  float* ws = (dw || db) ? static_cast<float*>(workspace) : nullptr;
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(nb), dim3(LN_NT), 0, s, static_cast<const bf16_t*>(dy),
                     lddy, static_cast<const bf16_t*>(x), ldx, static_cast<const bf16_t*>(w), mean,
                     rstd, static_cast<bf16_t*>(dx), lddx, (int)accumulate_dx, ws, rows, (int)cols);
  GVL_LAUNCH_CHECK("gvl_layernorm_bwd");
  if (ws) {
    const int g2 = (int)((2 * cols + 63) / 64);
    hipLaunchKernelGGL(ln_bwd_finalize, dim3(g2), dim3(256), 0, s, ws, nb, (int)cols,
                       static_cast<bf16_t*>(dw), static_cast<bf16_t*>(db), (int)accumulate_wb);
    GVL_LAUNCH_CHECK("gvl_layernorm_bwd(finalize)");
  }
  return 0;
}
