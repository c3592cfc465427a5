// Optimizer path over flat bf16 arenas + small fused elementwise helpers.
//  - grad norm: grid-stride sum of squares (16-B loads) -> per-block partials -> one block
//    finishes ||g|| and the clip coefficient on the device (no host sync);
//  - AdamW: one streaming pass, p/g/m/v bf16 in, p/m/v bf16 out, fp32 opmath, the clip
//    coefficient applied to g on the fly (torch _fused_adamw_ semantics, decoupled decay).
// All HBM-bound: AdamW moves 14 B/param, the norm 2 B/param.
#include "common.h"
#include "capi_util.h"
#include "../../include/gvl.h"

namespace {

constexpr int RED_NT = 256;
constexpr int RED_MAXB = 1024;

int red_blocks(int64_t n8) {
  int64_t nb = (n8 + RED_NT - 1) / RED_NT;
  if (nb > RED_MAXB) nb = RED_MAXB;
  if (nb < 1) nb = 1;
  return (int)nb;
}

__global__ __launch_bounds__(RED_NT) void sumsq_kernel(const bf16_t* __restrict__ g, int64_t n,
                                                       float* __restrict__ partial) {
  __shared__ float red[RED_NT / 64];
  float s = 0.f;
  const int64_t n8 = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * RED_NT + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * RED_NT) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(g + i * 8), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += f[k] * f[k];
  }
  if (blockIdx.x == 0) {
    for (int64_t i = n8 * 8 + threadIdx.x; i < n; i += RED_NT) {
      const float v = bf2f(g[i]);
      s += v * v;
    }
  }
  s = block_sum<RED_NT>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(RED_NT) void norm_finish_kernel(const float* __restrict__ partial,
                                                             int nb, float max_norm,
                                                             float* __restrict__ out) {
  __shared__ float red[RED_NT / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += RED_NT) s += partial[i];
  s = block_sum<RED_NT>(s, red);
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(s);
    out[0] = nrm;
    out[1] = fminf(1.f, max_norm / (nrm + 1e-6f));
  }
}

struct AdamP {
  float lr, b1, b2, eps, wd, bc1, bc2_sqrt;
};

GVL_DEV void adam_elem(float& p, float g, float& m, float& v, const AdamP& a, bool decay) {
  if (decay) p = p * (1.f - a.lr * a.wd);
  m = a.b1 * m + (1.f - a.b1) * g;
  v = a.b2 * v + (1.f - a.b2) * g * g;
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p - (a.lr / a.bc1) * m / denom;
}

__global__ __launch_bounds__(256) void adamw_kernel(bf16_t* __restrict__ p,
                                                    const bf16_t* __restrict__ g,
                                                    bf16_t* __restrict__ m, bf16_t* __restrict__ v,
                                                    int64_t n, int64_t n_decay, AdamP a,
                                                    const float* __restrict__ gscale,
                                                    const float* __restrict__ hyper) {
  const float cs = gscale ? *gscale : 1.f;
  if (hyper) {  // device-resident {lr, step}: a captured step reads this step's values
    a.lr = hyper[0];
    a.bc1 = 1.f - powf(a.b1, hyper[1]);
    a.bc2_sqrt = sqrtf(1.f - powf(a.b2, hyper[1]));
  }
  const int64_t n8 = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float fp[8], fg[8], fm[8], fv[8];
    unpack8(*reinterpret_cast<const uint4*>(p + i * 8), fp);
    unpack8(*reinterpret_cast<const uint4*>(g + i * 8), fg);
    unpack8(*reinterpret_cast<const uint4*>(m + i * 8), fm);
    unpack8(*reinterpret_cast<const uint4*>(v + i * 8), fv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      // clip_grad_norm_ scales the bf16 grad in place before the step: round like it
      const float gk = bf2f(f2bf(fg[k] * cs));
      adam_elem(fp[k], gk, fm[k], fv[k], a, (i * 8 + k) < n_decay);
    }
    *reinterpret_cast<uint4*>(p + i * 8) = pack8(fp);
    *reinterpret_cast<uint4*>(m + i * 8) = pack8(fm);
    *reinterpret_cast<uint4*>(v + i * 8) = pack8(fv);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = n8 * 8 + threadIdx.x; i < n; i += 256) {
      float fp = bf2f(p[i]), fm = bf2f(m[i]), fv = bf2f(v[i]);
      const float gk = bf2f(f2bf(bf2f(g[i]) * cs));
      adam_elem(fp, gk, fm, fv, a, i < n_decay);
      p[i] = f2bf(fp); m[i] = f2bf(fm); v[i] = f2bf(fv);
    }
  }
}

// Mixed-precision AdamW: fp32 master weights and moments, the bf16 compute copy the model
// reads written alongside (28 B/param).  Keeps updates smaller than a bf16 ulp of the
// weight (LayerNorm gains ~1.0 have ulp 2^-7 >> lr) instead of rounding them away, so the
// trajectory follows the reference's fp32 CPU path (the parity oracle).
__global__ __launch_bounds__(256) void adamw_master_kernel(
    bf16_t* __restrict__ p, float* __restrict__ pm, const bf16_t* __restrict__ g,
    float* __restrict__ m, float* __restrict__ v, int64_t n, int64_t n_decay, AdamP a,
    const float* __restrict__ gscale, const float* __restrict__ hyper) {
  const float cs = gscale ? *gscale : 1.f;
  if (hyper) {
    a.lr = hyper[0];
    a.bc1 = 1.f - powf(a.b1, hyper[1]);
    a.bc2_sqrt = sqrtf(1.f - powf(a.b2, hyper[1]));
  }
  const int64_t n8 = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float fg[8], fp[8], fm[8], fv[8];
    unpack8(*reinterpret_cast<const uint4*>(g + i * 8), fg);
    const float4* P4 = reinterpret_cast<const float4*>(pm + i * 8);
    const float4* M4 = reinterpret_cast<const float4*>(m + i * 8);
    const float4* V4 = reinterpret_cast<const float4*>(v + i * 8);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 a4 = P4[h], b4 = M4[h], c4 = V4[h];
      fp[4 * h] = a4.x; fp[4 * h + 1] = a4.y; fp[4 * h + 2] = a4.z; fp[4 * h + 3] = a4.w;
      fm[4 * h] = b4.x; fm[4 * h + 1] = b4.y; fm[4 * h + 2] = b4.z; fm[4 * h + 3] = b4.w;
      fv[4 * h] = c4.x; fv[4 * h + 1] = c4.y; fv[4 * h + 2] = c4.z; fv[4 * h + 3] = c4.w;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float gk = bf2f(f2bf(fg[k] * cs));
      adam_elem(fp[k], gk, fm[k], fv[k], a, (i * 8 + k) < n_decay);
    }
    float4* Pw = reinterpret_cast<float4*>(pm + i * 8);
    float4* Mw = reinterpret_cast<float4*>(m + i * 8);
    float4* Vw = reinterpret_cast<float4*>(v + i * 8);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      Pw[h] = make_float4(fp[4 * h], fp[4 * h + 1], fp[4 * h + 2], fp[4 * h + 3]);
      Mw[h] = make_float4(fm[4 * h], fm[4 * h + 1], fm[4 * h + 2], fm[4 * h + 3]);
      Vw[h] = make_float4(fv[4 * h], fv[4 * h + 1], fv[4 * h + 2], fv[4 * h + 3]);
    }
    *reinterpret_cast<uint4*>(p + i * 8) = pack8(fp);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = n8 * 8 + threadIdx.x; i < n; i += 256) {
      float fp = pm[i], fm = m[i], fv = v[i];
      const float gk = bf2f(f2bf(bf2f(g[i]) * cs));
      adam_elem(fp, gk, fm, fv, a, i < n_decay);
      pm[i] = fp; m[i] = fm; v[i] = fv;
      p[i] = f2bf(fp);
    }
  }
}

// Column sums (bias gradients), HBM-bound: 2 B read per element.  Block (cx, s): 16
// column-threads x 8 columns (16-B loads, 256-B row segments) x 16 row groups over rows
// [s*chunk, (s+1)*chunk), 8 independent loads in flight per thread; the row groups reduce
// through LDS into ws[s][cols].  The split count is sized for >= ~768 blocks (the chip needs
// ~64 KiB of loads in flight per CU) and stays <= 128 so the finishing kernel reads at most
// 16 partials per thread, all in flight at once.
constexpr int CS_COLS = 128;
constexpr int CS_MAX_SPLITS = 128;

__global__ __launch_bounds__(256) void colsum_partial_kernel(const bf16_t* __restrict__ x,
                                                             int64_t rows, int64_t cols, int64_t ld,
                                                             int64_t chunk, float* __restrict__ ws) {
  __shared__ float red[16][CS_COLS + 4];
  const int ct = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int64_t c = (int64_t)blockIdx.x * CS_COLS + ct * 8;
  const int64_t r0 = (int64_t)blockIdx.y * chunk;
  const int64_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int64_t r = r0 + rg;
    for (; r + 112 < r1; r += 128) {
      uint4 u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = *reinterpret_cast<const uint4*>(x + (r + 16 * k) * ld + c);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[0] += lo_bf(u[k].x); s[1] += hi_bf(u[k].x); s[2] += lo_bf(u[k].y); s[3] += hi_bf(u[k].y);
        s[4] += lo_bf(u[k].z); s[5] += hi_bf(u[k].z); s[6] += lo_bf(u[k].w); s[7] += hi_bf(u[k].w);
      }
    }
    for (; r < r1; r += 16) {
      const uint4 u = *reinterpret_cast<const uint4*>(x + r * ld + c);
      s[0] += lo_bf(u.x); s[1] += hi_bf(u.x); s[2] += lo_bf(u.y); s[3] += hi_bf(u.y);
      s[4] += lo_bf(u.z); s[5] += hi_bf(u.z); s[6] += lo_bf(u.w); s[7] += hi_bf(u.w);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rg][ct * 8 + k] = s[k];
  __syncthreads();
  const int i = threadIdx.x & (CS_COLS - 1), half = threadIdx.x >> 7;
  const int64_t cc = (int64_t)blockIdx.x * CS_COLS + i;
  float t = 0.f;
#pragma unroll
  for (int g = 0; g < 8; ++g) t += red[8 * half + g][i];
  __syncthreads();
  if (half) red[0][i] = t;
  __syncthreads();
  if (!half && cc < cols) ws[(int64_t)blockIdx.y * cols + cc] = t + red[0][i];
}

// Batched column sums (gvl_colsum_batched): problem blockIdx.z (partial) / blockIdx.y (finish)
constexpr int CS_MAX_BATCH = 16;
struct ColsumBatch {
  const bf16_t* x[CS_MAX_BATCH];
  bf16_t* out[CS_MAX_BATCH];
};

// Block: 32 columns x 8 partial groups; each thread sums <= 16 partials (independent loads).
__global__ __launch_bounds__(256) void colsum_finish_kernel(const float* __restrict__ ws, int nb,
                                                            int64_t cols, bf16_t* __restrict__ out,
                                                            int acc) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t c = (int64_t)blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < cols) {
    float v[CS_MAX_SPLITS / 8];
#pragma unroll
    for (int j = 0; j < CS_MAX_SPLITS / 8; ++j) {
      const int k = g + 8 * j;
      v[j] = k < nb ? ws[(int64_t)k * cols + c] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < CS_MAX_SPLITS / 8; ++j) s += v[j];
  }
  red[g][cl] = s;
  __syncthreads();
  if (g != 0 || c >= cols) return;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) t += red[k][cl];
  if (acc) t += bf2f(out[c]);
  out[c] = f2bf(t);
}

__global__ __launch_bounds__(256) void colsum_partial_batched_kernel(ColsumBatch bt, int64_t rows,
                                                                     int64_t cols, int64_t ld,
                                                                     int64_t chunk, float* ws) {
  // one problem per blockIdx.z; the body is colsum_partial_kernel's
  __shared__ float red[16][CS_COLS + 4];
  const bf16_t* __restrict__ x = bt.x[blockIdx.z];
  float* __restrict__ w = ws + (int64_t)blockIdx.z * gridDim.y * cols;
  const int ct = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int64_t c = (int64_t)blockIdx.x * CS_COLS + ct * 8;
  const int64_t r0 = (int64_t)blockIdx.y * chunk;
  const int64_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int64_t r = r0 + rg;
    for (; r + 112 < r1; r += 128) {
      uint4 u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = *reinterpret_cast<const uint4*>(x + (r + 16 * k) * ld + c);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[0] += lo_bf(u[k].x); s[1] += hi_bf(u[k].x); s[2] += lo_bf(u[k].y); s[3] += hi_bf(u[k].y);
        s[4] += lo_bf(u[k].z); s[5] += hi_bf(u[k].z); s[6] += lo_bf(u[k].w); s[7] += hi_bf(u[k].w);
      }
    }
    for (; r < r1; r += 16) {
      const uint4 u = *reinterpret_cast<const uint4*>(x + r * ld + c);
      s[0] += lo_bf(u.x); s[1] += hi_bf(u.x); s[2] += lo_bf(u.y); s[3] += hi_bf(u.y);
      s[4] += lo_bf(u.z); s[5] += hi_bf(u.z); s[6] += lo_bf(u.w); s[7] += hi_bf(u.w);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rg][ct * 8 + k] = s[k];
  __syncthreads();
  const int i = threadIdx.x & (CS_COLS - 1), half = threadIdx.x >> 7;
  const int64_t cc = (int64_t)blockIdx.x * CS_COLS + i;
  float t = 0.f;
#pragma unroll
  for (int g = 0; g < 8; ++g) t += red[8 * half + g][i];
  __syncthreads();
  if (half) red[0][i] = t;
  __syncthreads();
  if (!half && cc < cols) w[(int64_t)blockIdx.y * cols + cc] = t + red[0][i];
}

__global__ __launch_bounds__(256) void colsum_finish_batched_kernel(const float* ws, int nb,
                                                                    int64_t cols, ColsumBatch bt,
                                                                    int acc) {
  __shared__ float red[8][33];
  const float* __restrict__ w = ws + (int64_t)blockIdx.y * nb * cols;
  bf16_t* __restrict__ out = bt.out[blockIdx.y];
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t c = (int64_t)blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < cols) {
    float v[CS_MAX_SPLITS / 8];
#pragma unroll
    for (int j = 0; j < CS_MAX_SPLITS / 8; ++j) {
      const int k = g + 8 * j;
      v[j] = k < nb ? w[(int64_t)k * cols + c] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < CS_MAX_SPLITS / 8; ++j) s += v[j];
  }
  red[g][cl] = s;
  __syncthreads();
  if (g != 0 || c >= cols) return;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) t += red[k][cl];
  if (acc) t += bf2f(out[c]);
  out[c] = f2bf(t);
}

int colsum_blocks(int64_t rows, int64_t cols, int64_t* chunk) {
  const int64_t cb = (cols + CS_COLS - 1) / CS_COLS;
  int64_t nb = (768 + cb - 1) / cb;
  const int64_t by_rows = (rows + 63) / 64;  // >= 64 rows (4 per row group) per block
  if (nb > by_rows) nb = by_rows;
  if (nb > CS_MAX_SPLITS) nb = CS_MAX_SPLITS;
  if (nb < 1) nb = 1;
  *chunk = (rows + nb - 1) / nb;
  return (int)nb;
}

__global__ __launch_bounds__(256) void dropout_apply_kernel(const bf16_t* __restrict__ in,
                                                            int64_t ldi, bf16_t* __restrict__ out,
                                                            int64_t ldo, int64_t rows, int64_t cols,
                                                            uint64_t seed0, const uint64_t* seed_ptr,
                                                            uint32_t thresh, float scale) {
  const uint64_t seed = seed_eff(seed0, seed_ptr);
  const int64_t total = rows * cols;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / cols, c = e - r * cols;
    const float v = bf2f(in[r * ldi + c]);
    out[r * ldo + c] = f2bf(rng_keep(seed, (uint64_t)e, thresh) ? v * scale : 0.f);
  }
}

// 8 columns per thread (16-B loads / stores; cols, strides % 8 == 0 and 16-B aligned rows):
// the scalar form above moved 2 B per access (1.2 TB/s on the Q-Former bridge's 4096 x 768)
__global__ __launch_bounds__(256) void dropout_apply8_kernel(const bf16_t* __restrict__ in,
                                                             int64_t ldi, bf16_t* __restrict__ out,
                                                             int64_t ldo, int64_t rows, int64_t cols,
                                                             uint64_t seed0, const uint64_t* seed_ptr,
                                                             uint32_t thresh, float scale) {
  const uint64_t seed = seed_eff(seed0, seed_ptr);
  const int64_t c8 = cols >> 3, total = rows * c8;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / c8, c = (e - r * c8) * 8;
    const uint4 u = *reinterpret_cast<const uint4*>(in + r * ldi + c);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    uint32_t o[4];
    const uint64_t e0 = (uint64_t)(r * cols + c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = rng_keep(seed, e0 + 2 * k, thresh) ? lo_bf(w[k]) * scale : 0.f;
      const float b = rng_keep(seed, e0 + 2 * k + 1, thresh) ? hi_bf(w[k]) * scale : 0.f;
      o[k] = pack2(a, b);
    }
    *reinterpret_cast<uint4*>(out + r * ldo + c) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

__global__ __launch_bounds__(RED_NT) void gate_bwd8_kernel(const bf16_t* __restrict__ dx,
                                                           const bf16_t* __restrict__ y,
                                                           const bf16_t* __restrict__ gate,
                                                           bf16_t* __restrict__ dy, int64_t n8,
                                                           float* __restrict__ partial) {
  __shared__ float red[RED_NT / 64];
  const float t = tanhf(bf2f(*gate));
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * RED_NT + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * RED_NT) {
    const uint4 d = reinterpret_cast<const uint4*>(dx)[i], yy = reinterpret_cast<const uint4*>(y)[i];
    const uint32_t dw[4] = {d.x, d.y, d.z, d.w}, yw[4] = {yy.x, yy.y, yy.z, yy.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d0 = lo_bf(dw[k]), d1 = hi_bf(dw[k]);
      s += d0 * lo_bf(yw[k]) + d1 * hi_bf(yw[k]);
      o[k] = pack2(t * d0, t * d1);
    }
    reinterpret_cast<uint4*>(dy)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
  s = block_sum<RED_NT>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(RED_NT) void gate_bwd_kernel(const bf16_t* __restrict__ dx,
                                                          const bf16_t* __restrict__ y,
                                                          const bf16_t* __restrict__ gate,
                                                          bf16_t* __restrict__ dy, int64_t n,
                                                          float* __restrict__ partial) {
  __shared__ float red[RED_NT / 64];
  const float t = tanhf(bf2f(*gate));
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * RED_NT + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * RED_NT) {
    const float d = bf2f(dx[i]);
    s += d * bf2f(y[i]);
    dy[i] = f2bf(t * d);
  }
  s = block_sum<RED_NT>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(RED_NT) void gate_finish_kernel(const float* __restrict__ partial,
                                                             int nb, const bf16_t* __restrict__ gate,
                                                             float* __restrict__ out) {
  __shared__ float red[RED_NT / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += RED_NT) s += partial[i];
  s = block_sum<RED_NT>(s, red);
  if (threadIdx.x == 0) {
    const float t = tanhf(bf2f(*gate));
    out[0] += s * (1.f - t * t);
  }
}

// gate_finish into a bf16 gradient (the sunk tanh-gate parameter's): g = bf16(g + bf16(dg)),
// the same two roundings as autograd's bf16 gate grad added by AccumulateGrad
__global__ __launch_bounds__(RED_NT) void gate_finish_bf16_kernel(const float* __restrict__ partial,
                                                                  int nb, const bf16_t* __restrict__ gate,
                                                                  bf16_t* __restrict__ g) {
  __shared__ float red[RED_NT / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += RED_NT) s += partial[i];
  s = block_sum<RED_NT>(s, red);
  if (threadIdx.x == 0) {
    const float t = tanhf(bf2f(*gate));
    const float dg = bf2f(f2bf(s * (1.f - t * t)));
    *g = f2bf(bf2f(*g) + dg);
  }
}

__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float* __restrict__ in,
                                                          bf16_t* __restrict__ out, int64_t n,
                                                          int acc) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float v = in[i];
    if (acc) v += bf2f(out[i]);
    out[i] = f2bf(v);
  }
}

int ew_blocks(int64_t n) {
  int64_t nb = (n + 255) / 256;
  if (nb > 4096) nb = 4096;
  if (nb < 1) nb = 1;
  return (int)nb;
}

}  // namespace

extern "C" int64_t gvl_grad_norm_workspace_size(int64_t n) {
  return (int64_t)red_blocks(n >> 3) * (int64_t)sizeof(float);
}

extern "C" int gvl_grad_norm(const void* g, int64_t n, float max_norm, void* workspace, float* out,
                             gvl_stream_t stream) {
  GVL_REQUIRE(g && workspace && out, "gvl_grad_norm: null buffer");
  GVL_REQUIRE(gvl::aligned16(g), "gvl_grad_norm: g must be 16-byte aligned");
  const int nb = red_blocks(n >> 3);
  hipStream_t s = gvl::as_stream(stream);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(RED_NT), 0, s, static_cast<const bf16_t*>(g), n,
                     static_cast<float*>(workspace));
  GVL_LAUNCH_CHECK("gvl_grad_norm(sumsq)");
  hipLaunchKernelGGL(norm_finish_kernel, dim3(1), dim3(RED_NT), 0, s,
                     static_cast<const float*>(workspace), nb, max_norm, out);
  GVL_LAUNCH_CHECK("gvl_grad_norm(finish)");
  return 0;
}

extern "C" int gvl_adamw(void* p, const void* g, void* m, void* v, int64_t n, int64_t n_decay,
                         float lr, float beta1, float beta2, float eps, float weight_decay,
                         int64_t step, const float* grad_scale, gvl_stream_t stream) {
  GVL_REQUIRE(p && g && m && v, "gvl_adamw: null buffer");
  GVL_REQUIRE(step >= 1, "gvl_adamw: step must be >= 1");
  GVL_REQUIRE(gvl::aligned16(p) && gvl::aligned16(g) && gvl::aligned16(m) && gvl::aligned16(v),
              "gvl_adamw: arenas must be 16-byte aligned");
  if (n == 0) return 0;
  AdamP a;
  a.lr = lr; a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.wd = weight_decay;
  a.bc1 = (float)(1.0 - pow((double)beta1, (double)step));
  a.bc2_sqrt = (float)sqrt(1.0 - pow((double)beta2, (double)step));
  hipLaunchKernelGGL(adamw_kernel, dim3(ew_blocks(n >> 3)), dim3(256), 0, gvl::as_stream(stream),
                     static_cast<bf16_t*>(p), static_cast<const bf16_t*>(g),
                     static_cast<bf16_t*>(m), static_cast<bf16_t*>(v), n, n_decay, a, grad_scale,
                     nullptr);
  GVL_LAUNCH_CHECK("gvl_adamw");
  return 0;
}

extern "C" int gvl_adamw_dev(void* p, const void* g, void* m, void* v, int64_t n, int64_t n_decay,
                             const float* hyper, float beta1, float beta2, float eps,
                             float weight_decay, const float* grad_scale, gvl_stream_t stream) {
  GVL_REQUIRE(p && g && m && v && hyper, "gvl_adamw_dev: null buffer");
  GVL_REQUIRE(gvl::aligned16(p) && gvl::aligned16(g) && gvl::aligned16(m) && gvl::aligned16(v),
              "gvl_adamw_dev: arenas must be 16-byte aligned");
  if (n == 0) return 0;
  AdamP a;
  a.lr = 0.f; a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.wd = weight_decay;
  a.bc1 = 1.f; a.bc2_sqrt = 1.f;
  hipLaunchKernelGGL(adamw_kernel, dim3(ew_blocks(n >> 3)), dim3(256), 0, gvl::as_stream(stream),
                     static_cast<bf16_t*>(p), static_cast<const bf16_t*>(g),
                     static_cast<bf16_t*>(m), static_cast<bf16_t*>(v), n, n_decay, a, grad_scale,
                     hyper);
  GVL_LAUNCH_CHECK("gvl_adamw_dev");
  return 0;
}

extern "C" int gvl_adamw_master_dev(void* p, float* p_master, const void* g, float* m, float* v,
                                    int64_t n, int64_t n_decay, const float* hyper, float beta1,
                                    float beta2, float eps, float weight_decay,
                                    const float* grad_scale, gvl_stream_t stream) {
  GVL_REQUIRE(p && p_master && g && m && v && hyper, "gvl_adamw_master_dev: null buffer");
  GVL_REQUIRE(gvl::aligned16(p) && gvl::aligned16(g) && gvl::aligned16(p_master) &&
                  gvl::aligned16(m) && gvl::aligned16(v),
              "gvl_adamw_master_dev: arenas must be 16-byte aligned");
  if (n == 0) return 0;
  AdamP a;
  a.lr = 0.f; a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.wd = weight_decay;
  a.bc1 = 1.f; a.bc2_sqrt = 1.f;
  hipLaunchKernelGGL(adamw_master_kernel, dim3(ew_blocks(n >> 3)), dim3(256), 0,
                     gvl::as_stream(stream), static_cast<bf16_t*>(p), p_master,
                     static_cast<const bf16_t*>(g), m, v, n, n_decay, a, grad_scale, hyper);
  GVL_LAUNCH_CHECK("gvl_adamw_master_dev");
  return 0;
}

extern "C" int64_t gvl_colsum_workspace_size(int64_t rows, int64_t cols) {
  int64_t chunk;
  return (int64_t)colsum_blocks(rows, cols, &chunk) * cols * (int64_t)sizeof(float);
}

extern "C" int gvl_colsum(const void* x, int64_t rows, int64_t cols, int64_t ld, void* out,
                          int32_t accumulate, void* workspace, gvl_stream_t stream) {
  GVL_REQUIRE(cols % 8 == 0 && ld % 8 == 0, "gvl_colsum: cols/ld must be multiples of 8");
  GVL_REQUIRE(workspace && out, "gvl_colsum: null buffer");
  GVL_REQUIRE(rows == 0 || gvl::aligned16(x), "gvl_colsum: x must be 16-byte aligned");
  if (cols == 0) return 0;
  int64_t chunk;
  const int nb = colsum_blocks(rows, cols, &chunk);
  hipStream_t s = gvl::as_stream(stream);
  if (rows == 0) {
    (void)hipMemsetAsync(workspace, 0, cols * sizeof(float), s);
  } else {
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((unsigned)((cols + CS_COLS - 1) / CS_COLS), nb),
                       dim3(256), 0, s,
                       static_cast<const bf16_t*>(x), rows, cols, ld, chunk,
                       static_cast<float*>(workspace));
    GVL_LAUNCH_CHECK("gvl_colsum(partial)");
  }
  hipLaunchKernelGGL(colsum_finish_kernel, dim3((unsigned)((cols + 31) / 32)), dim3(256), 0, s,
                     static_cast<const float*>(workspace), rows == 0 ? 1 : nb, cols,
                     static_cast<bf16_t*>(out), (int)accumulate);
  GVL_LAUNCH_CHECK("gvl_colsum(finish)");
  return 0;
}

// Row splits per problem of a batched column sum: the whole launch still has >= ~768 blocks.
static int colsum_blocks_batched(int64_t rows, int64_t cols, int count, int64_t* chunk) {
  const int64_t cb = (cols + CS_COLS - 1) / CS_COLS;
  int64_t nb = (768 + cb * count - 1) / (cb * count);
  const int64_t by_rows = (rows + 63) / 64;
  if (nb > by_rows) nb = by_rows;
  if (nb > CS_MAX_SPLITS) nb = CS_MAX_SPLITS;
  if (nb < 1) nb = 1;
  *chunk = (rows + nb - 1) / nb;
  return (int)nb;
}

extern "C" int64_t gvl_colsum_batched_workspace_size(int32_t count, int64_t rows, int64_t cols) {
  int64_t chunk;
  return (int64_t)count * colsum_blocks_batched(rows, cols, count, &chunk) * cols *
         (int64_t)sizeof(float);
}

extern "C" int gvl_colsum_batched(const void* const* x, void* const* out, int32_t count,
                                  int64_t rows, int64_t cols, int64_t ld, int32_t accumulate,
                                  void* workspace, gvl_stream_t stream) {
  GVL_REQUIRE(x && out && count >= 1 && count <= CS_MAX_BATCH,
              "gvl_colsum_batched: 1..%d problems", CS_MAX_BATCH);
  GVL_REQUIRE(cols % 8 == 0 && ld % 8 == 0 && rows > 0, "gvl_colsum_batched: bad shape");
  GVL_REQUIRE(workspace, "gvl_colsum_batched: null workspace");
  ColsumBatch bt{};
  for (int i = 0; i < count; ++i) {
    GVL_REQUIRE(x[i] && out[i] && gvl::aligned16(x[i]), "gvl_colsum_batched: bad operand %d", i);
    bt.x[i] = static_cast<const bf16_t*>(x[i]);
    bt.out[i] = static_cast<bf16_t*>(out[i]);
  }
  int64_t chunk;
  const int nb = colsum_blocks_batched(rows, cols, count, &chunk);
  hipStream_t s = gvl::as_stream(stream);
  hipLaunchKernelGGL(colsum_partial_batched_kernel,
                     dim3((unsigned)((cols + CS_COLS - 1) / CS_COLS), nb, count), dim3(256), 0, s,
                     bt, rows, cols, ld, chunk, static_cast<float*>(workspace));
  GVL_LAUNCH_CHECK("gvl_colsum_batched(partial)");
  hipLaunchKernelGGL(colsum_finish_batched_kernel, dim3((unsigned)((cols + 31) / 32), count),
                     dim3(256), 0, s, static_cast<const float*>(workspace), nb, cols, bt,
                     (int)accumulate);
  GVL_LAUNCH_CHECK("gvl_colsum_batched(finish)");
  return 0;
}

extern "C" int gvl_dropout_mask_apply(const void* in, int64_t ld_in, void* out, int64_t ld_out,
                                      int64_t rows, int64_t cols, float p, uint64_t seed,
                                      const uint64_t* seed_ptr, gvl_stream_t stream) {
  GVL_REQUIRE(p >= 0.f && p < 1.f, "gvl_dropout_mask_apply: p out of range");
  if (rows * cols == 0) return 0;
  const uint32_t thresh = (uint32_t)((double)p * 4294967296.0);
  if (cols % 8 == 0 && ld_in % 8 == 0 && ld_out % 8 == 0 && gvl::aligned16(in) && gvl::aligned16(out)) {
    hipLaunchKernelGGL(dropout_apply8_kernel, dim3(ew_blocks(rows * cols / 8)), dim3(256), 0,
                       gvl::as_stream(stream), static_cast<const bf16_t*>(in), ld_in,
                       static_cast<bf16_t*>(out), ld_out, rows, cols, seed, seed_ptr, thresh,
                       1.f / (1.f - p));
    GVL_LAUNCH_CHECK("gvl_dropout_mask_apply");
    return 0;
  }
  hipLaunchKernelGGL(dropout_apply_kernel, dim3(ew_blocks(rows * cols)), dim3(256), 0,
                     gvl::as_stream(stream), static_cast<const bf16_t*>(in), ld_in,
                     static_cast<bf16_t*>(out), ld_out, rows, cols, seed, seed_ptr, thresh,
                     1.f / (1.f - p));
  GVL_LAUNCH_CHECK("gvl_dropout_mask_apply");
  return 0;
}

extern "C" int64_t gvl_gate_bwd_workspace_size(int64_t n) {
  return (int64_t)red_blocks(n) * (int64_t)sizeof(float);
}

static int gate_bwd_impl(const void* dx, const void* y, const void* gate, void* dy, float* gate_grad,
                         void* gate_grad_bf16, int64_t n, void* workspace, gvl_stream_t stream) {
  GVL_REQUIRE(dx && y && gate && dy && (gate_grad || gate_grad_bf16) && workspace,
              "gvl_gate_bwd: null buffer");
  const int nb = red_blocks(n);
  hipStream_t s = gvl::as_stream(stream);
  const bool vec = n % 8 == 0 && gvl::aligned16(dx) && gvl::aligned16(y) && gvl::aligned16(dy);
  const int nb8 = red_blocks(n >> 3);  // <= nb: the workspace (red_blocks(n) floats) covers it
  if (vec)
    hipLaunchKernelGGL(gate_bwd8_kernel, dim3(nb8), dim3(RED_NT), 0, s, static_cast<const bf16_t*>(dx),
                       static_cast<const bf16_t*>(y), static_cast<const bf16_t*>(gate),
                       static_cast<bf16_t*>(dy), n >> 3, static_cast<float*>(workspace));
  else
    hipLaunchKernelGGL(gate_bwd_kernel, dim3(nb), dim3(RED_NT), 0, s, static_cast<const bf16_t*>(dx),
                       static_cast<const bf16_t*>(y), static_cast<const bf16_t*>(gate),
                       static_cast<bf16_t*>(dy), n, static_cast<float*>(workspace));
  GVL_LAUNCH_CHECK("gvl_gate_bwd");
  if (gate_grad_bf16)
    hipLaunchKernelGGL(gate_finish_bf16_kernel, dim3(1), dim3(RED_NT), 0, s,
                       static_cast<const float*>(workspace), vec ? nb8 : nb,
                       static_cast<const bf16_t*>(gate), static_cast<bf16_t*>(gate_grad_bf16));
  else
    hipLaunchKernelGGL(gate_finish_kernel, dim3(1), dim3(RED_NT), 0, s,
                       static_cast<const float*>(workspace), vec ? nb8 : nb,
                       static_cast<const bf16_t*>(gate), gate_grad);
  GVL_LAUNCH_CHECK("gvl_gate_bwd(finish)");
  return 0;
}

extern "C" int gvl_gate_bwd(const void* dx, const void* y, const void* gate, void* dy,
                            float* gate_grad, int64_t n, void* workspace, gvl_stream_t stream) {
  return gate_bwd_impl(dx, y, gate, dy, gate_grad, nullptr, n, workspace, stream);
}

extern "C" int gvl_gate_bwd_acc_bf16(const void* dx, const void* y, const void* gate, void* dy,
                                     void* gate_grad, int64_t n, void* workspace,
                                     gvl_stream_t stream) {
  GVL_REQUIRE(gate_grad != nullptr, "gvl_gate_bwd_acc_bf16: null gate_grad");
  return gate_bwd_impl(dx, y, gate, dy, nullptr, gate_grad, n, workspace, stream);
}

extern "C" int gvl_f32_to_bf16(const float* in, void* out, int64_t n, int32_t accumulate,
                               gvl_stream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(ew_blocks(n)), dim3(256), 0, gvl::as_stream(stream),
                     in, static_cast<bf16_t*>(out), n, (int)accumulate);
  GVL_LAUNCH_CHECK("gvl_f32_to_bf16");
  return 0;
}
