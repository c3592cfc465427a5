// Incremental decoding: single-query attention over a KV cache and a fused
// temperature / top-k / top-p sampler.  Both are latency-bound (one new token per sequence).
//
// attn_decode_kernel: one 256-thread workgroup per (head, sequence).  Pass 1 scores every
// cached key against the new query (one key per thread, 8 x 16-B loads of its 64-dim row) into
// an LDS score array, block max/sum in fp32; pass 2 accumulates p_t * v_t with 8 threads per
// value row (16-B loads, 32 rows in flight per sweep) and folds the 32 partial rows in LDS.
//
// sample_kernel: one 1024-thread workgroup per row; the row (V <= 65536) sits in registers as
// contiguous 64-element chunks.  softmax(logits / T) -> top-k by an 8-bit radix select on the
// probability bits -> top-p by a radix search on probability MASS (the kept set is the
// reference's sorted-cumsum prefix: every token whose preceding cumulative probability is
// <= top_p, gpt2_linear/data.py:117-122) -> inverse-CDF draw of the caller's uniform u in
// token-index order (block prefix scan of the per-thread kept mass).
#include "common.h"
#include "capi_util.h"
#include "../../include/gvl.h"

namespace {

constexpr int DEC_NT = 256;
constexpr int DEC_MAXT = 4096;
constexpr float DEC_L2E = 1.4426950408889634f;

struct DecP {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  int64_t Tk, q_sb, k_sb, k_st, v_sb, v_st, o_sb;
  float scale;
};

__global__ __launch_bounds__(DEC_NT) void attn_decode_kernel(DecP p) {
  __shared__ float qs[64];
  __shared__ float sc[DEC_MAXT];
  __shared__ float red[DEC_NT / 64];
  __shared__ float part[32][65];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  if (tid < 64) qs[tid] = bf2f(p.q[b * p.q_sb + h * 64 + tid]) * (p.scale * DEC_L2E);
  __syncthreads();
  float q[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) q[d] = qs[d];
  const bf16_t* kb = p.k + b * p.k_sb + h * 64;
  float mx = -INFINITY;
  for (int64_t t = tid; t < p.Tk; t += DEC_NT) {
    const uint4* row = reinterpret_cast<const uint4*>(kb + t * p.k_st);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float f[8];
      unpack8(row[c], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s = fmaf(q[8 * c + j], f[j], s);
    }
    sc[t] = s;
    mx = fmaxf(mx, s);
  }
  mx = block_max<DEC_NT>(mx, red);
  float l = 0.f;
  for (int64_t t = tid; t < p.Tk; t += DEC_NT) {
    const float e = __builtin_amdgcn_exp2f(sc[t] - mx);
    sc[t] = e;
    l += e;
  }
  l = block_sum<DEC_NT>(l, red);  // (its barriers also publish sc[])
  const int d8 = tid & 7, tg = tid >> 3;
  const bf16_t* vb = p.v + b * p.v_sb + h * 64 + d8 * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t t = tg; t < p.Tk; t += 32) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(vb + t * p.v_st), f);
    const float w = sc[t];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = fmaf(w, f[j], acc[j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[tg][d8 * 8 + j] = acc[j];
  __syncthreads();
  if (tid < 64) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 32; ++g) s += part[g][tid];
    p.o[b * p.o_sb + h * 64 + tid] = f2bf(s / l);
  }
}

constexpr int SMP_NT = 1024;
constexpr int SMP_E = 64;  // elements per thread: V <= 65536

struct SampP {
  const void* logits;
  int64_t ld, V;
  int f32;
  float inv_temp;
  int top_k;
  float top_p;
  const float* u;
  int64_t* out;
};

// Exclusive prefix sum over the block (SMP_NT threads); `sh` holds SMP_NT/64 floats.
GVL_DEV float block_exscan(float v, float* sh, float* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  __syncthreads();
  if (lane == 63) sh[w] = x;
  __syncthreads();
  float base = 0.f, tot = 0.f;
#pragma unroll
  for (int i = 0; i < SMP_NT / 64; ++i) {
    if (i < w) base += sh[i];
    tot += sh[i];
  }
  *total = tot;
  return base + x - v;
}

// Keep every element > thr and the first n (in token-index order) of those == thr — the
// reference's sorted order breaks ties by index (a stable sort); zero the rest.  Returns the
// kept mass.  Chunks are contiguous per thread, so a block scan of per-thread tie counts gives
// each tied element its index-order rank.
GVL_DEV float keep_at_least(float (&x)[SMP_E], int E, int64_t i0, int64_t V, float thr,
                            uint32_t n, float* red) {
  float ties = 0.f;
#pragma unroll
  for (int j = 0; j < SMP_E; ++j)
    if (j < E && i0 + j < V && x[j] == thr && x[j] > 0.f) ties += 1.f;
  float tot;
  float rank = block_exscan(ties, red, &tot);
  float z = 0.f;
#pragma unroll
  for (int j = 0; j < SMP_E; ++j) {
    if (x[j] > thr) {
      z += x[j];
    } else if (x[j] == thr && x[j] > 0.f && j < E && i0 + j < V) {
      if (rank < (float)n) z += x[j];
      else x[j] = 0.f;
      rank += 1.f;
    } else {
      x[j] = 0.f;
    }
  }
  return block_sum<SMP_NT>(z, red);
}

__global__ __launch_bounds__(SMP_NT) void sample_kernel(SampP p) {
  __shared__ float red[SMP_NT / 64];
  __shared__ uint32_t hist[256];
  __shared__ float histf[256];
  __shared__ uint32_t sel[2];
  __shared__ float c_above;
  const int tid = threadIdx.x;
  const int64_t row = blockIdx.x;
  const int E = (int)((p.V + SMP_NT - 1) / SMP_NT);
  const int64_t i0 = (int64_t)tid * E;
  float x[SMP_E];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < SMP_E; ++j) {
    const int64_t i = i0 + j;
    float v = -INFINITY;
    if (j < E && i < p.V) {
      v = p.f32 ? reinterpret_cast<const float*>(p.logits)[row * p.ld + i]
                : bf2f(reinterpret_cast<const bf16_t*>(p.logits)[row * p.ld + i]);
      v *= p.inv_temp;
    }
    x[j] = v;
    mx = fmaxf(mx, v);
  }
  mx = block_max<SMP_NT>(mx, red);
  float z = 0.f;
#pragma unroll
  for (int j = 0; j < SMP_E; ++j) {
    x[j] = (x[j] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f((x[j] - mx) * DEC_L2E);
    z += x[j];
  }
  z = block_sum<SMP_NT>(z, red);

  if (p.top_k > 0 && p.top_k < p.V) {  // k-th largest probability: radix select on its bits
    uint32_t prefix = 0, msk = 0;
    uint32_t kk = (uint32_t)p.top_k;
    for (int shift = 24; shift >= 0; shift -= 8) {
      if (tid < 256) hist[tid] = 0;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < SMP_E; ++j) {
        const uint32_t bits = __float_as_uint(x[j]);
        if (j < E && i0 + j < p.V && (bits & msk) == prefix) atomicAdd(&hist[(bits >> shift) & 255], 1u);
      }
      __syncthreads();
      if (tid == 0) {
        uint32_t c = 0, chosen = 0;
        for (int bb = 255; bb >= 0; --bb) {
          if (c + hist[bb] >= kk) { chosen = (uint32_t)bb; break; }
          c += hist[bb];
        }
        sel[0] = chosen;
        sel[1] = kk - c;
      }
      __syncthreads();
      prefix |= sel[0] << shift;
      msk |= 255u << shift;
      kk = sel[1];
      __syncthreads();
    }
    z = keep_at_least(x, E, i0, p.V, __uint_as_float(prefix), kk, red);
  }

  if (p.top_p < 1.f) {  // smallest top-mass prefix whose cumulative probability exceeds top_p
    const float target = p.top_p * z;
    uint32_t prefix = 0, msk = 0;
    float above = 0.f;
    for (int shift = 24; shift >= 0; shift -= 8) {
      if (tid < 256) histf[tid] = 0.f;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < SMP_E; ++j) {
        const uint32_t bits = __float_as_uint(x[j]);
        if (x[j] > 0.f && (bits & msk) == prefix) atomicAdd(&histf[(bits >> shift) & 255], x[j]);
      }
      __syncthreads();
      if (tid == 0) {
        float c = above;
        uint32_t chosen = 0;
        for (int bb = 255; bb >= 0; --bb) {
          if (c + histf[bb] > target) { chosen = (uint32_t)bb; break; }
          c += histf[bb];
          chosen = (uint32_t)bb;  // (rounding: never crossed -> the lowest bin with mass)
        }
        sel[0] = chosen;
        c_above = c;
      }
      __syncthreads();
      prefix |= sel[0] << shift;
      msk |= 255u << shift;
      above = c_above;
      __syncthreads();
    }
    // above = mass strictly above thr; the sorted list crosses top_p inside the tie group
    // at thr after n = floor((target - above) / thr) + 1 of its (index-ordered) members
    const float thr = __uint_as_float(prefix);
    const float need = thr > 0.f ? floorf((target - above) / thr) + 1.f : 1.f;
    z = keep_at_least(x, E, i0, p.V, thr, (uint32_t)fmaxf(need, 1.f), red);
  }

  // inverse CDF in token-index order
  float s = 0.f;
  int last = 0;
#pragma unroll
  for (int j = 0; j < SMP_E; ++j) {
    s += x[j];
    if (x[j] > 0.f) last = j;
  }
  float tot;
  const float pre = block_exscan(s, red, &tot);
  const float target = p.u[row] * tot;
  if (tid == 0) {
    sel[0] = 0xFFFFFFFFu;  // drawn index
    sel[1] = 0;            // fallback: the highest-index kept token (target rounded to tot)
  }
  __syncthreads();
  if (s > 0.f) {
    atomicMax(&sel[1], (uint32_t)(i0 + last));
    if (pre <= target && target < pre + s) {
      float acc = pre;
      int pick = last;
      bool found = false;
#pragma unroll
      for (int j = 0; j < SMP_E; ++j) {
        if (!found && x[j] > 0.f) {
          acc += x[j];
          if (acc > target) {
            pick = j;
            found = true;
          }
        }
      }
      atomicMin(&sel[0], (uint32_t)(i0 + pick));
    }
  }
  __syncthreads();
  if (tid == 0) p.out[row] = (int64_t)(sel[0] != 0xFFFFFFFFu ? sel[0] : sel[1]);
}

}  // namespace

extern "C" int gvl_attn_decode(const void* q, int64_t q_sb, const void* k, int64_t k_sb,
                               int64_t k_st, const void* v, int64_t v_sb, int64_t v_st, void* o,
                               int64_t o_sb, int64_t B, int64_t H, int64_t Tk, float scale,
                               gvl_stream_t stream) {
  GVL_REQUIRE(q && k && v && o, "gvl_attn_decode: null buffer");
  GVL_REQUIRE(Tk > 0 && Tk <= DEC_MAXT, "gvl_attn_decode: Tk=%lld out of range (1..%d)",
              (long long)Tk, DEC_MAXT);
  GVL_REQUIRE(k_st % 8 == 0 && v_st % 8 == 0 && k_sb % 8 == 0 && v_sb % 8 == 0 &&
                  gvl::aligned16(k) && gvl::aligned16(v),
              "gvl_attn_decode: K/V rows must be 16-byte aligned");
  if (B == 0 || H == 0) return 0;
  DecP p{static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k),
         static_cast<const bf16_t*>(v), static_cast<bf16_t*>(o), Tk, q_sb, k_sb, k_st,
         v_sb, v_st, o_sb, scale};
  hipLaunchKernelGGL(attn_decode_kernel, dim3((unsigned)H, (unsigned)B), dim3(DEC_NT), 0,
                     gvl::as_stream(stream), p);
  GVL_LAUNCH_CHECK("gvl_attn_decode");
  return 0;
}

extern "C" int gvl_sample(const void* logits, int64_t ld, int32_t logits_fp32, int64_t rows,
                          int64_t V, float temperature, int32_t top_k, float top_p,
                          const float* u, int64_t* out, gvl_stream_t stream) {
  GVL_REQUIRE(logits && u && out, "gvl_sample: null buffer");
  GVL_REQUIRE(V > 0 && V <= (int64_t)SMP_NT * SMP_E, "gvl_sample: V=%lld unsupported", (long long)V);
  GVL_REQUIRE(temperature > 0.f && top_p > 0.f && top_p <= 1.f && top_k >= 0,
              "gvl_sample: bad temperature / top_k / top_p");
  if (rows == 0) return 0;
  SampP p{logits, ld, V, logits_fp32, 1.f / temperature, top_k, top_p, u, out};
  hipLaunchKernelGGL(sample_kernel, dim3((unsigned)rows), dim3(SMP_NT), 0, gvl::as_stream(stream),
                     p);
  GVL_LAUNCH_CHECK("gvl_sample");
  return 0;
}
