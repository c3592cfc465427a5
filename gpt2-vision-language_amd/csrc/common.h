// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of libgvl.
// bf16 is carried as raw 16-bit words (uint16_t) in memory; arithmetic is fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GVL_DEV __device__ __forceinline__

typedef uint16_t bf16_t;
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4_t lds_short4_t;

GVL_DEV float bf2f(uint32_t x) { return __uint_as_float(x << 16); }
GVL_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN-preserving
  return __builtin_bit_cast(bf16_t, b);
}
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));
GVL_DEV uint32_t pack2(float lo, float hi) {  // one v_cvt_pk_bf16_f32 (RNE)
  const bf16x2_t b = __builtin_convertvector(float2_t{lo, hi}, bf16x2_t);
  return __builtin_bit_cast(uint32_t, b);
}
GVL_DEV float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
GVL_DEV float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
GVL_DEV void unpack8(const uint4& u, float (&f)[8]) {
  f[0] = lo_bf(u.x); f[1] = hi_bf(u.x); f[2] = lo_bf(u.y); f[3] = hi_bf(u.y);
  f[4] = lo_bf(u.z); f[5] = hi_bf(u.z); f[6] = lo_bf(u.w); f[7] = hi_bf(u.w);
}
GVL_DEV uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// 16x16x32 bf16 MFMA: D = A(16x32) * B(32x16) + C.
// Lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]; D[4(l>>4)+r][l&15].
GVL_DEV float4_t mfma16(const short8_t& a, const short8_t& b, const float4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Transposed LDS read (ds_read_b64_tr_b16): per 16-lane group, lane 4q+p supplies the
// address of row q, cols 4p..4p+3 of a 4x16 block; lane i receives column i of rows 0..3.
GVL_DEV short4_t lds_read_tr(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4_t*)(lds_ptr));
}

GVL_DEV float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
GVL_DEV float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Wave reductions without LDS round trips (__shfl_xor lowers to ds_bpermute_b32 plus an
// lgkmcnt(0) wait per step): DPP within each 16-lane row (xor 1, xor 2, then the 8- and 16-lane
// mirrors, each pairing two already-uniform halves), then the gfx950 row swaps (l ^ 16, l ^ 32),
// all VALU.  Every step combines two equal-valued groups, so every lane ends with the same bits.
template <int CTRL>
GVL_DEV float dpp_src(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <bool MAX>
GVL_DEV float dpp_op(float a, float b) { return MAX ? fmaxf(a, b) : a + b; }
template <bool MAX>
GVL_DEV float row16_reduce(float v) {
  v = dpp_op<MAX>(v, dpp_src<0xB1>(v));   // quad_perm [1,0,3,2]: l ^ 1
  v = dpp_op<MAX>(v, dpp_src<0x4E>(v));   // quad_perm [2,3,0,1]: l ^ 2
  v = dpp_op<MAX>(v, dpp_src<0x141>(v));  // row_half_mirror: the other quad of the 8
  return dpp_op<MAX>(v, dpp_src<0x140>(v));  // row_mirror: the other 8 of the 16
}
template <bool MAX>
GVL_DEV float swap16_reduce(float v) {  // op(v(l), v(l ^ 16))
  const uint32_t u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return dpp_op<MAX>(__uint_as_float(a[0]), __uint_as_float(a[1]));
}
template <bool MAX>
GVL_DEV float swap32_reduce(float v) {  // op(v(l), v(l ^ 32))
  const uint32_t u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return dpp_op<MAX>(__uint_as_float(a[0]), __uint_as_float(a[1]));
}
GVL_DEV float wave_sum_v(float v) { return swap32_reduce<false>(swap16_reduce<false>(row16_reduce<false>(v))); }
GVL_DEV float wave_max_v(float v) { return swap32_reduce<true>(swap16_reduce<true>(row16_reduce<true>(v))); }
GVL_DEV float half_sum_v(float v) { return swap16_reduce<false>(row16_reduce<false>(v)); }  // per 32 lanes

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
// V: the wave step by wave_sum_v (VALU) instead of warp_sum (LDS permutes).
template <int NT, bool V = false>
GVL_DEV float block_sum(float v, float* red) {
  v = V ? wave_sum_v(v) : warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}
template <int NT, bool V = false>
GVL_DEV float block_max(float v, float* red) {
  v = V ? wave_max_v(v) : warp_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s = fmaxf(s, red[i]);
  return s;
}

// GELU variants used by the reference: nn.GELU(approximate='tanh') in the GPT-2 MLP
// (source/gpt2/train_gpt2.py:52) and exact-erf nn.GELU() in the Q-Former MLP
// (source/gpt2_q_former/model.py:126-130).
// These run in GEMM epilogues over every element of the MLP hidden layer, where the VALU
// cost of libm tanhf/erff (~60 instructions) outweighed the tile's MFMA time; they are
// written on bare v_exp_f32 / v_rcp_f32 instead:
//   0.5 (1 + tanh(u)) = sigmoid(2u)   and   1 - tanh(u)^2 = 4 s (1 - s),
// and erf by Abramowitz-Stegun 7.1.26 (|err| < 1.5e-7).  Both stay far inside the bf16
// rounding of the stored values.
GVL_DEV float fast_sigmoid(float z) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * z));
}
// s = sigmoid(2u), u = k0 (x + k1 x^3), with 2 k0 log2(e) folded into the polynomial.
GVL_DEV float gelu_tanh_sig(float x, float x2) {
  constexpr float A = 2.f * 0.7978845608028654f * 1.4426950408889634f, B = A * 0.044715f;
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * fmaf(B, x2, A)));
}
GVL_DEV float gelu_tanh(float x) { return x * gelu_tanh_sig(x, x * x); }
// CLIP's quick-GELU x * sigmoid(1.702 x) (transformers QuickGELUActivation), one exp + rcp
GVL_DEV float quick_gelu(float x) {
  constexpr float A = 1.702f * 1.4426950408889634f;
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-A * x));
}
GVL_DEV float dgelu_tanh(float x) {
  // d/dx x s(2u) = s + 2 k0 x s (1 - s) (1 + 3 k1 x^2)
  constexpr float C = 2.f * 0.7978845608028654f, D = 3.f * 0.044715f * C;
  const float x2 = x * x;
  const float s = gelu_tanh_sig(x, x2);
  return fmaf(x * s * (1.f - s), fmaf(D, x2, C), s);
}
// GELU and its derivative at once (one sigmoid / one erf), for the forward epilogues that
// store gelu'(x) for the backward instead of x.
GVL_DEV void gelu_dgelu_tanh(float x, float& g, float& dg) {
  constexpr float C = 2.f * 0.7978845608028654f, D = 3.f * 0.044715f * C;
  const float x2 = x * x;
  const float s = gelu_tanh_sig(x, x2);
  g = x * s;
  dg = fmaf(x * s * (1.f - s), fmaf(D, x2, C), s);
}
GVL_DEV float fast_erf(float x);
GVL_DEV void gelu_dgelu_erf(float x, float& g, float& dg) {
  const float cdf2 = 1.f + fast_erf(x * 0.7071067811865476f);  // 2 Phi(x)
  g = 0.5f * x * cdf2;
  dg = fmaf(x * 0.3989422804014327f, __builtin_amdgcn_exp2f(-0.7213475204444817f * x * x), 0.5f * cdf2);
}
GVL_DEV float fast_erf(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * a);
  const float poly =
      t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float r = 1.f - poly * __builtin_amdgcn_exp2f(-1.4426950408889634f * a * a);
  return copysignf(r, x);
}
GVL_DEV float gelu_erf(float x) { return 0.5f * x * (1.f + fast_erf(x * 0.7071067811865476f)); }
GVL_DEV float dgelu_erf(float x) {
  return 0.5f * (1.f + fast_erf(x * 0.7071067811865476f)) +
         x * 0.3989422804014327f * __builtin_amdgcn_exp2f(-0.7213475204444817f * x * x);
}

// Counter-based RNG for dropout masks (splitmix64 finaliser over (seed, index)).
GVL_DEV uint32_t rng_u32(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}
// Effective dropout seed: the call's seed, re-keyed by a device-side step offset when one is
// given (graph replays advance the offset on the device, so a captured step draws fresh masks).
GVL_DEV uint64_t seed_eff(uint64_t seed, const uint64_t* off) {
  if (off == nullptr) return seed;
  uint64_t z = *off;
  if (z == 0) return seed;
  z = (z + 0x632BE59BD9B4E019ull) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return seed ^ (z ^ (z >> 31));
}
// keep with probability 1-p: compare against threshold p * 2^32
GVL_DEV bool rng_keep(uint64_t seed, uint64_t idx, uint32_t thresh) {
  return rng_u32(seed, idx) >= thresh;
}
