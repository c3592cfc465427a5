// Fused softmax cross-entropy over bf16 logits (fp32 math): one 512-thread block per
// target row (V need not be a multiple of 8: the row buffer is padded to a multiple of 8
// columns and the tail columns count as -inf / get a zero gradient), the whole row held in registers (<= 16 x 16-B chunks per thread, V <= 65536),
// so logits are read from HBM once and dlogits = softmax - onehot written once.  512 threads
// keep the row buffer at 64 VGPRs, so 2+ rows per CU are resident and one row's reductions
// overlap another's loads; exponentials are bare v_exp_f32 on log2e-prescaled inputs.
// HBM-bound: 2*V (read) + 2*V (write) bytes per row.
#include "common.h"
#include "capi_util.h"
#include "../../include/gvl.h"

namespace {

#ifndef GVL_CE_NT  // threads per row (A/B: 1024 holds 8 chunks per thread instead of 16)
#define GVL_CE_NT 512
#endif
constexpr int CE_NT = GVL_CE_NT;
// cache policy A/B (build time): GVL_CE_LDNT=1 nontemporal logit loads, GVL_CE_STNT=1
// nontemporal dlogits stores
#ifndef GVL_CE_LDNT
#define GVL_CE_LDNT 0
#endif
#ifndef GVL_CE_STNT
#define GVL_CE_STNT 0
#endif
typedef uint32_t ce_u32x4 __attribute__((ext_vector_type(4)));
GVL_DEV uint4 ce_load(const bf16_t* p) {
  if constexpr (GVL_CE_LDNT)
    return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const ce_u32x4*>(p)));
  return *reinterpret_cast<const uint4*>(p);
}
GVL_DEV void ce_store(bf16_t* p, uint4 v) {
  if constexpr (GVL_CE_STNT) __builtin_nontemporal_store(__builtin_bit_cast(ce_u32x4, v), reinterpret_cast<ce_u32x4*>(p));
  else *reinterpret_cast<uint4*>(p) = v;
}
// row max / sum wave steps by DPP + lane swaps (common.h wave_max_v / wave_sum_v); 0: LDS permutes
#ifndef GVL_CE_DPP
#define GVL_CE_DPP 1
#endif
constexpr int CE_MAXC = 8192 / CE_NT;  // 16-B chunks per thread: V <= 65536
constexpr float CE_L2E = 1.4426950408889634f;

// bf16 -inf in columns [nvalid, 8) of an 8-column chunk (exp2 of it is exactly 0, so the
// softmax ignores them and their dlogits come out 0)
GVL_DEV uint4 mask_tail(uint4 u, int64_t nvalid) {
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (2 * k >= nvalid) w[k] = (w[k] & 0xFFFF0000u) | 0xFF80u;
    if (2 * k + 1 >= nvalid) w[k] = (w[k] & 0x0000FFFFu) | 0xFF800000u;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ __launch_bounds__(CE_NT) void ce_row_kernel(
    const bf16_t* __restrict__ logits, int64_t ldl, int64_t V, int64_t rpg, int64_t gstride,
    int64_t roff, const int64_t* __restrict__ targets, const uint8_t* __restrict__ mask,
    float* __restrict__ row_loss, bf16_t* __restrict__ dlogits, int64_t ldd) {
  __shared__ float red[CE_NT / 64];
  const int64_t r = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t lrow = (r / rpg) * gstride + roff + (r % rpg);
  const bf16_t* src = logits + lrow * ldl;
  bf16_t* dst = dlogits ? dlogits + r * ldd : nullptr;
  const int64_t tgt = targets[r];
  const bool valid = (tgt != -100) && (mask == nullptr || mask[r] != 0);
  const int nch = (int)((V + 7) >> 3);
  if (valid && (tgt < 0 || tgt >= V)) {
    // out-of-range class index (torch raises; the host-side check in gvl.functional does
    // too): never read outside the row, poison the loss instead
    if (dst)
      for (int c = tid; c < nch; c += CE_NT)
        *reinterpret_cast<uint4*>(dst + (int64_t)c * 8) = make_uint4(0, 0, 0, 0);
    if (tid == 0) row_loss[r] = __int_as_float(0x7fc00000);
    return;
  }
  if (!valid) {
    if (dst) {
      for (int c = tid; c < nch; c += CE_NT)
        *reinterpret_cast<uint4*>(dst + (int64_t)c * 8) = make_uint4(0, 0, 0, 0);
    }
    if (tid == 0) row_loss[r] = 0.f;
    return;
  }
  uint4 buf[CE_MAXC];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < CE_MAXC; ++i) {
    const int c = tid + i * CE_NT;
    if (c < nch) {
      buf[i] = ce_load(src + (int64_t)c * 8);
      if ((int64_t)c * 8 + 8 > V) buf[i] = mask_tail(buf[i], V - (int64_t)c * 8);
      const uint32_t w[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) mx = fmaxf(mx, fmaxf(lo_bf(w[k]), hi_bf(w[k])));
    }
  }
  mx = block_max<CE_NT, GVL_CE_DPP>(mx, red);
  const float mxl = mx * CE_L2E;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CE_MAXC; ++i) {
    const int c = tid + i * CE_NT;
    if (c < nch) {
      const uint32_t w[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        s += __builtin_amdgcn_exp2f(fmaf(lo_bf(w[k]), CE_L2E, -mxl)) +
             __builtin_amdgcn_exp2f(fmaf(hi_bf(w[k]), CE_L2E, -mxl));
    }
  }
  s = block_sum<CE_NT, GVL_CE_DPP>(s, red);
  const float lse = mx + __logf(s);
  if (tid == 0) row_loss[r] = lse - bf2f(src[tgt]);
  if (dst) {
    const float inv = 1.f / s;
#pragma unroll
    for (int i = 0; i < CE_MAXC; ++i) {
      const int c = tid + i * CE_NT;
      if (c < nch) {
        const uint32_t w[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
        uint32_t o[4];
        const int64_t base = (int64_t)c * 8;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float a = __builtin_amdgcn_exp2f(fmaf(lo_bf(w[k]), CE_L2E, -mxl)) * inv;
          float b = __builtin_amdgcn_exp2f(fmaf(hi_bf(w[k]), CE_L2E, -mxl)) * inv;
          if (base + 2 * k == tgt) a -= 1.f;
          if (base + 2 * k + 1 == tgt) b -= 1.f;
          o[k] = pack2(a, b);
        }
        ce_store(dst + base, make_uint4(o[0], o[1], o[2], o[3]));
      }
    }
  }
}

// HAS_MASK as a template argument: a per-row `mask == nullptr ||` test put a branch with a full
// vmcnt(0) wait into every unrolled row.
template <bool HAS_MASK>
__global__ __launch_bounds__(1024) void ce_finalize_kernel(const float* __restrict__ row_loss,
                                                           const int64_t* __restrict__ targets,
                                                           const uint8_t* __restrict__ mask,
                                                           int64_t rows, int mask_mode,
                                                           float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f, n = 0.f;
  // branch-free loads (every row's loss slot is in bounds; an ignored row's value is selected
  // away), unrolled: the rows' target, mask and loss loads all in flight together.  The loss
  // load behind the `valid` branch waited for the target first, one round trip after the other
  // for each of a thread's 16 rows (17 us for the LM's 16384 rows).
#pragma unroll 8
  for (int64_t r = threadIdx.x; r < rows; r += 1024) {
    const float l = row_loss[r];
    const bool mk = !HAS_MASK || mask[r] != 0;
    const bool valid = (targets[r] != -100) && mk;
    s += valid ? l : 0.f;
    // masked mean divides by sum(mask) (gpt2_cross-att/model.py:184-185); the ignore_index
    // mean by the number of non-ignored targets (F.cross_entropy default)
    if (mask_mode ? mk : valid) n += 1.f;
  }
  s = block_sum<1024>(s, red);
  n = block_sum<1024>(n, red);
  if (threadIdx.x == 0) {
    float inv = mask_mode ? 1.f / fmaxf(n, 1.f) : 1.f / n;  // 0/0 -> nan like torch
    out[0] = (n == 0.f && !mask_mode) ? __int_as_float(0x7fc00000) : s * inv;
    out[1] = inv;
  }
}

}  // namespace

extern "C" int gvl_cross_entropy(const void* logits, int64_t ldl, int64_t rows, int64_t vocab,
                                 int64_t rows_per_group, int64_t group_stride, int64_t row_offset,
                                 const int64_t* targets, const uint8_t* mask, int32_t mask_mode,
                                 float* row_loss, void* dlogits, int64_t ldd, float* out,
                                 gvl_stream_t stream) {
  const int64_t vpad = (vocab + 7) / 8 * 8;
  GVL_REQUIRE(vocab > 0 && vpad / 8 <= (int64_t)CE_NT * CE_MAXC,
              "gvl_cross_entropy: vocab=%lld unsupported (1..65536)", (long long)vocab);
  GVL_REQUIRE(ldl % 8 == 0 && ldl >= vpad && (!dlogits || (ldd % 8 == 0 && ldd >= vpad)),
              "gvl_cross_entropy: row strides must be multiples of 8 covering the vocab rounded "
              "up to 8 (ldl=%lld ldd=%lld vocab=%lld)", (long long)ldl, (long long)ldd,
              (long long)vocab);
  GVL_REQUIRE(rows_per_group > 0, "gvl_cross_entropy: rows_per_group must be > 0");
  GVL_REQUIRE(row_loss && out && targets, "gvl_cross_entropy: null buffer");
  hipStream_t s = gvl::as_stream(stream);
  if (rows > 0) {
    hipLaunchKernelGGL(ce_row_kernel, dim3((unsigned)rows), dim3(CE_NT), 0, s,
                       static_cast<const bf16_t*>(logits), ldl, vocab, rows_per_group, group_stride,
                       row_offset, targets, mask, row_loss, static_cast<bf16_t*>(dlogits), ldd);
    GVL_LAUNCH_CHECK("gvl_cross_entropy(rows)");
  }
  if (mask)
    hipLaunchKernelGGL(ce_finalize_kernel<true>, dim3(1), dim3(1024), 0, s, row_loss, targets, mask,
                       rows, (int)mask_mode, out);
  else
    hipLaunchKernelGGL(ce_finalize_kernel<false>, dim3(1), dim3(1024), 0, s, row_loss, targets, mask,
                       rows, (int)mask_mode, out);
  GVL_LAUNCH_CHECK("gvl_cross_entropy(finalize)");
  return 0;
}
