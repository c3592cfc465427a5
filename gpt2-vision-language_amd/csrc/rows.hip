// Grouped row copy (HBM-bound, 16-B accesses, one wave per destination row): the caption
// path's row placements that ATen would otherwise run as copy / fill kernels —
//   * the image tokens written in front of the text embeddings (the torch.cat of
//     gpt2_linear/model.py:191), and the learned queries broadcast over the batch
//     (gpt2_q_former/model.py:160-161, query_tokens.expand(B, -1, -1));
//   * the text-row gradient of the lm_head placed into the [B, S, C] decoder gradient with
//     the image rows zeroed (the loss covers the text slice only, gpt2_linear/model.py:219-230).
#include "common.h"
#include "capi_util.h"
#include "../../include/gvl.h"

namespace {

// dst row (g, r), r < dst_rows: copied from src row (g, r - dst_off) when
// dst_off <= r < dst_off + T, else zeroed (zero_rest) or left alone.
__global__ __launch_bounds__(256) void copy_rows_kernel(const bf16_t* __restrict__ src,
                                                        int64_t ld_src, int64_t src_rows,
                                                        int64_t src_off, bf16_t* __restrict__ dst,
                                                        int64_t ld_dst, int64_t dst_rows,
                                                        int64_t dst_off, int64_t T, int64_t G,
                                                        int cols, int zero_rest) {
  const int64_t span = zero_rest ? dst_rows : T;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= G * span) return;
  const int lane = threadIdx.x & 63;
  const int64_t g = w / span, i = w % span;
  const int64_t r = zero_rest ? i : dst_off + i;  // destination row within the group
  const int64_t t = r - dst_off;
  bf16_t* d = dst + (g * dst_rows + r) * ld_dst;
  if (t >= 0 && t < T) {
    const bf16_t* s = src + (g * src_rows + src_off + t) * ld_src;
    for (int c = lane * 8; c < cols; c += 512)
      *reinterpret_cast<uint4*>(d + c) = *reinterpret_cast<const uint4*>(s + c);
  } else {
    for (int c = lane * 8; c < cols; c += 512) *reinterpret_cast<uint4*>(d + c) = make_uint4(0, 0, 0, 0);
  }
}

}  // namespace

extern "C" int gvl_copy_rows(const void* src, int64_t ld_src, int64_t src_rows, int64_t src_off,
                             void* dst, int64_t ld_dst, int64_t dst_rows, int64_t dst_off,
                             int64_t T, int64_t G, int64_t cols, int32_t zero_rest,
                             gvl_stream_t stream) {
  GVL_REQUIRE(cols % 8 == 0 && ld_src % 8 == 0 && ld_dst % 8 == 0 && cols <= ld_dst,
              "gvl_copy_rows: cols and strides must be multiples of 8 elements");
  GVL_REQUIRE(gvl::aligned16(src) && gvl::aligned16(dst), "gvl_copy_rows: 16-B alignment");
  GVL_REQUIRE(T >= 0 && G >= 0 && dst_off >= 0 && dst_off + T <= dst_rows && src_rows >= 0,
              "gvl_copy_rows: rows out of range");
  const int64_t n = G * (zero_rest ? dst_rows : T);
  if (n == 0) return 0;
  hipLaunchKernelGGL(copy_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0,
                     gvl::as_stream(stream), static_cast<const bf16_t*>(src), ld_src, src_rows,
                     src_off, static_cast<bf16_t*>(dst), ld_dst, dst_rows, dst_off, T, G, (int)cols,
                     (int)zero_rest);
  GVL_LAUNCH_CHECK("gvl_copy_rows");
  return 0;
}
