// Embedding gather/scatter (K1) and CLIP-token pooling (K15). Both HBM-bound, 16-B
// vector accesses, one wave (embedding) / one block (pool) per output row.
#include "common.h"
#include "capi_util.h"
#include "../../include/gvl.h"

namespace {

// out[row(r)] = wte[idx[r]] + wpe[r % T]; row(r) = (r/T)*S + off + r%T.
__global__ __launch_bounds__(256) void emb_fwd_kernel(const int64_t* __restrict__ idx,
                                                      const bf16_t* __restrict__ wte,
                                                      const bf16_t* __restrict__ wpe,
                                                      bf16_t* __restrict__ out, int64_t n, int64_t T,
                                                      int C, int64_t S, int64_t off, int64_t V) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t t = r % T;
  const int64_t orow = (r / T) * S + off + t;
  // an id outside [0, V) never reads outside wte: it embeds as row 0 (the host-side check
  // in gvl.functional raises on it first, as nn.Embedding does)
  const int64_t id = idx[r];
  const bf16_t* a = wte + ((id >= 0 && id < V) ? id : 0) * (int64_t)C;
  const bf16_t* b = wpe + t * (int64_t)C;
  bf16_t* o = out + orow * (int64_t)C;
  for (int c = lane * 8; c < C; c += 512) {
    const uint4 u = *reinterpret_cast<const uint4*>(a + c);
    const uint4 v = *reinterpret_cast<const uint4*>(b + c);
    uint4 w;
    w.x = pack2(lo_bf(u.x) + lo_bf(v.x), hi_bf(u.x) + hi_bf(v.x));
    w.y = pack2(lo_bf(u.y) + lo_bf(v.y), hi_bf(u.y) + hi_bf(v.y));
    w.z = pack2(lo_bf(u.z) + lo_bf(v.z), hi_bf(u.z) + hi_bf(v.z));
    w.w = pack2(lo_bf(u.w) + lo_bf(v.w), hi_bf(u.w) + hi_bf(v.w));
    *reinterpret_cast<uint4*>(o + c) = w;
  }
}

__global__ __launch_bounds__(256) void emb_bwd_kernel(const int64_t* __restrict__ idx,
                                                      const bf16_t* __restrict__ dout,
                                                      float* __restrict__ dwte,
                                                      float* __restrict__ dwpe, int64_t n, int64_t T,
                                                      int C, int64_t S, int64_t off, int64_t V) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t t = r % T;
  const int64_t orow = (r / T) * S + off + t;
  const bf16_t* g = dout + orow * (int64_t)C;
  const int64_t id = idx[r];
  float* a = (dwte && id >= 0 && id < V) ? dwte + id * (int64_t)C : nullptr;
  float* b = dwpe ? dwpe + t * (int64_t)C : nullptr;
  for (int c = lane * 2; c < C; c += 128) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(g + c);
    const float g0 = lo_bf(u), g1 = hi_bf(u);
    if (a) { atomicAdd(a + c, g0); atomicAdd(a + c + 1, g1); }
    if (b) { atomicAdd(b + c, g0); atomicAdd(b + c + 1, g1); }
  }
}

// ---- deterministic embedding backward (ABI v6) -------------------------------------------
// dwte[v] += sum of dout rows of the tokens with id v, in token order, one fp32 sum per row
// and ONE bf16 read-modify-write per touched row (no atomics: bit-identical run to run).
// A chunk of <= EMB_CHUNK tokens is sorted by the unique key (id << 14 | position) in two
// launches: every 1024-key tile is bitonic-sorted in LDS by its own block (emb_tile_kernel),
// then each key's global rank = its index in its tile + the number of smaller keys in every
// other tile (binary searches in LDS, emb_rank_kernel) scatters it to its sorted slot.  Then
// one wave per sorted slot: the head of each run of equal ids sums its run and updates the
// row.  Larger inputs run chunk after chunk (stream-ordered, so a row touched by two chunks
// is updated in chunk order).  Out-of-range ids get the reserved id field EMB_BAD_ID (still
// unique keys: the position is kept) and are skipped.
constexpr int EMB_CHUNK = 16384;  // 14-bit positions
constexpr int EMB_TILE = 1024;
constexpr uint32_t EMB_BAD_ID = 0x3FFFFu;
constexpr int EMB_MAXC = 1024;    // 64 lanes x 8 bf16 x 2 slices

__global__ __launch_bounds__(EMB_TILE / 2) void emb_tile_kernel(const int64_t* __restrict__ idx,
                                                                int64_t base, int n, int64_t V,
                                                                uint32_t* __restrict__ tiles) {
  __shared__ uint32_t s[EMB_TILE];
  const int t0 = blockIdx.x * EMB_TILE;
  for (int i = threadIdx.x; i < EMB_TILE; i += EMB_TILE / 2) {
    const int p = t0 + i;
    uint32_t key = 0xFFFFFFFFu;  // pad: >= every real key, never ranked below n
    if (p < n) {
      const int64_t id = idx[base + p];
      key = ((id >= 0 && id < V) ? (uint32_t)id : EMB_BAD_ID) << 14 | (uint32_t)p;
    }
    s[i] = key;
  }
  __syncthreads();
  const int t = threadIdx.x;
  for (int k = 2; k <= EMB_TILE; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
      const int l = i + j;
      const uint32_t a = s[i], b = s[l];
      const bool up = (i & k) == 0;
      if ((a > b) == up) { s[i] = b; s[l] = a; }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < EMB_TILE; i += EMB_TILE / 2) tiles[t0 + i] = s[i];
}

// lower_bound: number of entries of the sorted tile p[0, EMB_TILE) that are < key
GVL_DEV int emb_count_less(const uint32_t* p, uint32_t key) {
  int lo = 0;
#pragma unroll
  for (int step = EMB_TILE / 2; step > 0; step >>= 1)
    if (p[lo + step - 1] < key) lo += step;
  return lo + (p[lo] < key ? 1 : 0);
}

__global__ __launch_bounds__(EMB_TILE) void emb_rank_kernel(const uint32_t* __restrict__ tiles,
                                                            int ntiles, int n,
                                                            uint32_t* __restrict__ out) {
  extern __shared__ uint32_t all[];
  for (int i = threadIdx.x; i < ntiles * EMB_TILE; i += EMB_TILE) all[i] = tiles[i];
  __syncthreads();
  const int me = blockIdx.x;
  const uint32_t key = all[me * EMB_TILE + threadIdx.x];
  int rank = threadIdx.x;
  for (int u = 0; u < ntiles; ++u)
    if (u != me) rank += emb_count_less(all + u * EMB_TILE, key);
  if (rank < n) out[rank] = key;
}

// Load order: the run head's key and its predecessor together; then the wte row, the first dout
// row and the NEXT key together (and each further dout row with the key after it), so a run of
// one token — most of them — costs three dependent round trips instead of five.
__global__ __launch_bounds__(256) void emb_seg_kernel(const uint32_t* __restrict__ keys, int n,
                                                       int64_t base, const bf16_t* __restrict__ dout,
                                                       bf16_t* __restrict__ dwte, int64_t T,
                                                       int C, int64_t S, int64_t off) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const uint32_t key = keys[i];
  const uint32_t prev = keys[i > 0 ? i - 1 : i];
  const uint32_t id = key >> 14;
  if (id == EMB_BAD_ID) return;
  if (i > 0 && (prev >> 14) == id) return;  // not the head of its run
  const int lane = threadIdx.x & 63;
  bf16_t* w = dwte + (int64_t)id * C;
  uint4 wu[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = lane * 8 + h * 512;
    if (c < C) wu[h] = *reinterpret_cast<const uint4*>(w + c);
  }
  float acc[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[h][e] = 0.f;
  uint32_t kj = key;
  for (int j = i;;) {
    const int64_t r = base + (int64_t)(kj & 0x3FFFu);
    const bf16_t* g = dout + ((r / T) * S + off + r % T) * (int64_t)C;
    uint4 u[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = lane * 8 + h * 512;
      if (c < C) u[h] = *reinterpret_cast<const uint4*>(g + c);
    }
    const uint32_t kn = j + 1 < n ? keys[j + 1] : 0xFFFFFFFFu;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = lane * 8 + h * 512;
      if (c < C) {
        acc[h][0] += lo_bf(u[h].x); acc[h][1] += hi_bf(u[h].x); acc[h][2] += lo_bf(u[h].y);
        acc[h][3] += hi_bf(u[h].y); acc[h][4] += lo_bf(u[h].z); acc[h][5] += hi_bf(u[h].z);
        acc[h][6] += lo_bf(u[h].w); acc[h][7] += hi_bf(u[h].w);
      }
    }
    if ((kn >> 14) != id) break;
    kj = kn;
    ++j;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = lane * 8 + h * 512;
    if (c < C) {
      const uint4 uw = wu[h];
      uint4 o;
      o.x = pack2(lo_bf(uw.x) + acc[h][0], hi_bf(uw.x) + acc[h][1]);
      o.y = pack2(lo_bf(uw.y) + acc[h][2], hi_bf(uw.y) + acc[h][3]);
      o.z = pack2(lo_bf(uw.z) + acc[h][4], hi_bf(uw.z) + acc[h][5]);
      o.w = pack2(lo_bf(uw.w) + acc[h][6], hi_bf(uw.w) + acc[h][7]);
      *reinterpret_cast<uint4*>(w + c) = o;
    }
  }
}

// dwpe[t] += sum over sequences g of dout[g*S + off + t], one wave per position t.
__global__ __launch_bounds__(256) void emb_pos_kernel(const bf16_t* __restrict__ dout,
                                                       bf16_t* __restrict__ dwpe, int64_t G,
                                                       int64_t T, int C, int64_t S, int64_t off) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int lane = threadIdx.x & 63;
  float acc[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[h][e] = 0.f;
  // four rows' loads in flight, then summed in sequence order (fixed order: deterministic)
  for (int64_t g0 = 0; g0 < G; g0 += 4) {
    uint4 u[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bf16_t* src = dout + ((g0 + q < G ? g0 + q : g0) * S + off + t) * (int64_t)C;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = lane * 8 + h * 512;
        u[q][h] = c < C ? *reinterpret_cast<const uint4*>(src + c) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (g0 + q >= G) break;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        acc[h][0] += lo_bf(u[q][h].x); acc[h][1] += hi_bf(u[q][h].x); acc[h][2] += lo_bf(u[q][h].y);
        acc[h][3] += hi_bf(u[q][h].y); acc[h][4] += lo_bf(u[q][h].z); acc[h][5] += hi_bf(u[q][h].z);
        acc[h][6] += lo_bf(u[q][h].w); acc[h][7] += hi_bf(u[q][h].w);
      }
    }
  }
  bf16_t* w = dwpe + t * (int64_t)C;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = lane * 8 + h * 512;
    if (c < C) {
      const uint4 u = *reinterpret_cast<const uint4*>(w + c);
      uint4 o;
      o.x = pack2(lo_bf(u.x) + acc[h][0], hi_bf(u.x) + acc[h][1]);
      o.y = pack2(lo_bf(u.y) + acc[h][2], hi_bf(u.y) + acc[h][3]);
      o.z = pack2(lo_bf(u.z) + acc[h][4], hi_bf(u.z) + acc[h][5]);
      o.w = pack2(lo_bf(u.w) + acc[h][6], hi_bf(u.w) + acc[h][7]);
      *reinterpret_cast<uint4*>(w + c) = o;
    }
  }
}

// Pool: block per (b, o), o in [0, 33): o=0 is CLS, o=1+i*8+j the adaptive-avg window
// rows [floor(i*s/4), ceil((i+1)*s/4)), cols [floor(j*s/8), ceil((j+1)*s/8)); then the
// 33 tokens are L2-normalised with F.normalize's max(||x||, 1e-12).
constexpr int POOL_NT = 256;
constexpr int POOL_MAXD = 4;  // D <= 1024
constexpr int POOL_WIN = 8;   // pooling windows up to 8 patches (side 16: 4 x 2) take the unrolled path

template <typename TIn>
GVL_DEV float ld_in(const TIn* p);
template <>
GVL_DEV float ld_in<float>(const float* p) { return *p; }
template <>
GVL_DEV float ld_in<bf16_t>(const bf16_t* p) { return bf2f(*p); }

template <typename TIn>
__global__ __launch_bounds__(POOL_NT) void pool_kernel(const TIn* __restrict__ in, void* out,
                                                       int out_f32, int64_t L, int D, int side,
                                                       int normalize) {
  __shared__ float red[POOL_NT / 64];
  const int64_t b = blockIdx.y;
  const int o = blockIdx.x;
  const TIn* base = in + b * L * (int64_t)D;
  float acc[POOL_MAXD];
  int r0 = 0, r1 = 1, c0 = 0, c1 = 1;
  if (o > 0) {
    const int i = (o - 1) >> 3, j = (o - 1) & 7;
    r0 = (i * side) / 4;
    r1 = ((i + 1) * side + 3) / 4;
    c0 = (j * side) / 8;
    c1 = ((j + 1) * side + 7) / 8;
  }
  const int wc = c1 - c0, nwin = (r1 - r0) * wc;
  const float inv_cnt = 1.f / (float)nwin;
  float ss = 0.f;
  if (nwin <= POOL_WIN) {
    // the window's loads unrolled with clamped indices (no branch between them), so every load of
    // the block is in flight before the first add waits (a runtime-bounded loop issued one
    // dependent load per iteration: 8 round trips per column at side 16)
    float v[POOL_MAXD][POOL_WIN];
#pragma unroll
    for (int k = 0; k < POOL_MAXD; ++k) {
      const int d = threadIdx.x + k * POOL_NT;
      const int dc = d < D ? d : 0;
#pragma unroll
      for (int t = 0; t < POOL_WIN; ++t) {
        const int tc = t < nwin ? t : 0;
        const int y = r0 + tc / wc, x = c0 + tc % wc;
        const int64_t row = o == 0 ? 0 : 1 + (int64_t)y * side + x;
        v[k][t] = ld_in<TIn>(base + row * D + dc);
      }
    }
#pragma unroll
    for (int k = 0; k < POOL_MAXD; ++k) {
      const int d = threadIdx.x + k * POOL_NT;
      float a = 0.f;
      if (o == 0) {
        a = v[k][0];
      } else {
#pragma unroll
        for (int t = 0; t < POOL_WIN; ++t) a += t < nwin ? v[k][t] : 0.f;
        a *= inv_cnt;
      }
      if (d >= D) a = 0.f;
      acc[k] = a;
      ss += a * a;
    }
  } else {
#pragma unroll
    for (int k = 0; k < POOL_MAXD; ++k) {
      const int d = threadIdx.x + k * POOL_NT;
      float a = 0.f;
      if (d < D) {
        if (o == 0) {
          a = ld_in<TIn>(base + d);
        } else {
          for (int y = r0; y < r1; ++y)
            for (int x = c0; x < c1; ++x) a += ld_in<TIn>(base + (1 + (int64_t)y * side + x) * D + d);
          a *= inv_cnt;
        }
      }
      acc[k] = a;
      ss += a * a;
    }
  }
  ss = block_sum<POOL_NT>(ss, red);
  const float scale = normalize ? 1.f / fmaxf(sqrtf(ss), 1e-12f) : 1.f;
  const int64_t orow = (b * 33 + o) * (int64_t)D;
#pragma unroll
  for (int k = 0; k < POOL_MAXD; ++k) {
    const int d = threadIdx.x + k * POOL_NT;
    if (d < D) {
      const float v = acc[k] * scale;
      if (out_f32) reinterpret_cast<float*>(out)[orow + d] = v;
      else reinterpret_cast<bf16_t*>(out)[orow + d] = f2bf(v);
    }
  }
}

// fp32 input, D % 4 == 0, windows of <= WIN patches (the CLIP features of the caption steps:
// side 16 -> 8, side 14 -> 12): thread t owns columns 4t..4t+3 and issues its window's WIN 16-B
// loads at once (pool_kernel moves 4 B per load instruction: 32 of them per thread at D = 768).
// Same per-column summation order as pool_kernel.
template <int WIN>
__global__ __launch_bounds__(POOL_NT) void pool4_kernel(const float* __restrict__ in, void* out,
                                                        int out_f32, int64_t L, int D, int side,
                                                        int normalize) {
  __shared__ float red[POOL_NT / 64];
  const int64_t b = blockIdx.y;
  const int o = blockIdx.x;
  const float* base = in + b * L * (int64_t)D;
  int r0 = 0, r1 = 1, c0 = 0, c1 = 1;
  if (o > 0) {
    const int i = (o - 1) >> 3, j = (o - 1) & 7;
    r0 = (i * side) / 4;
    r1 = ((i + 1) * side + 3) / 4;
    c0 = (j * side) / 8;
    c1 = ((j + 1) * side + 7) / 8;
  }
  const int wc = c1 - c0, nwin = (r1 - r0) * wc;
  const float inv_cnt = 1.f / (float)nwin;
  const int d = 4 * threadIdx.x;
  const int dc = d < D ? d : 0;
  float4 v[WIN];
#pragma unroll
  for (int t = 0; t < WIN; ++t) {
    const int tc = t < nwin ? t : 0;
    const int y = r0 + tc / wc, x = c0 + tc % wc;
    const int64_t row = o == 0 ? 0 : 1 + (int64_t)y * side + x;
    v[t] = *reinterpret_cast<const float4*>(base + row * D + dc);
  }
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (o == 0) {
    a[0] = v[0].x, a[1] = v[0].y, a[2] = v[0].z, a[3] = v[0].w;
  } else {
#pragma unroll
    for (int t = 0; t < WIN; ++t)
      if (t < nwin) a[0] += v[t].x, a[1] += v[t].y, a[2] += v[t].z, a[3] += v[t].w;
#pragma unroll
    for (int e = 0; e < 4; ++e) a[e] *= inv_cnt;
  }
  float ss = 0.f;
  if (d < D) ss = a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
  ss = block_sum<POOL_NT>(ss, red);
  const float scale = normalize ? 1.f / fmaxf(sqrtf(ss), 1e-12f) : 1.f;
  if (d >= D) return;
  const int64_t orow = (b * 33 + o) * (int64_t)D;
  if (out_f32) {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + orow + d) =
        make_float4(a[0] * scale, a[1] * scale, a[2] * scale, a[3] * scale);
  } else {
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(out) + orow + d) =
        make_uint2(pack2(a[0] * scale, a[1] * scale), pack2(a[2] * scale, a[3] * scale));
  }
}

// F.normalize(dim=-1, eps=1e-12) of bf16 / fp32 rows (D <= 1024), one block per row.
template <typename T>
__global__ __launch_bounds__(POOL_NT) void l2norm_rows_kernel(const T* __restrict__ in,
                                                              T* __restrict__ out, int D) {
  __shared__ float red[POOL_NT / 64];
  const int64_t r = blockIdx.x;
  float v[POOL_MAXD];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < POOL_MAXD; ++k) {
    const int d = threadIdx.x + k * POOL_NT;
    v[k] = d < D ? ld_in<T>(in + r * D + d) : 0.f;
    ss += v[k] * v[k];
  }
  ss = block_sum<POOL_NT>(ss, red);
  const float scale = 1.f / fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
  for (int k = 0; k < POOL_MAXD; ++k) {
    const int d = threadIdx.x + k * POOL_NT;
    if (d < D) {
      if constexpr (sizeof(T) == 4) out[r * D + d] = v[k] * scale;
      else out[r * D + d] = f2bf(v[k] * scale);
    }
  }
}

}  // namespace

extern "C" int gvl_embedding_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out,
                                 int64_t n_tokens, int64_t T, int64_t C, int64_t vocab,
                                 int64_t out_rows_per_seq, int64_t out_offset,
                                 gvl_stream_t stream) {
  GVL_REQUIRE(C % 8 == 0, "gvl_embedding_fwd: C must be a multiple of 8");
  GVL_REQUIRE(T > 0 && vocab > 0, "gvl_embedding_fwd: T and vocab must be > 0");
  if (n_tokens == 0) return 0;
  hipLaunchKernelGGL(emb_fwd_kernel, dim3((unsigned)((n_tokens + 3) / 4)), dim3(256), 0,
                     gvl::as_stream(stream), idx, static_cast<const bf16_t*>(wte),
                     static_cast<const bf16_t*>(wpe), static_cast<bf16_t*>(out), n_tokens, T, (int)C,
                     out_rows_per_seq, out_offset, vocab);
  GVL_LAUNCH_CHECK("gvl_embedding_fwd");
  return 0;
}

extern "C" int gvl_embedding_bwd(const int64_t* idx, const void* dout, float* dwte_acc,
                                 float* dwpe_acc, int64_t n_tokens, int64_t T, int64_t C,
                                 int64_t vocab, int64_t out_rows_per_seq, int64_t out_offset,
                                 gvl_stream_t stream) {
  GVL_REQUIRE(C % 2 == 0 && T > 0 && vocab > 0, "gvl_embedding_bwd: bad shape");
  if (n_tokens == 0) return 0;
  hipLaunchKernelGGL(emb_bwd_kernel, dim3((unsigned)((n_tokens + 3) / 4)), dim3(256), 0,
                     gvl::as_stream(stream), idx, static_cast<const bf16_t*>(dout), dwte_acc,
                     dwpe_acc, n_tokens, T, (int)C, out_rows_per_seq, out_offset, vocab);
  GVL_LAUNCH_CHECK("gvl_embedding_bwd");
  return 0;
}

extern "C" int64_t gvl_embedding_bwd_workspace(int64_t n_tokens) {
  // sorted tiles (padded to whole tiles) + the merged keys of one chunk
  const int64_t n = n_tokens < EMB_CHUNK ? n_tokens : EMB_CHUNK;
  return (n + EMB_TILE - 1) / EMB_TILE * EMB_TILE + n;
}

extern "C" int gvl_embedding_bwd_det(const int64_t* idx, const void* dout, void* dwte, void* dwpe,
                                     int64_t n_tokens, int64_t T, int64_t C, int64_t vocab,
                                     int64_t out_rows_per_seq, int64_t out_offset,
                                     uint32_t* keys, int64_t keys_count, gvl_stream_t stream) {
  GVL_REQUIRE(C % 8 == 0 && C <= EMB_MAXC && T > 0 && vocab > 0,
              "gvl_embedding_bwd_det: bad shape (C %% 8 == 0, C <= %d)", EMB_MAXC);
  GVL_REQUIRE(vocab < (1ll << 18) - 1, "gvl_embedding_bwd_det: vocab must be < 2^18 - 1");
  GVL_REQUIRE(n_tokens % T == 0, "gvl_embedding_bwd_det: n_tokens must be a multiple of T");
  if (n_tokens == 0) return 0;
  hipStream_t s = gvl::as_stream(stream);
  if (dwte) {
    GVL_REQUIRE(keys && keys_count >= gvl_embedding_bwd_workspace(n_tokens),
                "gvl_embedding_bwd_det: key workspace too small");
    for (int64_t base = 0; base < n_tokens; base += EMB_CHUNK) {
      const int n = (int)((n_tokens - base) < EMB_CHUNK ? (n_tokens - base) : EMB_CHUNK);
      const int nt = (n + EMB_TILE - 1) / EMB_TILE;
      uint32_t* tiles = keys + n;
      hipLaunchKernelGGL(emb_tile_kernel, dim3(nt), dim3(EMB_TILE / 2), 0, s, idx, base, n, vocab,
                         tiles);
      hipLaunchKernelGGL(emb_rank_kernel, dim3(nt), dim3(EMB_TILE), nt * EMB_TILE * sizeof(uint32_t),
                         s, (const uint32_t*)tiles, nt, n, keys);
      hipLaunchKernelGGL(emb_seg_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s,
                         (const uint32_t*)keys, n, base, static_cast<const bf16_t*>(dout),
                         static_cast<bf16_t*>(dwte), T, (int)C, out_rows_per_seq, out_offset);
    }
  }
  if (dwpe)
    hipLaunchKernelGGL(emb_pos_kernel, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, s,
                       static_cast<const bf16_t*>(dout), static_cast<bf16_t*>(dwpe), n_tokens / T,
                       T, (int)C, out_rows_per_seq, out_offset);
  GVL_LAUNCH_CHECK("gvl_embedding_bwd_det");
  return 0;
}

extern "C" int gvl_pool_clip_ex(const void* in, int32_t in_fp32, void* out, int32_t out_fp32,
                                int64_t B, int64_t L, int64_t D, int32_t normalize,
                                gvl_stream_t stream) {
  const int64_t N = L - 1;
  int side = 0;
  while ((int64_t)(side + 1) * (side + 1) <= N) ++side;
  GVL_REQUIRE((int64_t)side * side == N && side > 0,
              "gvl_pool_clip: expected square grid, got N=%lld", (long long)N);
  GVL_REQUIRE(D > 0 && D <= POOL_NT * POOL_MAXD, "gvl_pool_clip: D=%lld unsupported", (long long)D);
  if (B == 0) return 0;
  dim3 grid(33, (unsigned)B);
  hipStream_t s = gvl::as_stream(stream);
  // pool4_kernel<8 | 16> by the largest of the 32 windows (side 16: 4 x 2, side 14: 4 x 3)
  int max_win = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) {
      const int nw = (((i + 1) * side + 3) / 4 - (i * side) / 4) * (((j + 1) * side + 7) / 8 - (j * side) / 8);
      max_win = nw > max_win ? nw : max_win;
    }
  const bool vec_ok = in_fp32 && D % 4 == 0 && gvl::aligned16(in) &&
                      (out_fp32 ? gvl::aligned16(out) : reinterpret_cast<uintptr_t>(out) % 8 == 0);
  if (vec_ok && max_win <= 8)
    hipLaunchKernelGGL(pool4_kernel<8>, grid, dim3(POOL_NT), 0, s, static_cast<const float*>(in),
                       out, (int)out_fp32, L, (int)D, side, (int)normalize);
  else if (vec_ok && max_win <= 16)
    hipLaunchKernelGGL(pool4_kernel<16>, grid, dim3(POOL_NT), 0, s, static_cast<const float*>(in),
                       out, (int)out_fp32, L, (int)D, side, (int)normalize);
  else if (in_fp32)
    hipLaunchKernelGGL(pool_kernel<float>, grid, dim3(POOL_NT), 0, s, static_cast<const float*>(in),
                       out, (int)out_fp32, L, (int)D, side, (int)normalize);
  else
    hipLaunchKernelGGL(pool_kernel<bf16_t>, grid, dim3(POOL_NT), 0, s,
                       static_cast<const bf16_t*>(in), out, (int)out_fp32, L, (int)D, side,
                       (int)normalize);
  GVL_LAUNCH_CHECK("gvl_pool_clip");
  return 0;
}

extern "C" int gvl_pool_clip(const void* in, int32_t in_fp32, void* out, int32_t out_fp32,
                             int64_t B, int64_t L, int64_t D, gvl_stream_t stream) {
  return gvl_pool_clip_ex(in, in_fp32, out, out_fp32, B, L, D, 1, stream);
}

extern "C" int gvl_l2_normalize_rows(const void* in, void* out, int32_t fp32, int64_t rows,
                                     int64_t D, gvl_stream_t stream) {
  GVL_REQUIRE(D > 0 && D <= POOL_NT * POOL_MAXD, "gvl_l2_normalize_rows: D=%lld unsupported",
              (long long)D);
  if (rows == 0) return 0;
  hipStream_t s = gvl::as_stream(stream);
  if (fp32)
    hipLaunchKernelGGL(l2norm_rows_kernel<float>, dim3((unsigned)rows), dim3(POOL_NT), 0, s,
                       static_cast<const float*>(in), static_cast<float*>(out), (int)D);
  else
    hipLaunchKernelGGL(l2norm_rows_kernel<bf16_t>, dim3((unsigned)rows), dim3(POOL_NT), 0, s,
                       static_cast<const bf16_t*>(in), static_cast<bf16_t*>(out), (int)D);
  GVL_LAUNCH_CHECK("gvl_l2_normalize_rows");
  return 0;
}
