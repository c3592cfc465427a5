// bf16 GEMM on gfx950 MFMA (v_mfma_f32_16x16x32_bf16) with a fused epilogue — entry point
// and the register-staged fallback kernel (any K % 8 == 0, tails in every dimension).
//
// Fallback tile 128x128x64, 256 threads = 4 waves in 2x2, each wave a 64x64 sub-tile of
// 4x4 MFMA tiles.  Operands are register-staged through a double-buffered LDS image:
//   K-contiguous operand  -> [128 rows][64 k]   128-B rows, 16-B chunk XOR (row>>1)&7,
//                            fragments by ds_read_b128 (conflict-free for 16x16x32 maps);
//   MN-contiguous operand -> [64 k][128 cols]   256-B rows, chunk XOR fT(k),
//                            fragments by two ds_read_b64_tr_b16 (hardware transpose).
// The MFMA is issued with operands swapped (B-fragment as "A") so each lane owns one
// output row and four consecutive output columns -> 8-byte epilogue stores.
// Workgroups are remapped so that consecutive tiles share an XCD (L2) — T1 of the guide.
// The fast path (gemm_lds.hip: LDS-DMA staging, 256-wide tiles) is used whenever K % 64 == 0.
#include <stdlib.h>

#include "common.h"
#include "capi_util.h"
#include "gemm_common.h"
#include "../../include/gvl.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int STAGE_BYTES = 2 * 16384;  // A image + B image

GVL_DEV int swz_k(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
GVL_DEV int fT(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }
GVL_DEV int swz_t(int krow, int chunk) { return krow * 256 + ((chunk ^ fT(krow)) << 4); }

// Global -> registers for one 128x64 (or 64x128) operand tile.
template <bool MN>
GVL_DEV void load_tile(uint4 (&r)[4], const bf16_t* __restrict__ X, int64_t ld, int64_t r0,
                       int64_t R, int64_t k0, int64_t K, int tid) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    int64_t row, col;
    bool ok;
    if (!MN) {
      const int rr = (tid >> 3) + 32 * it, ch = tid & 7;
      row = r0 + rr;
      col = k0 + ch * 8;
      ok = (row < R) && (col < K);
    } else {
      const int kr = (tid >> 4) + 16 * it, ch = tid & 15;
      row = k0 + kr;
      col = r0 + ch * 8;
      ok = (row < K) && (col < R);
    }
    if (ok) {
      r[it] = *reinterpret_cast<const uint4*>(X + row * ld + col);
    } else {
      r[it] = make_uint4(0, 0, 0, 0);
    }
  }
}

template <bool MN>
GVL_DEV void store_tile(const uint4 (&r)[4], char* lds, int tid) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    int off;
    if (!MN) {
      off = swz_k((tid >> 3) + 32 * it, tid & 7);
    } else {
      off = swz_t((tid >> 4) + 16 * it, tid & 15);
    }
    *reinterpret_cast<uint4*>(lds + off) = r[it];
  }
}

// Fragment of a 16(row) x 32(k) operand slab: rows/cols [c0, c0+16), k-step s (k 32s..32s+31).
template <bool MN>
GVL_DEV short8_t read_frag(const char* lds, int c0, int s, int lane) {
  if (!MN) {
    const int row = c0 + (lane & 15), ch = 4 * s + (lane >> 4);
    return *reinterpret_cast<const short8_t*>(lds + swz_k(row, ch));
  } else {
    const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int krow = 32 * s + 8 * G + q;
    const int ch = (c0 >> 3) + (p >> 1);
    const int f = fT(krow);
    const int off1 = krow * 256 + ((ch ^ f) << 4) + (p & 1) * 8;
    const int off2 = off1 + 4 * 256;  // krow+4 has the same fT
    short4_t lo = lds_read_tr(lds + off1);
    short4_t hi = lds_read_tr(lds + off2);
    short8_t r;
    r.lo = lo;
    r.hi = hi;
    return r;
  }
}

template <bool AMN, bool BMN>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(GemmP p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD; give each XCD a
  // contiguous range of tiles (row-major over (tm, tn)) so A panels are L2 hits.
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  float4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((p.K + BK - 1) / BK);
  uint4 ra[4], rb[4];
  load_tile<AMN>(ra, p.A, p.lda, m0, p.M, 0, p.K, tid);
  load_tile<BMN>(rb, p.B, p.ldb, n0, p.N, 0, p.K, tid);
  store_tile<AMN>(ra, smem, tid);
  store_tile<BMN>(rb, smem + 16384, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool more = (kt + 1) < nk;
    if (more) {
      load_tile<AMN>(ra, p.A, p.lda, m0, p.M, (int64_t)(kt + 1) * BK, p.K, tid);
      load_tile<BMN>(rb, p.B, p.ldb, n0, p.N, (int64_t)(kt + 1) * BK, p.K, tid);
    }
    const char* sa = smem + (kt & 1) * STAGE_BYTES;
    const char* sb = sa + 16384;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      short8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<AMN>(sa, wm * 64 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<BMN>(sb, wn * 64 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    }
    if (more) {
      char* dst = smem + ((kt + 1) & 1) * STAGE_BYTES;
      store_tile<AMN>(ra, dst, tid);
      store_tile<BMN>(rb, dst + 16384, tid);
    }
    __syncthreads();
  }
  gemm_epilogue<4, 4>(p, acc, m0 + wm * 64, n0 + wn * 64, lane);
}

// GVL_GEMM_IMPL=regstage|lds|ring|pp picks the kernel family (0|1|2|3, default 3: the
// four-wave kernels for narrow outputs, the persistent ping-pong kernel where it fills the
// chip, else the 128x128 ring); GVL_GEMM_CFG forces a tile config of that family (impl 3:
// 3 = the persistent kernel, 10 = the four-wave kernel, 11 = the default routing without it).
struct GemmEnv {
  int impl = 3, cfg = -1, group = 0;  // group 0: by shape (gemm_group)
  GemmEnv() {
    const char* gr = getenv("GVL_GEMM_GROUP");
    if (gr && atoi(gr) > 0) group = atoi(gr);
    const char* s = getenv("GVL_GEMM_IMPL");
    if (s && s[0] == 'r' && s[1] == 'e') impl = 0;
    if (s && s[0] == 'l') impl = 1;
    if (s && s[0] == 'r' && s[1] == 'i') impl = 2;
    if (s && s[0] == 'p') impl = 3;
    const char* c = getenv("GVL_GEMM_CFG");
    if (c) cfg = atoi(c);
  }
};
GemmEnv& env() {
  static GemmEnv e;
  return e;
}

// Tile rows per L2 group of the tile walk (gemm_tile_of).  GVL_GEMM_WALK_RULE (A/B, build
// time): 0 = 8 everywhere; 1 = 4 for M >= 12288 (the LM's 16384-token GEMMs), else 8;
// 2 (default) = 4 for M or K >= 12288 (also the LM's weight gradients over 16384 tokens), else
// 8 — LM step 856k -> 862k tokens/s, Q-Former unchanged (profiles/r3/gemm_walk_group_ab_r3s2.txt).
// GVL_GEMM_GROUP=n overrides it for every GEMM.
#ifndef GVL_GEMM_WALK_RULE
#define GVL_GEMM_WALK_RULE 2
#endif
int gemm_group(const gvl_gemm_desc* d) {
  if (env().group > 0) return env().group;
  if (GVL_GEMM_WALK_RULE == 1 && d->m >= 12288) return 4;
  if (GVL_GEMM_WALK_RULE == 2 && (d->m >= 12288 || d->k >= 12288)) return 4;
  return 8;
}

void fill_params(const gvl_gemm_desc* d, GemmP& p) {
  p.A = static_cast<const bf16_t*>(d->a);
  p.B = static_cast<const bf16_t*>(d->b);
  p.C = d->c;
  p.M = d->m; p.N = d->n; p.K = d->k;
  p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc;
  p.alpha = d->alpha;
  p.alpha_ptr = d->alpha_ptr;
  p.bias = static_cast<const bf16_t*>(d->bias);
  p.pre_out = static_cast<bf16_t*>(d->pre_out);
  p.pre_in = static_cast<const bf16_t*>(d->pre_in);
  p.ldp = d->ldp;
  p.residual = static_cast<const bf16_t*>(d->residual);
  p.ldr = d->ldr;
  p.gate = static_cast<const bf16_t*>(d->gate);
  p.seed = d->seed;
  p.seed_ptr = static_cast<const uint64_t*>(d->seed_ptr);
  p.has_drop = d->drop_p > 0.f;
  p.drop_scale = p.has_drop ? 1.f / (1.f - d->drop_p) : 1.f;
  p.drop_thresh = (uint32_t)((double)d->drop_p * 4294967296.0);
  p.act = d->act; p.dact = d->dact; p.c_f32 = d->c_fp32;
  p.splits = 1;
  p.cnt = 0;
  p.st_nt = 0;
  p.bn = 256;
  p.bm = 256;
  p.kper = d->k;
  p.group = gemm_group(d);
  p.ws = (d->workspace && gvl::aligned16(d->workspace) && d->n % 4 == 0)
             ? static_cast<float*>(d->workspace) : nullptr;
  p.ws_bytes = p.ws ? d->workspace_bytes : 0;
  p.tickets = d->tickets;
  p.nticket = d->tickets ? d->ticket_count : 0;
  p.batch = 1;
  p.grouped = 0;
  p.alpha_mask = 0;
}

}  // namespace

namespace gvl {
bool pp3_combine_forced() { return env().impl >= 3 && env().cfg == 13; }
}  // namespace gvl

extern "C" int gvl_gemm_tune(int32_t impl, int32_t cfg) {
  GVL_REQUIRE(impl >= 0 && impl <= 3 && cfg >= -1 && cfg <= 13, "gvl_gemm_tune: bad arguments");
  env().impl = impl;
  env().cfg = cfg;
  return 0;
}

extern "C" int gvl_gemm_kernel_name(const gvl_gemm_desc* d, char* buf, int32_t len) {
  GVL_REQUIRE(d && buf && len > 0, "gvl_gemm_kernel_name: bad arguments");
  const char* tf[2] = {"false", "true"};
  if (env().impl >= 3 && (env().cfg < 0 || env().cfg == 12)) {
    GemmP q;
    fill_params(d, q);
    if (gvl::gemm_w4x_plan(q, d->a_mn, d->b_mn, env().cfg == 12)) {
      snprintf(buf, len, "gemm_w4x_kernel<%d, %d, %s, %s, %d, false>", q.bm, d->a_mn ? q.bn : 192,
               tf[d->a_mn != 0], tf[d->b_mn != 0], gvl::gemm_epi_kind(q));
      return 0;
    }
  }
  if (env().impl >= 3 && gvl::gemm_ring_ok(d)) {
    GemmP p;
    fill_params(d, p);
    const int cfg = env().cfg;
    if ((cfg < 0 || cfg == 10) && gvl::gemm_w4_plan(p, d->a_mn, cfg == 10)) {
      // (cfg 11: default routing with the four-wave kernel off)
      const char* epi[EPI_KINDS] = {"0", "1", "2", "3", "4", "5", "6", "7", "8", "9", "10", "11", "12", "13", "14"};
      if (gvl::gemm_w4d_ok(p))
        snprintf(buf, len, "%s<%s, %s>", gvl::gemm_w4_rows128(p) ? "gemm_w4dm_kernel" : "gemm_w4d_kernel",
                 tf[d->b_mn != 0], epi[gvl::gemm_epi_kind(p)]);
      else
        snprintf(buf, len, "%s<3, %s, %s>",
                 gvl::gemm_w4_rows96(p, d->b_mn != 0) ? "gemm_w4r_kernel"
                 : gvl::gemm_w4_cols96(p, d->b_mn != 0) ? "gemm_w4n_kernel"
                 : gvl::gemm_w4_rows128(p) ? "gemm_w4m_kernel" : "gemm_w4_kernel",
                 tf[d->b_mn != 0], epi[gvl::gemm_w4_epi_kind(p)]);
    } else if (gvl::gemm_pp3_plan(p, cfg == 3 || cfg == 10)) {
      const char* epi[EPI_KINDS] = {"0", "1", "2", "3", "4", "5", "6", "7", "8", "9", "10", "11", "12", "13", "14"};
      const bool slab = p.splits > 1 && !(p.splits == 2 && p.tickets);  // partials-only kernel
      snprintf(buf, len, "gemm_pp3_kernel<4, %s, %s, %s, %d, %d>", tf[d->a_mn != 0], tf[d->b_mn != 0],
               epi[slab ? 0 : gvl::gemm_epi_kind(p)], p.bn, p.bm);
    } else {
      snprintf(buf, len, "%s, %s, %s>", gvl::gemm_ring_name(gvl::gemm_ring_pick(d->m, d->n, d->k, -1, d->a_mn)),
               tf[d->a_mn != 0], tf[d->b_mn != 0]);
    }
  } else if (env().impl == 2 && gvl::gemm_ring_ok(d)) {
    const int cfg = gvl::gemm_ring_pick(d->m, d->n, d->k, env().cfg, d->a_mn);
    snprintf(buf, len, "%s, %s, %s>", gvl::gemm_ring_name(cfg), tf[d->a_mn != 0], tf[d->b_mn != 0]);
  } else if (env().impl >= 1 && gvl::gemm_lds_ok(d)) {
    const int cfg = gvl::gemm_lds_pick(d->m, d->n, d->k, env().cfg > 2 ? -1 : env().cfg);
    const int bm[3] = {256, 256, 128}, bn[3] = {256, 128, 128}, wm[3] = {2, 4, 2}, wn[3] = {4, 2, 2};
    snprintf(buf, len, "gemm_lds_kernel<%d, %d, %d, %d, %s, %s>", bm[cfg], bn[cfg], wm[cfg],
             wn[cfg], tf[d->a_mn != 0], tf[d->b_mn != 0]);
  } else {
    snprintf(buf, len, "gemm_bf16_kernel<%s, %s>", tf[d->a_mn != 0], tf[d->b_mn != 0]);
  }
  return 0;
}

extern "C" int gvl_gemm(const gvl_gemm_desc* d, gvl_stream_t stream) {
  GVL_REQUIRE(d != nullptr, "gvl_gemm: null descriptor");
  GVL_REQUIRE(d->m >= 0 && d->n >= 0 && d->k >= 0, "gvl_gemm: negative size");
  if (d->m == 0 || d->n == 0) return 0;
  GVL_REQUIRE(d->a && d->b && d->c, "gvl_gemm: null operand");
  // 16-B vector loads run along K only for K-contiguous operands
  GVL_REQUIRE((d->a_mn && d->b_mn) || d->k % 8 == 0,
              "gvl_gemm: K=%lld must be a multiple of 8", (long long)d->k);
  GVL_REQUIRE(d->n % 4 == 0, "gvl_gemm: N=%lld must be a multiple of 4", (long long)d->n);
  GVL_REQUIRE(!d->a_mn || d->m % 8 == 0, "gvl_gemm: M must be a multiple of 8 for MN-major A");
  GVL_REQUIRE(!d->b_mn || d->n % 8 == 0, "gvl_gemm: N must be a multiple of 8 for MN-major B");
  GVL_REQUIRE(d->lda % 8 == 0 && d->ldb % 8 == 0 && d->ldc % 4 == 0,
              "gvl_gemm: leading dims must be multiples of 8 (lda, ldb) / 4 (ldc)");
  GVL_REQUIRE(gvl::aligned16(d->a) && gvl::aligned16(d->b) && gvl::aligned8(d->c),
              "gvl_gemm: operands must be 16-byte aligned");
  GVL_REQUIRE(d->act >= 0 && d->act <= 5 && d->dact >= 0 && d->dact <= 3, "gvl_gemm: bad act");
  GVL_REQUIRE(d->act != 5 || (d->pre_out == nullptr && d->dact == 0), "gvl_gemm: act 5 (quick-GELU) "
              "has no pre-activation output and no dact");
  GVL_REQUIRE(!d->dact || (d->pre_in && d->ldp % 4 == 0), "gvl_gemm: dact needs pre_in");
  GVL_REQUIRE(!d->residual || d->ldr % 4 == 0, "gvl_gemm: ldr must be a multiple of 4");
  GVL_REQUIRE(d->drop_p >= 0.f && d->drop_p < 1.f, "gvl_gemm: drop_p out of range");
  GemmP p;
  fill_params(d, p);
  hipStream_t s = gvl::as_stream(stream);
  if (env().impl >= 3 && (env().cfg < 0 || env().cfg == 12) &&
      gvl::gemm_w4x_try(p, d->a_mn, d->b_mn, env().cfg == 12, s)) {  // AGPR four-wave kernel
    GVL_LAUNCH_CHECK("gvl_gemm(w4x)");
    return 0;
  }
  if (env().impl >= 3 && gvl::gemm_ring_ok(d)) {
    const int cfg = env().cfg;
    GemmP q = p;
    if (cfg == 10 && gvl::gemm_w4_plan(p, d->a_mn, true)) {
      gvl::gemm_w4_launch(p, d->b_mn, s);
    } else if (cfg != 11 && cfg != 13 && cfg != 3 && cfg != 10 && gvl::gemm_w4_try(p, d->a_mn, d->b_mn, s)) {
    } else if (gvl::gemm_pp3_plan(q, cfg == 3 || cfg == 10)) {
      gvl::gemm_pp3_launch(q, d->a_mn, d->b_mn, s);
    } else {
      gvl::gemm_ring_launch(p, d->a_mn, d->b_mn, gvl::gemm_ring_pick(d->m, d->n, d->k, -1, d->a_mn), s);
    }
    GVL_LAUNCH_CHECK("gvl_gemm(pp)");
    return 0;
  }
  if (env().impl == 2 && gvl::gemm_ring_ok(d)) {
    const int cfg = gvl::gemm_ring_pick(d->m, d->n, d->k, env().cfg, d->a_mn);
    gvl::gemm_ring_launch(p, d->a_mn, d->b_mn, cfg, s);
    GVL_LAUNCH_CHECK("gvl_gemm(ring)");
    return 0;
  }
  if (env().impl >= 1 && gvl::gemm_lds_ok(d)) {
    const int cfg = gvl::gemm_lds_pick(d->m, d->n, d->k, env().cfg > 2 ? -1 : env().cfg);
    gvl::gemm_lds_launch(p, d->a_mn, d->b_mn, cfg, s);
    GVL_LAUNCH_CHECK("gvl_gemm(lds)");
    return 0;
  }
  p.tiles_m = (int)((d->m + BM - 1) / BM);
  p.tiles_n = (int)((d->n + BN - 1) / BN);
  const int grid = p.tiles_m * p.tiles_n;
  if (!d->a_mn && !d->b_mn) gvl::launch_timed(gemm_bf16_kernel<false, false>, dim3(grid), dim3(NT), 0, s, p);
  else if (!d->a_mn && d->b_mn) gvl::launch_timed(gemm_bf16_kernel<false, true>, dim3(grid), dim3(NT), 0, s, p);
  else if (d->a_mn && !d->b_mn) gvl::launch_timed(gemm_bf16_kernel<true, false>, dim3(grid), dim3(NT), 0, s, p);
  else gvl::launch_timed(gemm_bf16_kernel<true, true>, dim3(grid), dim3(NT), 0, s, p);
  GVL_LAUNCH_CHECK("gvl_gemm");
  return 0;
}

// Batched GEMM: count problems of one shape / layout (only the operand pointers differ), as
// one persistent launch of gemm_pp3_kernel whose work items walk every problem's tiles — the
// deferred weight gradients of the 12 GPT-2 blocks (gvl/functional.py): each is too small
// (9-36 tiles of 256x256 at K = 16384 tokens) to fill the chip without a K split and fp32
// slabs, together they do.  Epilogue: plain or C += AB (residual == c, fused accumulation);
// anything else, or an unsupported shape, runs the problems one by one through gvl_gemm.
// name of the kernel instance the last batched call launched ("" after a per-problem fallback)
static thread_local char g_batched_name[128];

static int gemm_batched_impl(const gvl_gemm_desc* d, void* const* dbias, int32_t count,
                             gvl_stream_t stream) {
  g_batched_name[0] = 0;
  GVL_REQUIRE(d != nullptr && count >= 1, "gvl_gemm_batched: bad arguments");
  bool ok = count > 1 && count <= GVL_MAX_BATCH && env().impl >= 3 && env().cfg < 0;
  // fused bias gradients: weight-gradient layout (both operands MN-contiguous), C += AB
  if (dbias) ok = ok && d[0].a_mn && d[0].b_mn && d[0].residual != nullptr;
  for (int i = 0; ok && i < count; ++i) {
    const gvl_gemm_desc& e = d[i];
    ok = gvl::gemm_ring_ok(&e) && e.m == d[0].m && e.n == d[0].n && e.k == d[0].k &&
         e.lda == d[0].lda && e.ldb == d[0].ldb && e.ldc == d[0].ldc && e.a_mn == d[0].a_mn &&
         e.b_mn == d[0].b_mn && e.alpha == d[0].alpha && !e.alpha_ptr && !e.bias && !e.act &&
         !e.dact && !e.gate && e.drop_p == 0.f && !e.c_fp32 && e.m > 0 && e.n > 0 &&
         gvl::aligned16(e.c) && (e.residual == nullptr || (e.residual == e.c && e.ldr == e.ldc)) &&
         ((e.residual == nullptr) == (d[0].residual == nullptr));
  }
  if (!ok) {
    GVL_REQUIRE(!dbias, "gvl_gemm_batched_dbias: shape not batchable (use gvl_colsum)");
    for (int i = 0; i < count; ++i) {
      const int rc = gvl_gemm(&d[i], stream);
      if (rc) return rc;
    }
    return 0;
  }
  GemmP p;
  fill_params(&d[0], p);
  for (int i = 0; i < GVL_MAX_BATCH; ++i) p.Db[i] = (dbias && i < count) ? dbias[i] : nullptr;
  float* const ws = p.ws;  // kept for the two-way split below
  const int64_t ws_bytes = p.ws_bytes;
  uint32_t* const tickets = p.tickets;
  const int nticket = p.nticket;
  p.ws = nullptr;  // whole-K tiles: the batch fills the chip
  p.ws_bytes = 0;
  p.tickets = nullptr;
  p.nticket = 0;
  p.batch = count;
  for (int i = 0; i < count; ++i) {
    p.Ab[i] = static_cast<const bf16_t*>(d[i].a);
    p.Bb[i] = static_cast<const bf16_t*>(d[i].b);
    p.Cb[i] = d[i].c;
  }
  if (d[0].a_mn && d[0].b_mn && gvl::gemm_w4x_batched_try(p, gvl::as_stream(stream))) {
    GemmP q = p;
    gvl::w4x_dw_plan(q);
    snprintf(g_batched_name, sizeof g_batched_name, "gemm_w4x_kernel<256, %d, true, true, %d, false>",
             q.bn, gvl::gemm_epi_kind(p));
    GVL_LAUNCH_CHECK("gvl_gemm_batched(w4x)");
    return 0;
  }
  if (gvl::gemm_pp3_plan(p, true) && p.splits == 1) {
    // tile shape for the whole batch (the plan sized it for one problem): 256 rows, 256 or
    // 192 columns, whichever fills the last round of CUs better (192 counted at 0.9)
    const int64_t cus = gvl::num_cus(), tm = (p.M + 255) / 256;
    auto fill = [&](int64_t tiles) {
      return (double)tiles / (double)(((tiles + cus - 1) / cus) * cus);
    };
    const double e256 = fill(count * tm * ((p.N + 255) / 256));
    const double e192 = (p.N % 64 == 0 && p.N >= 384) ? 0.9 * fill(count * tm * ((p.N + 191) / 192)) : 0.0;
    p.bm = 256;
    p.bn = e192 > e256 ? 192 : 256;
    p.tiles_m = (int)tm;
    p.tiles_n = (int)((p.N + p.bn - 1) / p.bn);
    // Two-way K split combined in-launch (gemm_pp3_kernel: per-problem fp32 partial slabs in
    // the workspace, tickets per tile and wave; bias gradients by gvl_colsum_batched after
    // it, since the fused row sums would need their own combine) when the batch's
    // whole-K tiles leave most CUs idle through one long round: the 12 attn.c_proj weight
    // gradients (768 x 768, K = 16384) are 144 tiles of 256 x 192 on 256 CUs; split, 216
    // half-K 256 x 256 items.  Estimate as in the planner (gemm_plan.hip): rounds x (32-deep
    // K-steps + 6), a 192-wide step counted 0.75 / 0.9, ~4 for the combine; required >= 10 %
    // better.  GVL_BATCHED_SPLIT=0 turns it off (A/B).
    static const bool split_on = [] {
      const char* e = getenv("GVL_BATCHED_SPLIT");
      return !(e && e[0] == '0');
    }();
    const int64_t tn256 = (p.N + 255) / 256, items2 = 2 * (int64_t)count * tm * tn256;
    const int64_t need = (int64_t)count * 2 * p.M * p.N * 4;
    // a split batch's bias gradients go to gvl_colsum_batched after the GEMM: every one of its
    // preconditions is checked here, before anything is launched, so it cannot fail once the
    // GEMM has added into C (a failure then would make the caller redo the weight gradients)
    bool colsum_ok = gvl_colsum_batched_workspace_size(count, p.K, p.M) <= ws_bytes &&
                     p.M % 8 == 0 && d[0].lda % 8 == 0;
    for (int i = 0; dbias && colsum_ok && i < count; ++i)
      colsum_ok = dbias[i] != nullptr && gvl::aligned16(d[i].a);
    if (split_on && ws && tickets && p.K % 64 == 0 && p.K / 2 >= 256 &&
        (int64_t)count * tm * tn256 * 8 <= nticket && need <= ws_bytes && (!dbias || colsum_ok)) {
      auto est = [&](int64_t items, double steps, double w) {
        return (double)((items + cus - 1) / cus) * (steps + 6.0) * w;
      };
      const double t1 = est((int64_t)count * p.tiles_m * p.tiles_n, p.K / 32.0,
                            p.bn == 192 ? 0.75 / 0.9 : 1.0);
      const double t2 = est(items2, p.K / 64.0, 1.0) + 4.0;
      if (t2 < 0.9 * t1) {
        p.bn = 256;
        p.tiles_n = (int)tn256;
        p.splits = 2;
        p.kper = p.K / 2;
        p.ws = ws;
        p.ws_bytes = ws_bytes;
        p.tickets = tickets;
        p.nticket = nticket;
      }
    }
  } else {
    GVL_REQUIRE(!dbias, "gvl_gemm_batched_dbias: shape not batchable (use gvl_colsum)");
    for (int i = 0; i < count; ++i) {
      const int rc = gvl_gemm(&d[i], stream);
      if (rc) return rc;
    }
    return 0;
  }
  {
    const char* tf[2] = {"false", "true"};
    snprintf(g_batched_name, sizeof g_batched_name, "gemm_pp3_kernel<4, %s, %s, %d, %d, %d>",
             tf[d[0].a_mn != 0], tf[d[0].b_mn != 0], gvl::gemm_epi_kind(p), p.bn, p.bm);
  }
  gvl::gemm_pp3_launch(p, d[0].a_mn, d[0].b_mn, gvl::as_stream(stream));
  GVL_LAUNCH_CHECK("gvl_gemm_batched");
  if (dbias && p.splits == 2) {  // dbias[i] += column sums of dY_i = A_i stored [K][M]
    const void* xs[GVL_MAX_BATCH];
    for (int i = 0; i < count; ++i) xs[i] = d[i].a;
    // preconditions checked above: a failure here is a launch error, reported as -2 (never the
    // -1 "nothing launched, use the unfused path" answer)
    if (gvl_colsum_batched(xs, dbias, count, p.K, p.M, d[0].lda, 1, ws, stream) != 0) return -2;
  }
  return 0;
}

extern "C" int gvl_gemm_batched(const gvl_gemm_desc* d, int32_t count, gvl_stream_t stream) {
  return gemm_batched_impl(d, nullptr, count, stream);
}

// Grouped weight gradients (ABI v9): count problems of possibly different shapes, each
// dW_i += dY_i^T X_i (a_mn = b_mn = 1, residual == c, same alpha), dbias[i] (may be null) +=
// column sums of dY_i, in one launch of the AGPR four-wave kernel.  0: launched; -1: the
// problems do not qualify, nothing launched (the caller runs them another way).
extern "C" int gvl_gemm_grouped(const gvl_gemm_desc* d, void* const* dbias, int32_t count,
                                gvl_stream_t stream) {
  g_batched_name[0] = 0;
  GVL_REQUIRE(d != nullptr && count >= 1, "gvl_gemm_grouped: bad arguments");
  if (count > GVL_MAX_GROUP || env().impl < 3 || env().cfg >= 0) return -1;
  // ABI v11: one device scale for the problems that carry it (the lm_head's weight grad)
  const void* ap = nullptr;
  uint64_t amask = 0;
  for (int i = 0; i < count; ++i) {
    if (!d[i].alpha_ptr) continue;
    if (!ap) ap = d[i].alpha_ptr;
    amask |= uint64_t(1) << i;
  }
  for (int i = 0; i < count; ++i) {
    const gvl_gemm_desc& e = d[i];
    if (!(e.a_mn && e.b_mn && e.residual == e.c && e.ldr == e.ldc && e.alpha == d[0].alpha &&
          (!e.alpha_ptr || !ap || e.alpha_ptr == ap) && !e.bias && !e.act && !e.dact && !e.gate && e.drop_p == 0.f && !e.c_fp32 &&
          e.m > 0 && e.n > 0 && e.k > 0 && e.m < (1 << 30) && e.n < (1 << 30) && e.k < (1 << 30) &&
          e.lda < (1 << 30) && e.ldb < (1 << 30) && e.ldc < (1 << 30) && gvl::aligned16(e.a) && gvl::aligned16(e.b) &&
          gvl::aligned16(e.c)))
      return -1;
  }
  GemmP p;
  fill_params(&d[0], p);
  p.ws = nullptr;
  p.ws_bytes = 0;
  p.tickets = nullptr;
  p.nticket = 0;
  p.batch = count;
  p.alpha_ptr = static_cast<const float*>(ap);
  p.alpha_mask = amask;
  for (int i = 0; i < GVL_MAX_GROUP; ++i) p.Db[i] = (dbias && i < count) ? dbias[i] : nullptr;
  for (int i = 0; i < count; ++i) {
    p.Ab[i] = static_cast<const bf16_t*>(d[i].a);
    p.Bb[i] = static_cast<const bf16_t*>(d[i].b);
    p.Cb[i] = d[i].c;
    p.Mb[i] = (int32_t)d[i].m, p.Nb[i] = (int32_t)d[i].n, p.Kb[i] = (int32_t)d[i].k;
    p.ldab[i] = (int32_t)d[i].lda, p.ldbb[i] = (int32_t)d[i].ldb, p.ldcb[i] = (int32_t)d[i].ldc;
  }
  if (!gvl::gemm_w4x_grouped_try(p, gvl::as_stream(stream))) return -1;
  snprintf(g_batched_name, sizeof g_batched_name, "gemm_w4x_kernel<256, %d, true, true, %d, true>", p.bn,
           EPI_RES);
  GVL_LAUNCH_CHECK("gvl_gemm_grouped");
  return 0;
}

extern "C" int gvl_gemm_batched_kernel_name(char* buf, int32_t len) {
  GVL_REQUIRE(buf && len > 0, "gvl_gemm_batched_kernel_name: bad arguments");
  snprintf(buf, len, "%s", g_batched_name);
  return 0;
}

extern "C" int gvl_gemm_batched_dbias(const gvl_gemm_desc* d, void* const* dbias, int32_t count,
                                      gvl_stream_t stream) {
  GVL_REQUIRE(dbias != nullptr, "gvl_gemm_batched_dbias: null dbias");
  return gemm_batched_impl(d, dbias, count, stream);
}
