// LDS-DMA ring helpers shared by the ring / ping-pong GEMM kernels (gemm_ring.hip,
// gemm_pp3.h, gemm_w4.hip): K-steps of 32, one slot per step, swizzle applied on the DMA source.
#pragma once
#include "common.h"

namespace gvl_ring {

constexpr int KS = 32;  // K-step depth
typedef __attribute__((address_space(3))) void lds_void_t;

GVL_DEV int f64b(int row) { return (row >> 1) & 2; }                          // 64-B rows
GVL_DEV int fT(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }           // 256-B rows

GVL_DEV __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffff ? bytes : 0x7fffffff));
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

template <int R, bool MN, int NWV>
struct Step {
  static constexpr int BYTES = R * KS * 2;
  static constexpr int NINSTR = BYTES / 1024;

  GVL_DEV static void issue(__amdgpu_buffer_rsrc_t rs, int64_t ld, int64_t r0, int64_t k0,
                            char* lds, int wave, int lane) {
#pragma unroll
    for (int t = 0; t < NINSTR / NWV; ++t) {
      const int j = t * NWV + wave;
      int64_t off_elems;
      if (!MN) {
        const int row = 16 * j + (lane >> 2);
        const int lc = (lane & 3) ^ f64b(row);
        off_elems = (r0 + row) * ld + k0 + lc * 8;
      } else {
        const int half = j >> 3, kr = 4 * (j & 7) + (lane >> 4);
        const int lc = (lane & 15) ^ fT(kr);
        off_elems = (k0 + kr) * ld + r0 + half * 128 + lc * 8;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + j * 1024), 16,
                                               (int)(off_elems * 2), 0, 0, 0);
    }
  }

  // Persistent kernels: this wave's DMA pieces as per-lane byte offsets of the k = 0 step of
  // a tile at r0 (computed once per tile); step k adds k * step_bytes(ld) as the scalar
  // soffset, so the per-step issue is address-arithmetic free.
  static constexpr int PER = NINSTR / NWV;
  GVL_DEV static void base_offsets(int64_t ld, int64_t r0, int64_t k0, int wave, int lane,
                                   int (&off)[PER]) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int j = t * NWV + wave;
      int64_t e;
      if (!MN) {
        const int row = 16 * j + (lane >> 2);
        e = (r0 + row) * ld + k0 + ((lane & 3) ^ f64b(row)) * 8;
      } else {
        const int half = j >> 3, kr = 4 * (j & 7) + (lane >> 4);
        e = (k0 + kr) * ld + r0 + half * 128 + ((lane & 15) ^ fT(kr)) * 8;
      }
      off[t] = (int)(e * 2);
    }
  }
  GVL_DEV static int step_bytes(int64_t ld) { return MN ? (int)(KS * ld * 2) : KS * 2; }
  GVL_DEV static void issue_at(__amdgpu_buffer_rsrc_t rs, const int (&off)[PER], int kbytes,
                               char* lds, int wave) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int j = t * NWV + wave;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + j * 1024), 16, off[t],
                                               kbytes, 0, 0);
    }
  }

  // 16x32 operand fragment for rows/cols [c0, c0+16) of this K-step.
  GVL_DEV static short8_t frag(const char* lds, int c0, int lane) {
    if (!MN) {
      const int row = c0 + (lane & 15), ch = lane >> 4;
      return *reinterpret_cast<const short8_t*>(lds + row * 64 + ((ch ^ f64b(row)) << 4));
    } else {
      const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
      const int half = c0 >> 7, cl = c0 & 127;
      const int kr = 8 * G + q;
      const int ch = (cl >> 3) + (p >> 1);
      const char* base = lds + half * (KS * 256);
      const int off1 = kr * 256 + ((ch ^ fT(kr)) << 4) + (p & 1) * 8;
      short8_t r;
      r.lo = lds_read_tr(base + off1);
      r.hi = lds_read_tr(base + off1 + 4 * 256);
      return r;
    }
  }
};

// 192-wide operand slab of a 32-deep K-step (gemm_pp3_kernel with BN = 192: 8 waves, so
// waves 0-3 issue two of the 12 DMA pieces and waves 4-7 one, piece j = wave + 8 t, j < 12;
// gemm_w4x_kernel: 4 waves, three pieces each).
//  * K-contiguous: [192 rows][32] 64-B rows, the Step image;
//  * MN-contiguous: cols 0-127 as the Step [32][128] half (256-B rows, fT swizzle), cols
//    128-191 as [32][64] 128-B rows at +8 KiB, chunk c of k-row kr at c ^ f2(kr) (conflict-free
//    ds_read_b64_tr_b16 lane groups for the fragment pattern below).
GVL_DEV int f2(int k) { return (((k >> 1) & 1) | ((k >> 2) & 2)) << 1; }  // 128-B rows

template <bool MN, int NWV = 8>
struct Step192 {
  static constexpr int R = 192;
  static constexpr int BYTES = R * KS * 2;
  static constexpr int NINSTR = BYTES / 1024;                // 12
  static constexpr int PER = (NINSTR + NWV - 1) / NWV;      // 8 waves: 2 for waves 0-3, 1 for 4-7
  GVL_DEV static int64_t elem(int64_t ld, int64_t r0, int64_t k0, int j, int lane) {
    if (!MN) {
      const int row = 16 * j + (lane >> 2);
      return (r0 + row) * ld + k0 + ((lane & 3) ^ f64b(row)) * 8;
    }
    if (j < 8) {
      const int kr = 4 * j + (lane >> 4);
      return (k0 + kr) * ld + r0 + ((lane & 15) ^ fT(kr)) * 8;
    }
    const int kr = 8 * (j - 8) + (lane >> 3);
    return (k0 + kr) * ld + r0 + 128 + ((lane & 7) ^ f2(kr)) * 8;
  }
  GVL_DEV static void base_offsets(int64_t ld, int64_t r0, int64_t k0, int wave, int lane,
                                   int (&off)[PER]) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int j = t * NWV + wave;
      off[t] = j < NINSTR ? (int)(elem(ld, r0, k0, j, lane) * 2) : 0;
    }
  }
  GVL_DEV static int step_bytes(int64_t ld) { return MN ? (int)(KS * ld * 2) : KS * 2; }
  GVL_DEV static void issue_at(__amdgpu_buffer_rsrc_t rs, const int (&off)[PER], int kbytes,
                               char* lds, int wave) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int j = t * NWV + wave;
      if (j < NINSTR)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(lds + j * 1024), 16, off[t],
                                                 kbytes, 0, 0);
    }
  }
  GVL_DEV static short8_t frag(const char* lds, int c0, int lane) {
    if (!MN) {
      const int row = c0 + (lane & 15), ch = lane >> 4;
      return *reinterpret_cast<const short8_t*>(lds + row * 64 + ((ch ^ f64b(row)) << 4));
    }
    const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int kr = 8 * G + q;
    short8_t r;
    if (c0 < 128) {
      const int ch = (c0 >> 3) + (p >> 1);
      const int off1 = kr * 256 + ((ch ^ fT(kr)) << 4) + (p & 1) * 8;
      r.lo = lds_read_tr(lds + off1);
      r.hi = lds_read_tr(lds + off1 + 4 * 256);
    } else {
      const int ch = ((c0 - 128) >> 3) + (p >> 1);
      const char* base = lds + 8192;
      const int off1 = kr * 128 + ((ch ^ f2(kr)) << 4) + (p & 1) * 8;
      r.lo = lds_read_tr(base + off1);
      r.hi = lds_read_tr(base + off1 + 4 * 128);
    }
    return r;
  }
};

// s_waitcnt vmcnt(n * PER) for a runtime n in [0, MAXN]: the count must be an immediate.
template <int PER, int MAXN>
GVL_DEV void wait_vm_steps(int n) {
  if (MAXN >= 4 && n >= 4) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PER) : "memory"); return; }
  if (MAXN >= 3 && n == 3) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER) : "memory"); return; }
  if (MAXN >= 2 && n == 2) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory"); return; }
  if (MAXN >= 1 && n == 1) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 * PER) : "memory"); return; }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

GVL_DEV void barrier_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

}  // namespace gvl_ring
