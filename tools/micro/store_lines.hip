// Store-pattern microbenchmark: does a 16-B-per-lane store instruction cost per 128-B line it
// touches?  Every workgroup (256 threads, one per CU) writes T tiles of 256 rows x 192 bf16
// columns of a row-major [M, ld] matrix, as a GEMM epilogue does:
//   A: 16 rows x 64 B per wave instruction (lane: row l & 15, 16-B chunk l >> 4) — the
//      persistent / four-wave kernels' epilogue16 pattern (each 128-B line half-written);
//   B:  8 rows x 128 B per wave instruction (lane: row l >> 3, chunk l & 7) — whole lines.
// Same bytes, same addresses.  Prints us per launch for each (hipEvents, median of 5 x 20).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

template <int PAT>
__global__ __launch_bounds__(256) void store_tiles(uint4* __restrict__ c, int ld_chunks, int tiles_m,
                                                   int tiles_n, int T) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint4 v = make_uint4(lane, wave, blockIdx.x, 7);
  for (int t = 0; t < T; ++t) {
    const int tile = blockIdx.x + t * gridDim.x;
    const int tm = tile / tiles_n % tiles_m, tn = tile % tiles_n;
    // wave w owns rows 64 w .. 64 w + 63 of the tile, all 24 chunks (384 B) of each row
    const int r0 = tm * 256 + wave * 64, c0 = tn * 24;
    if (PAT == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)        // 16-row groups
#pragma unroll
        for (int s = 0; s < 6; ++s) {    // 64-B segments
          const int r = r0 + 16 * i + (lane & 15), ch = c0 + 4 * s + (lane >> 4);
          c[(size_t)r * ld_chunks + ch] = v;
        }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)        // 8-row groups
#pragma unroll
        for (int s = 0; s < 3; ++s) {    // 128-B lines
          const int r = r0 + 8 * i + (lane >> 3), ch = c0 + 8 * s + (lane & 7);
          c[(size_t)r * ld_chunks + ch] = v;
        }
    }
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  struct Case { int M, N; const char* name; };
  const Case cases[] = {{16384, 3072, "c_fc out 16384 x 3072"}, {8064, 3072, "8064 x 3072"},
                        {16384, 50304 / 192 * 192, "lm_head-like 16384 x 50112"}};
  for (const Case& cs : cases) {
    const int tiles_m = cs.M / 256, tiles_n = cs.N / 192, tiles = tiles_m * tiles_n;
    const int G = std::min(tiles, cus), T = tiles / G;
    uint4* c = nullptr;
    hipMalloc(&c, (size_t)cs.M * cs.N * 2);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int pat = 0; pat < 2; ++pat) {
      std::vector<float> ts;
      for (int rep = 0; rep < 6; ++rep) {
        hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) {
          if (pat == 0) store_tiles<0><<<G, 256>>>(c, cs.N / 8, tiles_m, tiles_n, T);
          else store_tiles<1><<<G, 256>>>(c, cs.N / 8, tiles_m, tiles_n, T);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep) ts.push_back(ms * 1000.f / 20);
      }
      std::sort(ts.begin(), ts.end());
      const double gb = (double)G * T * 256 * 192 * 2 / 1e9;
      printf("%-28s pattern %s: %8.1f us  (%.2f TB/s, %d tiles per CU)\n", cs.name,
             pat ? "B (8 rows x 128 B)" : "A (16 rows x 64 B)", ts[2], gb / ts[2] * 1e-3 * 1e6 / 1e6, T);
    }
    hipFree(c);
  }
  return 0;
}
