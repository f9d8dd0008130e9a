// Store-pattern microbenchmark: how fast can a persistent grid write a bf16 [M][N] output tile by
// tile with (a) the MFMA fragment layout the conv epilogues use (per store instruction 16 rows ×
// 32 B: lane = row l&15, 4-column group l>>4, 8 B per lane), (b) full-row coalesced 16-B lanes
// (a wave instruction covers 4 rows × 256 B), (c) fragment layout with 16 B per lane (8 columns:
// 16 rows × 64 B per instruction).  Tiles of 256 × 128 (8 waves, 64 × 64 per wave), as the
// LDS-DMA conv kernel.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/store_pattern dev/tools/store_pattern.hip && /tmp/store_pattern
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

template <int PAT>
__global__ void __launch_bounds__(512, 1) store_kernel(uint16_t* __restrict__ out, int M, int N,
                                                        int tiles_per_block) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / 2, wn = wid % 2;
  const int ntn = N / 128;
  const int t0 = blockIdx.x * tiles_per_block;
  const int ntiles = (M / 256) * ntn;
  for (int t = t0; t < t0 + tiles_per_block && t < ntiles; ++t) {
    const int bm0 = (t / ntn) * 256, bn0 = (t % ntn) * 128;
    if (PAT == 0) {  // fragment layout, 8 B per lane
#pragma unroll
      for (int rm = 0; rm < 4; ++rm)
#pragma unroll
        for (int rn = 0; rn < 4; ++rn) {
          const int m = bm0 + wm * 64 + rm * 16 + (lane & 15);
          const int n = bn0 + wn * 64 + rn * 16 + (lane >> 4) * 4;
          v2u32 v = {(uint32_t)(m + rn), (uint32_t)n};
          *(v2u32*)(out + (long)m * N + n) = v;
        }
    } else if (PAT == 1) {  // coalesced: 16 lanes per 256-B row, 4 rows per instruction
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = bm0 + wid * 32 + i * 4 + (lane >> 4);
        const int n = bn0 + (lane & 15) * 8;
        v4u32 v = {(uint32_t)m, (uint32_t)n, (uint32_t)i, 0u};
        *(v4u32*)(out + (long)m * N + n) = v;
      }
    } else {  // fragment rows, 16 B per lane (8 columns): 16 rows × 64 B per instruction
#pragma unroll
      for (int rm = 0; rm < 4; ++rm)
#pragma unroll
        for (int rn = 0; rn < 2; ++rn) {
          const int m = bm0 + wm * 64 + rm * 16 + (lane & 15);
          const int n = bn0 + wn * 64 + rn * 32 + (lane >> 4) * 8;
          v4u32 v = {(uint32_t)m, (uint32_t)n, (uint32_t)rn, 0u};
          *(v4u32*)(out + (long)m * N + n) = v;
        }
    }
  }
}

int main() {
  const int N = 256;
  const int M = 802816;  // ResNet-50 b256, 56×56 pixels: 411 MB of bf16 at N = 256
  uint16_t* out;
  hipMalloc(&out, (size_t)M * N * 2);
  const int ntiles = (M / 256) * (N / 128);
  for (int blocks : {256, 512, 1024, 2048}) {
    const int tpb = (ntiles + blocks - 1) / blocks;
    for (int pat = 0; pat < 3; ++pat) {
      auto k = pat == 0 ? store_kernel<0> : pat == 1 ? store_kernel<1> : store_kernel<2>;
      hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, out, M, N, tpb);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, out, M, N, tpb);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 100.0;
      printf("blocks %5d pattern %d: %7.1f us  %5.2f TB/s\n", blocks, pat, us,
             (double)M * N * 2 / (us * 1e-6) / 1e12);
    }
  }
  hipFree(out);
  return 0;
}
