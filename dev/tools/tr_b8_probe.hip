// Probe of gfx950 ds_read_b64_tr_b8 semantics (exact integer data): LDS byte (row, col) of a
// [32 rows][64 cols] image holds row*64+col (mod 256 → we store row in the high nibble path via two
// images: one with the row index, one with the column index).  Every lane supplies an address
// chosen by a hypothesis (lane 2q+p of each 16-lane group: row q, columns 8p..8p+7 of block
// (row0 = 8*group, col0 = 16*group)), and writes back its 8 received bytes for both images.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) uint8_t lds_u8_t;

__global__ void probe(uint8_t* out_row, uint8_t* out_col) {
  __shared__ __attribute__((aligned(16))) uint8_t img_r[32 * 64];
  __shared__ __attribute__((aligned(16))) uint8_t img_c[32 * 64];
  const int t = threadIdx.x;
  for (int i = t; i < 32 * 64; i += 64) {
    img_r[i] = (uint8_t)(i / 64);
    img_c[i] = (uint8_t)(i % 64);
  }
  __syncthreads();
  const int g = t >> 4, i = t & 15, q = i >> 1, p = i & 1;
  const int row = 8 * (g & 3), col = 16 * (g & 3);
  const uint32_t off = (uint32_t)((row + q) * 64 + col + 8 * p);
  uint64_t vr, vc;
  const uint32_t ar = (uint32_t)(size_t)(lds_u8_t*)img_r + off;
  const uint32_t ac = (uint32_t)(size_t)(lds_u8_t*)img_c + off;
  asm volatile("ds_read_b64_tr_b8 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(vr) : "v"(ar) : "memory");
  asm volatile("ds_read_b64_tr_b8 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(vc) : "v"(ac) : "memory");
  for (int j = 0; j < 8; ++j) {
    out_row[t * 8 + j] = (uint8_t)(vr >> (8 * j));
    out_col[t * 8 + j] = (uint8_t)(vc >> (8 * j));
  }
}

int main() {
  uint8_t *dr, *dc;
  hipMalloc(&dr, 512);
  hipMalloc(&dc, 512);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dr, dc);
  uint8_t hr[512], hc[512];
  hipMemcpy(hr, dr, 512, hipMemcpyDeviceToHost);
  hipMemcpy(hc, dc, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 8; ++j) printf(" (%2d,%2d)", hr[l * 8 + j], hc[l * 8 + j]);
    printf("\n");
  }
  return 0;
}
