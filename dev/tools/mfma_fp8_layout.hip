// Determines the A/B lane layout of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3, unit E8M0
// scales) with exact small-integer data (guide §3: check every non-bf16 map before relying on
// it).  Candidates for lane l, byte j (0..31):
//   H1: k = 32·(l>>4) + j                      (contiguous 32-deep slice per lane group)
//   H2: k = 8·(l>>4) + 32·(j>>3) + (j&7)       (four 16x16x32 blocks)
// Prints the max |error| of each candidate vs the host product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <math.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void mm(const v8i* a, const v8i* b, f4* c) {
  const int l = threadIdx.x;
  f4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, 127, 0, 127);
  c[l] = acc;
}

static uint8_t e4m3(int v) {  // exact for v in [-2, 2]
  switch (v) {
    case 0: return 0x00;
    case 1: return 0x38;
    case 2: return 0x40;
    case -1: return 0xB8;
    case -2: return 0xC0;
  }
  return 0;
}

int main() {
  int A[16][128], B[128][16];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 128; ++k) A[i][k] = ((i * 7 + k * 3) % 5) - 2;
  for (int k = 0; k < 128; ++k)
    for (int j = 0; j < 16; ++j) B[k][j] = ((k * 5 + j * 11 + 1) % 5) - 2;
  float ref[16][16];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      float s = 0;
      for (int k = 0; k < 128; ++k) s += A[i][k] * B[k][j];
      ref[i][j] = s;
    }
  v8i *da, *db;
  f4* dc;
  hipMalloc(&da, 64 * 32);
  hipMalloc(&db, 64 * 32);
  hipMalloc(&dc, 64 * 16);
  for (int h = 1; h <= 2; ++h) {
    uint8_t ha[64][32], hb[64][32];
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        const int k = h == 1 ? 32 * (l >> 4) + j : 8 * (l >> 4) + 32 * (j >> 3) + (j & 7);
        ha[l][j] = e4m3(A[l & 15][k]);  // A[row = l&15][k]
        hb[l][j] = e4m3(B[k][l & 15]);  // B[k][col = l&15]
      }
    hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, da, db, dc);
    float hc[64][4];
    hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
    float err = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        const int col = l & 15, row = (l >> 4) * 4 + r;  // C/D map (dtype independent)
        err = fmaxf(err, fabsf(hc[l][r] - ref[row][col]));
      }
    printf("H%d max_abs_err %.3f\n", h, err);
  }
  return 0;
}
