// Microbenchmark of the LDS → MFMA inner loop of the LDS-DMA conv kernel (no global traffic):
// 512-thread workgroups (8 waves, 4×2), a 256×128×64 KC-swizzled bf16 tile pair in LDS, each wave
// a 64×64 sub-tile (4×4 v_mfma_f32_16x16x32_bf16 per 32-deep slice).  Variants differ only in
// the read / wait / MFMA schedule.  Build + run (on the GPU box):
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mm dev/tools/mfma_lds_micro.hip && /tmp/mm
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char_t;

constexpr int BM = 256, BN = 128, BK = 64, WM = 4, WN = 2, TM = 64, TN = 64, RM = 4, RN = 4;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;

__device__ __forceinline__ int kc_off(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}
__device__ __forceinline__ bf16x8 rd(uint32_t base, int row, int chunk) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(base + (uint32_t)kc_off(row, chunk)) : "memory");
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ void wait0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int V>
__global__ void __launch_bounds__(512, 1) kern(float* out, int steps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  for (int i = tid; i < (A_BYTES + B_BYTES) / 4; i += 512) ((float*)smem)[i] = 0.001f * (i & 255);
  __syncthreads();
  const uint32_t As = (uint32_t)(size_t)(lds_char_t*)smem, Bs = As + A_BYTES;
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  auto load = [&](int kk, bf16x8(&a)[RM], bf16x8(&b)[RN]) {
#pragma unroll
    for (int r = 0; r < RM; ++r) a[r] = rd(As, wm * TM + r * 16 + (lane & 15), kk * 4 + (lane >> 4));
#pragma unroll
    for (int r = 0; r < RN; ++r) b[r] = rd(Bs, wn * TN + r * 16 + (lane & 15), kk * 4 + (lane >> 4));
  };
  auto mm = [&](const bf16x8(&a)[RM], const bf16x8(&b)[RN]) {
    if (V == 3) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    if (V == 3) __builtin_amdgcn_s_setprio(0);
  };
  bf16x8 a0[RM], b0[RN], a1[RM], b1[RN];
  if (V == 0 || V == 3 || V == 4) {
    // current schedule: reads(k1) → MFMA(k0) → wait → barrier → reads(next k0) → MFMA(k1) → wait
    load(0, a0, b0);
    wait0();
    for (int s = 0; s < steps; ++s) {
      load(1, a1, b1);
      mm(a0, b0);
      wait0();
      if (V != 4) asm volatile("s_barrier" ::: "memory");
      load(0, a0, b0);
      mm(a1, b1);
      wait0();
    }
  } else if (V == 1) {
    // all 16 reads of a step up front, one wait, 32 MFMAs, barrier
    for (int s = 0; s < steps; ++s) {
      load(0, a0, b0);
      load(1, a1, b1);
      wait0();
      mm(a0, b0);
      mm(a1, b1);
      asm volatile("s_barrier" ::: "memory");
    }
  } else if (V == 2) {
    // compiler-scheduled plain LDS loads (no asm), barrier per step
    for (int s = 0; s < steps; ++s) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 a[RM], b[RN];
#pragma unroll
        for (int r = 0; r < RM; ++r)
          a[r] = *(const bf16x8*)(smem + kc_off(wm * TM + r * 16 + (lane & 15), kk * 4 + (lane >> 4)));
#pragma unroll
        for (int r = 0; r < RN; ++r)
          b[r] = *(const bf16x8*)(smem + A_BYTES + kc_off(wn * TN + r * 16 + (lane & 15), kk * 4 + (lane >> 4)));
        mm(a, b);
      }
      __syncthreads();
    }
  } else if (V == 5) {
    // MFMA only (operands in registers): the pipe's ceiling
    load(0, a0, b0);
    load(1, a1, b1);
    wait0();
    for (int s = 0; s < steps; ++s) {
      mm(a0, b0);
      mm(a1, b1);
    }
  }
  float t = 0;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * 512 + tid] = t;
}

template <int V>
void run(const char* name, float* out, int blocks, int steps) {
  auto k = kern<V>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, A_BYTES + B_BYTES);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), A_BYTES + B_BYTES, 0, out, steps);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), A_BYTES + B_BYTES, 0, out, steps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double flop = 2.0 * BM * BN * BK * (double)steps * blocks;
  printf("%-40s %8.1f us  %7.0f TF\n", name, best * 1e3, flop / (best * 1e-3) / 1e12);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 512 * 4 * 4);
  const int blocks = 256, steps = 2000;
  run<5>("V5 mfma only (regs)", out, blocks, steps);
  run<0>("V0 current (split reads, barrier)", out, blocks, steps);
  run<3>("V3 current + s_setprio", out, blocks, steps);
  run<4>("V4 current, no barrier", out, blocks, steps);
  run<1>("V1 16 reads, 1 wait, 32 mfma, barrier", out, blocks, steps);
  run<2>("V2 compiler-scheduled, syncthreads", out, blocks, steps);
  hipFree(out);
  return 0;
}
