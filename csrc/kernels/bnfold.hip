// Per-step weight preparation of a training BN folded into its 1×1 consumer conv (ops/bnfold.py):
//   forward: W' = W·diag(a) in the compute dtype and the bias W·b — one launch, one workgroup per
//            output channel row (K×C is at most 2048² here: a few µs, instead of the five
//            PyTorch launches of float copy, multiply, cast, gemv and add it replaced);
//   backward: dW[k][c] *= a[c] on the fp32 weight gradient, in place.
// a = coef[0], b = coef[1] (bn_finalize layout: fp32 [4][Cp]).
#include "common.h"
#include "kernels.h"

namespace tdl {
namespace {

constexpr int FT = 256;

template <typename T>
__global__ void __launch_bounds__(FT) bn_fold_weight_kernel(const T* __restrict__ w,
                                                           const float* __restrict__ coef, int C,
                                                           int ldcoef, T* __restrict__ wout,
                                                           const float* __restrict__ bias_in,
                                                           float* __restrict__ bias_out) {
  const int k = blockIdx.x;
  const T* row = w + (long)k * C;
  T* orow = wout + (long)k * C;
  float acc = 0.f;
  for (int c = threadIdx.x; c < C; c += FT) {
    float v;
    if constexpr (sizeof(T) == 2) v = bf2f(row[c]); else v = (float)row[c];
    const float a = coef[c], b = coef[ldcoef + c];
    if constexpr (sizeof(T) == 2) orow[c] = f2bf(v * a); else orow[c] = v * a;
    acc = fmaf(v, b, acc);
  }
  // workgroup reduction of Σ_c W[k][c]·b[c] (fixed order: deterministic)
  __shared__ float red[FT / 64];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < FT / 64; ++i) s += red[i];
    bias_out[k] = s + (bias_in ? bias_in[k] : 0.f);
  }
}

__global__ void __launch_bounds__(FT) scale_cols_kernel(float* __restrict__ dw,
                                                        const float* __restrict__ a, long n, int C) {
  const long i = blockIdx.x * (long)FT + threadIdx.x;
  if (i < n) dw[i] *= a[i % C];
}

}  // namespace

void bn_fold_weight_launch(const void* w, bool bf16, const float* coef, int K, int C, int ldcoef,
                           void* wout, const float* bias_in, float* bias_out, hipStream_t st) {
  if (K <= 0 || C <= 0) return;
  if (bf16)
    hipLaunchKernelGGL(bn_fold_weight_kernel<bf16_t>, dim3(K), dim3(FT), 0, st,
                       (const bf16_t*)w, coef, C, ldcoef, (bf16_t*)wout, bias_in, bias_out);
  else
    hipLaunchKernelGGL(bn_fold_weight_kernel<float>, dim3(K), dim3(FT), 0, st, (const float*)w,
                       coef, C, ldcoef, (float*)wout, bias_in, bias_out);
}

void scale_cols_launch(float* dw, const float* a, long n, int C, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scale_cols_kernel, dim3((unsigned)((n + FT - 1) / FT)), dim3(FT), 0, st, dw,
                     a, n, C);
}

}  // namespace tdl
