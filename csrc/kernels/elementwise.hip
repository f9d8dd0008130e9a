// Vectorised elementwise kernels (16-B bf16 vectors per lane, grid-stride, scalar tails).
#include "common.h"
#include "kernels.h"

namespace tdl {
namespace {

constexpr int NT = 256;
inline int blocks_for(long n) {
  return (int)std::min<long>(4096, std::max<long>(1, (n + NT - 1) / NT));
}

__global__ void relu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                bf16_t* __restrict__ dx, long n) {
  const long nv = n / 8;
  const long stride = (long)gridDim.x * NT;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < nv; i += stride) {
    float g[8], v[8];
    unpack8(((const uint4*)dy)[i], g);
    unpack8(((const uint4*)y)[i], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = v[j] > 0.f ? g[j] : 0.f;
    ((uint4*)dx)[i] = pack8(g);
  }
  for (long i = nv * 8 + blockIdx.x * (long)NT + threadIdx.x; i < n; i += stride)
    dx[i] = bf2f(y[i]) > 0.f ? dy[i] : (bf16_t)0;
}

__global__ void add_act_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                               bf16_t* __restrict__ y, long n, int relu) {
  const long nv = n / 8;
  const long stride = (long)gridDim.x * NT;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < nv; i += stride) {
    float va[8];
    unpack8(((const uint4*)a)[i], va);
    if (b) {
      float vb[8];
      unpack8(((const uint4*)b)[i], vb);
#pragma unroll
      for (int j = 0; j < 8; ++j) va[j] += vb[j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) va[j] = fmaxf(va[j], 0.f);
    }
    ((uint4*)y)[i] = pack8(va);
  }
  for (long i = nv * 8 + blockIdx.x * (long)NT + threadIdx.x; i < n; i += stride) {
    float v = bf2f(a[i]) + (b ? bf2f(b[i]) : 0.f);
    if (relu) v = fmaxf(v, 0.f);
    y[i] = f2bf(v);
  }
}

__global__ void scale_kernel(const void* __restrict__ x, const float* __restrict__ s,
                             void* __restrict__ y, long n, int bf16) {
  const float k = *s;
  const long stride = (long)gridDim.x * NT;
  if (bf16) {
    const bf16_t* xb = (const bf16_t*)x;
    bf16_t* yb = (bf16_t*)y;
    for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += stride) yb[i] = f2bf(bf2f(xb[i]) * k);
  } else {
    const float* xf = (const float*)x;
    float* yf = (float*)y;
    for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += stride) yf[i] = xf[i] * k;
  }
}

__global__ void sigmoid_threshold_kernel(const void* __restrict__ x, int bf16,
                                         float* __restrict__ prob, float* __restrict__ pred, long n,
                                         float thr) {
  const long stride = (long)gridDim.x * NT;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += stride) {
    const float v = bf16 ? bf2f(((const bf16_t*)x)[i]) : ((const float*)x)[i];
    const float p = 1.f / (1.f + __expf(-v));
    prob[i] = p;
    pred[i] = p > thr ? 1.f : 0.f;
  }
}

}  // namespace

void relu_bwd_launch(const bf16_t* dy, const bf16_t* y, bf16_t* dx, long n, hipStream_t st) {
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(blocks_for(n / 8 + 1)), dim3(NT), 0, st, dy, y, dx, n);
}

void add_act_launch(const bf16_t* a, const bf16_t* b, bf16_t* y, long n, bool relu, hipStream_t st) {
  hipLaunchKernelGGL(add_act_kernel, dim3(blocks_for(n / 8 + 1)), dim3(NT), 0, st, a, b, y, n,
                     relu ? 1 : 0);
}

void scale_by_scalar_launch(const void* x, const float* s, void* y, long n, bool bf16,
                            hipStream_t st) {
  hipLaunchKernelGGL(scale_kernel, dim3(blocks_for(n)), dim3(NT), 0, st, x, s, y, n, bf16 ? 1 : 0);
}

void sigmoid_threshold_launch(const void* x, bool x_bf16, float* prob, float* pred, long n,
                              float thr, hipStream_t st) {
  hipLaunchKernelGGL(sigmoid_threshold_kernel, dim3(blocks_for(n)), dim3(NT), 0, st, x,
                     x_bf16 ? 1 : 0, prob, pred, n, thr);
}

}  // namespace tdl
