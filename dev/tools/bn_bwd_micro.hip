// Isolates the fixed cost seen in bwd_apply_vec_kernel at small M·C (≈40 µs at 6 MB tensors
// while the forward apply takes 5 µs).  Variants: V bit0 = skip block-0 dγ/dβ copy, bit1 = no
// coefficient math from red/gamma (use coef only), bit2 = no relu mask.
#include "../csrc/kernels/bn.hip"
#include <stdio.h>
#include <vector>
using namespace tdl;
using tdl::NT;

template <int V>
__global__ void __launch_bounds__(NT) k(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                        const float* __restrict__ coef, const float* __restrict__ red,
                                        const float* __restrict__ gamma, bf16_t* __restrict__ dx,
                                        float* __restrict__ dgamma, long nvec, int C, float ic) {
  if (!(V & 1) && blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += NT) dgamma[c] = red[C + c];
  }
  const int cvecs = C >> 3;
  const long stride = (long)gridDim.x * NT;
  long i = blockIdx.x * (long)NT + threadIdx.x;
  float A[8], Bc[8], Cc[8], Sc[8], Sh[8];
  const int cv = (int)(i % cvecs);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cv * 8 + j;
    Sc[j] = coef[c];
    Sh[j] = coef[C + c];
    if (V & 2) {
      A[j] = Sc[j]; Bc[j] = Sh[j]; Cc[j] = 0.f;
    } else {
      const float mean = coef[2 * C + c], inv = coef[3 * C + c];
      const float a = gamma[c] * inv;
      const float b = -a * inv * red[C + c] * ic;
      A[j] = a; Bc[j] = b; Cc[j] = -a * red[c] * ic - b * mean;
    }
  }
  for (; i < nvec; i += stride) {
    float g[8], vx[8];
    unpack8(((const uint4*)dy)[i], g);
    unpack8(((const uint4*)x)[i], vx);
    if (!(V & 4)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = vx[j] * Sc[j] + Sh[j] > 0.f ? g[j] : 0.f;
    }
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = A[j] * g[j] + Bc[j] * vx[j] + Cc[j];
    ((uint4*)dx)[i] = pack8(o);
  }
}

template <int V>
float run(const bf16_t* dy, const bf16_t* x, const float* coef, const float* red, const float* gam,
          bf16_t* dx, float* dg, long n, int C) {
  const int blocks = (int)std::min<long>(2048, (n / 8 + NT - 1) / NT);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(NT), 0, 0, dy, x, coef, red, gam, dx, dg, n / 8, C, 1e-5f);
  hipEventRecord(a);
  for (int it = 0; it < 50; ++it)
    hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(NT), 0, 0, dy, x, coef, red, gam, dx, dg, n / 8, C, 1e-5f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000 / 50;
}

float run_real(const bf16_t* dy, const bf16_t* x, const float* coef, const float* red, const float* gam,
               bf16_t* dx, float* dg, long n, int C, int relu, bool with_dg) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w)
    bn_bwd_apply_launch(dy, nullptr, x, coef, red, gam, dx, nullptr, with_dg ? dg : nullptr, nullptr, n / C, C, 1e5f, relu, 0);
  hipEventRecord(a);
  for (int it = 0; it < 50; ++it)
    bn_bwd_apply_launch(dy, nullptr, x, coef, red, gam, dx, nullptr, with_dg ? dg : nullptr, nullptr, n / C, C, 1e5f, relu, 0);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000 / 50;
}

float run_reduce(const bf16_t* dy, const bf16_t* x, const float* coef, float* red, long n, int C, int relu) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) bn_bwd_reduce_launch(dy, x, x, coef, red, n / C, C, relu, 0);
  hipEventRecord(a);
  for (int it = 0; it < 50; ++it) bn_bwd_reduce_launch(dy, x, x, coef, red, n / C, C, relu, 0);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000 / 50;
}

int main() {
  const int shapes[][2] = {{128 * 49, 512}, {128 * 196, 256}, {128 * 196, 1024}, {128 * 784, 512}, {128 * 3136, 64}, {128 * 3136, 256}};
  for (auto& s : shapes) {
    const long M = s[0];
    const int C = s[1];
    const long n = M * C;
    bf16_t *dy, *x, *dx;
    float *coef, *red, *gam, *dg;
    hipMalloc(&dy, n * 2);
    hipMalloc(&x, n * 2);
    hipMalloc(&dx, n * 2);
    hipMalloc(&coef, 4 * C * 4);
    hipMalloc(&red, 2 * C * 4);
    hipMalloc(&gam, C * 4);
    hipMalloc(&dg, C * 4);
    std::vector<uint16_t> h(n);
    for (long i = 0; i < n; ++i) h[i] = 0x3f80 ^ ((i * 2654435761u) & 0x807f);
    hipMemcpy(dy, h.data(), n * 2, hipMemcpyHostToDevice);
    hipMemcpy(x, h.data(), n * 2, hipMemcpyHostToDevice);
    std::vector<float> hc(4 * C, 0.5f);
    hipMemcpy(coef, hc.data(), 4 * C * 4, hipMemcpyHostToDevice);
    hipMemcpy(red, hc.data(), 2 * C * 4, hipMemcpyHostToDevice);
    hipMemcpy(gam, hc.data(), C * 4, hipMemcpyHostToDevice);
    printf("M=%ld C=%d %.1f MB: V0 %.1f  V1 %.1f  V2 %.1f  V4 %.1f  V7 %.1f us\n", M, C, n * 2 / 1e6,
           run<0>(dy, x, coef, red, gam, dx, dg, n, C), run<1>(dy, x, coef, red, gam, dx, dg, n, C),
           run<2>(dy, x, coef, red, gam, dx, dg, n, C), run<4>(dy, x, coef, red, gam, dx, dg, n, C),
           run<7>(dy, x, coef, red, gam, dx, dg, n, C));
    printf("   real: relu2 %.1f  relu0 %.1f  relu2+dg %.1f us\n", run_real(dy, x, coef, red, gam, dx, dg, n, C, 2, false),
           run_real(dy, x, coef, red, gam, dx, dg, n, C, 0, false), run_real(dy, x, coef, red, gam, dx, dg, n, C, 2, true));
    float* red2;
    hipMalloc(&red2, 2 * C * 4);
    printf("   reduce: relu2 %.1f  relu1 %.1f us\n", run_reduce(dy, x, coef, red2, n, C, 2),
           run_reduce(dy, x, coef, red2, n, C, 1));
    hipFree(red2);
    hipFree(dy); hipFree(x); hipFree(dx); hipFree(coef); hipFree(red); hipFree(gam); hipFree(dg);
  }
  return 0;
}
