// The reference's `_upsample` (symmetric 1-px pad → TF1 legacy bilinear → crop) as a separable
// linear map with ≤2 taps per output row/column (tap tables built on the host).
// idx layout per axis (int32): [i0(O) | i1(O) | lo(I) | hi(I)], wt (fp32): [w0(O) | w1(O)];
// lo/hi = the (inclusive) range of outputs whose taps touch input index i — so the backward is a
// deterministic gather over that range instead of an atomic scatter.
#include "common.h"
#include "kernels.h"

namespace tdl {
namespace {

constexpr int NT = 256;
inline int blocks_for(long n) { return (int)std::min<long>(8192, std::max<long>(1, (n + NT - 1) / NT)); }

template <int V, typename T>
__global__ void up_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                              const int* __restrict__ ih, const float* __restrict__ wh,
                              const int* __restrict__ iw, const float* __restrict__ ww, int N, int H,
                              int W, int C, int Ho, int Wo, int ldy) {
  // ldy: pixel stride of y in elements (C, or wider: y is a channel slice of a concat buffer)
  const int cv = C / V;
  const long total = (long)N * Ho * Wo * cv;
  for (long t = blockIdx.x * (long)NT + threadIdx.x; t < total; t += (long)gridDim.x * NT) {
    const int c = (int)(t % cv) * V;
    long p = t / cv;
    const int j = (int)(p % Wo);
    p /= Wo;
    const int i = (int)(p % Ho);
    const int n = (int)(p / Ho);
    const int a0 = ih[i], a1 = ih[Ho + i];
    const float u0 = wh[i], u1 = wh[Ho + i];
    const int b0 = iw[j], b1 = iw[Wo + j];
    const float v0 = ww[j], v1 = ww[Wo + j];
    const int rows[2] = {a0, a1};
    const int cols[2] = {b0, b1};
    const float wr[2] = {u0, u1};
    const float wc[2] = {v0, v1};
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float wgt = wr[r] * wc[q];
        const T* src = x + (((long)n * H + rows[r]) * W + cols[q]) * C + c;
        float v[V];
        if constexpr (V == 8) load8(src, v);
        else v[0] = load1(src);
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] += wgt * v[k];
      }
    T* dst = y + (((long)n * Ho + i) * Wo + j) * ldy + c;
    if constexpr (V == 8) store8(dst, acc);
    else store1(dst, acc[0]);
  }
}

template <int V, typename T>
__global__ void up_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx,
                              const int* __restrict__ ih, const float* __restrict__ wh,
                              const int* __restrict__ iw, const float* __restrict__ ww, int N, int H,
                              int W, int C, int Ho, int Wo, int ldd) {
  // ldd: pixel stride of dy in elements (a channel slice of a concat buffer's gradient)
  const int cv = C / V;
  const long total = (long)N * H * W * cv;
  for (long t = blockIdx.x * (long)NT + threadIdx.x; t < total; t += (long)gridDim.x * NT) {
    const int c = (int)(t % cv) * V;
    long p = t / cv;
    const int b = (int)(p % W);
    p /= W;
    const int a = (int)(p % H);
    const int n = (int)(p / H);
    const int ilo = ih[2 * Ho + a], ihi = ih[2 * Ho + H + a];
    const int jlo = iw[2 * Wo + b], jhi = iw[2 * Wo + W + b];
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    for (int i = ilo; i <= ihi; ++i) {
      const float wi = (ih[i] == a ? wh[i] : 0.f) + (ih[Ho + i] == a ? wh[Ho + i] : 0.f);
      if (wi == 0.f) continue;
      for (int j = jlo; j <= jhi; ++j) {
        const float wj = (iw[j] == b ? ww[j] : 0.f) + (iw[Wo + j] == b ? ww[Wo + j] : 0.f);
        if (wj == 0.f) continue;
        const T* src = dy + (((long)n * Ho + i) * Wo + j) * ldd + c;
        float v[V];
        if constexpr (V == 8) load8(src, v);
        else v[0] = load1(src);
        const float wgt = wi * wj;
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] += wgt * v[k];
      }
    }
    T* dst = dx + (((long)n * H + a) * W + b) * C + c;
    if constexpr (V == 8) store8(dst, acc);
    else store1(dst, acc[0]);
  }
}

}  // namespace

template <typename T>
static void upsample_fwd_impl(const T* x, T* y, const int* ih, const float* wh, const int* iw,
                         const float* ww, int N, int H, int W, int C, int Ho, int Wo,
                         hipStream_t st, int ldy) {
  const long n = (long)N * Ho * Wo * C;
  if (ldy <= 0) ldy = C;
  if (C % 8 == 0 && ldy % 8 == 0)
    hipLaunchKernelGGL((up_fwd_kernel<8, T>), dim3(blocks_for(n / 8)), dim3(NT), 0, st, x, y, ih, wh, iw, ww,
                       N, H, W, C, Ho, Wo, ldy);
  else
    hipLaunchKernelGGL((up_fwd_kernel<1, T>), dim3(blocks_for(n)), dim3(NT), 0, st, x, y, ih, wh, iw, ww, N,
                       H, W, C, Ho, Wo, ldy);
}

template <typename T>
static void upsample_bwd_impl(const T* dy, T* dx, const int* ih, const float* wh,
                         const int* iw, const float* ww, int N, int H, int W, int C, int Ho, int Wo,
                         hipStream_t st, int ldd) {
  const long n = (long)N * H * W * C;
  if (ldd <= 0) ldd = C;
  if (C % 8 == 0 && ldd % 8 == 0)
    hipLaunchKernelGGL((up_bwd_kernel<8, T>), dim3(blocks_for(n / 8)), dim3(NT), 0, st, dy, dx, ih, wh, iw,
                       ww, N, H, W, C, Ho, Wo, ldd);
  else
    hipLaunchKernelGGL((up_bwd_kernel<1, T>), dim3(blocks_for(n)), dim3(NT), 0, st, dy, dx, ih, wh, iw, ww,
                       N, H, W, C, Ho, Wo, ldd);
}


#define TDL_UP_ENTRY(T)                                                                           \
  void upsample_fwd_launch(const T* x, T* y, const int* ih, const float* wh, const int* iw,       \
                           const float* ww, int N, int H, int W, int C, int Ho, int Wo,           \
                           hipStream_t st, int ldy) {                                             \
    upsample_fwd_impl<T>(x, y, ih, wh, iw, ww, N, H, W, C, Ho, Wo, st, ldy);                       \
  }                                                                                               \
  void upsample_bwd_launch(const T* dy, T* dx, const int* ih, const float* wh, const int* iw,     \
                           const float* ww, int N, int H, int W, int C, int Ho, int Wo,           \
                           hipStream_t st, int ldd) {                                             \
    upsample_bwd_impl<T>(dy, dx, ih, wh, iw, ww, N, H, W, C, Ho, Wo, st, ldd);                     \
  }
TDL_UP_ENTRY(bf16_t)
TDL_UP_ENTRY(float)
#undef TDL_UP_ENTRY

}  // namespace tdl
