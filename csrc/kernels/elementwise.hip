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

// Row packing of a few-channel image for its k×k stem conv (ops/conv.py row_pack): t[n][h][wo] =
// the S·Cr values x[n][h][wo·sw − pl + s][c] (s < S, c < Cr; zero outside the row) followed by zero
// padding to Cp.  The k×k conv over x is then a k×1 conv over t whose GEMM K is R·Cp (168 for the
// 7×7 RGB stem) instead of R·S·8 (392 with the channels padded to 8).  One thread per 16-B chunk.
__global__ void row_pack_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ t, long chunks,
                                int H, int W, int Cx, int Cr, int S, int sw, int pl, int Wo, int Cp) {
  const int cpc = Cp >> 3;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < chunks;
       i += (long)gridDim.x * blockDim.x) {
    const long row = i / cpc;  // (n, h, wo)
    const int q = (int)(i - row * cpc);
    const int wo = (int)(row % Wo);
    const long nh = row / Wo;  // n·H + h
    const int w0 = wo * sw - pl;
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      uint32_t pair = 0;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int e = q * 8 + j + h2, s = e / Cr, c = e - s * Cr, wi = w0 + s;
        uint32_t b = 0;
        if (s < S && (unsigned)wi < (unsigned)W) b = x[(nh * W + wi) * Cx + c];
        pair |= b << (16 * h2);
      }
      v[j >> 1] = pair;
    }
    *(uint4*)(t + i * 8) = make_uint4(v[0], v[1], v[2], v[3]);
  }
}

// the RGB stem's case (input padded to 8 channels, 7 taps × 3 channels → 24): one thread per
// output row — seven 16-B pixel loads (neighbouring rows share them through the caches), three
// 16-B stores; the generic kernel's per-element 2-byte loads ran at ~2.6 TB/s
template <int S, int CR, int CP>
__global__ void row_pack_px8_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ t, long rows,
                                    int W, int sw, int pl, int Wo) {
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < rows;
       r += (long)gridDim.x * blockDim.x) {
    const int wo = (int)(r % Wo);
    const long nh = r / Wo;
    const int w0 = wo * sw - pl;
    uint4 px[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int wi = w0 + s;
      px[s] = (unsigned)wi < (unsigned)W ? *(const uint4*)(x + (nh * W + wi) * 8)
                                         : make_uint4(0, 0, 0, 0);
    }
    uint32_t o[CP / 2];
#pragma unroll
    for (int j = 0; j < CP / 2; ++j) o[j] = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint32_t w4[4] = {px[s].x, px[s].y, px[s].z, px[s].w};
#pragma unroll
      for (int c = 0; c < CR; ++c) {
        const int e = s * CR + c;
        const uint32_t v = (w4[c >> 1] >> (16 * (c & 1))) & 0xffffu;
        o[e >> 1] |= v << (16 * (e & 1));
      }
    }
    uint4* dst = (uint4*)(t + r * CP);
#pragma unroll
    for (int q = 0; q < CP / 8; ++q) dst[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  }
}

// The same packing with the image row staged in LDS: one workgroup per (n, h) input row (grid-
// stride over rows) loads the row's W pixels with one 16-B load each, then writes the packed row
// as consecutive 16-B chunks (Wo·CP/8 of them, lane-contiguous: every wave store is one
// contiguous run).  The per-thread version loaded 7 overlapping pixels per output column and
// wrote 48-B strided chunks (2.75 TB/s); here each input byte is fetched once.
template <int S, int CR, int CP, int WMAX>
__global__ void __launch_bounds__(256) row_pack_lds_kernel(const bf16_t* __restrict__ x,
                                                           bf16_t* __restrict__ t, long rows, int W,
                                                           int sw, int pl, int Wo) {
  __shared__ uint16_t px[WMAX][8];
  const int tid = threadIdx.x;
  const int nchunk = Wo * (CP / 8);
  for (long row = blockIdx.x; row < rows; row += gridDim.x) {
    const uint4* src = (const uint4*)(x + row * (long)W * 8);
    for (int w = tid; w < W; w += 256) *(uint4*)px[w] = src[w];
    __syncthreads();
    uint4* dst = (uint4*)(t + row * (long)Wo * CP);
    for (int q = tid; q < nchunk; q += 256) {
      const int wo = q / (CP / 8), part = q - wo * (CP / 8);
      const int w0 = wo * sw - pl;
      uint32_t v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t pair = 0;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int e = part * 8 + 2 * j + h2, s = e / CR, c = e - s * CR, wi = w0 + s;
          const uint32_t b = (s < S && (unsigned)wi < (unsigned)W) ? px[wi][c] : 0u;
          pair |= b << (16 * h2);
        }
        v[j] = pair;
      }
      dst[q] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    __syncthreads();
  }
}

}  // namespace

void row_pack_launch(const bf16_t* x, bf16_t* t, int N, int H, int W, int Cx, int Cr, int S,
                     int sw, int pl, int Wo, int Cp, hipStream_t st) {
  const long chunks = (long)N * H * Wo * (Cp / 8);
  if (chunks == 0) return;
  static const bool lds = getenv("TDL_ROWPACK_LDS") == nullptr || atoi(getenv("TDL_ROWPACK_LDS")) != 0;
  if (Cx == 8 && Cr == 3 && S == 7 && Cp == 24 && W <= 256 && lds) {
    const long rows = (long)N * H;  // image rows
    const int blocks = (int)std::min<long>(16384, rows);
    hipLaunchKernelGGL((row_pack_lds_kernel<7, 3, 24, 256>), dim3(blocks), dim3(256), 0, st, x, t,
                       rows, W, sw, pl, Wo);
    return;
  }
  if (Cx == 8 && Cr == 3 && S == 7 && Cp == 24) {
    const long rows = (long)N * H * Wo;
    const int blocks = (int)std::min<long>(16384, (rows + 255) / 256);
    hipLaunchKernelGGL((row_pack_px8_kernel<7, 3, 24>), dim3(blocks), dim3(256), 0, st, x, t, rows, W,
                       sw, pl, Wo);
    return;
  }
  const int blocks = (int)std::min<long>(8192, (chunks + 255) / 256);
  hipLaunchKernelGGL(row_pack_kernel, dim3(blocks), dim3(256), 0, st, x, t, chunks, H, W, Cx, Cr,
                     S, sw, pl, Wo, Cp);
}

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

// fp32 ↔ bf16 conversion (RNE) of flat buffers — the bf16 gradient buckets' pack / unpack
// (parallel/bucketer.py); 8 elements per thread, grid-stride, scalar tail
__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  const long n8 = n / 8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    const float4 a = ((const float4*)x)[2 * i], b = ((const float4*)x)[2 * i + 1];
    ((uint4*)y)[i] = make_uint4(cvt_pk_bf16(a.x, a.y), cvt_pk_bf16(a.z, a.w), cvt_pk_bf16(b.x, b.y),
                                cvt_pk_bf16(b.z, b.w));
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) y[n8 * 8 + threadIdx.x] = f2bf(x[n8 * 8 + threadIdx.x]);
}

__global__ void bf16_to_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long n) {
  const long n8 = n / 8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    float f[8];
    unpack8(((const uint4*)x)[i], f);
    ((float4*)y)[2 * i] = make_float4(f[0], f[1], f[2], f[3]);
    ((float4*)y)[2 * i + 1] = make_float4(f[4], f[5], f[6], f[7]);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) y[n8 * 8 + threadIdx.x] = bf2f(x[n8 * 8 + threadIdx.x]);
}

void convert_launch(const void* x, bool x_bf16, void* y, long n, hipStream_t st) {
  if (n <= 0) return;
  const int blocks = (int)std::min<long>(4096, std::max<long>(1, (n / 8 + NT - 1) / NT));
  if (x_bf16)
    hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(blocks), dim3(NT), 0, st, (const bf16_t*)x,
                       (float*)y, n);
  else
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(blocks), dim3(NT), 0, st, (const float*)x,
                       (bf16_t*)y, n);
}

void sigmoid_threshold_launch(const void* x, bool x_bf16, float* prob, float* pred, long n,
                              float thr, hipStream_t st) {
  hipLaunchKernelGGL(sigmoid_threshold_kernel, dim3(blocks_for(n)), dim3(NT), 0, st, x,
                     x_bf16 ? 1 : 0, prob, pred, n, thr);
}

}  // namespace tdl
