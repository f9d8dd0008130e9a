// fp8 (OCP e4m3fn, gfx950) quantisation with per-tensor scaling for the fp8 forward convolution
// (ResNet-152 fp8 weights/activations on the CDNA4 fp8 MFMA).
//
//   amax      : |x|max over a bf16 tensor → an amax slot (common.h: spread partial maxima, one
//               atomicMax on the IEEE bits per workgroup — valid for values ≥ 0)
//   quantize  : scale = amax / 448 (E4M3 max normal), y8 = sat(x / scale) as e4m3; the scale is
//               also written to device memory for the GEMM epilogue (acc · s_x · s_w).  Delayed
//               scaling: the scale comes from the previous call's slot while this call measures
//               its own amax (one pass, no host sync, no memset)
//   dequantize: tests / debugging
// Everything stays on the device: no host synchronisation for the scale.
#include "common.h"
#include "kernels.h"

namespace tdl {
namespace {

constexpr int NT = 256;
constexpr float E4M3_MAX = 448.f;

__global__ void __launch_bounds__(NT) amax_kernel(const bf16_t* __restrict__ x, long nvec,
                                                  float* __restrict__ slot) {
  float m = 0.f;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < nvec; i += (long)gridDim.x * NT) {
    float v[8];
    unpack8(((const uint4*)x)[i], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
  }
  amax_publish(slot, m);
}

__device__ __forceinline__ uint32_t pack4_e4m3(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

constexpr float E5M2_MAX = 57344.f;

__device__ __forceinline__ uint32_t pack4_e5m2(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, v, true);
  return (uint32_t)v;
}

// e5m2 flavour of quantize_kernel (same delayed-scaling slots)
__global__ void __launch_bounds__(NT) quantize_e5m2_kernel(const bf16_t* __restrict__ x, long n16,
                                                           const float* __restrict__ prev,
                                                           float* __restrict__ meas,
                                                           float* __restrict__ clr,
                                                           float* __restrict__ scale_out,
                                                           uint8_t* __restrict__ y, float margin) {
  const float am = fmaxf(amax_read(prev) * margin, 1e-30f);
  const float inv = E5M2_MAX / am;
  if (blockIdx.x == 0 && threadIdx.x == 0 && scale_out) *scale_out = am / E5M2_MAX;
  if (clr) amax_clear(clr);
  float m = 0.f;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n16; i += (long)gridDim.x * NT) {
    float v[16];
    unpack8(((const uint4*)x)[2 * i], v);
    unpack8(((const uint4*)x)[2 * i + 1], v + 8);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      m = fmaxf(m, fabsf(v[j]));
      v[j] = fminf(fmaxf(v[j] * inv, -E5M2_MAX), E5M2_MAX);
    }
    uint4 o;
    o.x = pack4_e5m2(v[0], v[1], v[2], v[3]);
    o.y = pack4_e5m2(v[4], v[5], v[6], v[7]);
    o.z = pack4_e5m2(v[8], v[9], v[10], v[11]);
    o.w = pack4_e5m2(v[12], v[13], v[14], v[15]);
    ((uint4*)y)[i] = o;
  }
  if (meas) amax_publish(meas, m);
}

// one 64×64 byte tile per workgroup: 16-B row loads → LDS (padded rows) → 16-B column stores
__global__ void __launch_bounds__(256) multi_transpose_kernel(const uint8_t* __restrict__ src,
                                                              uint8_t* __restrict__ dst,
                                                              const long* __restrict__ tiles) {
  __shared__ uint8_t t[64][64 + 16];
  const long* d = tiles + 4 * (long)blockIdx.x;
  const long off = d[0], rows = d[1], cols = d[2], id = d[3];
  const long tcols = (cols + 63) / 64;
  const long r0 = (id / tcols) * 64, c0 = (id % tcols) * 64;
  const int tr = threadIdx.x >> 2, tc = (threadIdx.x & 3) * 16;
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (r0 + tr < rows && c0 + tc < cols) v = *(const uint4*)(src + off + (r0 + tr) * cols + c0 + tc);
  *(uint4*)&t[tr][tc] = v;
  __syncthreads();
  // output row = source column c0 + tr, 16 consecutive source rows r0 + tc … +15
  if (c0 + tr < cols && r0 + tc < rows) {
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      w[q] = (uint32_t)t[tc + 4 * q][tr] | ((uint32_t)t[tc + 4 * q + 1][tr] << 8) |
             ((uint32_t)t[tc + 4 * q + 2][tr] << 16) | ((uint32_t)t[tc + 4 * q + 3][tr] << 24);
    *(uint4*)(dst + off + (c0 + tr) * rows + r0 + tc) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

__global__ void dequantize_e5m2_kernel(const uint8_t* __restrict__ y, long n,
                                       const float* __restrict__ scale, float* __restrict__ out) {
  const float s = *scale;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = __builtin_amdgcn_cvt_f32_bf8((int)y[i], 0) * s;
}

// 16 elements per thread: two 16-B bf16 vectors in, one 16-B e4m3 vector out.  scale = amax(slot
// `prev`)/448; with `meas` the |x|max of this call is accumulated into `meas` (the next call's
// scale: delayed scaling) and `clr` is cleared for the call after.
__global__ void __launch_bounds__(NT) quantize_kernel(const bf16_t* __restrict__ x, long n16,
                                                      const float* __restrict__ prev,
                                                      float* __restrict__ meas, float* __restrict__ clr,
                                                      float* __restrict__ scale_out,
                                                      uint8_t* __restrict__ y, float margin) {
  const float am = fmaxf(amax_read(prev) * margin, 1e-12f);
  const float inv = E4M3_MAX / am;
  if (blockIdx.x == 0 && threadIdx.x == 0 && scale_out) *scale_out = am / E4M3_MAX;
  if (clr) amax_clear(clr);
  float m = 0.f;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n16; i += (long)gridDim.x * NT) {
    float v[16];
    unpack8(((const uint4*)x)[2 * i], v);
    unpack8(((const uint4*)x)[2 * i + 1], v + 8);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      m = fmaxf(m, fabsf(v[j]));
      v[j] = fminf(fmaxf(v[j] * inv, -E4M3_MAX), E4M3_MAX);
    }
    uint4 o;
    o.x = pack4_e4m3(v[0], v[1], v[2], v[3]);
    o.y = pack4_e4m3(v[4], v[5], v[6], v[7]);
    o.z = pack4_e4m3(v[8], v[9], v[10], v[11]);
    o.w = pack4_e4m3(v[12], v[13], v[14], v[15]);
    ((uint4*)y)[i] = o;
  }
  if (meas) amax_publish(meas, m);
}

// All fp8 weights of a model in ONE launch (after each optimizer step): the bf16 compute copies
// live in one flat buffer (models/params.py), the e4m3 copies in a parallel flat byte buffer.
// Work list: chunk c = (segment, start, len, first) with len % 16 == 0; each segment (weight
// tensor) has its own delayed-scaling amax ring rings[seg] = fp32[3][AMAX_SLOT] and scale
// scales[seg].  prime = 1: measure |w|max into slot `phase` only (first call).
__global__ void __launch_bounds__(NT) multi_quantize_kernel(const bf16_t* __restrict__ src,
                                                            uint8_t* __restrict__ dst,
                                                            const long* __restrict__ chunks,
                                                            float* __restrict__ rings,
                                                            float* __restrict__ scales, int phase,
                                                            int prime, float margin) {
  const long* c = chunks + 4 * (long)blockIdx.x;
  const long seg = c[0], start = c[1], n16 = c[2] / 16;
  float* ring = rings + seg * 3 * AMAX_SLOT;
  float* prev = ring + phase * AMAX_SLOT;
  const uint4* s4 = (const uint4*)(src + start);
  float m = 0.f;
  if (prime) {
    for (long i = threadIdx.x; i < n16; i += NT) {
      float v[16];
      unpack8(s4[2 * i], v);
      unpack8(s4[2 * i + 1], v + 8);
#pragma unroll
      for (int j = 0; j < 16; ++j) m = fmaxf(m, fabsf(v[j]));
    }
    amax_publish(prev, m);
    return;
  }
  const float am = fmaxf(amax_read(prev) * margin, 1e-12f);
  const float inv = E4M3_MAX / am;
  if (c[3] && threadIdx.x == 0) scales[seg] = am / E4M3_MAX;
  if (c[3] && threadIdx.x < AMAX_SPREAD)
    ring[(phase + 2) % 3 * AMAX_SLOT + threadIdx.x * AMAX_STRIDE] = 0.f;
  uint4* d4 = (uint4*)(dst + start);
  for (long i = threadIdx.x; i < n16; i += NT) {
    float v[16];
    unpack8(s4[2 * i], v);
    unpack8(s4[2 * i + 1], v + 8);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      m = fmaxf(m, fabsf(v[j]));
      v[j] = fminf(fmaxf(v[j] * inv, -E4M3_MAX), E4M3_MAX);
    }
    uint4 o;
    o.x = pack4_e4m3(v[0], v[1], v[2], v[3]);
    o.y = pack4_e4m3(v[4], v[5], v[6], v[7]);
    o.z = pack4_e4m3(v[8], v[9], v[10], v[11]);
    o.w = pack4_e4m3(v[12], v[13], v[14], v[15]);
    d4[i] = o;
  }
  amax_publish(ring + (phase + 1) % 3 * AMAX_SLOT, m);
}

__global__ void dequantize_kernel(const uint8_t* __restrict__ y, long n, const float* __restrict__ scale,
                                  float* __restrict__ out) {
  const float s = *scale;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int w = (int)y[i];
    out[i] = __builtin_amdgcn_cvt_f32_fp8(w, 0) * s;
  }
}

// End-of-step roll of every delayed-scaling amax ring (graph-capturable: the slot roles are fixed,
// the data moves): slot 0 (read by the next call) ← max(slot 1 (accumulated by this step's call),
// decay · slot 0) — an exponentially forgetting amax history: with decay > 0 a step whose |x|max
// dips does not shrink the scale at once, so the next step's larger values are not clipped —
// slot 1 ← 0.  rings: n ring base addresses (fp32 [3][AMAX_SLOT] each)
__global__ void __launch_bounds__(NT) roll_kernel(const unsigned long long* __restrict__ rings,
                                                  float decay) {
  float* r = (float*)rings[blockIdx.x];
  for (int t = threadIdx.x; t < AMAX_SLOT; t += NT) {
    r[t] = fmaxf(r[AMAX_SLOT + t], decay * r[t]);
    r[AMAX_SLOT + t] = 0.f;
  }
}

inline int grid_for(long n) { return (int)std::min<long>(4096, std::max<long>(1, (n + NT - 1) / NT)); }

}  // namespace

// delayed-scaling policy (TDL_FP8_MARGIN / TDL_FP8_MARGIN_E5M2 / TDL_FP8_AMAX_DECAY, or
// fp8_set_policy): scale = margin · amax_history / fp8_max.  Defaults from the memorisation sweep
// (dev/tools/fp8_policy_sweep.py, profiles/r05_fp8_numerics.txt): e4m3 margin 1 (2 was worse:
// a binade of precision lost at the bottom for no clipping saved), e5m2 margin 16 (loss tail
// 0.023 vs 0.030 at 4: e5m2's 32 binades afford it, a clipped gradient biases the update), no
// amax decay (0.9 did not help)
static float g_policy[3] = {-1.f, -1.f, -1.f};
static float env_f(const char* name, float dflt) {
  const char* e = getenv(name);
  return e ? (float)atof(e) : dflt;
}
Fp8Policy fp8_policy() {
  static const Fp8Policy env{env_f("TDL_FP8_MARGIN", 1.f), env_f("TDL_FP8_MARGIN_E5M2", 16.f),
                             env_f("TDL_FP8_AMAX_DECAY", 0.f)};
  return Fp8Policy{g_policy[0] >= 0.f ? g_policy[0] : env.margin_e4m3,
                   g_policy[1] >= 0.f ? g_policy[1] : env.margin_e5m2,
                   g_policy[2] >= 0.f ? g_policy[2] : env.decay};
}
void fp8_set_policy(float margin_e4m3, float margin_e5m2, float decay) {
  g_policy[0] = margin_e4m3;
  g_policy[1] = margin_e5m2;
  g_policy[2] = decay;
}

void fp8_roll_launch(const unsigned long long* rings, int n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(roll_kernel, dim3(n), dim3(NT), 0, st, rings, fp8_policy().decay);
}

void fp8_amax_launch(const bf16_t* x, long n, float* slot, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(amax_kernel, dim3(grid_for(n / 8)), dim3(NT), 0, st, x, n / 8, slot);
}

void fp8_quantize_launch(const bf16_t* x, long n, const float* prev, float* meas, float* clr,
                         float* scale_out, uint8_t* y, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(quantize_kernel, dim3(grid_for(n / 16)), dim3(NT), 0, st, x, n / 16, prev, meas,
                     clr, scale_out, y, meas ? fp8_policy().margin_e4m3 : 1.f);  // (JIT: exact)
}

void fp8_multi_quantize_launch(const bf16_t* src, uint8_t* dst, const long* chunks, int nchunks,
                               float* rings, float* scales, int phase, bool prime, hipStream_t st) {
  if (nchunks <= 0) return;
  hipLaunchKernelGGL(multi_quantize_kernel, dim3(nchunks), dim3(NT), 0, st, src, dst, chunks, rings,
                     scales, phase, prime ? 1 : 0, fp8_policy().margin_e4m3);
}

void fp8_quantize_e5m2_launch(const bf16_t* x, long n, const float* prev, float* meas, float* clr,
                              float* scale_out, uint8_t* y, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(quantize_e5m2_kernel, dim3(grid_for(n / 16)), dim3(NT), 0, st, x, n / 16, prev,
                     meas, clr, scale_out, y, meas ? fp8_policy().margin_e5m2 : 1.f);
}

void fp8_dequantize_e5m2_launch(const uint8_t* y, long n, const float* scale, float* out,
                                hipStream_t st) {
  hipLaunchKernelGGL(dequantize_e5m2_kernel, dim3(grid_for(n)), dim3(NT), 0, st, y, n, scale, out);
}

void fp8_multi_transpose_launch(const uint8_t* src, uint8_t* dst, const long* tiles, int ntiles,
                                hipStream_t st) {
  if (ntiles <= 0) return;
  hipLaunchKernelGGL(multi_transpose_kernel, dim3(ntiles), dim3(256), 0, st, src, dst, tiles);
}

void fp8_dequantize_launch(const uint8_t* y, long n, const float* scale, float* out, hipStream_t st) {
  hipLaunchKernelGGL(dequantize_kernel, dim3(grid_for(n)), dim3(NT), 0, st, y, n, scale, out);
}

}  // namespace tdl
