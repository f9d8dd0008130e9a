// BatchNorm (NHWC) kernels for gfx950 — memory-bound: every pass reads/writes 16-B bf16 vectors
// (8 channels per lane); per-channel reductions go lanes → LDS → one contiguous atomic row per
// workgroup.  A generic scalar path handles C % 8 != 0 (the reference preset's 258-wide block2).
//
//   bn_stats       Σx, Σx² (when the producer conv did not fuse them into its epilogue)
//   bn_finalize    mean, invstd, scale=γ·invstd, shift=β−mean·scale; moving averages (TF decay)
//   bn_apply       y = act(x·scale + shift [+ res])
//   bn_bwd_reduce  Σg, Σg·x̂   (g = dy·[y>0] when the forward had a ReLU; the mask comes from y
//                  (relu 1), from x·scale+shift (2, no residual) or from a 1-bit-per-element mask
//                  the forward apply wrote (3, residual BN: saves re-reading y twice)
//   bn_bwd_apply   dx = γ·invstd·(g − Σg/M − x̂·Σg·x̂/M);  dres = g
#include "common.h"
#include "kernels.h"

namespace tdl {
namespace {

constexpr int NT = 256;

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

__device__ __forceinline__ void unpack(const uint4& v, float f[8]) { unpack8(v, f); }

// ---------------------------------------------------------------------------------------------
// generic: each block covers 64 channels (one per lane) × a row range, 4 waves stride the rows
// ---------------------------------------------------------------------------------------------
template <int KIND>  // 0: stats(x) ; 1: bwd reduce(dy,y,x)
__global__ void reduce_scalar_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ y,
                                     const bf16_t* __restrict__ x, const float* __restrict__ coef,
                                     float* __restrict__ out, long M, int C, long rows_per_block,
                                     int relu, float* __restrict__ slab) {
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float s0 = 0.f, s1 = 0.f;
  if (c < C) {
    if (KIND == 0) {
      for (long r = r0 + w; r < r1; r += 4) {
        const float v = bf2f(a[r * C + c]);
        s0 += v;
        s1 += v * v;
      }
    } else {
      const float mean = coef[2 * C + c], inv = coef[3 * C + c];
      for (long r = r0 + w; r < r1; r += 4) {
        float g = bf2f(a[r * C + c]);
        if (relu == 1 && bf2f(y[r * C + c]) <= 0.f) g = 0.f;
        if (relu == 2 && bf2f(x[r * C + c]) * coef[c] + coef[C + c] <= 0.f) g = 0.f;
        const float xh = (bf2f(x[r * C + c]) - mean) * inv;
        s0 += g;
        s1 += g * xh;
      }
    }
  }
  red[0][w][lane] = s0;
  red[1][w][lane] = s1;
  __syncthreads();
  if (w == 0 && c < C) {
    const float a0 = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
    const float a1 = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
    if (slab) {  // deterministic mode: this block's row of the slab (det.hip)
      slab[blockIdx.x * 2L * C + c] = a0;
      slab[blockIdx.x * 2L * C + C + c] = a1;
    } else {
      atomicAdd(out + c, a0);
      atomicAdd(out + C + c, a1);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// vector path (C % 8 == 0, C/8 <= 256): thread = (row lane, channel vector)
typedef uint32_t nt_u32x4 __attribute__((ext_vector_type(4)));
// 16-B global load / store, optionally non-temporal (streamed once: keep it out of the caches the
// concurrent side-stream weight-gradient GEMMs reuse)
template <bool NTM>
__device__ __forceinline__ uint4 ld16(const void* p, long k) {
  if constexpr (NTM) {
    const nt_u32x4 v = __builtin_nontemporal_load((const nt_u32x4*)p + k);
    return make_uint4(v[0], v[1], v[2], v[3]);
  } else {
    return ((const uint4*)p)[k];
  }
}
template <bool NTM>
__device__ __forceinline__ void st16(void* p, long k, const uint4& v) {
  if constexpr (NTM) {
    nt_u32x4 w;
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    __builtin_nontemporal_store(w, (nt_u32x4*)p + k);
  } else {
    ((uint4*)p)[k] = v;
  }
}

// ---------------------------------------------------------------------------------------------
template <int KIND, int U, bool NTM = false>
__global__ void __launch_bounds__(NT) reduce_vec_kernel(const bf16_t* __restrict__ a,
                                                        const bf16_t* __restrict__ y,
                                                        const bf16_t* __restrict__ x,
                                                        const float* __restrict__ coef,
                                                        float* __restrict__ out, long M, int C,
                                                        long rows_per_block, int relu, long lda,
                                                        float* __restrict__ slab) {
  // lda: row stride (elements) of `a` (C, or wider for a channel slice of a concat gradient)
  __shared__ float red[2][NT][9];  // +1 pad against bank conflicts
  const int cvecs = C >> 3;
  const int rpp = NT / cvecs;  // rows per pass
  const int t = threadIdx.x;
  const int cv = t % cvecs, rl = t / cvecs;
  const long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float s0[8], s1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
  if (rl < rpp) {
    float mean[8], inv[8], sc[8], sh[8];
    if (KIND == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mean[j] = coef[2 * C + cv * 8 + j];
        inv[j] = coef[3 * C + cv * 8 + j];
        sc[j] = coef[cv * 8 + j];
        sh[j] = coef[C + cv * 8 + j];
      }
    }
    // U rows in flight per thread: all loads of a group are issued before any use
    long r = r0 + rl;
    for (; r < r1; r += U * rpp) {
      uint4 la[U], lx[U], ly[U];
      uint32_t lm[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long rr = r + u * rpp;
        const long row = rr < r1 ? rr : r;
        const long off = row * C + cv * 8;
        la[u] = ld16<NTM>(a + row * lda + cv * 8, 0);
        if (KIND == 1) lx[u] = ld16<NTM>(x + off, 0);
        if (KIND == 1 && relu == 1) ly[u] = ld16<NTM>(y + off, 0);
        if (KIND == 1 && relu == 3) lm[u] = ((const uint8_t*)y)[off >> 3];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
      if (r + u * rpp >= r1) break;
      float va[8];
      unpack(la[u], va);
      if (KIND == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s0[j] += va[j];
          s1[j] += va[j] * va[j];
        }
      } else {
        float vx[8];
        unpack(lx[u], vx);
        if (relu == 1) {
          float vy[8];
          unpack(ly[u], vy);
#pragma unroll
          for (int j = 0; j < 8; ++j) va[j] = vy[j] > 0.f ? va[j] : 0.f;
        } else if (relu == 2) {  // y = relu(x·scale + shift): the mask without reading y
#pragma unroll
          for (int j = 0; j < 8; ++j) va[j] = vx[j] * sc[j] + sh[j] > 0.f ? va[j] : 0.f;
        } else if (relu == 3) {  // bit mask written by the forward apply (1/16 of y's bytes)
#pragma unroll
          for (int j = 0; j < 8; ++j) va[j] = (lm[u] >> j) & 1u ? va[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (vx[j] - mean[j]) * inv[j];
          s0[j] += va[j];
          s1[j] += va[j] * xh;
        }
      }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][t][j] = s0[j];
    red[1][t][j] = s1[j];
  }
  __syncthreads();
  // threads t < 2*C: one output channel each (contiguous atomics)
  for (int o = t; o < 2 * C; o += NT) {
    const int which = o / C, c = o - which * C;
    const int v = c >> 3, j = c & 7;
    float s = 0.f;
    for (int r = 0; r < rpp; ++r) s += red[which][r * cvecs + v][j];
    if (slab)
      slab[blockIdx.x * 2L * C + which * C + c] = s;
    else
      atomicAdd(out + which * C + c, s);
  }
}

// Backward sums of two BNs fed the same gradient g = dy (no ReLU mask left: the residual BN of a
// downsampling bottleneck and its shortcut BN, whose output the residual BN adds): one pass reads
// dy once for both — out = (Σg, Σg·x̂) of x (coef), out2 = (Σg, Σg·x2) raw (bn_bwd_apply
// red_raw).  Same thread layout as reduce_vec_kernel (C % 8 == 0, C / 8 <= NT).
template <int U, bool NTM = false>
__global__ void __launch_bounds__(NT) reduce2_vec_kernel(const bf16_t* __restrict__ a,
                                                         const bf16_t* __restrict__ x,
                                                         const bf16_t* __restrict__ x2,
                                                         const float* __restrict__ coef,
                                                         float* __restrict__ out,
                                                         float* __restrict__ out2, long M, int C,
                                                         long rows_per_block,
                                                         float* __restrict__ slab) {
  __shared__ float red[3][NT][9];
  const int cvecs = C >> 3;
  const int rpp = NT / cvecs;
  const int t = threadIdx.x;
  const int cv = t % cvecs, rl = t / cvecs;
  const long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float s0[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = s2[j] = 0.f;
  if (rl < rpp) {
    float mean[8], inv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mean[j] = coef[2 * C + cv * 8 + j];
      inv[j] = coef[3 * C + cv * 8 + j];
    }
    for (long r = r0 + rl; r < r1; r += U * rpp) {
      uint4 la[U], lx[U], lx2[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long rr = r + u * rpp;
        const long off = (rr < r1 ? rr : r) * C + cv * 8;
        la[u] = ld16<NTM>(a + off, 0);
        lx[u] = ld16<NTM>(x + off, 0);
        lx2[u] = ld16<NTM>(x2 + off, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r + u * rpp >= r1) break;
        float va[8], vx[8], vx2[8];
        unpack(la[u], va);
        unpack(lx[u], vx);
        unpack(lx2[u], vx2);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s0[j] += va[j];
          s1[j] += va[j] * ((vx[j] - mean[j]) * inv[j]);
          s2[j] = fmaf(va[j], vx2[j], s2[j]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][t][j] = s0[j];
    red[1][t][j] = s1[j];
    red[2][t][j] = s2[j];
  }
  __syncthreads();
  for (int o = t; o < 3 * C; o += NT) {
    const int which = o / C, c = o - which * C;
    const int v = c >> 3, j = c & 7;
    float sum = 0.f;
    for (int r = 0; r < rpp; ++r) sum += red[which][r * cvecs + v][j];
    if (slab) {  // row layout [Σg | Σg·x̂ | Σg | Σg·x2]: out = cols [0, 2C), out2 = [2C, 4C)
      float* row = slab + blockIdx.x * 4L * C;
      if (which == 0) {
        row[c] = sum;
        row[2 * C + c] = sum;
      } else if (which == 1) {
        row[C + c] = sum;
      } else {
        row[3 * C + c] = sum;
      }
    } else if (which == 0) {
      atomicAdd(out + c, sum);
      atomicAdd(out2 + c, sum);
    } else if (which == 1) {
      atomicAdd(out + C + c, sum);
    } else {
      atomicAdd(out2 + C + c, sum);
    }
  }
}

template <int KIND>
void reduce_launch(const bf16_t* a, const bf16_t* y, const bf16_t* x, const float* coef, float* out,
                   long M, int C, int relu, hipStream_t st, long lda = 0) {
  if (lda <= 0) lda = C;
  if (M <= 0) return;
  if (C % 8 == 0 && C / 8 <= NT) {
    // ≈ one or two workgroups per CU, ≥ 16 rows per thread: few atomics per output address
    // (every workgroup adds one row of 2C partial sums)
    const int cvecs = C / 8, rpp = NT / cvecs;
    static const int cap = env_int("TDL_BN_RED_BLOCKS", 1024);
    static const int u = env_int("TDL_BN_RED_U", 4);
    static const int minr = env_int("TDL_BN_RED_MINR", 8);
    static const bool ntm = env_int("TDL_BN_NT", 1) != 0;  // non-temporal streaming
    // optional cap on the atomics per launch (every workgroup adds 2C partial sums): measured
    // (dev/tools/bn_micro.py) 1 Mi: b256 reduce total 2.92 -> 2.85 ms but b1024 8.43 -> 8.86 ms —
    // fewer workgroups cost more bandwidth than the atomics save; off by default
    static const long atom = env_int("TDL_BN_RED_ATOM", 1 << 30);
    const long cap_atom = std::max<long>(128, atom / (2L * C));
    long blocks = std::min<long>(std::min<long>(cap, cap_atom), std::max<long>(1, M / (rpp * minr)));
    long rpb = (M + blocks - 1) / blocks;
    blocks = (M + rpb - 1) / rpb;
    float* slab = deterministic() ? det_slab((size_t)blocks * 2 * C, st) : nullptr;
    if (u == 8)
      if (ntm)
        hipLaunchKernelGGL((reduce_vec_kernel<KIND, 8, true>), dim3(blocks), dim3(NT), 0, st, a, y, x,
                           coef, out, M, C, rpb, relu, lda, slab);
      else
        hipLaunchKernelGGL((reduce_vec_kernel<KIND, 8>), dim3(blocks), dim3(NT), 0, st, a, y, x, coef,
                           out, M, C, rpb, relu, lda, slab);
    else if (u == 2)
      if (ntm)
        hipLaunchKernelGGL((reduce_vec_kernel<KIND, 2, true>), dim3(blocks), dim3(NT), 0, st, a, y, x,
                           coef, out, M, C, rpb, relu, lda, slab);
      else
        hipLaunchKernelGGL((reduce_vec_kernel<KIND, 2>), dim3(blocks), dim3(NT), 0, st, a, y, x, coef,
                           out, M, C, rpb, relu, lda, slab);
    else
      if (ntm)
        hipLaunchKernelGGL((reduce_vec_kernel<KIND, 4, true>), dim3(blocks), dim3(NT), 0, st, a, y, x,
                           coef, out, M, C, rpb, relu, lda, slab);
      else
        hipLaunchKernelGGL((reduce_vec_kernel<KIND, 4>), dim3(blocks), dim3(NT), 0, st, a, y, x, coef,
                           out, M, C, rpb, relu, lda, slab);
    if (slab) slab_sum_launch(slab, out, (int)blocks, 2L * C, 2L * C, st);
  } else {
    long blocks = std::min<long>(512, std::max<long>(1, M / 64));
    long rpb = (M + blocks - 1) / blocks;
    blocks = (M + rpb - 1) / rpb;
    float* slab = deterministic() ? det_slab((size_t)blocks * 2 * C, st) : nullptr;
    hipLaunchKernelGGL(reduce_scalar_kernel<KIND>, dim3(blocks, (C + 63) / 64), dim3(NT), 0, st, a, y,
                       x, coef, out, M, C, rpb, relu, slab);
    if (slab) slab_sum_launch(slab, out, (int)blocks, 2L * C, 2L * C, st);
  }
}

__global__ void finalize_kernel(const float* __restrict__ stats, float* __restrict__ coef,
                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                float* __restrict__ rmean, float* __restrict__ rvar, int C,
                                int c_run, float count, float decay, float eps, int training) {
  // channels [c_run, C) are physical padding (zero γ/β, zero input): no moving statistics
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mean, var;
  if (training) {
    mean = stats[c] / count;
    var = fmaxf(stats[C + c] / count - mean * mean, 0.f);
    const float unb = count > 1.f ? var * count / (count - 1.f) : var;
    if (c < c_run) {
      rmean[c] = decay * rmean[c] + (1.f - decay) * mean;
      rvar[c] = decay * rvar[c] + (1.f - decay) * unb;
    }
  } else {
    mean = c < c_run ? rmean[c] : 0.f;
    var = c < c_run ? rvar[c] : 1.f;
  }
  const float inv = rsqrtf(var + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float sc = g * inv;
  coef[c] = sc;
  coef[C + c] = beta[c] - mean * sc;
  coef[2 * C + c] = mean;
  coef[3 * C + c] = inv;
}

// y = act(x·scale + shift [+ res]).  When the grid stride is a multiple of the channel-vector
// count (always for power-of-two C ≤ 2048) each thread's channel vector is loop-invariant, so its
// 16 coefficients are loaded once into registers.
// Optional fp8 side output (delayed scaling, fp8 forward convs): y8 = e4m3(sat(y·448/amax_prev))
// in the same pass, scale_out = amax_prev/448 for the consumer GEMM, and this call's |y|max into
// amax_out (the next call's scale) — amax slots as in common.h.  y8 is skipped while amax_prev is
// still 0 (first call).
__device__ __forceinline__ uint32_t e4m3x4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

template <int U, bool NTM = false>
__global__ void __launch_bounds__(NT) apply_vec_kernel(const bf16_t* __restrict__ x,
                                                       const float* __restrict__ coef,
                                                       const bf16_t* __restrict__ res,
                                                       bf16_t* __restrict__ y, long nvec, int C,
                                                       int relu, uint8_t* __restrict__ y8,
                                                       const float* __restrict__ amax_prev,
                                                       float* __restrict__ scale_out,
                                                       float* __restrict__ amax_out,
                                                       float* __restrict__ amax_zero,
                                                       uint8_t* __restrict__ mask, int ldy_v,
                                                       float margin) {
  // ldy_v: y's row stride in 8-element vectors (C/8 contiguous; wider when y is a channel slice
  // of a concat buffer — the concat-free ASPP / decoder)
  float inv8 = 0.f, vmax = 0.f;
  bool emit8 = false;
  if (amax_out) {
    // a zero (or never-set) previous |y|max falls back to unit scale: the e4m3 copy is always
    // written when requested, so a consumer never reads uninitialised bytes
    const float ap0 = amax_read(amax_prev) * margin;  // (fp8_policy: headroom over the history)
    const float ap = ap0 > 0.f ? ap0 : 448.f;
    emit8 = y8 != nullptr;
    inv8 = 448.f / ap;
    if (blockIdx.x == 0 && threadIdx.x == 0 && scale_out) *scale_out = ap / 448.f;
    amax_clear(amax_zero);  // the slot the next call accumulates into
  }
  const int cvecs = C >> 3;
  const long stride = (long)gridDim.x * NT;
  const bool hoist = (stride % cvecs) == 0;
  long i = blockIdx.x * (long)NT + threadIdx.x;
  float sc[8], sh[8];
  auto load_coef = [&](int cv) {
    const float4 s0 = *(const float4*)(coef + cv * 8), s1 = *(const float4*)(coef + cv * 8 + 4);
    const float4 h0 = *(const float4*)(coef + C + cv * 8), h1 = *(const float4*)(coef + C + cv * 8 + 4);
    sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
    sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w;
    sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
  };
  if (hoist) load_coef((int)(i % cvecs));
  for (; i < nvec; i += U * stride) {
    uint4 lx[U], lr[U];  // U vectors per thread in flight: all loads issued before any use
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long k = i + u * stride < nvec ? i + u * stride : i;
      lx[u] = ld16<NTM>(x, k);
      if (res) lr[u] = ld16<NTM>(res, k);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
    const long k = i + u * stride;
    if (k >= nvec) break;
    if (!hoist) load_coef((int)(k % cvecs));
    float v[8];
    unpack(lx[u], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] * sc[j] + sh[j];
    if (res) {
      float r[8];
      unpack(lr[u], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    const uint4 packed = pack8(v);
    // (y == nullptr: e4m3 copy only — an fp8-only BN output, ops/bn.py)
    if (y) st16<NTM>(y, ldy_v == cvecs ? k : (k / cvecs) * ldy_v + k % cvecs, packed);
    if (mask) {  // ReLU mask of the stored bf16 values, one bit per element (backward relu mode 3)
      float q[8];
      unpack8(packed, q);
      uint32_t b = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) b |= (q[j] > 0.f ? 1u : 0u) << j;
      mask[k] = (uint8_t)b;
    }
    if (amax_out) {
      float q[8];
      unpack8(packed, q);  // quantise the stored bf16 values (what the bf16 path would read)
#pragma unroll
      for (int j = 0; j < 8; ++j) vmax = fmaxf(vmax, fabsf(q[j]));
      if (emit8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = fminf(fmaxf(q[j] * inv8, -448.f), 448.f);
        uint2 o;
        o.x = e4m3x4(q[0], q[1], q[2], q[3]);
        o.y = e4m3x4(q[4], q[5], q[6], q[7]);
        ((uint2*)y8)[k] = o;
      }
    }
    }
  }
  if (amax_out) amax_publish(amax_out, vmax);
}

__global__ void apply_scalar_kernel(const bf16_t* __restrict__ x, const float* __restrict__ coef,
                                    const bf16_t* __restrict__ res, bf16_t* __restrict__ y, long n,
                                    int C, int relu) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    float v = bf2f(x[i]) * coef[c] + coef[C + c];
    if (res) v += bf2f(res[i]);
    if (relu) v = fmaxf(v, 0.f);
    y[i] = f2bf(v);
  }
}

// dx = γ·invstd·(g − Σg/M − x̂·Σg·x̂/M) folded into dx = A·g + B·x + Cc per channel:
//   A = γ·invstd,  B = −A·invstd·Σg·x̂/M,  Cc = −A·Σg/M − B·mean.
// Coefficients are hoisted into registers (loop-invariant channel vector, see apply_vec_kernel).
// Block 0 also writes dγ = Σg·x̂ and dβ = Σg straight into the flat gradient buffer.
__device__ __forceinline__ void load8f(const float* p, float* f) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

__device__ __forceinline__ uint32_t e5m2x4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, v, true);
  return (uint32_t)v;
}

template <bool HOIST, int U, bool NTM = false>
__global__ void __launch_bounds__(NT) bwd_apply_vec_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const bf16_t* __restrict__ x,
    const float* __restrict__ coef, const float* __restrict__ red, const float* __restrict__ gamma,
    bf16_t* __restrict__ dx, bf16_t* __restrict__ dres, float* __restrict__ dgamma,
    float* __restrict__ dbeta, long nvec, int C, float inv_count, int relu,
    uint8_t* __restrict__ dx8, const float* __restrict__ amax_prev, float* __restrict__ scale_out,
    float* __restrict__ amax_out, float* __restrict__ amax_zero, int red_raw, int ldd_v,
    const bf16_t* __restrict__ dadd, float margin) {
  // dadd (optional, shaped like dx): another consumer's gradient of x added to dx in this pass
  // (a DeepLab unit input feeds its pre-activation BN and, as the identity shortcut, the
  // residual of conv3's epilogue) instead of autograd summing the two
  // ldd_v: dy's row stride in 8-element vectors (a channel slice of a concat gradient when > C/8)
  // red_raw: red = (Σg, Σg·x) accumulated by the producing dgrad's epilogue (conv_common.h);
  // Σg·x̂ = invstd·(Σg·x − mean·Σg) here
  // optional e5m2 side output of dx (fp8 dgrad of the producing conv; delayed scaling with
  // `margin` (fp8_policy, default 16×) headroom over the previous |dx|max: gradients can grow step
  // to step, e5m2 has 30 binades to spare, a clipped gradient biases the update)
  float inv8 = 0.f, vmax = 0.f;
  bool emit8 = false;
  if (amax_out) {
    // a zero previous |dx|max (e.g. a step whose loss gradient was exactly zero) falls back to
    // unit scale: dx8 is always written when requested (values clamped to ±57344), never left
    // as uninitialised bytes behind a zero scale
    const float ap0 = amax_read(amax_prev) * margin;
    const float ap = ap0 > 0.f ? ap0 : 57344.f;
    emit8 = dx8 != nullptr;
    inv8 = 57344.f / ap;
    if (blockIdx.x == 0 && threadIdx.x == 0 && scale_out) *scale_out = ap / 57344.f;
    amax_clear(amax_zero);
  }
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += NT) {
      if (dgamma)
        dgamma[c] = red_raw ? coef[3 * C + c] * (red[C + c] - coef[2 * C + c] * red[c]) : red[C + c];
      if (dbeta) dbeta[c] = red[c];
    }
  }
  const int cvecs = C >> 3;
  const long stride = (long)gridDim.x * NT;
  long i = blockIdx.x * (long)NT + threadIdx.x;
  float A[8], Bc[8], Cc[8], Sc[8], Sh[8];
  auto load_coef = [&](int cv) {
    float mean[8], inv[8], s0[8], s1[8], gm[8];
    load8f(coef + cv * 8, Sc);
    load8f(coef + C + cv * 8, Sh);
    load8f(coef + 2 * C + cv * 8, mean);
    load8f(coef + 3 * C + cv * 8, inv);
    load8f(red + cv * 8, s0);
    load8f(red + C + cv * 8, s1);
    if (red_raw) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s1[j] = inv[j] * (s1[j] - mean[j] * s0[j]);
    }
    if (gamma) {
      load8f(gamma + cv * 8, gm);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) gm[j] = 1.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = gm[j] * inv[j];
      const float b = -a * inv[j] * s1[j] * inv_count;
      A[j] = a;
      Bc[j] = b;
      Cc[j] = -a * s0[j] * inv_count - b * mean[j];
    }
  };
  if (HOIST) load_coef((int)(i % cvecs));
  for (; i < nvec; i += U * stride) {
    // U vectors per thread in flight: every load of the group is issued before any use
    uint4 lg[U], lx[U], ly[U], la[U];
    uint32_t lm[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long k = i + u * stride < nvec ? i + u * stride : i;
      lg[u] = ld16<NTM>(dy, ldd_v == cvecs ? k : (k / cvecs) * ldd_v + k % cvecs);
      lx[u] = ld16<NTM>(x, k);
      if (dadd) la[u] = ld16<NTM>(dadd, k);
      if (relu == 1) ly[u] = ((const uint4*)y)[k];
      if (relu == 3) lm[u] = ((const uint8_t*)y)[k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long k = i + u * stride;
      if (k >= nvec) break;
      if (!HOIST) load_coef((int)(k % cvecs));
      float g[8], vx[8];
      unpack(lg[u], g);
      unpack(lx[u], vx);
      if (relu == 1) {
        float vy[8];
        unpack(ly[u], vy);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = vy[j] > 0.f ? g[j] : 0.f;
      } else if (relu == 2) {  // mask recomputed from x (no residual): one tensor read saved
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = vx[j] * Sc[j] + Sh[j] > 0.f ? g[j] : 0.f;
      } else if (relu == 3) {  // bit mask from the forward apply (residual BN: y not re-read)
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = (lm[u] >> j) & 1u ? g[j] : 0.f;
      }
      if (dres) ((uint4*)dres)[k] = pack8(g);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = A[j] * g[j] + Bc[j] * vx[j] + Cc[j];
      if (dadd) {
        float va[8];
        unpack(la[u], va);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += va[j];
      }
      const uint4 packed = pack8(o);
      if (dx) st16<NTM>(dx, k, packed);  // (null: the e5m2 copy only, bindings bn_bwd_apply)
      if (amax_out) {
        float q[8];
        unpack8(packed, q);  // quantise the stored bf16 values
#pragma unroll
        for (int j = 0; j < 8; ++j) vmax = fmaxf(vmax, fabsf(q[j]));
        if (emit8) {
#pragma unroll
          for (int j = 0; j < 8; ++j) q[j] = fminf(fmaxf(q[j] * inv8, -57344.f), 57344.f);
          uint2 w;
          w.x = e5m2x4(q[0], q[1], q[2], q[3]);
          w.y = e5m2x4(q[4], q[5], q[6], q[7]);
          ((uint2*)dx8)[k] = w;
        }
      }
    }
  }
  if (amax_out) amax_publish(amax_out, vmax);
}

__global__ void bwd_apply_scalar_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                        const bf16_t* __restrict__ x, const float* __restrict__ coef,
                                        const float* __restrict__ red,
                                        const float* __restrict__ gamma, bf16_t* __restrict__ dx,
                                        bf16_t* __restrict__ dres, float* __restrict__ dgamma,
                                        float* __restrict__ dbeta, long n, int C, float inv_count,
                                        int relu, int red_raw) {
  auto s1_of = [&](int c) {
    return red_raw ? coef[3 * C + c] * (red[C + c] - coef[2 * C + c] * red[c]) : red[C + c];
  };
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      if (dgamma) dgamma[c] = s1_of(c);
      if (dbeta) dbeta[c] = red[c];
    }
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    float g = bf2f(dy[i]);
    if (relu == 1 && bf2f(y[i]) <= 0.f) g = 0.f;
    if (relu == 2 && bf2f(x[i]) * coef[c] + coef[C + c] <= 0.f) g = 0.f;
    if (dres) dres[i] = f2bf(g);
    const float mean = coef[2 * C + c], inv = coef[3 * C + c];
    const float k = (gamma ? gamma[c] : 1.f) * inv;
    const float xh = (bf2f(x[i]) - mean) * inv;
    dx[i] = f2bf(k * (g - red[c] * inv_count - xh * s1_of(c) * inv_count));
  }
}

inline int ew_blocks(long n, int cvecs = 1, int per_thread = 1) {
  // block count whose grid stride (blocks·NT vectors) is a multiple of the channel-vector count:
  // each thread's channel vector is then loop-invariant and the kernels hoist the per-channel
  // coefficients into registers (C = 728 or 1536 in Xception-41 are not powers of two)
  static const long cap = env_int("TDL_BN_EW_BLOCKS", 1024);
  long b = std::max<long>(1, (n + (long)NT * per_thread - 1) / ((long)NT * per_thread));
  b = std::min<long>(b, cap);
  int g = NT, c = std::max(cvecs, 1);
  while (c) {  // gcd(NT, cvecs)
    const int t = g % c;
    g = c;
    c = t;
  }
  const long b0 = std::max(cvecs, 1) / g;
  return (int)(((b + b0 - 1) / b0) * b0);
}

}  // namespace

void bn_stats_launch(const bf16_t* x, float* stats, long M, int C, hipStream_t st) {
  reduce_launch<0>(x, nullptr, nullptr, nullptr, stats, M, C, 0, st);
}

void bn_finalize_launch(const float* stats, float* coef, const float* gamma, const float* beta,
                        float* rmean, float* rvar, int C, int c_run, float count, float decay,
                        float eps, bool training, hipStream_t st) {
  hipLaunchKernelGGL(finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, stats, coef, gamma,
                     beta, rmean, rvar, C, c_run, count, decay, eps, training ? 1 : 0);
}

void bn_apply_launch(const bf16_t* x, const float* coef, const bf16_t* res, bf16_t* y, long M,
                     int C, bool relu, hipStream_t st, uint8_t* y8, const float* amax_prev,
                     float* scale_out, float* amax_out, float* amax_zero, uint8_t* mask,
                     long ldy) {
  const long n = M * C;
  if (ldy <= 0) ldy = C;
  if (C % 8 == 0) {
    static const int u = env_int("TDL_BN_APPLY_U", 1);
    static const bool ntm = env_int("TDL_BN_NT", 1) != 0;  // non-temporal streaming
    auto k = ntm ? apply_vec_kernel<1, true>
                 : (u == 2 ? apply_vec_kernel<2> : u == 4 ? apply_vec_kernel<4> : apply_vec_kernel<1>);
    hipLaunchKernelGGL(k, dim3(ew_blocks(n / 8, C / 8, u)), dim3(NT), 0, st, x, coef, res, y, n / 8, C,
                       relu ? 1 : 0, y8, amax_prev, scale_out, amax_out, amax_zero, mask,
                       (int)(ldy / 8), fp8_policy().margin_e4m3);
  } else {
    hipLaunchKernelGGL(apply_scalar_kernel, dim3(ew_blocks(n)), dim3(NT), 0, st, x, coef, res, y, n,
                       C, relu ? 1 : 0);
  }
}

void bn_bwd_reduce_launch(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* coef,
                          float* red, long M, int C, int relu, hipStream_t st, long ldd) {
  reduce_launch<1>(dy, y, x, coef, red, M, C, relu, st, ldd);
}

bool bn_bwd_reduce2_launch(const bf16_t* dy, const bf16_t* x, const bf16_t* x2, const float* coef,
                           float* red, float* red2, long M, int C, hipStream_t st) {
  if (M <= 0 || C % 8 || C / 8 > NT) return false;
  const int cvecs = C / 8, rpp = NT / cvecs;
  static const int cap = env_int("TDL_BN_RED_BLOCKS", 1024);
  long blocks = std::min<long>(cap, std::max<long>(1, M / (rpp * 8)));
  const long rpb = (M + blocks - 1) / blocks;
  blocks = (M + rpb - 1) / rpb;
  static const bool ntm = env_int("TDL_BN_NT", 1) != 0;  // non-temporal streaming
  float* slab = deterministic() ? det_slab((size_t)blocks * 4 * C, st) : nullptr;
  if (ntm)
    hipLaunchKernelGGL((reduce2_vec_kernel<4, true>), dim3(blocks), dim3(NT), 0, st, dy, x, x2, coef, red,
                       red2, M, C, rpb, slab);
  else
    hipLaunchKernelGGL((reduce2_vec_kernel<4>), dim3(blocks), dim3(NT), 0, st, dy, x, x2, coef, red, red2,
                       M, C, rpb, slab);
  if (slab) {
    slab_sum_launch(slab, red, (int)blocks, 2L * C, 4L * C, st);
    slab_sum_launch(slab + 2 * C, red2, (int)blocks, 2L * C, 4L * C, st);
  }
  return true;
}

void bn_bwd_apply_launch(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* coef,
                         const float* red, const float* gamma, bf16_t* dx, bf16_t* dres,
                         float* dgamma, float* dbeta, long M, int C, float count, int relu,
                         hipStream_t st, uint8_t* dx8, const float* amax_prev, float* scale_out,
                         float* amax_out, float* amax_zero, bool red_raw, long ldd,
                         const bf16_t* dadd) {
  const long n = M * C;
  if (ldd <= 0) ldd = C;
  if (C % 8 == 0) {
    static const int u = env_int("TDL_BN_BWD_U", 2);
    const int blocks = ew_blocks(n / 8, C / 8, u);
    const bool hoist = ((long)blocks * NT) % (C / 8) == 0;
    static const bool ntm = env_int("TDL_BN_NT", 1) != 0;  // non-temporal streaming
    auto k = hoist ? (ntm ? bwd_apply_vec_kernel<true, 2, true>
                          : u == 2 ? bwd_apply_vec_kernel<true, 2>
                                   : u == 4 ? bwd_apply_vec_kernel<true, 4> : bwd_apply_vec_kernel<true, 1>)
                   : bwd_apply_vec_kernel<false, 1>;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(NT), 0, st, dy, y, x, coef, red, gamma, dx, dres, dgamma,
                       dbeta, n / 8, C, 1.f / count, relu, dx8, amax_prev, scale_out, amax_out,
                       amax_zero, red_raw ? 1 : 0, (int)(ldd / 8), dadd, fp8_policy().margin_e5m2);
  } else {
    hipLaunchKernelGGL(bwd_apply_scalar_kernel, dim3(ew_blocks(n)), dim3(NT), 0, st, dy, y, x, coef,
                       red, gamma, dx, dres, dgamma, dbeta, n, C, 1.f / count, relu,
                       red_raw ? 1 : 0);
  }
}

}  // namespace tdl
