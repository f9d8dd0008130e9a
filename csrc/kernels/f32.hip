// fp32 training path — the reference's own precision (/root/reference/model.py has no dtype
// option; its published training speed, Test.ipynb:212-213, is fp32).  Every GPU op of the
// DeepLab preset has an fp32 kernel here or an fp32 instantiation of its type-generic kernel
// (pool.hip, upsample.hip), so `--dtype fp32` trains with fp32 operands end to end:
//
//   * convolution: implicit GEMM on v_mfma_f32_32x32x2_f32 (fp32 operands, fp32 accumulate —
//     no bf16 / tf32-style rounding of the inputs), 128×128×16 workgroup tiles, 4 waves of
//     64×64 (2×2 MFMA blocks), register-staged double-buffered LDS, k-major LDS images so every
//     fragment read is one conflict-free ds_read_b32 per lane; the same kernel computes the
//     forward (bias / residual / ReLU / BN-statistics epilogue), the input gradient (strided and
//     dilated taps masked by divisibility; accumulate for residual-gradient joins) and the weight
//     gradient (split over pixels, fp32 atomics into dW);
//   * BatchNorm statistics / apply (+residual +ReLU, strided destination) / backward reduce /
//     backward apply (+residual gradient, +linked residual add, in-kernel dγ/dβ), channel column
//     sums (bias gradients), ReLU backward and add(+ReLU);
//   * depthwise convolution forward / input gradient / weight gradient (+bias gradient).
//
// The fp32 MFMA issues 1/16 of the bf16 FLOP rate per instruction: 32 MFMAs per 16-deep K-step
// keep a wave busy for ~2k cycles, so the register-staged loads and the per-K-step tap arithmetic
// hide behind them (no LDS-DMA pipeline needed at this arithmetic intensity).
#include "common.h"
#include "kernels.h"

namespace tdl {
namespace {

constexpr int CT = 256;             // conv workgroup: 4 waves in a 2×2 grid, 64×64 outputs each
constexpr int BM = 128, BN = 128, BK = 16;
constexpr int LDP = 128 + 4;        // LDS row = one k: rows k and k+8 land 32 banks apart

enum { C_FWD = 0, C_DGRAD = 1, C_WGRAD = 2 };

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// 4 consecutive floats p[0..3] of which the first n are valid (n ≤ 0: none).  vec: the row
// length is a multiple of 4 (aligned float4 loads); otherwise element loads (classifier heads
// with a class count that is not a multiple of 4)
__device__ __forceinline__ float4 ld4(const float* p, int n, bool vec) {
  if (n <= 0) return f4zero();
  if (vec) return *(const float4*)p;
  return make_float4(p[0], n > 1 ? p[1] : 0.f, n > 2 ? p[2] : 0.f, n > 3 ? p[3] : 0.f);
}

// GEMM views (m = output row, n = output column, reduction in 16-deep K-steps q):
//   FWD   m = output pixel, n = output channel, q = (tap r,s) × 16-channel chunk of C
//   DGRAD m = input pixel,  n = input channel,  q = (tap r,s) × 16-channel chunk of K
//   WGRAD m = output channel, n = (r,s,c) of dW [K][R][S][C], q = 16-pixel chunk of N·Ho·Wo
// Workgroup tile TBM × TBN (64 or 128 each), 4 waves in a 2×2 grid, each wave (TBM/2) × (TBN/2) =
// FM × FN blocks of 32×32.  Operand staging per K-step (an operand with R rows is R×16 floats =
// R/64 float4 loads per thread; 256 % R == 0, so a thread keeps one row / column group):
//   "row" operands (FWD A/B, DGRAD A): thread owns row t % R and k offsets 4·((t + 256j) / R)
//   "col" operands (DGRAD B, WGRAD A/B): thread owns columns 4·(t % (R/4)) … +3 and k rows
//   (t + 256j) / (R/4)
// Small problems take smaller tiles (conv_f32_launch): the reference preset's 13×13 maps at batch
// 64 are 170 workgroups of 128×128 — two thirds of the chip, one wave of work — but 676 of 64×64.
template <int R>
struct RowPat {  // "row" staging: row, and the k offset of load j
  static constexpr int L = R / 64;
  __device__ __forceinline__ static int row(int t) { return t % R; }
  __device__ __forceinline__ static int k4(int t, int j) { return ((t + 256 * j) / R) * 4; }
};
template <int R>
struct ColPat {  // "col" staging: first column, and the k row of load j
  static constexpr int L = R / 64;
  __device__ __forceinline__ static int col(int t) { return (t % (R / 4)) * 4; }
  __device__ __forceinline__ static int kr(int t, int j) { return (t + 256 * j) / (R / 4); }
};

// (launch bounds: ≥ 2 waves per SIMD — without it hipcc parks the accumulators in AGPRs next to
// ~140–200 VGPRs, 1–2 waves per SIMD; with it 106–139 VGPRs and no AGPRs: 3–4 waves per SIMD,
// no scratch)
template <int MODE, int TBM = BM, int TBN = BN>
__global__ void __launch_bounds__(CT, 2) conv_f32_kernel(ConvF32Args a, int M, int Ng, int nq,
                                                      int cch, int qps, int tiles_n) {
  static_assert((TBM == 64 || TBM == 128) && (TBN == 64 || TBN == 128), "tiles of 64 / 128");
  constexpr int FM = TBM / 64, FN = TBN / 64;  // 32×32 blocks per wave
  constexpr bool A_ROW = MODE != C_WGRAD, B_ROW = MODE == C_FWD;
  constexpr int LA = TBM / 64, LB = TBN / 64;  // float4 loads per thread per operand
  __shared__ __attribute__((aligned(16))) float As[2][BK][LDP];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][LDP];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int l31 = lane & 31, hk = lane >> 5;
  const int tile = blockIdx.x;
  const int m0 = (tile / tiles_n) * TBM, n0 = (tile % tiles_n) * TBN;
  const int q0 = blockIdx.y * qps, q1 = min(nq, q0 + qps);
  const int H = a.H, W = a.W, C = a.C, K = a.K, S = a.S, Ho = a.Ho, Wo = a.Wo;

  // ---- per-thread loader state (fixed over the K loop)
  const int ra_ = A_ROW ? RowPat<TBM>::row(t) : ColPat<TBM>::col(t);  // A row / first column
  const int rb_ = B_ROW ? RowPat<TBN>::row(t) : ColPat<TBN>::col(t);  // B row / first column
  int pa_n = 0, pa_h = 0, pa_w = 0;  // A row pixel (FWD: output, DGRAD: input)
  bool a_ok = false, b_ok = false;
  int wr_r = 0, wr_s = 0, wr_c = 0;  // WGRAD: this thread's dW columns (r, s, c)
  if (MODE == C_FWD || MODE == C_DGRAD) {
    const int m = m0 + ra_;
    a_ok = m < M;
    const int PW = MODE == C_FWD ? Wo : W, PH = MODE == C_FWD ? Ho : H;
    const int mm = a_ok ? m : 0;
    pa_w = mm % PW;
    const int tq = mm / PW;
    pa_h = tq % PH;
    pa_n = tq / PH;
    b_ok = n0 + rb_ < (MODE == C_FWD ? K : C);
  } else {
    const int n = n0 + rb_;
    b_ok = n < Ng;
    const int nn = b_ok ? n : 0;
    const int rs = nn / C;
    wr_c = nn - rs * C;
    wr_r = rs / S;
    wr_s = rs - wr_r * S;
  }

  float4 ra[LA], rb[LB];
  auto load = [&](int q) {
    if (MODE == C_FWD) {
      // q is uniform: the tap / chunk decomposition stays in scalar registers
      const int qu = __builtin_amdgcn_readfirstlane(q);
      const int tap = qu / cch, cq = qu - tap * cch;
      const int r = tap / S, s = tap - r * S;
      const int hi = pa_h * a.sh - a.ph + r * a.dh, wi = pa_w * a.sw - a.pw + s * a.dw;
      const bool pv = a_ok && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
      const float* src = a.x + (((long)pa_n * H + hi) * W + wi) * C + cq * BK;
#pragma unroll
      for (int j = 0; j < LA; ++j) {
        const int c = cq * BK + RowPat<TBM>::k4(t, j);
        ra[j] = pv && c < C ? *(const float4*)(src + RowPat<TBM>::k4(t, j)) : f4zero();
      }
      const float* wsrc = a.w + (((long)(n0 + rb_) * a.R + r) * S + s) * C + cq * BK;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const int c = cq * BK + RowPat<TBN>::k4(t, j);
        rb[j] = b_ok && c < C ? *(const float4*)(wsrc + RowPat<TBN>::k4(t, j)) : f4zero();
      }
    } else if (MODE == C_DGRAD) {
      const int qu = __builtin_amdgcn_readfirstlane(q);
      const int tap = qu / cch, cq = qu - tap * cch;
      const int r = tap / S, s = tap - r * S;
      const int hn = pa_h + a.ph - r * a.dh, wn_ = pa_w + a.pw - s * a.dw;
      // (stride 1, the common case, needs no per-lane division; the branch is uniform)
      const int ho = hn < 0 ? -1 : a.sh == 1 ? hn : hn / a.sh;
      const int wo = wn_ < 0 ? -1 : a.sw == 1 ? wn_ : wn_ / a.sw;
      const bool pv = a_ok && ho >= 0 && wo >= 0 && ho * a.sh == hn && wo * a.sw == wn_ &&
                      ho < Ho && wo < Wo;
      const float* src = a.dy + (((long)pa_n * Ho + ho) * Wo + wo) * K + cq * BK;
      const bool kv = (K & 3) == 0;
#pragma unroll
      for (int j = 0; j < LA; ++j) {
        const int kk = RowPat<TBM>::k4(t, j);
        ra[j] = pv ? ld4(src + kk, K - cq * BK - kk, kv) : f4zero();
      }
      const long kstride = (long)a.R * S * C;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const int kb = cq * BK + ColPat<TBN>::kr(t, j);
        rb[j] = b_ok && kb < K ? *(const float4*)(a.w + ((long)kb * a.R + r) * S * C + (long)s * C +
                                                  n0 + rb_)
                               : f4zero();
      }
      (void)kstride;
    } else {
      const long P = (long)a.N * Ho * Wo;
      const bool kv = (K & 3) == 0;
#pragma unroll
      for (int j = 0; j < LA; ++j) {
        const long p = (long)q * BK + ColPat<TBM>::kr(t, j);
        ra[j] = p < P ? ld4(a.dy + p * K + m0 + ra_, K - m0 - ra_, kv) : f4zero();
      }
      const int HoWo = Ho * Wo;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const long p = (long)q * BK + ColPat<TBN>::kr(t, j);
        float4 v = f4zero();
        if (b_ok && p < P) {
          const int pn = (int)fdiv((uint32_t)p, a.fd_HoWo), rem = (int)p - pn * HoWo;
          const int ho = (int)fdiv((uint32_t)rem, a.fd_Wo), wo = rem - ho * Wo;
          const int hi = ho * a.sh - a.ph + wr_r * a.dh, wi = wo * a.sw - a.pw + wr_s * a.dw;
          if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W)
            v = *(const float4*)(a.x + (((long)pn * H + hi) * W + wi) * C + wr_c);
        }
        rb[j] = v;
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < LA; ++j) {
      if (A_ROW) {
        const int k4 = RowPat<TBM>::k4(t, j);
        As[buf][k4 + 0][ra_] = ra[j].x; As[buf][k4 + 1][ra_] = ra[j].y;
        As[buf][k4 + 2][ra_] = ra[j].z; As[buf][k4 + 3][ra_] = ra[j].w;
      } else {
        *(float4*)&As[buf][ColPat<TBM>::kr(t, j)][ra_] = ra[j];
      }
    }
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      if (B_ROW) {
        const int k4 = RowPat<TBN>::k4(t, j);
        Bs[buf][k4 + 0][rb_] = rb[j].x; Bs[buf][k4 + 1][rb_] = rb[j].y;
        Bs[buf][k4 + 2][rb_] = rb[j].z; Bs[buf][k4 + 3][rb_] = rb[j].w;
      } else {
        *(float4*)&Bs[buf][ColPat<TBN>::kr(t, j)][rb_] = rb[j];
      }
    }
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  if (q0 < q1) {
    load(q0);
    store(0);
    __syncthreads();
    for (int q = q0; q < q1; ++q) {
      const int buf = (q - q0) & 1;
      const bool more = q + 1 < q1;
      if (more) load(q + 1);  // in flight under this K-step's MFMAs
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        // MFMA k-slot hk of step kk reads LDS row 8·hk + kk (same permutation for A and B)
        const float* ar = &As[buf][8 * hk + kk][wm * (TBM / 2) + l31];
        const float* br = &Bs[buf][8 * hk + kk][wn * (TBN / 2) + l31];
        float bv[FN];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) bv[fn] = br[32 * fn];
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const float av = ar[32 * fm];
#pragma unroll
          for (int fn = 0; fn < FN; ++fn)
            acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[fn], acc[fm][fn], 0, 0, 0);
        }
      }
      if (more) store(buf ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue: lane holds column l31 of each 32×32 block, rows (v&3) + 8(v>>2) + 4·hk
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int col = n0 + wn * (TBN / 2) + fn * 32 + l31;
    float s0 = 0.f, s1 = 0.f;
    float bias = 0.f;
    if (MODE == C_FWD && a.bias && col < K) bias = a.bias[col];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wm * (TBM / 2) + fm * 32 + (v & 3) + 8 * (v >> 2) + 4 * hk;
        float val = acc[fm][fn][v];
        if (MODE == C_FWD) {
          if (row < M && col < K) {
            const long o = (long)row * K + col;
            val += bias;
            if (a.res) val += a.res[o];
            if (a.relu) val = fmaxf(val, 0.f);
            a.out[o] = val;
            s0 += val;
            s1 += val * val;
          }
        } else if (MODE == C_DGRAD) {
          if (row < M && col < C) {
            const long o = (long)row * C + col;
            a.out[o] = a.accumulate ? a.out[o] + val : val;
          }
        } else if (row < K && col < Ng) {
          const long o = (long)row * Ng + col;
          if (a.slab)
            a.slab[(long)blockIdx.y * K * Ng + o] = val;  // this split's partial slab
          else
            a.out[o] = a.accumulate ? a.out[o] + val : val;
        }
      }
    }
    if (MODE == C_FWD && a.stats) {
      s0 += __shfl_xor(s0, 32, 64);
      s1 += __shfl_xor(s1, 32, 64);
      if (hk == 0 && col < K) {
        unsafeAtomicAdd(a.stats + col, s0);
        unsafeAtomicAdd(a.stats + K + col, s1);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// channel reductions over [M][C] (row stride lda): per-column float4 partial sums in registers,
// an LDS reduction over the block's row lanes, one fp32 atomic per column per block.
//   MODE 0: (Σx, Σx²)            BN forward statistics
//   MODE 1: Σx                   bias gradient (column sums)
//   MODE 2: (Σg, Σg·x̂)           BN backward, g = dy·mask (relu 1: y > 0, 2: x·scale+shift > 0)
constexpr int RT = 256;

template <int MODE>
__global__ void __launch_bounds__(RT) chan_reduce_f32(const float* __restrict__ a,
                                                      const float* __restrict__ x,
                                                      const float* __restrict__ y,
                                                      const float* __restrict__ coef,
                                                      float* __restrict__ out, long M, int C,
                                                      long lda, int relu, int cvb) {
  __shared__ float4 red0[RT], red1[RT];
  const int cv = C >> 2;
  const int tx = threadIdx.x % cvb, ty = threadIdx.x / cvb, rpb = RT / cvb;
  const int v4 = blockIdx.y * cvb + tx;
  const bool cvalid = v4 < cv;
  const int c = v4 * 4;
  float4 s0 = f4zero(), s1 = f4zero();
  float4 sc = f4zero(), sh = f4zero(), mean = f4zero(), inv = f4zero();
  if (MODE == 2 && cvalid) {
    sc = *(const float4*)(coef + c);
    sh = *(const float4*)(coef + C + c);
    mean = *(const float4*)(coef + 2 * C + c);
    inv = *(const float4*)(coef + 3 * C + c);
  }
  if (cvalid) {
    for (long m = (long)blockIdx.x * rpb + ty; m < M; m += (long)gridDim.x * rpb) {
      float4 v = *(const float4*)(a + m * lda + c);
      if (MODE == 0) {
        s0.x += v.x; s0.y += v.y; s0.z += v.z; s0.w += v.w;
        s1.x += v.x * v.x; s1.y += v.y * v.y; s1.z += v.z * v.z; s1.w += v.w * v.w;
      } else if (MODE == 1) {
        s0.x += v.x; s0.y += v.y; s0.z += v.z; s0.w += v.w;
      } else {
        const float4 xv = *(const float4*)(x + m * C + c);
        if (relu == 1) {
          const float4 yv = *(const float4*)(y + m * C + c);
          v.x = yv.x > 0.f ? v.x : 0.f; v.y = yv.y > 0.f ? v.y : 0.f;
          v.z = yv.z > 0.f ? v.z : 0.f; v.w = yv.w > 0.f ? v.w : 0.f;
        } else if (relu == 2) {
          v.x = xv.x * sc.x + sh.x > 0.f ? v.x : 0.f; v.y = xv.y * sc.y + sh.y > 0.f ? v.y : 0.f;
          v.z = xv.z * sc.z + sh.z > 0.f ? v.z : 0.f; v.w = xv.w * sc.w + sh.w > 0.f ? v.w : 0.f;
        }
        s0.x += v.x; s0.y += v.y; s0.z += v.z; s0.w += v.w;
        s1.x += v.x * (xv.x - mean.x) * inv.x; s1.y += v.y * (xv.y - mean.y) * inv.y;
        s1.z += v.z * (xv.z - mean.z) * inv.z; s1.w += v.w * (xv.w - mean.w) * inv.w;
      }
    }
  }
  red0[threadIdx.x] = s0;
  red1[threadIdx.x] = s1;
  __syncthreads();
  if (ty == 0 && cvalid) {
    for (int j = 1; j < rpb; ++j) {
      const float4 p = red0[j * cvb + tx], q = red1[j * cvb + tx];
      s0.x += p.x; s0.y += p.y; s0.z += p.z; s0.w += p.w;
      s1.x += q.x; s1.y += q.y; s1.z += q.z; s1.w += q.w;
    }
    unsafeAtomicAdd(out + c + 0, s0.x); unsafeAtomicAdd(out + c + 1, s0.y);
    unsafeAtomicAdd(out + c + 2, s0.z); unsafeAtomicAdd(out + c + 3, s0.w);
    if (MODE != 1) {
      unsafeAtomicAdd(out + C + c + 0, s1.x); unsafeAtomicAdd(out + C + c + 1, s1.y);
      unsafeAtomicAdd(out + C + c + 2, s1.z); unsafeAtomicAdd(out + C + c + 3, s1.w);
    }
  }
}

void chan_reduce_launch(int mode, const float* a, const float* x, const float* y, const float* coef,
                        float* out, long M, int C, long lda, int relu, hipStream_t st) {
  const int cv = C / 4;
  int cvb = 1;
  while (cvb < cv && cvb < 64) cvb <<= 1;
  const int gy = (cv + cvb - 1) / cvb;
  const long rpb = RT / cvb;
  // ≥ 16 rows per thread, ≤ ~1024 blocks in all (one atomic per column per block)
  const long gx = std::max<long>(1, std::min<long>((M + rpb * 16 - 1) / (rpb * 16), 1024 / gy));
  const dim3 grid((unsigned)gx, (unsigned)gy);
  if (mode == 0)
    hipLaunchKernelGGL(chan_reduce_f32<0>, grid, dim3(RT), 0, st, a, x, y, coef, out, M, C, lda, relu,
                       cvb);
  else if (mode == 1)
    hipLaunchKernelGGL(chan_reduce_f32<1>, grid, dim3(RT), 0, st, a, x, y, coef, out, M, C, lda, relu,
                       cvb);
  else
    hipLaunchKernelGGL(chan_reduce_f32<2>, grid, dim3(RT), 0, st, a, x, y, coef, out, M, C, lda, relu,
                       cvb);
}

// column sums for any column count: 64 columns × 4 row lanes per block, one atomic per column
__global__ void __launch_bounds__(256) colsum_scalar_f32(const float* __restrict__ x,
                                                         float* __restrict__ out, long M, int C,
                                                         long ldx) {
  __shared__ float red[256];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + tx;
  float s = 0.f;
  if (c < C)
    for (long m = (long)blockIdx.x * 4 + ty; m < M; m += (long)gridDim.x * 4) s += x[m * ldx + c];
  red[threadIdx.x] = s;
  __syncthreads();
  if (ty == 0 && c < C) unsafeAtomicAdd(out + c, s + red[64 + tx] + red[128 + tx] + red[192 + tx]);
}

inline int eblocks(long n) { return (int)std::min<long>(8192, std::max<long>(1, (n + 255) / 256)); }

// y[m·ldy + c] = act(x·scale + shift [+ res])
__global__ void __launch_bounds__(256) bn_apply_f32(const float* __restrict__ x,
                                                    const float* __restrict__ coef,
                                                    const float* __restrict__ res,
                                                    float* __restrict__ y, long M, int C, long ldy,
                                                    int relu) {
  const int cv = C >> 2;
  const long n = M * cv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long m = i / cv;
    const int c = (int)(i - m * cv) * 4;
    const float4 v = ((const float4*)x)[i];
    const float4 sc = *(const float4*)(coef + c), sh = *(const float4*)(coef + C + c);
    float4 o = make_float4(v.x * sc.x + sh.x, v.y * sc.y + sh.y, v.z * sc.z + sh.z,
                           v.w * sc.w + sh.w);
    if (res) {
      const float4 r = ((const float4*)res)[i];
      o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
    }
    if (relu) {
      o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
    }
    *(float4*)(y + m * ldy + c) = o;
  }
}

// dx = γ·invstd·(g − Σg/M − x̂·Σg·x̂/M) [+ dadd], g = dy·mask; dres = g; block 0 writes dγ, dβ
__global__ void __launch_bounds__(256) bn_bwd_apply_f32(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ x,
    const float* __restrict__ coef, const float* __restrict__ red, const float* __restrict__ gamma,
    float* __restrict__ dx, float* __restrict__ dres, float* __restrict__ dgamma,
    float* __restrict__ dbeta, const float* __restrict__ dadd, long M, int C, long ldd,
    float inv_count, int relu) {
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += 256) {
      if (dgamma) dgamma[c] = red[C + c];
      if (dbeta) dbeta[c] = red[c];
    }
  }
  const int cv = C >> 2;
  const long n = M * cv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long m = i / cv;
    const int c = (int)(i - m * cv) * 4;
    float g[4], xv[4], o[4];
    const float4 gv = *(const float4*)(dy + m * ldd + c);
    const float4 xx = ((const float4*)x)[i];
    g[0] = gv.x; g[1] = gv.y; g[2] = gv.z; g[3] = gv.w;
    xv[0] = xx.x; xv[1] = xx.y; xv[2] = xx.z; xv[3] = xx.w;
    if (relu == 1) {
      const float4 yv = ((const float4*)y)[i];
      const float yy[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = yy[j] > 0.f ? g[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cc = c + j;
      if (relu == 2) g[j] = xv[j] * coef[cc] + coef[C + cc] > 0.f ? g[j] : 0.f;
      const float mean = coef[2 * C + cc], inv = coef[3 * C + cc];
      const float ga = (gamma ? gamma[cc] : 1.f) * inv;
      const float b = -ga * inv * red[C + cc] * inv_count;
      o[j] = ga * g[j] + b * xv[j] + (-ga * red[cc] * inv_count - b * mean);
    }
    if (dres) ((float4*)dres)[i] = make_float4(g[0], g[1], g[2], g[3]);
    if (dadd) {
      const float4 ad = ((const float4*)dadd)[i];
      o[0] += ad.x; o[1] += ad.y; o[2] += ad.z; o[3] += ad.w;
    }
    ((float4*)dx)[i] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// relu_bwd: dx = dy·[y > 0];  add_act: y = act(a [+ b])
__global__ void __launch_bounds__(256) relu_bwd_f32(const float4* __restrict__ dy,
                                                    const float4* __restrict__ y,
                                                    float4* __restrict__ dx, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 g = dy[i], v = y[i];
    dx[i] = make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f,
                        v.w > 0.f ? g.w : 0.f);
  }
}

__global__ void __launch_bounds__(256) add_act_f32(const float4* __restrict__ a,
                                                   const float4* __restrict__ b,
                                                   float4* __restrict__ y, long n4, int relu) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 v = a[i];
    if (b) {
      const float4 w = b[i];
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    if (relu) {
      v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    }
    y[i] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// depthwise k×k (depth multiplier 1), weights [R][S][C]; one thread per 4-channel vector
__global__ void __launch_bounds__(256) dw_fwd_f32(DwF32Args a) {
  const int cv = a.C >> 2;
  const long n = (long)a.N * a.Ho * a.Wo * cv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % cv) * 4;
    long p = i / cv;
    const int wo = (int)(p % a.Wo);
    p /= a.Wo;
    const int ho = (int)(p % a.Ho);
    const int nn = (int)(p / a.Ho);
    float4 acc = a.bias ? *(const float4*)(a.bias + c) : f4zero();
    for (int r = 0; r < a.R; ++r) {
      const int hi = ho * a.sh - a.ph + r * a.dh;
      if ((unsigned)hi >= (unsigned)a.H) continue;
      for (int s = 0; s < a.S; ++s) {
        const int wi = wo * a.sw - a.pw + s * a.dwl;
        if ((unsigned)wi >= (unsigned)a.W) continue;
        const float4 xv = *(const float4*)(a.x + (((long)nn * a.H + hi) * a.W + wi) * a.C + c);
        const float4 wv = *(const float4*)(a.w + ((long)r * a.S + s) * a.C + c);
        acc.x += xv.x * wv.x; acc.y += xv.y * wv.y; acc.z += xv.z * wv.z; acc.w += xv.w * wv.w;
      }
    }
    if (a.relu) {
      acc.x = fmaxf(acc.x, 0.f); acc.y = fmaxf(acc.y, 0.f);
      acc.z = fmaxf(acc.z, 0.f); acc.w = fmaxf(acc.w, 0.f);
    }
    ((float4*)a.out)[i] = acc;
  }
}

// dx[n,h,w,c] = Σ_{r,s} dy[n,(h+ph−r·dh)/sh,(w+pw−s·dw)/sw,c]·w[r,s,c] over divisible, in-range taps
__global__ void __launch_bounds__(256) dw_dgrad_f32(DwF32Args a) {
  const int cv = a.C >> 2;
  const long n = (long)a.N * a.H * a.W * cv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int c = (int)(i % cv) * 4;
    long p = i / cv;
    const int w = (int)(p % a.W);
    p /= a.W;
    const int h = (int)(p % a.H);
    const int nn = (int)(p / a.H);
    float4 acc = f4zero();
    for (int r = 0; r < a.R; ++r) {
      const int hn = h + a.ph - r * a.dh;
      if (hn < 0 || hn % a.sh) continue;
      const int ho = hn / a.sh;
      if (ho >= a.Ho) continue;
      for (int s = 0; s < a.S; ++s) {
        const int wn = w + a.pw - s * a.dwl;
        if (wn < 0 || wn % a.sw) continue;
        const int wo = wn / a.sw;
        if (wo >= a.Wo) continue;
        const float4 g = *(const float4*)(a.dy + (((long)nn * a.Ho + ho) * a.Wo + wo) * a.C + c);
        const float4 wv = *(const float4*)(a.w + ((long)r * a.S + s) * a.C + c);
        acc.x += g.x * wv.x; acc.y += g.y * wv.y; acc.z += g.z * wv.z; acc.w += g.w * wv.w;
      }
    }
    if (a.dadd) {
      const float4 d = ((const float4*)a.dadd)[i];
      acc.x += d.x; acc.y += d.y; acc.z += d.z; acc.w += d.w;
    }
    ((float4*)a.out)[i] = acc;
  }
}

// dW[r,s,c] += Σ_pixels dy·x (taps ≤ 9), db[c] += Σ dy: block = cvb channel vectors × rpb pixel
// lanes, register partials per tap, LDS reduction over the pixel lanes, fp32 atomics
constexpr int DW_MAXT = 9;
__global__ void __launch_bounds__(256) dw_wgrad_f32(DwF32Args a, int cvb) {
  __shared__ float4 red[256];
  const int cv = a.C >> 2;
  const int tx = threadIdx.x % cvb, ty = threadIdx.x / cvb, rpb = 256 / cvb;
  const int v4 = blockIdx.y * cvb + tx;
  const bool cvalid = v4 < cv;
  const int c = v4 * 4;
  const int T = a.R * a.S;
  float4 acc[DW_MAXT + 1];
#pragma unroll
  for (int j = 0; j <= DW_MAXT; ++j) acc[j] = f4zero();
  const long P = (long)a.N * a.Ho * a.Wo;
  if (cvalid) {
    for (long p = (long)blockIdx.x * rpb + ty; p < P; p += (long)gridDim.x * rpb) {
      const int wo = (int)(p % a.Wo);
      const long q = p / a.Wo;
      const int ho = (int)(q % a.Ho);
      const int nn = (int)(q / a.Ho);
      const float4 g = *(const float4*)(a.dy + p * a.C + c);
      acc[DW_MAXT].x += g.x; acc[DW_MAXT].y += g.y; acc[DW_MAXT].z += g.z; acc[DW_MAXT].w += g.w;
#pragma unroll
      for (int j = 0; j < DW_MAXT; ++j) {
        if (j >= T) continue;  // (no break: the loop must unroll or acc[] goes to scratch)
        const int r = j / a.S, s = j - r * a.S;
        const int hi = ho * a.sh - a.ph + r * a.dh, wi = wo * a.sw - a.pw + s * a.dwl;
        if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) continue;
        const float4 xv = *(const float4*)(a.x + (((long)nn * a.H + hi) * a.W + wi) * a.C + c);
        acc[j].x += g.x * xv.x; acc[j].y += g.y * xv.y; acc[j].z += g.z * xv.z; acc[j].w += g.w * xv.w;
      }
    }
  }
#pragma unroll
  for (int j = 0; j <= DW_MAXT; ++j) {
    if (j < T || j == DW_MAXT) {
      __syncthreads();
      red[threadIdx.x] = acc[j];
      __syncthreads();
      if (ty == 0 && cvalid) {
        float4 s = acc[j];
        for (int k = 1; k < rpb; ++k) {
          const float4 o = red[k * cvb + tx];
          s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
        }
        float* dst = j == DW_MAXT ? (a.db ? a.db + c : nullptr) : a.dwt + (long)j * a.C + c;
        if (dst) {
          unsafeAtomicAdd(dst + 0, s.x); unsafeAtomicAdd(dst + 1, s.y);
          unsafeAtomicAdd(dst + 2, s.z); unsafeAtomicAdd(dst + 3, s.w);
        }
      }
    }
  }
}

// row packing of a few-channel image for its k×k stem conv (elementwise.hip row_pack_kernel's
// fp32 form): t[n][h][wo][e] = x[n][h][wo·sw − pl + e / Cr][e % Cr] for e < S·Cr, zero elsewhere
__global__ void __launch_bounds__(256) row_pack_f32(const float* __restrict__ x,
                                                    float* __restrict__ t, long n, int W, int Cx,
                                                    int Cr, int S, int sw, int pl, int Wo, int Cp) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long row = i / Cp;
    const int e = (int)(i - row * Cp);
    const int wo = (int)(row % Wo);
    const long nh = row / Wo;
    const int s = e / Cr, c = e - s * Cr, wi = wo * sw - pl + s;
    t[i] = s < S && (unsigned)wi < (unsigned)W ? x[(nh * W + wi) * Cx + c] : 0.f;
  }
}

}  // namespace

// ------------------------------------------------------------------------------------ launchers
void row_pack_f32_launch(const float* x, float* t, int N, int H, int W, int Cx, int Cr, int S,
                         int sw, int pl, int Wo, int Cp, hipStream_t st) {
  const long n = (long)N * H * Wo * Cp;
  hipLaunchKernelGGL(row_pack_f32, dim3(eblocks(n)), dim3(256), 0, st, x, t, n, W, Cx, Cr, S, sw, pl,
                     Wo, Cp);
}
// WGRAD: split the pixel reduction until the grid holds ~4 workgroups per CU, ≥ 16 K-steps each
static void wgrad_plan(const ConvF32Args& a, int* qps, int* splits) {
  const int M = a.K, Ng = a.R * a.S * a.C;
  const int nq = (int)(((long)a.N * a.Ho * a.Wo + BK - 1) / BK);
  const long tiles = (long)((M + BM - 1) / BM) * ((Ng + BN - 1) / BN);
  const long want = std::max<long>(1, 1024 / tiles);
  *qps = (int)std::max<long>(16, (nq + want - 1) / want);
  *splits = std::max(1, (nq + *qps - 1) / *qps);
}

int conv_f32_wgrad_splits(const ConvF32Args& a) {
  int qps, splits;
  wgrad_plan(a, &qps, &splits);
  return splits;
}

static int g_f32_tile[2] = {0, 0};
void conv_f32_set_tile(int tbm, int tbn) {
  const bool ok = (tbm == 64 || tbm == 128) && (tbn == 64 || tbn == 128);
  g_f32_tile[0] = ok ? tbm : 0;
  g_f32_tile[1] = ok ? tbn : 0;
}

static void conv_f32_launch(int mode, const ConvF32Args& a0, hipStream_t st) {
  ConvF32Args a = a0;
  a.fd_HoWo = make_fastdiv((uint32_t)std::max(1, a.Ho * a.Wo));
  a.fd_Wo = make_fastdiv((uint32_t)std::max(1, a.Wo));
  int M, Ng, nq, cch = 1;
  if (mode == C_FWD) {
    M = a.N * a.Ho * a.Wo; Ng = a.K; cch = (a.C + BK - 1) / BK; nq = a.R * a.S * cch;
  } else if (mode == C_DGRAD) {
    M = a.N * a.H * a.W; Ng = a.C; cch = (a.K + BK - 1) / BK; nq = a.R * a.S * cch;
  } else {
    M = a.K; Ng = a.R * a.S * a.C; nq = (int)(((long)a.N * a.Ho * a.Wo + BK - 1) / BK);
  }
  if (M <= 0 || Ng <= 0 || nq <= 0) return;
  // tile: 128×128, unless that leaves the chip under-filled (FWD / DGRAD): then the shape among
  // 128×128 / 64×128 / 128×64 / 64×64 whose workgroup count best fills whole waves of 256 CUs
  // (ties: the bigger tile) — TDL_F32_TILE=0 keeps 128×128
  static const bool small_on = getenv("TDL_F32_TILE") == nullptr || atoi(getenv("TDL_F32_TILE"));
  int tbm = 128, tbn = 128;
  if (mode != C_WGRAD && g_f32_tile[0] > 0) {  // forced (tests: every tile shape)
    tbm = g_f32_tile[0];
    tbn = g_f32_tile[1];
  } else if (mode != C_WGRAD && small_on) {
    const int cand[4][2] = {{128, 128}, {64, 128}, {128, 64}, {64, 64}};
    double best = -1.0;
    for (const auto& cdm : cand) {
      const long nt = (long)((M + cdm[0] - 1) / cdm[0]) * ((Ng + cdm[1] - 1) / cdm[1]);
      const long slots = 256L * ((nt + 255) / 256);
      // fill of the last wave of workgroups; a bigger tile is worth ~10 % of fill
      const double score = (double)nt / slots + (cdm[0] * cdm[1] == 128 * 128 ? 0.1 : cdm[0] * cdm[1] == 64 * 64 ? 0.0 : 0.05);
      if (score > best + 1e-9) {
        best = score;
        tbm = cdm[0];
        tbn = cdm[1];
      }
    }
  }
  const int tiles_m = (M + tbm - 1) / tbm;
  const int tiles_n = (Ng + tbn - 1) / tbn;
  const long tiles = (long)tiles_m * tiles_n;
  int qps = nq, splits = 1;
  if (mode == C_WGRAD) wgrad_plan(a, &qps, &splits);
  const dim3 grid((unsigned)tiles, (unsigned)splits);
#define TDL_F32_LAUNCH(MODE_, TM_, TN_)                                                         \
  hipLaunchKernelGGL((conv_f32_kernel<MODE_, TM_, TN_>), grid, dim3(CT), 0, st, a, M, Ng, nq, cch, qps, \
                     tiles_n)
  if (mode == C_WGRAD) {
    TDL_F32_LAUNCH(C_WGRAD, 128, 128);
  } else if (mode == C_FWD) {
    if (tbm == 128 && tbn == 128) TDL_F32_LAUNCH(C_FWD, 128, 128);
    else if (tbm == 64 && tbn == 128) TDL_F32_LAUNCH(C_FWD, 64, 128);
    else if (tbm == 128) TDL_F32_LAUNCH(C_FWD, 128, 64);
    else TDL_F32_LAUNCH(C_FWD, 64, 64);
  } else {
    if (tbm == 128 && tbn == 128) TDL_F32_LAUNCH(C_DGRAD, 128, 128);
    else if (tbm == 64 && tbn == 128) TDL_F32_LAUNCH(C_DGRAD, 64, 128);
    else if (tbm == 128) TDL_F32_LAUNCH(C_DGRAD, 128, 64);
    else TDL_F32_LAUNCH(C_DGRAD, 64, 64);
  }
#undef TDL_F32_LAUNCH
}

void conv_f32_fwd_launch(const ConvF32Args& a, hipStream_t st) { conv_f32_launch(C_FWD, a, st); }
void conv_f32_dgrad_launch(const ConvF32Args& a, hipStream_t st) { conv_f32_launch(C_DGRAD, a, st); }
void conv_f32_wgrad_launch(const ConvF32Args& a0, hipStream_t st) {
  const long n = (long)a0.K * a0.R * a0.S * a0.C;
  const int splits = conv_f32_wgrad_splits(a0);
  ConvF32Args a = a0;
  if (splits == 1) a.slab = nullptr;  // one split: dW written (or accumulated) directly
  conv_f32_launch(C_WGRAD, a, st);
  if (splits > 1) splitk_reduce_launch(a.slab, a.out, n, splits, a.accumulate != 0, st);
}

void colsum_f32_launch(const float* x, float* out, long M, int C, long ldx, hipStream_t st) {
  if (C % 4 == 0 && ldx % 4 == 0) {
    chan_reduce_launch(1, x, nullptr, nullptr, nullptr, out, M, C, ldx, 0, st);
    return;
  }
  const int gy = (C + 63) / 64;
  const long gx = std::max<long>(1, std::min<long>((M + 63) / 64, 256 / gy));
  hipLaunchKernelGGL(colsum_scalar_f32, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, st, x, out, M,
                     C, ldx);
}
void bn_stats_f32_launch(const float* x, float* stats, long M, int C, hipStream_t st) {
  chan_reduce_launch(0, x, nullptr, nullptr, nullptr, stats, M, C, C, 0, st);
}
void bn_bwd_reduce_f32_launch(const float* dy, const float* y, const float* x, const float* coef,
                              float* red, long M, int C, int relu, long ldd, hipStream_t st) {
  chan_reduce_launch(2, dy, x, y, coef, red, M, C, ldd, relu, st);
}
void bn_apply_f32_launch(const float* x, const float* coef, const float* res, float* y, long M,
                         int C, bool relu, long ldy, hipStream_t st) {
  hipLaunchKernelGGL(bn_apply_f32, dim3(eblocks(M * (C / 4))), dim3(256), 0, st, x, coef, res, y, M,
                     C, ldy, (int)relu);
}
void bn_bwd_apply_f32_launch(const float* dy, const float* y, const float* x, const float* coef,
                             const float* red, const float* gamma, float* dx, float* dres,
                             float* dgamma, float* dbeta, const float* dadd, long M, int C,
                             float count, int relu, long ldd, hipStream_t st) {
  const float inv_count = count > 0.f && count < 3.0e38f ? 1.f / count : 0.f;
  hipLaunchKernelGGL(bn_bwd_apply_f32, dim3(eblocks(M * (C / 4))), dim3(256), 0, st, dy, y, x, coef,
                     red, gamma, dx, dres, dgamma, dbeta, dadd, M, C, ldd, inv_count, relu);
}
void relu_bwd_f32_launch(const float* dy, const float* y, float* dx, long n, hipStream_t st) {
  hipLaunchKernelGGL(relu_bwd_f32, dim3(eblocks(n / 4)), dim3(256), 0, st, (const float4*)dy,
                     (const float4*)y, (float4*)dx, n / 4);
}
void add_act_f32_launch(const float* a, const float* b, float* y, long n, bool relu,
                        hipStream_t st) {
  hipLaunchKernelGGL(add_act_f32, dim3(eblocks(n / 4)), dim3(256), 0, st, (const float4*)a,
                     (const float4*)b, (float4*)y, n / 4, (int)relu);
}
void dwconv_f32_fwd_launch(const DwF32Args& a, hipStream_t st) {
  hipLaunchKernelGGL(dw_fwd_f32, dim3(eblocks((long)a.N * a.Ho * a.Wo * (a.C / 4))), dim3(256), 0, st,
                     a);
}
void dwconv_f32_dgrad_launch(const DwF32Args& a, hipStream_t st) {
  hipLaunchKernelGGL(dw_dgrad_f32, dim3(eblocks((long)a.N * a.H * a.W * (a.C / 4))), dim3(256), 0,
                     st, a);
}
void dwconv_f32_wgrad_launch(const DwF32Args& a, hipStream_t st) {
  const int cv = a.C / 4;
  int cvb = 1;
  while (cvb < cv && cvb < 64) cvb <<= 1;
  const int gy = (cv + cvb - 1) / cvb;
  const long rpb = 256 / cvb, P = (long)a.N * a.Ho * a.Wo;
  const long gx = std::max<long>(1, std::min<long>((P + rpb * 32 - 1) / (rpb * 32), 512 / gy));
  hipLaunchKernelGGL(dw_wgrad_f32, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, st, a, cvb);
}

}  // namespace tdl
