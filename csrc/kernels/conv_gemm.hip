// MFMA implicit-GEMM convolution for gfx950 (MI355X / CDNA4), NHWC activations, KRSC weights, bf16
// operands, fp32 accumulation.
//
// One kernel template serves the three convolution GEMMs:
//
//   mode   GEMM C[M][N] = Σ_k A[m][k]·B[n][k]                A operand            B operand
//   FWD    y[m=(n,ho,wo)][co]    k = (r,s,ci)   M=N·Ho·Wo     x gathered (k-contig) w[co][k] (k-contig)
//   DGRAD  dx[m=(n,h,w)][ci]     k = (r,s,co)   M=N·H·W       dy gathered (k-contig) w[co][r][s][ci] (n-contig)
//   WGRAD  dw[m=co][n=(r,s,ci)]  k = (n,ho,wo)  split-K       dy[p][co] (m-contig)   x gathered (n-contig)
//
// Operands whose 16-B global vectors run along K ("KC") are staged into an LDS image
// [rows][64] (128-B rows, 16-B chunk index XOR ((row>>1)&7): conflict-free ds_read_b128 for the
// 16x16x32 fragment pattern).  Operands whose vectors run along M/N ("MC", i.e. K is strided in
// memory) are staged as [64 k-rows][cols] (32-B pair index XOR f(k)) and read with gfx950's
// ds_read_b64_tr_b16 hardware transpose, so dgrad needs no weight transpose and wgrad no
// activation transpose.  Staging is register double-buffered (global→VGPR for tile t+1 is in
// flight while the MFMAs consume tile t from LDS; one barrier per 64-deep K step).
//
// Tile: BM×BN×64 per 256-thread workgroup, 2×2 waves, each wave (BM/2)×(BN/2) as 16×16 MFMA
// tiles (v_mfma_f32_16x16x32_bf16).  The MFMA is issued with the operands swapped (D = Bᵀ·Aᵀ) so
// each lane ends up holding 4 consecutive output channels of one output row → 8-B bf16 / 16-B
// fp32 vector stores.  Epilogue options: bias, ReLU, and per-channel Σy / Σy² of the stored bf16
// values (BatchNorm statistics) reduced across lanes, then waves through LDS, then one contiguous
// atomicAdd row per workgroup.  Workgroup ids are remapped so each XCD owns a contiguous tile range.
#include "common.h"
#include "kernels.h"

namespace tdl {

namespace {

constexpr int BK = 64;
constexpr int NT = 256;
enum { FWD = 0, DGRAD = 1, WGRAD = 2 };

__device__ __forceinline__ int kc_off(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <int COLS>
__device__ __forceinline__ int mc_swz(int k) {
  if constexpr (COLS >= 128)
    return (k & 3) | (((k >> 3) & 1) << 2);
  else
    return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
}

template <int COLS>
__device__ __forceinline__ int mc_off(int k, int col) {
  return k * (COLS * 2) + (((col >> 4) ^ mc_swz<COLS>(k)) << 5) + ((col & 15) << 1);
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ bf16x8 read_kc(const char* tile, int row, int chunk) {
  uint4 v = *(const uint4*)(tile + kc_off(row, chunk));
  return __builtin_bit_cast(bf16x8, v);
}

template <int COLS>
__device__ __forceinline__ bf16x8 read_mc(const char* tile, int krow, int col) {
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + mc_off<COLS>(krow, col)));
  s16x4 hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + mc_off<COLS>(krow + 4, col)));
  s16x8 cat = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, cat);
}

// ---------------------------------------------------------------------------------------------
// generic per-element operand access (used when C or K is not a multiple of 8)
// A(m, k), B(n, k) in GEMM terms.
// ---------------------------------------------------------------------------------------------
template <int MODE>
__device__ __forceinline__ bf16_t elemA(const ConvArgs& a, int m, int k) {
  if (m >= a.M || k >= a.Kg) return 0;
  if constexpr (MODE == FWD) {
    const int HoWo = a.Ho * a.Wo;
    const int n = m / HoWo, rem = m - n * HoWo, ho = rem / a.Wo, wo = rem - ho * a.Wo;
    const int c = k % a.C, rs = k / a.C, r = rs / a.S, s = rs - r * a.S;
    const int hi = ho * a.sh - a.ph + r * a.dh, wi = wo * a.sw - a.pw + s * a.dw;
    if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) return 0;
    return a.x[(((long)n * a.H + hi) * a.W + wi) * a.C + c];
  } else if constexpr (MODE == DGRAD) {
    const int HW = a.H * a.W;
    const int n = m / HW, rem = m - n * HW, h = rem / a.W, w = rem - h * a.W;
    const int co = k % a.K, rs = k / a.K, r = rs / a.S, s = rs - r * a.S;
    int th = h + a.ph - r * a.dh, tw = w + a.pw - s * a.dw;
    if (th < 0 || tw < 0 || th % a.sh || tw % a.sw) return 0;
    th /= a.sh;
    tw /= a.sw;
    if (th >= a.Ho || tw >= a.Wo) return 0;
    return a.dy[(((long)n * a.Ho + th) * a.Wo + tw) * a.K + co];
  } else {  // WGRAD: A[m=co][k=p] = dy[p][co]
    return a.dy[(long)k * a.K + m];
  }
}

template <int MODE>
__device__ __forceinline__ bf16_t elemB(const ConvArgs& a, int n, int k) {
  if (n >= a.Ng || k >= a.Kg) return 0;
  if constexpr (MODE == FWD) {
    return a.w[(long)n * a.Kg + k];
  } else if constexpr (MODE == DGRAD) {  // B[n=ci][k=(r,s,co)] = w[co][r][s][ci]
    const int co = k % a.K, rs = k / a.K;
    return a.w[((long)co * a.R * a.S + rs) * a.C + n];
  } else {  // WGRAD: B[n=(r,s,ci)][k=p] = x[n_img, ho*sh-ph+r*dh, wo*sw-pw+s*dw, ci]
    const int HoWo = a.Ho * a.Wo;
    const int ni = k / HoWo, rem = k - ni * HoWo, ho = rem / a.Wo, wo = rem - ho * a.Wo;
    const int ci = n % a.C, rs = n / a.C, r = rs / a.S, s = rs - r * a.S;
    const int hi = ho * a.sh - a.ph + r * a.dh, wi = wo * a.sw - a.pw + s * a.dw;
    if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) return 0;
    return a.x[(((long)ni * a.H + hi) * a.W + wi) * a.C + ci];
  }
}

__device__ __forceinline__ uint4 gather8(const bf16_t* v) {
  return make_uint4((uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                    (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16));
}

// ---------------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------------
template <int MODE, int BM, int BN, bool ALIGNED, bool STATS>
__global__ void __launch_bounds__(NT, 2) conv_gemm_kernel(ConvArgs a) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM, TN = BN / WN, RM = TM / 16, RN = TN / 16;
  constexpr bool A_MC = (MODE == WGRAD), B_MC = (MODE != FWD);
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PA = BM * BK / 8 / NT, PB = BN * BK / 8 / NT;
  constexpr int A_CPR = BM / 8, B_CPR = BN / 8;  // MC: 16-B chunks per k-row
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = (a.Ng + BN - 1) / BN;
  const int ntm = (a.M + BM - 1) / BM;
  const int ntiles = ntn * ntm;
  int id = xcd_remap(blockIdx.x, gridDim.x);
  const int split = id / ntiles;
  const int tile = id - split * ntiles;
  const int bm0 = (tile / ntn) * BM, bn0 = (tile % ntn) * BN;

  const int nkt = (a.Kg + BK - 1) / BK;
  int kt0 = 0, kt1 = nkt;
  if constexpr (MODE == WGRAD) {
    kt0 = split * a.kps;
    kt1 = min(nkt, kt0 + a.kps);
  }

  // ---------------- per-thread precomputation (aligned path) ----------------
  // A side
  long a_base[PA];
  int a_p0[PA], a_p1[PA];
  // B side
  long b_base[PB];
  int b_p0[PB], b_p1[PB];
  int a_fix = 0, b_fix = 0, b_fix2 = 0;
  const int HoWo = a.Ho * a.Wo;
  if constexpr (ALIGNED) {
    if constexpr (MODE == FWD) {
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int m = bm0 + (tid >> 3) + i * (NT / 8);
        if (m < a.M) {
          const int n = m / HoWo, rem = m - n * HoWo, ho = rem / a.Wo, wo = rem - ho * a.Wo;
          a_base[i] = (long)n * a.H * a.W * a.C;
          a_p0[i] = ho * a.sh - a.ph;
          a_p1[i] = wo * a.sw - a.pw;
        } else {
          a_base[i] = 0;
          a_p0[i] = -(1 << 28);
          a_p1[i] = 0;
        }
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int n = bn0 + (tid >> 3) + i * (NT / 8);
        b_base[i] = (long)n * a.Kg;
        b_p0[i] = n < a.Ng;
        b_p1[i] = 0;
      }
    } else if constexpr (MODE == DGRAD) {
      const int HW = a.H * a.W;
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int m = bm0 + (tid >> 3) + i * (NT / 8);
        if (m < a.M) {
          const int n = m / HW, rem = m - n * HW, h = rem / a.W, w = rem - h * a.W;
          a_base[i] = (long)n * HoWo * a.K;
          a_p0[i] = h + a.ph;
          a_p1[i] = w + a.pw;
        } else {
          a_base[i] = 0;
          a_p0[i] = -(1 << 28);
          a_p1[i] = -(1 << 28);
        }
      }
      b_fix = bn0 + (tid % B_CPR) * 8;  // ci
    } else {  // WGRAD
      a_fix = bm0 + (tid % A_CPR) * 8;  // co
      const int nn = bn0 + (tid % B_CPR) * 8;
      if (nn < a.Ng) {
        const int ci = nn % a.C, rs = nn / a.C, r = rs / a.S, s = rs - r * a.S;
        b_fix = ci;
        b_fix2 = r * a.dh - a.ph;
        b_p0[0] = s * a.dw - a.pw;
      } else {
        b_fix = -1;
        b_fix2 = -(1 << 28);
        b_p0[0] = 0;
      }
    }
  }

  uint4 ra[PA], rb[PB];

  auto load_tiles = [&](int kt) {
    if constexpr (ALIGNED) {
      if constexpr (MODE == FWD) {
        const int k = kt * BK + (tid & 7) * 8;
        const bool kv = k < a.Kg;
        const int c = k % a.C, rs = k / a.C, r = rs / a.S, s = rs - r * a.S;
        const int ro = r * a.dh, so = s * a.dw;
#pragma unroll
        for (int i = 0; i < PA; ++i) {
          const int hi = a_p0[i] + ro, wi = a_p1[i] + so;
          const bool v = kv && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
          ra[i] = v ? *(const uint4*)(a.x + a_base[i] + ((long)hi * a.W + wi) * a.C + c)
                    : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) {
          const bool v = kv && b_p0[i];
          rb[i] = v ? *(const uint4*)(a.w + b_base[i] + k) : make_uint4(0, 0, 0, 0);
        }
      } else if constexpr (MODE == DGRAD) {
        const int k = kt * BK + (tid & 7) * 8;
        const bool kv = k < a.Kg;
        const int co = k % a.K, rs = k / a.K, r = rs / a.S, s = rs - r * a.S;
        const int ro = r * a.dh, so = s * a.dw;
#pragma unroll
        for (int i = 0; i < PA; ++i) {
          int th = a_p0[i] - ro, tw = a_p1[i] - so;
          bool v = kv && th >= 0 && tw >= 0;
          if (a.sh != 1) {
            v = v && (th % a.sh) == 0 && (tw % a.sw) == 0;
            th /= a.sh;
            tw /= a.sw;
          }
          v = v && th < a.Ho && tw < a.Wo;
          ra[i] = v ? *(const uint4*)(a.dy + a_base[i] + ((long)th * a.Wo + tw) * a.K + co)
                    : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) {
          const int kk = kt * BK + tid / B_CPR + i * (NT / B_CPR);
          const bool v = kk < a.Kg && b_fix < a.Ng;
          if (v) {
            const int co2 = kk % a.K, rs2 = kk / a.K;
            rb[i] = *(const uint4*)(a.w + ((long)co2 * a.R * a.S + rs2) * a.C + b_fix);
          } else {
            rb[i] = make_uint4(0, 0, 0, 0);
          }
        }
      } else {  // WGRAD
#pragma unroll
        for (int i = 0; i < PA; ++i) {
          const int p = kt * BK + tid / A_CPR + i * (NT / A_CPR);
          const bool v = p < a.Kg && a_fix < a.M;
          ra[i] = v ? *(const uint4*)(a.dy + (long)p * a.K + a_fix) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) {
          const int p = kt * BK + tid / B_CPR + i * (NT / B_CPR);
          bool v = p < a.Kg && b_fix >= 0;
          uint4 val = make_uint4(0, 0, 0, 0);
          if (v) {
            const int ni = p / HoWo, rem = p - ni * HoWo, ho = rem / a.Wo, wo = rem - ho * a.Wo;
            const int hi = ho * a.sh + b_fix2, wi = wo * a.sw + b_p0[0];
            if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
              val = *(const uint4*)(a.x + (((long)ni * a.H + hi) * a.W + wi) * a.C + b_fix);
          }
          rb[i] = val;
        }
      }
    } else {
      // generic element path
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        bf16_t e[8];
        if constexpr (!A_MC) {
          const int m = bm0 + (tid >> 3) + i * (NT / 8);
          const int k = kt * BK + (tid & 7) * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = elemA<MODE>(a, m, k + j);
        } else {
          const int k = kt * BK + tid / A_CPR + i * (NT / A_CPR);
          const int m = bm0 + (tid % A_CPR) * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = elemA<MODE>(a, m + j, k);
        }
        ra[i] = gather8(e);
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        bf16_t e[8];
        if constexpr (!B_MC) {
          const int n = bn0 + (tid >> 3) + i * (NT / 8);
          const int k = kt * BK + (tid & 7) * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = elemB<MODE>(a, n, k + j);
        } else {
          const int k = kt * BK + tid / B_CPR + i * (NT / B_CPR);
          const int n = bn0 + (tid % B_CPR) * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = elemB<MODE>(a, n + j, k);
        }
        rb[i] = gather8(e);
      }
    }
  };

  auto store_tiles = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      if constexpr (!A_MC) {
        *(uint4*)(As + kc_off((tid >> 3) + i * (NT / 8), tid & 7)) = ra[i];
      } else {
        *(uint4*)(As + mc_off<BM>(tid / A_CPR + i * (NT / A_CPR), (tid % A_CPR) * 8)) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      if constexpr (!B_MC) {
        *(uint4*)(Bs + kc_off((tid >> 3) + i * (NT / 8), tid & 7)) = rb[i];
      } else {
        *(uint4*)(Bs + mc_off<BN>(tid / B_CPR + i * (NT / B_CPR), (tid % B_CPR) * 8)) = rb[i];
      }
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    load_tiles(kt0);
    store_tiles(0);
  }
  __syncthreads();

  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) load_tiles(kt + 1);
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[RM], bfg[RN];
#pragma unroll
      for (int rm = 0; rm < RM; ++rm) {
        const int row = wm * TM + rm * 16;
        if constexpr (A_MC)
          af[rm] = read_mc<BM>(As, kk * 32 + 8 * (lane >> 4) + ((lane >> 2) & 3), row + 4 * (lane & 3));
        else
          af[rm] = read_kc(As, row + (lane & 15), kk * 4 + (lane >> 4));
      }
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) {
        const int row = wn * TN + rn * 16;
        if constexpr (B_MC)
          bfg[rn] = read_mc<BN>(Bs, kk * 32 + 8 * (lane >> 4) + ((lane >> 2) & 3), row + 4 * (lane & 3));
        else
          bfg[rn] = read_kc(Bs, row + (lane & 15), kk * 4 + (lane >> 4));
      }
#pragma unroll
      for (int rm = 0; rm < RM; ++rm)
#pragma unroll
        for (int rn = 0; rn < RN; ++rn)
          acc[rm][rn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[rn], af[rm], acc[rm][rn], 0, 0, 0);
    }
    if (more) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  // lane holds C[m = bm0 + wm*TM + rm*16 + (lane&15)][n = bn0 + wn*TN + rn*16 + (lane>>4)*4 + i]
  if constexpr (MODE == WGRAD) {
    float* out = (float*)a.out + (long)split * a.M * a.Ng;
    const bool vec = (a.Ng & 3) == 0;
#pragma unroll
    for (int rm = 0; rm < RM; ++rm) {
      const int m = bm0 + wm * TM + rm * 16 + (lane & 15);
      if (m >= a.M) continue;
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) {
        const int n0 = bn0 + wn * TN + rn * 16 + (lane >> 4) * 4;
        float* p = out + (long)m * a.Ng + n0;
        if (vec && n0 + 3 < a.Ng) {
          *(float4*)p = make_float4(acc[rm][rn][0], acc[rm][rn][1], acc[rm][rn][2], acc[rm][rn][3]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (n0 + i < a.Ng) p[i] = acc[rm][rn][i];
        }
      }
    }
  } else {
    bf16_t* out = (bf16_t*)a.out;
    const bool vec = ((a.ldc & 3) == 0);
    float s_sum[RN][4], s_sq[RN][4];
#pragma unroll
    for (int rn = 0; rn < RN; ++rn)
#pragma unroll
      for (int i = 0; i < 4; ++i) s_sum[rn][i] = s_sq[rn][i] = 0.f;
#pragma unroll
    for (int rm = 0; rm < RM; ++rm) {
      const int m = bm0 + wm * TM + rm * 16 + (lane & 15);
      const bool mv = m < a.M;
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) {
        const int n0 = bn0 + wn * TN + rn * 16 + (lane >> 4) * 4;
        float v[4];
        bf16_t h[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float t = acc[rm][rn][i];
          if (a.bias != nullptr && n0 + i < a.Ng) t += a.bias[n0 + i];
          if (a.relu) t = fmaxf(t, 0.f);
          h[i] = f2bf(t);
          v[i] = bf2f(h[i]);
        }
        if (mv) {
          bf16_t* p = out + (long)m * a.ldc + n0;
          if (vec && n0 + 3 < a.Ng) {
            *(uint2*)p = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16),
                                    (uint32_t)h[2] | ((uint32_t)h[3] << 16));
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (n0 + i < a.Ng) p[i] = h[i];
          }
          if constexpr (STATS) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              s_sum[rn][i] += v[i];
              s_sq[rn][i] += v[i] * v[i];
            }
          }
        }
      }
    }
    if constexpr (STATS) {
      // reduce over the 16 lanes that share (lane>>4): they hold different m of the same n
#pragma unroll
      for (int rn = 0; rn < RN; ++rn)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            s_sum[rn][i] += __shfl_xor(s_sum[rn][i], o, 64);
            s_sq[rn][i] += __shfl_xor(s_sq[rn][i], o, 64);
          }
        }
      // LDS: red[wm][2][BN]
      float* red = (float*)smem;  // main loop ended with a barrier: smem is free
      if ((lane & 15) == 0) {
#pragma unroll
        for (int rn = 0; rn < RN; ++rn)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int nl = wn * TN + rn * 16 + (lane >> 4) * 4 + i;
            red[(wm * 2 + 0) * BN + nl] = s_sum[rn][i];
            red[(wm * 2 + 1) * BN + nl] = s_sq[rn][i];
          }
      }
      __syncthreads();
      for (int t = tid; t < 2 * BN; t += NT) {
        const int which = t / BN, nl = t - which * BN;
        const int n = bn0 + nl;
        if (n < a.Ng) {
          float v = 0.f;
#pragma unroll
          for (int w = 0; w < WM; ++w) v += red[(w * 2 + which) * BN + nl];
          atomicAdd(a.stats + which * a.Ng + n, v);
        }
      }
    }
  }
}

// fp32 split-K slab reduction: out[i] (+)= Σ_z slab[z][i]
__global__ void splitk_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                     long n, int splits, int accumulate) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 s = accumulate ? ((const float4*)out)[i] : make_float4(0, 0, 0, 0);
    for (int z = 0; z < splits; ++z) {
      const float4 v = ((const float4*)(slab + (long)z * n))[i];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    ((float4*)out)[i] = s;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    float s = accumulate ? out[i] : 0.f;
    for (int z = 0; z < splits; ++z) s += slab[(long)z * n + i];
    out[i] = s;
  }
}

// column sums of a bf16 [P][K] matrix into fp32 out[K] (zeroed by caller): bias gradient
__global__ void colsum_kernel(const bf16_t* __restrict__ x, float* __restrict__ out, long P, int K,
                              long rows_per_block) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const long r0 = blockIdx.y * rows_per_block;
  const long r1 = min(P, r0 + rows_per_block);
  float s = 0.f;
  if (c < K)
    for (long r = r0 + w; r < r1; r += 4) s += bf2f(x[r * K + c]);
  red[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && c < K) atomicAdd(out + c, red[0][threadIdx.x] + red[1][threadIdx.x] +
                                              red[2][threadIdx.x] + red[3][threadIdx.x]);
}

template <int MODE, int BM, int BN, bool AL, bool ST>
void launch_t(const ConvArgs& a, int splits, hipStream_t st) {
  const int tiles = cdiv(a.M, BM) * cdiv(a.Ng, BN);
  hipLaunchKernelGGL((conv_gemm_kernel<MODE, BM, BN, AL, ST>), dim3(tiles * splits), dim3(NT), 0, st,
                     a);
}

template <int MODE, bool AL, bool ST>
void launch_cfg(const ConvArgs& a, int bm, int bn, int splits, hipStream_t st) {
  if (bm == 128 && bn == 128)
    launch_t<MODE, 128, 128, AL, ST>(a, splits, st);
  else if (bm == 128 && bn == 64)
    launch_t<MODE, 128, 64, AL, ST>(a, splits, st);
  else if (bm == 64 && bn == 128)
    launch_t<MODE, 64, 128, AL, ST>(a, splits, st);
  else
    launch_t<MODE, 64, 64, AL, ST>(a, splits, st);
}

}  // namespace

static void pick_tile(int M, int Ng, int& bm, int& bn) {
  bn = Ng <= 64 ? 64 : 128;
  bm = M <= 64 ? 64 : 128;
  // small problems: prefer more workgroups
  if (bm == 128 && bn == 128 && (long)cdiv(M, 128) * cdiv(Ng, 128) < 256) bn = 64;
  if (bm == 128 && (long)cdiv(M, bm) * cdiv(Ng, bn) < 256) bm = 64;
}

void conv_fwd_launch(const ConvArgs& a, hipStream_t st) {
  int bm, bn;
  pick_tile(a.M, a.Ng, bm, bn);
  const bool al = (a.C % 8 == 0) && (a.K % 8 == 0);
  const bool stats = a.stats != nullptr;
  if (al) {
    if (stats) launch_cfg<FWD, true, true>(a, bm, bn, 1, st);
    else launch_cfg<FWD, true, false>(a, bm, bn, 1, st);
  } else {
    if (stats) launch_cfg<FWD, false, true>(a, bm, bn, 1, st);
    else launch_cfg<FWD, false, false>(a, bm, bn, 1, st);
  }
}

void conv_dgrad_launch(const ConvArgs& a, hipStream_t st) {
  int bm, bn;
  pick_tile(a.M, a.Ng, bm, bn);
  const bool al = (a.C % 8 == 0) && (a.K % 8 == 0);
  if (al) launch_cfg<DGRAD, true, false>(a, bm, bn, 1, st);
  else launch_cfg<DGRAD, false, false>(a, bm, bn, 1, st);
}

void conv_wgrad_plan(int M, int Ng, long Kg, int* bm, int* bn, int* splits, int* kps) {
  *bm = M <= 64 ? 64 : 128;
  *bn = Ng <= 64 ? 64 : 128;
  const int tiles = cdiv(M, *bm) * cdiv(Ng, *bn);
  const int nkt = cdiv(Kg, BK);
  int target = 1024;  // ≈4 workgroups per CU over 256 CUs
  int s = std::max(1, std::min(nkt, target / std::max(tiles, 1)));
  int per = cdiv(nkt, s);
  per = std::max(per, 4);  // at least 4 K-steps per split
  *kps = per;
  *splits = cdiv(nkt, per);
}

void conv_wgrad_launch(const ConvArgs& a, int bm, int bn, int splits, float* out, bool accumulate,
                       hipStream_t st) {
  const bool al = (a.C % 8 == 0) && (a.K % 8 == 0);
  if (al) launch_cfg<WGRAD, true, false>(a, bm, bn, splits, st);
  else launch_cfg<WGRAD, false, false>(a, bm, bn, splits, st);
  const long n = (long)a.M * a.Ng;
  const int blocks = (int)std::min<long>(2048, std::max<long>(1, (n / 4 + 255) / 256));
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, (const float*)a.out, out,
                     n, splits, accumulate ? 1 : 0);
}

void colsum_launch(const bf16_t* x, float* out, long P, int K, hipStream_t st) {
  const long rpb = 1024;
  dim3 grid(cdiv(K, 64), (int)std::max<long>(1, (P + rpb - 1) / rpb));
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, st, x, out, P, K, rpb);
}

}  // namespace tdl
