// Shared pieces of the implicit-GEMM convolution kernels (conv_gemm.hip: register-staged
// 4-wave kernel; conv_glds.hip: LDS-DMA pipelined kernel): LDS image layouts, range-checked buffer
// access, per-tile geometry of the three conv GEMMs (FWD / DGRAD parity classes / WGRAD split-K).
#pragma once
#include "common.h"
#include "kernels.h"

namespace tdl {
namespace convk {

constexpr int BK = 64;
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

// Range-checked buffer access: an offset beyond the descriptor's byte count returns 0 on load
// and is dropped on store, so padding / ragged edges need no branch (a per-element branch around
// a load makes hipcc wait vmcnt(0) per element and serialises the staging pipeline).
constexpr uint32_t OOB = 0xFFFFFFF0u;
// byte offset of an invalid output row: row + column offsets (< 64 KiB) stay past any buffer the
// 32-bit range-checked descriptors address (hosts check out_bytes < ROW_OOB) without wrapping
constexpr uint32_t ROW_OOB = 0xF0000000u;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload16(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

__device__ __forceinline__ uint4 gather8(const bf16_t* v) {
  return make_uint4((uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                    (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16));
}

// ---------------------------------------------------------------------------------------------
// per-tile geometry
// ---------------------------------------------------------------------------------------------
struct Tile {
  int bm0, bn0;   // first row / column of the tile (class-local rows for DGRAD)
  int cls;        // DGRAD class
  int Mc, Kgc;    // rows / K of the (class) GEMM
  int kt0, kt1;   // K-step range (split range for WGRAD)
  int split;      // WGRAD split index
};

template <int MODE, int BM, int BN, int KS = BK>
__device__ __forceinline__ Tile tile_of(const ConvArgs& a, int t) {
  Tile T;
  const int ntn = (a.Ng + BN - 1) / BN;
  T.cls = 0;
  T.split = 0;
  T.Mc = a.M;
  T.Kgc = a.Kg;
  int local = t;
  if constexpr (MODE == DGRAD) {
    int c = 0;
    while (c + 1 < a.ncls && t >= a.cls_tile0[c + 1]) ++c;
    T.cls = c;
    local = t - a.cls_tile0[c];
    T.Mc = a.N * a.cls_Hc[c] * a.cls_Wc[c];
    T.Kgc = a.cls_Th[c] * a.cls_Tw[c] * a.K;
  } else if constexpr (MODE == WGRAD) {
    const int ntm = (a.M + BM - 1) / BM;
    const int nt = ntm * ntn;
    T.split = t / nt;
    local = t - T.split * nt;
  }
  if constexpr (MODE == FWD) {
    // workgroup b owns column tile (b % ntn) and row tiles [(b / ntn)·tpb, +tpb): its tiles share
    // bn0 (BN statistics accumulate in registers, one flush per workgroup) and the ntn workgroups
    // of a row group run together, re-reading the same A tiles from L2
    const int grp = local / (a.tpb * ntn), r = local - grp * a.tpb * ntn;
    T.bn0 = (r / a.tpb) * BN;
    T.bm0 = (grp * a.tpb + r % a.tpb) * BM;
  } else {
    T.bm0 = (local / ntn) * BM;
    T.bn0 = (local % ntn) * BN;
  }
  const int nkt = (T.Kgc + KS - 1) / KS;  // KS: GEMM K per step (64 bf16 / 128 fp8)
  if constexpr (MODE == WGRAD) {
    T.kt0 = T.split * a.kps;
    T.kt1 = min(nkt, T.kt0 + a.kps);
    if (T.kt1 <= T.kt0) T.kt1 = T.kt0 + 1;  // empty split: one zero step (slab must be written)
  } else {
    T.kt0 = 0;
    T.kt1 = max(nkt, 1);  // a class with no taps still writes its (zero) tile
  }
  return T;
}

// ---------------------------------------------------------------------------------------------
// generic per-element operand access (used when C or K is not a multiple of 8)
// ---------------------------------------------------------------------------------------------
template <int MODE>
__device__ __forceinline__ bf16_t elemA(const ConvArgs& a, const Tile& T, int m, int k) {
  if (m >= T.Mc || k >= T.Kgc) return 0;
  if constexpr (MODE == FWD) {
    const int HoWo = a.Ho * a.Wo;
    const int n = m / HoWo, rem = m - n * HoWo, ho = rem / a.Wo, wo = rem - ho * a.Wo;
    const int c = k % a.C, rs = k / a.C, r = rs / a.S, s = rs - r * a.S;
    const int hi = ho * a.sh - a.ph + r * a.dh, wi = wo * a.sw - a.pw + s * a.dw;
    if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) return 0;
    return a.x[(((long)n * a.H + hi) * a.W + wi) * a.C + c];
  } else if constexpr (MODE == DGRAD) {
    const int c = T.cls;
    const int Hc = a.cls_Hc[c], Wc = a.cls_Wc[c];
    const int n = m / (Hc * Wc), rem = m - n * Hc * Wc, i = rem / Wc, j = rem - i * Wc;
    const int psh = a.dg_masked ? 1 : a.sh, psw = a.dg_masked ? 1 : a.sw;
    const int h = a.cls_a[c] + psh * i, w = a.cls_b[c] + psw * j;
    const int co = k % a.K, t = k / a.K, th = t / a.cls_Tw[c], tw = t - th * a.cls_Tw[c];
    const int rsh = a.dg_masked ? 1 : a.sh, rsw = a.dg_masked ? 1 : a.sw;
    const int r = a.cls_r0[c] + rsh * th, s = a.cls_s0[c] + rsw * tw;
    int nh = h + a.ph - r * a.dh, nw = w + a.pw - s * a.dw;
    if (nh < 0 || nw < 0) return 0;
    if (a.dg_masked && (nh % a.sh || nw % a.sw)) return 0;
    const int ho = nh / a.sh, wo = nw / a.sw;
    if (ho >= a.Ho || wo >= a.Wo) return 0;
    return a.dy[(((long)n * a.Ho + ho) * a.Wo + wo) * a.K + co];
  } else {  // WGRAD: A[m=co][k=p] = dy[p][co]
    return a.dy[(long)k * a.K + m];
  }
}

template <int MODE>
__device__ __forceinline__ bf16_t elemB(const ConvArgs& a, const Tile& T, int n, int k) {
  if (n >= a.Ng || k >= T.Kgc) return 0;
  if constexpr (MODE == FWD) {
    return a.w[(long)n * a.Kg + k];
  } else if constexpr (MODE == DGRAD) {  // B[n=ci][k=(t,co)] = w[co][r][s][ci]
    const int c = T.cls;
    const int co = k % a.K, t = k / a.K, th = t / a.cls_Tw[c], tw = t - th * a.cls_Tw[c];
    const int rsh = a.dg_masked ? 1 : a.sh, rsw = a.dg_masked ? 1 : a.sw;
    const int r = a.cls_r0[c] + rsh * th, s = a.cls_s0[c] + rsw * tw;
    return a.w[(((long)co * a.R + r) * a.S + s) * a.C + n];
  } else {  // WGRAD: B[n=(r,s,ci)][k=p] = x[n_img, ho*sh-ph+r*dh, wo*sw-pw+s*dw, ci]
    const int HoWo = a.Ho * a.Wo;
    const int ni = k / HoWo, rem = k - ni * HoWo, ho = rem / a.Wo, wo = rem - ho * a.Wo;
    const int ci = n % a.C, rs = n / a.C, r = rs / a.S, s = rs - r * a.S;
    const int hi = ho * a.sh - a.ph + r * a.dh, wi = wo * a.sw - a.pw + s * a.dw;
    if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) return 0;
    return a.x[(((long)ni * a.H + hi) * a.W + wi) * a.C + ci];
  }
}

// global output row for a tile-local row (DGRAD classes interleave into the NHWC dx)
template <int MODE>
__device__ __forceinline__ long out_row(const ConvArgs& a, const Tile& T, int m) {
  if constexpr (MODE == DGRAD) {
    const int c = T.cls;
    const int Hc = a.cls_Hc[c], Wc = a.cls_Wc[c];
    const int n = m / (Hc * Wc), rem = m - n * Hc * Wc, i = rem / Wc, j = rem - i * Wc;
    const int psh = a.dg_masked ? 1 : a.sh, psw = a.dg_masked ? 1 : a.sw;
    const int h = a.cls_a[c] + psh * i, w = a.cls_b[c] + psw * j;
    return ((long)n * a.H + h) * a.W + w;
  } else {
    return m;
  }
}

// magic-number divisors of the geometry (host side; every conv kernel's row / tap arithmetic)
inline void set_fastdivs(ConvArgs& a) {
  a.fd_sh = make_fastdiv((uint32_t)std::max(1, a.sh));
  a.fd_sw = make_fastdiv((uint32_t)std::max(1, a.sw));
  for (int c = 0; c < MAX_DG_CLASSES; ++c) {
    a.cls_fdHW[c] = make_fastdiv((uint32_t)std::max(1, a.cls_Hc[c] * a.cls_Wc[c]));
    a.cls_fdW[c] = make_fastdiv((uint32_t)std::max(1, a.cls_Wc[c]));
  }
  a.fd_HoWo = make_fastdiv((uint32_t)std::max(1, a.Ho * a.Wo));
  a.fd_Wo = make_fastdiv((uint32_t)std::max(1, a.Wo));
  a.fd_C = make_fastdiv((uint32_t)std::max(1, a.C));
  a.fd_S = make_fastdiv((uint32_t)std::max(1, a.S));
}

// out_row with the prepared fast divisions (set_fastdivs) and 32-bit arithmetic
template <int MODE>
__device__ __forceinline__ uint32_t out_row_fast(const ConvArgs& a, const Tile& T, int m) {
  if constexpr (MODE == DGRAD) {
    const int c = T.cls;
    const uint32_t Hc = a.cls_Hc[c], Wc = a.cls_Wc[c];
    const uint32_t n = fdiv((uint32_t)m, a.cls_fdHW[c]);
    const uint32_t rem = (uint32_t)m - n * Hc * Wc;
    const uint32_t i = fdiv(rem, a.cls_fdW[c]);
    const uint32_t j = rem - i * Wc;
    const uint32_t psh = a.dg_masked ? 1u : (uint32_t)a.sh, psw = a.dg_masked ? 1u : (uint32_t)a.sw;
    const uint32_t h = (uint32_t)a.cls_a[c] + psh * i;
    const uint32_t w = (uint32_t)a.cls_b[c] + psw * j;
    return (n * (uint32_t)a.H + h) * (uint32_t)a.W + w;
  } else {
    return (uint32_t)m;
  }
}

}  // namespace convk
}  // namespace tdl
