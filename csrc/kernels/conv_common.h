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

// u = relu(a·z + b) of 8 consecutive bf16 channels (a folded training BN + ReLU, ConvArgs::aff),
// bit-identical to bn.hip apply_vec: one fma per element, ReLU, round-to-nearest-even
__device__ __forceinline__ uint4 aff_relu8(uint4 z, const float (&ca)[8], const float (&cb)[8]) {
  const uint32_t w[4] = {z.x, z.y, z.z, z.w};
  uint32_t o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float lo = fmaf(__uint_as_float(w[j] << 16), ca[2 * j], cb[2 * j]);
    const float hi = fmaf(__uint_as_float(w[j] & 0xffff0000u), ca[2 * j + 1], cb[2 * j + 1]);
    o[j] = relu_pk_bf16(cvt_pk_bf16(lo, hi));
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// the 8 (a, b) coefficient pairs of channels c … c+7 (ConvArgs::aff rows, ld = aff_ld)
__device__ __forceinline__ void aff_load8(const float* aff, int ld, int c, float (&ca)[8],
                                          float (&cb)[8]) {
  const float4 a0 = *(const float4*)(aff + c), a1 = *(const float4*)(aff + c + 4);
  const float4 b0 = *(const float4*)(aff + ld + c), b1 = *(const float4*)(aff + ld + c + 4);
  ca[0] = a0.x; ca[1] = a0.y; ca[2] = a0.z; ca[3] = a0.w;
  ca[4] = a1.x; ca[5] = a1.y; ca[6] = a1.z; ca[7] = a1.w;
  cb[0] = b0.x; cb[1] = b0.y; cb[2] = b0.z; cb[3] = b0.w;
  cb[4] = b1.x; cb[5] = b1.y; cb[6] = b1.z; cb[7] = b1.w;
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

// COLG: column-grouped order (FWD always; DGRAD with fused BN statistics, single class): a
// workgroup's tiles share one column tile, so its statistics flush once
template <int MODE, int BM, int BN, int KS = BK, bool COLG = (MODE == FWD)>
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
  if constexpr (COLG) {
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
    const int psh = a.dg_masked ? 1 : a.esh, psw = a.dg_masked ? 1 : a.esw;
    const int h = a.cls_a[c] + psh * i, w = a.cls_b[c] + psw * j;
    return ((long)n * a.eH + h) * a.eW + w;
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
// DGM: the kernel may run dg_masked problems (the register-staged kernel; the LDS-DMA kernel
// never does, and the extra uniform select cost it a scratch spill)
template <int MODE, bool DGM = false>
__device__ __forceinline__ uint32_t out_row_fast(const ConvArgs& a, const Tile& T, int m) {
  if constexpr (MODE == DGRAD) {
    const int c = T.cls;
    const uint32_t Hc = a.cls_Hc[c], Wc = a.cls_Wc[c];
    const uint32_t n = fdiv((uint32_t)m, a.cls_fdHW[c]);
    const uint32_t rem = (uint32_t)m - n * Hc * Wc;
    const uint32_t i = fdiv(rem, a.cls_fdW[c]);
    const uint32_t j = rem - i * Wc;
    const uint32_t psh = DGM && a.dg_masked ? 1u : (uint32_t)a.esh;
    const uint32_t psw = DGM && a.dg_masked ? 1u : (uint32_t)a.esw;
    const uint32_t h = (uint32_t)a.cls_a[c] + psh * i;
    const uint32_t w = (uint32_t)a.cls_b[c] + psw * j;
    return (n * (uint32_t)a.eH + h) * (uint32_t)a.eW + w;
  } else {
    return (uint32_t)m;
  }
}

// ---------------------------------------------------------------------------------------------
// bf16 output tile epilogue of both conv kernels (FWD y / DGRAD dx): bias, the DGRAD residual
// join (dx += …) and ReLU bit mask, ReLU, BN Σ/Σ² of the stored values (FWD) or the BN-backward
// sums Σg, Σg·x (DGRAD, x = a.bn_x), 16-B stores.
// ---------------------------------------------------------------------------------------------
// lane holds C[m = bm0 + wm*TM + rm*16 + (lane&15)][n = bn0 + wn*TN + rn*16 + (lane>>4)*4 + i].
// SCALE: multiply by `scale` first (fp8 GEMMs: the per-tensor operand scales); `no_mem`: issue no
// loads / stores (timing ablation).
// NJ: compile-time "no residual join" (its previous-dx registers are not allocated)
// FRES (FWD): add the residual a.res (laid out like the output) before the ReLU — the
// DeepLab unit's relu(conv3 + bias + shortcut) in one pass (the statistics then are those of
// the next unit's pre-activation BN input)
// ROWS: the caller supplies each fragment's output-row byte offset in rows_in[] (ROW_OOB for
// lanes without an output pixel — conv_halo.hip's padded / tail lanes, whose accumulators hold
// values that must not reach memory or the statistics, so STATS then masks by row validity)
// AFM (DGRAD with STATS): the ReLU mask of a folded BN (ConvArgs::aff) — a·x + b > 0 of the BN
// input x the statistics load anyway
// DGRAD epilogue operands loaded ahead (epi_preload_dgrad): the BN input x of the statistics,
// the ReLU mask words and the previous dx of a join — issued before the tile's K loop so their
// latency hides under it (conv_halo.hip conv_rw_kernel)
// cache policy of the bf16 output-tile stores (buffer instruction aux bits: 2 = nt, streamed).
// Non-temporal measured 2 % slower on ResNet-50 and Xception-41: the next BN pass reads the output
// back soon after, partly from the caches (profiles/r06_epilogue_nt.txt)
#ifndef TDL_EPI_STORE_AUX
#define TDL_EPI_STORE_AUX 0
#endif
constexpr int kEpiStoreAux = TDL_EPI_STORE_AUX;

template <int RM, int RN>
struct EpiPre {
  v2u32 xv[RM][RN];
  uint32_t mrow[RM][2];
  v2u32 pv[RM][RN];
};

// the loads store_tile_bf16<DGRAD, …, ROWS> would issue, into `p` (same addressing)
template <int RM, int RN, int TN, bool STATS, bool NJ>
__device__ __forceinline__ void epi_preload_dgrad(const ConvArgs& a, const Tile& T, int wn,
                                                  int lane, rsrc_t rout, const uint32_t* rbase,
                                                  EpiPre<RM, RN>& p) {
  const int c0 = T.bn0 + wn * TN + (lane >> 4) * 4;
  const bool cols_ok = T.bn0 + wn * TN + TN <= a.Ng;
  if constexpr (STATS) {
    const rsrc_t rbx = make_rsrc(a.bn_x, a.out_bytes);
#pragma unroll
    for (int rm = 0; rm < RM; ++rm)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) {
        const bool cv = cols_ok || c0 + rn * 16 < a.Ng;
        p.xv[rm][rn] = __builtin_amdgcn_raw_buffer_load_b64(
            rbx, cv ? rbase[rm] + (uint32_t)(c0 + rn * 16) * 2u : ROW_OOB, 0, 0);
      }
  }
  if (a.mask) {
    const rsrc_t rmask = make_rsrc(a.mask, a.out_bytes / 16u);
#pragma unroll
    for (int rm = 0; rm < RM; ++rm) {
      const uint32_t boff = (rbase[rm] / 2u + (uint32_t)(T.bn0 + wn * TN)) >> 3;
      const uint32_t o = rbase[rm] != ROW_OOB ? boff : OOB;
      if constexpr (TN == 64) {
        const v2u32 m2 = __builtin_amdgcn_raw_buffer_load_b64(rmask, o, 0, 0);
        p.mrow[rm][0] = m2[0];
        p.mrow[rm][1] = m2[1];
      } else {
        static_assert(TN == 32, "mask slab of 4 or 8 bytes");
        p.mrow[rm][0] = __builtin_amdgcn_raw_buffer_load_b32(rmask, o, 0, 0);
        p.mrow[rm][1] = 0;
      }
    }
  }
  if constexpr (!NJ) {
    if (a.beta) {
#pragma unroll
      for (int rm = 0; rm < RM; ++rm)
#pragma unroll
        for (int rn = 0; rn < RN; ++rn) {
          const bool cv = cols_ok || c0 + rn * 16 < a.Ng;
          p.pv[rm][rn] = __builtin_amdgcn_raw_buffer_load_b64(
              rout, cv ? rbase[rm] + (uint32_t)(c0 + rn * 16) * 2u : ROW_OOB, 0, 0);
        }
    }
  }
}

template <int MODE, int RM, int RN, int TM, int TN, bool BIAS, bool STATS, bool SCALE, bool DGM = false,
          bool NJ = false, bool FRES = false, bool ROWS = false, bool AFM = false, bool PRE = false,
          int RG = RM>
__device__ __forceinline__ void store_tile_bf16(const ConvArgs& a, const Tile& T,
                                                const f32x4 (&acc)[RM][RN], int wm, int wn,
                                                int lane, rsrc_t rout, float scale, bool no_mem,
                                                float (&s_sum)[RN][4], float (&s_sq)[RN][4],
                                                const uint32_t* rows_in = nullptr,
                                                const EpiPre<RM, RN>* pre = nullptr) {
  static_assert(!PRE || (MODE == DGRAD && ROWS && !AFM), "preloaded operands: DGRAD, rows given");
  static_assert(RG >= 1 && RM % RG == 0, "fragment-row groups");
  // Row byte offsets are 32-bit with invalid rows pushed past the buffer (ROW_OOB): a
  // fragment's store offset is then row base + a compile-time constant.  Rows past the GEMM's
  // M hold zeros (their A rows were fetched out of range), so the statistics need no mask.
  uint32_t rbase[RM];
#pragma unroll
  for (int rm = 0; rm < RM; ++rm) {
    if constexpr (ROWS) {
      rbase[rm] = rows_in[rm];
    } else {
      const int m = T.bm0 + wm * TM + rm * 16 + (lane & 15);
      rbase[rm] = m < T.Mc ? out_row_fast<MODE, DGM>(a, T, m) * (uint32_t)a.ldc * 2u : ROW_OOB;
    }
  }
  const int c0 = T.bn0 + wn * TN + (lane >> 4) * 4;  // this lane's column in fragment rn = 0
  const bool cols_ok = T.bn0 + wn * TN + TN <= a.Ng;   // wave-uniform: no ragged columns
  // Per fragment: two v_cvt_pk_bf16_f32, the ReLU as one packed int16 max per pair (a bf16
  // is negative iff its int16 pattern is), one 16-B store per fragment pair.  The earlier
  // per-element epilogue (64-bit row math, integer divisions, per-fragment validity selects,
  // runtime mask / join / ReLU tests on every value) cost ≈1,200 VALU instructions per wave
  // per tile — at 4 cycles per wave64 VALU op that, not HBM, paced the 1–4-K-step tiles of
  // 1×1 convs (dev/tools/dgrad_ablate.py: 129 µs for a 1×1 dgrad with no memory traffic).
  v4u32 bias_v[RN];
  if constexpr (BIAS) {
    const rsrc_t rbias = make_rsrc(a.bias, (uint32_t)a.Ng * 4u);
#pragma unroll
    for (int rn = 0; rn < RN; ++rn) {
      const int n0 = c0 + rn * 16;
      bias_v[rn] = __builtin_amdgcn_raw_buffer_load_b128(rbias, n0 < a.Ng ? n0 * 4u : OOB, 0, 0);
    }
  }
  // DGRAD residual join (dx += this dgrad: the previous dx is read back) and ReLU bit mask
  // (pre-masked join: a row's TN mask bits of the wave's columns in one 4- / 8-byte load,
  // ldc % 64 == 0).  Every load is issued before any is used — one memory round trip per
  // tile; interleaved load → use made hipcc wait vmcnt(0) per fragment, draining the next
  // tile's in-flight operand DMA each time.
  bool join_prev = false, join_mask = false;
  if constexpr (MODE == DGRAD) {
    join_prev = !NJ && a.beta && !no_mem;
    join_mask = a.mask && !no_mem;
  } else if constexpr (MODE == FWD && FRES) {
    join_prev = !no_mem;
  }
  uint32_t mrow[RM][2];
  v2u32 pv[RM][RN];
  // DGRAD BN-backward statistics (STATS): the BN input x at the stored positions — Σg·x with g
  // the stored (masked) dx; the BN backward converts to Σg·x̂ (bn.hip, red_raw)
  v2u32 xv[RM][RN];
  // folded BN + ReLU of this dgrad's output (ConvArgs::aff): dx is masked by a·x + b > 0 of the
  // BN input x the statistics read anyway — no bit mask exists (ops/bnconv.py)
  constexpr bool aff_mask = AFM && MODE == DGRAD && STATS;
  v4u32 aff_a[aff_mask ? RN : 1], aff_b[aff_mask ? RN : 1];
  if constexpr (aff_mask) {
    {
      const rsrc_t raff = make_rsrc(a.aff, (uint32_t)a.aff_ld * 8u);
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) {
        const int n0 = c0 + rn * 16;
        aff_a[rn] = __builtin_amdgcn_raw_buffer_load_b128(raff, n0 < a.Ng ? n0 * 4u : OOB, 0, 0);
        aff_b[rn] = __builtin_amdgcn_raw_buffer_load_b128(
            raff, n0 < a.Ng ? (uint32_t)(a.aff_ld + n0) * 4u : OOB, 0, 0);
      }
    }
  }
  const bool relu = a.relu;
  const bool wide = cols_ok;
  // RG < RM: the epilogue operands are loaded and consumed RG fragment rows at a time (two
  // memory round trips instead of one, half the live operand registers — the 256×128 tiles'
  // statistics + join epilogue otherwise spills)
#pragma unroll
  for (int g0 = 0; g0 < RM; g0 += RG) {
    if constexpr (PRE) {
#pragma unroll
      for (int rm = g0; rm < g0 + RG; ++rm) {
        mrow[rm][0] = pre->mrow[rm][0];
        mrow[rm][1] = pre->mrow[rm][1];
#pragma unroll
        for (int rn = 0; rn < RN; ++rn) {
          if constexpr (STATS) xv[rm][rn] = pre->xv[rm][rn];
          if constexpr (!NJ) pv[rm][rn] = pre->pv[rm][rn];
        }
      }
    } else if constexpr (MODE == DGRAD && STATS) {
      const rsrc_t rbx = make_rsrc(a.bn_x, no_mem ? 0u : a.out_bytes);
#pragma unroll
      for (int rm = g0; rm < g0 + RG; ++rm)
#pragma unroll
        for (int rn = 0; rn < RN; ++rn) {
          const bool cv = cols_ok || c0 + rn * 16 < a.Ng;
          xv[rm][rn] = __builtin_amdgcn_raw_buffer_load_b64(
              rbx, cv ? rbase[rm] + (uint32_t)(c0 + rn * 16) * 2u : ROW_OOB, 0, 0);
        }
    }
    if constexpr (MODE == DGRAD && !PRE) {
      if (join_mask) {
        const rsrc_t rmask = make_rsrc(a.mask, a.out_bytes / 16u);
#pragma unroll
        for (int rm = g0; rm < g0 + RG; ++rm) {
          const uint32_t boff = (rbase[rm] / 2u + (uint32_t)(T.bn0 + wn * TN)) >> 3;
          const uint32_t o = rbase[rm] != ROW_OOB ? boff : OOB;
          if constexpr (TN == 64) {
            const v2u32 m2 = __builtin_amdgcn_raw_buffer_load_b64(rmask, o, 0, 0);
            mrow[rm][0] = m2[0];
            mrow[rm][1] = m2[1];
          } else {
            static_assert(TN == 32, "mask slab of 4 or 8 bytes");
            mrow[rm][0] = __builtin_amdgcn_raw_buffer_load_b32(rmask, o, 0, 0);
            mrow[rm][1] = 0;
          }
        }
      }
    }
    if constexpr (((MODE == DGRAD && !NJ) || (MODE == FWD && FRES)) && !PRE) {
      if (join_prev) {
        // DGRAD: the previous dx of the output buffer itself; FWD: the residual tensor
        const rsrc_t rprev = MODE == FWD ? make_rsrc(a.res, a.out_bytes) : rout;
#pragma unroll
        for (int rm = g0; rm < g0 + RG; ++rm)
#pragma unroll
          for (int rn = 0; rn < RN; ++rn) {
            const bool cv = cols_ok || c0 + rn * 16 < a.Ng;
            pv[rm][rn] = __builtin_amdgcn_raw_buffer_load_b64(
                rprev, cv ? rbase[rm] + (uint32_t)(c0 + rn * 16) * 2u : ROW_OOB, 0, 0);
          }
      }
    }
#pragma unroll
    for (int rm = g0; rm < g0 + RG; ++rm) {
      v2u32 pk[RN];
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) {
        f32x4 t = acc[rm][rn];
        if constexpr (SCALE) t = t * scale;
        if constexpr (BIAS) {
#pragma unroll
          for (int i = 0; i < 4; ++i) t[i] += __uint_as_float(bias_v[rn][i]);
        }
        if constexpr ((MODE == DGRAD && !NJ) || (MODE == FWD && FRES)) {
          if (join_prev) {
            t[0] += __uint_as_float(pv[rm][rn][0] << 16);
            t[1] += __uint_as_float(pv[rm][rn][0] & 0xffff0000u);
            t[2] += __uint_as_float(pv[rm][rn][1] << 16);
            t[3] += __uint_as_float(pv[rm][rn][1] & 0xffff0000u);
          }
        }
        if constexpr (MODE == DGRAD) {
          if (join_mask) {
            // bit (rn·16 + group·4 + i) of the wave's TN-column slab; v_bfe_i32 → 0 / ~0
            const int sh = (rn & 1) * 16 + (lane >> 4) * 4;
            const uint32_t w = mrow[rm][rn >> 1];
#pragma unroll
            for (int i = 0; i < 4; ++i)
              t[i] = __uint_as_float(__float_as_uint(t[i]) &
                                     (uint32_t)__builtin_amdgcn_sbfe((int)w, sh + i, 1));
          }
        }
        if constexpr (aff_mask) {
          {
            const float z[4] = {__uint_as_float(xv[rm][rn][0] << 16),
                                __uint_as_float(xv[rm][rn][0] & 0xffff0000u),
                                __uint_as_float(xv[rm][rn][1] << 16),
                                __uint_as_float(xv[rm][rn][1] & 0xffff0000u)};
#pragma unroll
            for (int i = 0; i < 4; ++i)
              t[i] = fmaf(z[i], __uint_as_float(aff_a[rn][i]), __uint_as_float(aff_b[rn][i])) > 0.f
                         ? t[i] : 0.f;
          }
        }
        pk[rn][0] = cvt_pk_bf16(t[0], t[1]);
        pk[rn][1] = cvt_pk_bf16(t[2], t[3]);
        if (relu) {
          pk[rn][0] = relu_pk_bf16(pk[rn][0]);
          pk[rn][1] = relu_pk_bf16(pk[rn][1]);
        }
        // ragged column tiles: columns ≥ Ng hold zeros (B rows fetched out of range) and must
        // not be stored (they would land in the next row)
        const bool cv = cols_ok || c0 + rn * 16 < a.Ng;
        if (!no_mem && !wide)
          __builtin_amdgcn_raw_buffer_store_b64(pk[rn], rout, cv ? rbase[rm] + (uint32_t)(c0 + rn * 16) * 2u : ROW_OOB, 0, kEpiStoreAux);
        if constexpr (STATS && MODE == DGRAD) {
          // (Σg, Σg·x) of the stored bf16 g; rows past M store zeros (x reads there return 0)
          const float rg = (!ROWS || rbase[rm] != ROW_OOB) ? 1.f : 0.f;
          const float v0 = __uint_as_float(pk[rn][0] << 16) * rg, v1 = __uint_as_float(pk[rn][0] & 0xffff0000u) * rg;
          const float v2 = __uint_as_float(pk[rn][1] << 16) * rg, v3 = __uint_as_float(pk[rn][1] & 0xffff0000u) * rg;
          s_sum[rn][0] += v0; s_sum[rn][1] += v1; s_sum[rn][2] += v2; s_sum[rn][3] += v3;
          s_sq[rn][0] = fmaf(v0, __uint_as_float(xv[rm][rn][0] << 16), s_sq[rn][0]);
          s_sq[rn][1] = fmaf(v1, __uint_as_float(xv[rm][rn][0] & 0xffff0000u), s_sq[rn][1]);
          s_sq[rn][2] = fmaf(v2, __uint_as_float(xv[rm][rn][1] << 16), s_sq[rn][2]);
          s_sq[rn][3] = fmaf(v3, __uint_as_float(xv[rm][rn][1] & 0xffff0000u), s_sq[rn][3]);
        } else if constexpr (STATS) {
          // statistics of the stored bf16 values; rows past M are zero unless a bias was added
          const float rv = (!(BIAS || ROWS) || rbase[rm] != ROW_OOB) ? 1.f : 0.f;
          const float v0 = __uint_as_float(pk[rn][0] << 16) * rv, v1 = __uint_as_float(pk[rn][0] & 0xffff0000u) * rv;
          const float v2 = __uint_as_float(pk[rn][1] << 16) * rv, v3 = __uint_as_float(pk[rn][1] & 0xffff0000u) * rv;
          s_sum[rn][0] += v0; s_sum[rn][1] += v1; s_sum[rn][2] += v2; s_sum[rn][3] += v3;
          s_sq[rn][0] = fmaf(v0, v0, s_sq[rn][0]);
          s_sq[rn][1] = fmaf(v1, v1, s_sq[rn][1]);
          s_sq[rn][2] = fmaf(v2, v2, s_sq[rn][2]);
          s_sq[rn][3] = fmaf(v3, v3, s_sq[rn][3]);
        }
      }
      if (!no_mem && wide) {
        // 16-B stores: v_permlane16_swap trades the odd 16-lane rows of fragment p with the
        // even rows of fragment p+1, so lanes l and l^16 (column groups 2j, 2j+1 of one row)
        // each end up with 8 consecutive columns — even lanes of block p, odd lanes of block
        // p+1 — and an instruction writes 16 rows × 64 B instead of 16 rows × 32 B (half the
        // write requests: −20 % on the 1×1 dgrads, profiles/r02_dgrad_ablation.txt)
        const int g = lane >> 4;
        const uint32_t lcol = (uint32_t)(T.bn0 + wn * TN + (g & 1) * 16 + (g & ~1) * 4) * 2u;
#pragma unroll
        for (int p = 0; p < RN; p += 2) {
          const auto s0 = __builtin_amdgcn_permlane16_swap(pk[p][0], pk[p + 1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pk[p][1], pk[p + 1][1], false, false);
          v4u32 q;
          q[0] = s0[0]; q[1] = s1[0]; q[2] = s0[1]; q[3] = s1[1];
          __builtin_amdgcn_raw_buffer_store_b128(q, rout, rbase[rm] + lcol + (uint32_t)p * 32u, 0, kEpiStoreAux);
        }
      }
    }

  }
}

}  // namespace convk
}  // namespace tdl
