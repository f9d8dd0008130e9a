// MFMA implicit-GEMM convolution for gfx950 (MI355X / CDNA4), NHWC activations, KRSC weights, bf16
// operands, fp32 accumulation.
//
// One kernel template serves the three convolution GEMMs:
//
//   mode   GEMM C[M][N] = Σ_k A[m][k]·B[n][k]                A operand            B operand
//   FWD    y[m=(n,ho,wo)][co]    k = (r,s,ci)   M=N·Ho·Wo     x gathered (k-contig) w[co][k] (k-contig)
//   DGRAD  dx[m=(n,h,w)][ci]     k = (t,co)     per class     dy gathered (k-contig) w[co][r][s][ci] (n-contig)
//   WGRAD  dw[m=co][n=(r,s,ci)]  k = (n,ho,wo)  split-K       dy[p][co] (m-contig)   x gathered (n-contig)
//
// DGRAD parity classes: for stride s the input pixels split into s_h·s_w classes (h mod s_h,
// w mod s_w); inside a class exactly the taps r ≡ (h+pad) (mod s) contribute, and
// ho = (h + pad − r)/s is exact — so a strided dgrad is s² dense sub-GEMMs with no masked-out
// work (a 3×3/s2 dgrad does the FLOPs of the forward, not 4× that; a 1×1/s2 dgrad writes zeros
// for 3 of 4 classes).  Stride 1 is the single-class case (dilation allowed).
//
// Operands whose 16-B global vectors run along K ("KC") are staged into an LDS image
// [rows][64] (128-B rows, 16-B chunk index XOR ((row>>1)&7): conflict-free ds_read_b128 for the
// 16x16x32 fragment pattern).  Operands whose vectors run along M/N ("MC", i.e. K is strided in
// memory) are staged as [64 k-rows][cols] (32-B pair index XOR f(k)) and read with gfx950's
// ds_read_b64_tr_b16 hardware transpose, so dgrad needs no weight transpose and wgrad no
// activation transpose.  Staging is register double-buffered.
//
// Scheduling: a workgroup walks `tpb` consecutive output tiles as ONE flat sequence of 64-deep
// K steps; the global→VGPR loads of step s+1 (possibly the first step of the next tile) are in
// flight while the MFMAs of step s run, so small-K (1×1, Cin ≤ 128) convs are not serialised on
// per-tile load latency.  Workgroup ids are remapped so each XCD owns a contiguous tile range.
//
// Tile: BM×BN×64 per 256-thread workgroup, 2×2 waves, v_mfma_f32_16x16x32_bf16, operands swapped
// (D = Bᵀ·Aᵀ) so each lane holds 4 consecutive output channels of one output row → 8-B bf16 /
// 16-B fp32 vector stores.  Epilogue: bias, ReLU, and per-channel Σy / Σy² of the stored bf16
// values (BatchNorm statistics) reduced lanes → waves (LDS) → one contiguous atomic row per tile.
#include "conv_common.h"
#include "conv_route.h"
#include <stdexcept>
#include <string>

namespace tdl {

namespace {

constexpr int NT = 256;
using namespace convk;

// ---------------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------------
// AFF (aligned FWD / WGRAD): the input x is u = relu(a·x + b) of a folded training BN
// (ConvArgs::aff) — applied to the staged registers before the LDS store; loads that fell in the
// padding / past M or K (validity bit 0) stay 0
template <int MODE, int BM, int BN, bool ALIGNED, bool STATS, bool BIAS, bool AFF = false>
__global__ void __launch_bounds__(NT, 2) conv_gemm_kernel(ConvArgs a) {
  static_assert(!AFF || (ALIGNED && MODE != DGRAD), "folded BN: aligned FWD / WGRAD only");
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM, TN = BN / WN, RM = TM / 16, RN = TN / 16;
  constexpr bool A_MC = (MODE == WGRAD), B_MC = (MODE != FWD);
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PA = BM * BK / 8 / NT, PB = BN * BK / 8 / NT;
  constexpr int A_CPR = BM / 8, B_CPR = BN / 8;  // MC: 16-B chunks per k-row
  constexpr int RED_BYTES = STATS ? 2 * WM * BN * 4 : 0;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + RED_BYTES + 16];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_begin = blk * a.tpb;
  const int tile_end = min(a.cls_tile0[a.ncls], tile_begin + a.tpb);
  if (tile_begin >= tile_end) return;
  const int HoWo = a.Ho * a.Wo;
  const rsrc_t rx = make_rsrc(a.x, a.x_bytes);
  const rsrc_t rw = make_rsrc(a.w, a.w_bytes);
  const rsrc_t rdy = make_rsrc(a.dy, a.dy_bytes);
  const rsrc_t rout = make_rsrc(a.out, a.out_bytes);

  // ---------------- load-side per-tile state (aligned path) ----------------
  int a_base[PA];
  int a_p0[PA], a_p1[PA];
  int b_base[PB];
  int b_ok[PB];
  int a_fix = 0, b_fix = 0, b_fix2 = 0, b_fix3 = 0;
  float aff_a[8], aff_b[8];  // AFF: coefficients of this lane's 8 channels
  uint32_t aff_v = 0;        // AFF: validity bit per staged load of the folded operand

  auto prep_tile = [&](const Tile& T) {
    if constexpr (!ALIGNED) return;
    if constexpr (MODE == FWD) {
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int m = T.bm0 + (tid >> 3) + i * (NT / 8);
        if (m < T.Mc) {
          const int n = (int)fdiv((uint32_t)m, a.fd_HoWo), rem = m - n * HoWo;
          const int ho = (int)fdiv((uint32_t)rem, a.fd_Wo), wo = rem - ho * a.Wo;
          a_base[i] = n * a.H * a.W * a.C;
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
        const int n = T.bn0 + (tid >> 3) + i * (NT / 8);
        b_base[i] = n * a.Kg;
        b_ok[i] = n < a.Ng;
      }
    } else if constexpr (MODE == DGRAD) {
      const int c = T.cls;
      const int Hc = a.cls_Hc[c], Wc = a.cls_Wc[c], HWc = Hc * Wc;
      const int ca = a.cls_a[c], cb = a.cls_b[c], r0 = a.cls_r0[c], s0 = a.cls_s0[c];
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int m = T.bm0 + (tid >> 3) + i * (NT / 8);
        if (m < T.Mc) {
          const int n = m / HWc, rem = m - n * HWc, ii = rem / Wc, jj = rem - ii * Wc;
          const int h = ca + a.sh * ii, w = cb + a.sw * jj;
          a_base[i] = n * HoWo * a.K;
          // ho = (h + ph - r0·dh)/sh − th·step (exact for the class)
          a_p0[i] = (h + a.ph - r0 * a.dh) / a.sh;
          a_p1[i] = (w + a.pw - s0 * a.dw) / a.sw;
        } else {
          a_base[i] = 0;
          a_p0[i] = -(1 << 28);
          a_p1[i] = -(1 << 28);
        }
      }
      b_fix = T.bn0 + (tid % B_CPR) * 8;  // ci
    } else {  // WGRAD
      a_fix = T.bm0 + (tid % A_CPR) * 8;  // co
      const int nn = T.bn0 + (tid % B_CPR) * 8;
      if (nn < a.Ng) {
        const int rs = (int)fdiv((uint32_t)nn, a.fd_C), ci = nn - rs * a.C;
        const int r = (int)fdiv((uint32_t)rs, a.fd_S), s = rs - r * a.S;
        b_fix = ci;
        b_fix2 = r * a.dh - a.ph;
        b_fix3 = s * a.dw - a.pw;
        if constexpr (AFF) aff_load8(a.aff, a.aff_ld, ci, aff_a, aff_b);
      } else {
        b_fix = -1;
        b_fix2 = -(1 << 28);
        b_fix3 = 0;
      }
    }
  };

  uint4 ra[PA], rb[PB];

  auto load_step = [&](const Tile& T, int kt) {
    if constexpr (ALIGNED) {
      if constexpr (MODE == FWD) {
        const int k = kt * BK + (tid & 7) * 8;
        const bool kv = k < a.Kg;
        const int rs = (int)fdiv((uint32_t)k, a.fd_C), c = k - rs * a.C;
        const int r = (int)fdiv((uint32_t)rs, a.fd_S), s = rs - r * a.S;
        const int ro = r * a.dh, so = s * a.dw;
        if constexpr (AFF) {
          aff_load8(a.aff, a.aff_ld, kv ? c : 0, aff_a, aff_b);
          aff_v = 0;
        }
#pragma unroll
        for (int i = 0; i < PA; ++i) {
          const int hi = a_p0[i] + ro, wi = a_p1[i] + so;
          const bool v = kv && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
          const uint32_t off = (uint32_t)(a_base[i] + (hi * a.W + wi) * a.C + c) * 2u;
          ra[i] = bload16(rx, v ? off : OOB);
          if constexpr (AFF) aff_v |= (v ? 1u : 0u) << i;
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) {
          const bool v = kv && b_ok[i];
          rb[i] = bload16(rw, v ? (uint32_t)(b_base[i] + k) * 2u : OOB);
        }
      } else if constexpr (MODE == DGRAD) {
        const int c = T.cls;
        const int Tw = a.cls_Tw[c];
        const int step_h = a.sh == 1 ? a.dh : 1, step_w = a.sw == 1 ? a.dw : 1;
        const int k = kt * BK + (tid & 7) * 8;
        const bool kv = k < T.Kgc;
        const int co = k % a.K, t = k / a.K, th = t / Tw, tw = t - th * Tw;
        const int ro = th * step_h, so = tw * step_w;
#pragma unroll
        for (int i = 0; i < PA; ++i) {
          const int ho = a_p0[i] - ro, wo = a_p1[i] - so;
          const bool v = kv && (unsigned)ho < (unsigned)a.Ho && (unsigned)wo < (unsigned)a.Wo;
          const uint32_t off = (uint32_t)(a_base[i] + (ho * a.Wo + wo) * a.K + co) * 2u;
          ra[i] = bload16(rdy, v ? off : OOB);
        }
        const int r0 = a.cls_r0[c], s0 = a.cls_s0[c];
#pragma unroll
        for (int i = 0; i < PB; ++i) {
          const int kk = kt * BK + tid / B_CPR + i * (NT / B_CPR);
          const bool v = kk < T.Kgc && b_fix < a.Ng;
          const int co2 = kk % a.K, t2 = kk / a.K, th2 = t2 / Tw, tw2 = t2 - th2 * Tw;
          const int r = r0 + a.sh * th2, s = s0 + a.sw * tw2;
          const uint32_t off = (uint32_t)(((co2 * a.R + r) * a.S + s) * a.C + b_fix) * 2u;
          rb[i] = bload16(rw, v ? off : OOB);
        }
      } else {  // WGRAD
        if constexpr (AFF) aff_v = 0;
#pragma unroll
        for (int i = 0; i < PA; ++i) {
          const int p = kt * BK + tid / A_CPR + i * (NT / A_CPR);
          const bool v = p < a.Kg && a_fix < a.M;
          ra[i] = bload16(rdy, v ? (uint32_t)(p * a.K + a_fix) * 2u : OOB);
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) {
          const int p = kt * BK + tid / B_CPR + i * (NT / B_CPR);
          // magic-number divisions (set_fastdivs): `/` by a runtime divisor costs ~40 VALU each,
          // twice per load, in the K-step loop
          const int ni = (int)fdiv((uint32_t)p, a.fd_HoWo), rem = p - ni * HoWo;
          const int ho = (int)fdiv((uint32_t)rem, a.fd_Wo), wo = rem - ho * a.Wo;
          const int hi = ho * a.sh + b_fix2, wi = wo * a.sw + b_fix3;
          const bool v = p < a.Kg && b_fix >= 0 && (unsigned)hi < (unsigned)a.H &&
                         (unsigned)wi < (unsigned)a.W;
          const uint32_t off = (uint32_t)(((ni * a.H + hi) * a.W + wi) * a.C + b_fix) * 2u;
          rb[i] = bload16(rx, v ? off : OOB);
          if constexpr (AFF) aff_v |= (v ? 1u : 0u) << i;
        }
      }
    } else {
      // generic element path
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        bf16_t e[8];
        if constexpr (!A_MC) {
          const int m = T.bm0 + (tid >> 3) + i * (NT / 8);
          const int k = kt * BK + (tid & 7) * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = elemA<MODE>(a, T, m, k + j);
        } else {
          const int k = kt * BK + tid / A_CPR + i * (NT / A_CPR);
          const int m = T.bm0 + (tid % A_CPR) * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = elemA<MODE>(a, T, m + j, k);
        }
        ra[i] = gather8(e);
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        bf16_t e[8];
        if constexpr (!B_MC) {
          const int n = T.bn0 + (tid >> 3) + i * (NT / 8);
          const int k = kt * BK + (tid & 7) * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = elemB<MODE>(a, T, n, k + j);
        } else {
          const int k = kt * BK + tid / B_CPR + i * (NT / B_CPR);
          const int n = T.bn0 + (tid % B_CPR) * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = elemB<MODE>(a, T, n + j, k);
        }
        rb[i] = gather8(e);
      }
    }
  };

  auto store_step = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
    if constexpr (AFF) {  // the folded BN + ReLU, on the data that has arrived by now
      const uint4 zero = make_uint4(0, 0, 0, 0);
      if constexpr (MODE == FWD) {
#pragma unroll
        for (int i = 0; i < PA; ++i) ra[i] = (aff_v >> i) & 1u ? aff_relu8(ra[i], aff_a, aff_b) : zero;
      } else {
#pragma unroll
        for (int i = 0; i < PB; ++i) rb[i] = (aff_v >> i) & 1u ? aff_relu8(rb[i], aff_a, aff_b) : zero;
      }
    }
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
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  auto compute_step = [&](int buf) {
    const char* As = smem + buf * STAGE;
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
  };

  // per-lane BN statistics, accumulated over all tiles of the workgroup (they share bn0)
  float s_sum[RN][4], s_sq[RN][4];
#pragma unroll
  for (int rn = 0; rn < RN; ++rn)
#pragma unroll
    for (int i = 0; i < 4; ++i) s_sum[rn][i] = s_sq[rn][i] = 0.f;

  // lane holds C[m = bm0 + wm*TM + rm*16 + (lane&15)][n = bn0 + wn*TN + rn*16 + (lane>>4)*4 + i]
  //
  // bf16 epilogue for vector-aligned outputs (Ng, ldc % 4 == 0): the shared lean form
  // (conv_common.h store_tile_bf16)
  auto lean_epilogue = [&](const Tile& T) {
    store_tile_bf16<MODE, RM, RN, TM, TN, BIAS, STATS, false, true>(a, T, acc, wm, wn, lane, rout, 1.f,
                                                             false, s_sum, s_sq);
  };

  auto epilogue = [&](const Tile& T) {
    if constexpr (MODE == WGRAD) {
      if ((a.Ng & 3) == 0) {
        const uint32_t slab0 = (uint32_t)T.split * (uint32_t)(a.M * a.Ng);
#pragma unroll
        for (int rm = 0; rm < RM; ++rm) {
          const int m = T.bm0 + wm * TM + rm * 16 + (lane & 15);
#pragma unroll
          for (int rn = 0; rn < RN; ++rn) {
            const int n0 = T.bn0 + wn * TN + rn * 16 + (lane >> 4) * 4;
            const bool v = m < a.M && n0 < a.Ng;
            const uint32_t off = (slab0 + (uint32_t)(m * a.Ng + n0)) * 4u;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, acc[rm][rn]), rout,
                                                   v ? off : OOB, 0, 0);
          }
        }
      } else {
        float* out = (float*)a.out + (long)T.split * a.M * a.Ng;
#pragma unroll
        for (int rm = 0; rm < RM; ++rm) {
          const int m = T.bm0 + wm * TM + rm * 16 + (lane & 15);
          if (m >= a.M) continue;
#pragma unroll
          for (int rn = 0; rn < RN; ++rn) {
            const int n0 = T.bn0 + wn * TN + rn * 16 + (lane >> 4) * 4;
            float* p = out + (long)m * a.Ng + n0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (n0 + i < a.Ng) p[i] = acc[rm][rn][i];
          }
        }
      }
    } else {
      bf16_t* out = (bf16_t*)a.out;
      const bool fast = ((a.Ng & 3) == 0) && ((a.ldc & 3) == 0);
      if (fast && !(a.dbg & 1024)) {  // (dbg 1024: the per-element path, for A/B timing)
        lean_epilogue(T);
        return;
      }
      const rsrc_t rbias = make_rsrc(a.bias, a.bias ? (uint32_t)a.Ng * 4u : 0u);
      const rsrc_t rmask = make_rsrc(a.mask, a.mask ? a.out_bytes / 16u : 0u);
      // Phase 1 (fast layout): every epilogue load — bias, the DGRAD join's previous dx, the
      // ReLU mask — is issued before any is used (one memory round trip per tile instead of a
      // vmcnt(0) drain per fragment; see conv_glds.hip)
      long orows[RM];
      bool mvs[RM];
#pragma unroll
      for (int rm = 0; rm < RM; ++rm) {
        const int m = T.bm0 + wm * TM + rm * 16 + (lane & 15);
        mvs[rm] = m < T.Mc;
        orows[rm] = mvs[rm] ? out_row<MODE>(a, T, m) : 0;
      }
      v4u32 bias_v[RN];
      if constexpr (BIAS) {
        if (fast) {
#pragma unroll
          for (int rn = 0; rn < RN; ++rn) {
            const int n0 = T.bn0 + wn * TN + rn * 16 + (lane >> 4) * 4;
            bias_v[rn] = __builtin_amdgcn_raw_buffer_load_b128(rbias, n0 < a.Ng ? n0 * 4u : OOB, 0, 0);
          }
        }
      }
      uint64_t mrows[RM];
      v2u32 pvs[RM][RN];
#pragma unroll
      for (int rm = 0; rm < RM; ++rm) {
        mrows[rm] = ~0ull;
        if constexpr (MODE == DGRAD) {
          // DGRAD ReLU mask (pre-masked join): a row's TN mask bits of the wave's columns in one
          // 4- / 8-byte load (ldc % 64 == 0: byte-aligned slab), reused by every rn fragment
          if (a.mask) {
            const uint32_t boff = (uint32_t)((orows[rm] * a.ldc + T.bn0 + wn * TN) >> 3);
            if constexpr (TN == 64) {
              const v2u32 mv2 = __builtin_amdgcn_raw_buffer_load_b64(rmask, mvs[rm] ? boff : OOB, 0, 0);
              mrows[rm] = (uint64_t)mv2[0] | ((uint64_t)mv2[1] << 32);
            } else {
              static_assert(TN == 32, "mask slab of 4 or 8 bytes");
              mrows[rm] = __builtin_amdgcn_raw_buffer_load_b32(rmask, mvs[rm] ? boff : OOB, 0, 0);
            }
          }
          if (a.beta && fast) {  // residual-gradient join: dx += this conv's dgrad
#pragma unroll
            for (int rn = 0; rn < RN; ++rn) {
              const int n0 = T.bn0 + wn * TN + rn * 16 + (lane >> 4) * 4;
              const uint32_t poff = (uint32_t)(orows[rm] * a.ldc + n0) * 2u;
              pvs[rm][rn] = __builtin_amdgcn_raw_buffer_load_b64(rout, (mvs[rm] && n0 < a.Ng) ? poff : OOB, 0, 0);
            }
          }
        }
      }
      // Phase 2: combine and store
#pragma unroll
      for (int rm = 0; rm < RM; ++rm) {
        const bool mv = mvs[rm];
        const long orow = orows[rm];
        const uint64_t mrow = mrows[rm];
#pragma unroll
        for (int rn = 0; rn < RN; ++rn) {
          const int n0 = T.bn0 + wn * TN + rn * 16 + (lane >> 4) * 4;
          float bv[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (BIAS) {
            if (fast) {
#pragma unroll
              for (int i = 0; i < 4; ++i) bv[i] = __uint_as_float(bias_v[rn][i]);
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i) bv[i] = (n0 + i < a.Ng) ? a.bias[n0 + i] : 0.f;
            }
          }
          float v[4];
          bf16_t h[4];
          float prev[4] = {0.f, 0.f, 0.f, 0.f};
          uint32_t mbits = 0xFu;
          if constexpr (MODE == DGRAD) {
            if (a.mask) mbits = (uint32_t)(mrow >> (rn * 16 + (lane >> 4) * 4)) & 0xFu;
            if (a.beta) {  // residual-gradient join: dx += this conv's dgrad
              if (fast) {
                const v2u32 pv = pvs[rm][rn];
                prev[0] = __uint_as_float(pv[0] << 16);
                prev[1] = __uint_as_float(pv[0] & 0xffff0000u);
                prev[2] = __uint_as_float(pv[1] << 16);
                prev[3] = __uint_as_float(pv[1] & 0xffff0000u);
              } else if (mv) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                  prev[i] = (n0 + i < a.Ng) ? bf2f(out[orow * a.ldc + n0 + i]) : 0.f;
              }
            }
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float t = acc[rm][rn][i] + bv[i] + prev[i];
            if (!((mbits >> i) & 1u)) t = 0.f;
            if (a.relu) t = fmaxf(t, 0.f);
            h[i] = f2bf(t);
            v[i] = bf2f(h[i]);
          }
          if (fast) {
            const bool v_ok = mv && n0 < a.Ng;
            const uint32_t off = (uint32_t)(orow * a.ldc + n0) * 2u;
            v2u32 pk;
            pk[0] = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
            pk[1] = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
            __builtin_amdgcn_raw_buffer_store_b64(pk, rout, v_ok ? off : OOB, 0, 0);
            if constexpr (STATS) {
              const float msk = v_ok ? 1.f : 0.f;
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                s_sum[rn][i] += msk * v[i];
                s_sq[rn][i] += msk * v[i] * v[i];
              }
            }
          } else if (mv) {
            bf16_t* p = out + orow * a.ldc + n0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (n0 + i < a.Ng) p[i] = h[i];
            if constexpr (STATS) {
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const float msk = (n0 + i < a.Ng) ? 1.f : 0.f;
                s_sum[rn][i] += msk * v[i];
                s_sq[rn][i] += msk * v[i] * v[i];
              }
            }
          }
        }
      }
    }
  };

  auto flush_stats = [&](int bn0) {
    if constexpr (STATS && MODE != WGRAD) {
      const int nb = bn0;
      {
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
        float* red = (float*)(smem + 2 * STAGE);  // dedicated region (staging may be in flight)
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
          const int n = nb + nl;
          if (n < a.Ng) {
            float v = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) v += red[(w * 2 + which) * BN + nl];
            atomicAdd(a.stats + which * a.Ng + n, v);
          }
        }
      }
    }
  };

  // ---------------- flat (tile, k-step) pipeline ----------------
  int lt = tile_begin;             // load cursor
  Tile LT = tile_of<MODE, BM, BN>(a, lt);
  int lkt = LT.kt0;
  prep_tile(LT);
  Tile CT = LT;                    // compute cursor
  int ckt = lkt;
  zero_acc();
  load_step(LT, lkt);
  store_step(0);
  __syncthreads();
  int buf = 0;
  for (;;) {
    // advance the load cursor
    bool more = true;
    if (lkt + 1 < LT.kt1) {
      ++lkt;
    } else if (lt + 1 < tile_end) {
      ++lt;
      LT = tile_of<MODE, BM, BN>(a, lt);
      lkt = LT.kt0;
      prep_tile(LT);
    } else {
      more = false;
    }
    if (more) load_step(LT, lkt);
    compute_step(buf);
    if (ckt + 1 >= CT.kt1) {
      epilogue(CT);
      zero_acc();
      if (more) {
        CT = LT;   // next computed step is the first step of the (just loaded) next tile
        ckt = lkt;
      }
    } else {
      ++ckt;
    }
    if (!more) break;
    store_step(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  flush_stats(CT.bn0);
}

// fp32 split-K slab reduction: out[i] (+)= Σ_z slab[z][i].  2-D parallel: each workgroup owns
// PPB float4 positions × G split groups (G = 256/PPB), partial sums combined through LDS.
template <int G>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ slab,
                                                            float* __restrict__ out, long n,
                                                            int splits, int accumulate) {
  constexpr int PPB = 256 / G;
  __shared__ float4 part[G][PPB];
  const int pl = threadIdx.x % PPB, g = threadIdx.x / PPB;
  const long n4 = n / 4;
  const long i = blockIdx.x * (long)PPB + pl;
  float4 s = make_float4(0, 0, 0, 0);
  if (i < n4) {
    for (int z = g; z < splits; z += G) {
      const float4 v = ((const float4*)(slab + (long)z * n))[i];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  part[g][pl] = s;
  __syncthreads();
  if (g == 0 && i < n4) {
    float4 t = accumulate ? ((const float4*)out)[i] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < G; ++q) {
      t.x += part[q][pl].x;
      t.y += part[q][pl].y;
      t.z += part[q][pl].z;
      t.w += part[q][pl].w;
    }
    ((float4*)out)[i] = t;
  }
  // scalar tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long j = n4 * 4 + threadIdx.x;
    float t = accumulate ? out[j] : 0.f;
    for (int z = 0; z < splits; ++z) t += slab[(long)z * n + j];
    out[j] = t;
  }
}

// Bias gradient = column sums of a bf16 [P][K] matrix, in two deterministic launches without
// atomics or a memset: colsum_part_kernel writes one fp32 partial row per row-block into a slab,
// colsum_reduce_kernel sums the slab rows into out (overwrite, or accumulate).  Vector path
// (K % 8 == 0): a lane owns 8 channels (one 16-B load per row, 4 rows in flight), the 4 waves of
// a workgroup stride the rows and meet in LDS.
template <bool VEC>
__global__ void __launch_bounds__(256) colsum_part_kernel(const bf16_t* __restrict__ x,
                                                         float* __restrict__ part, long P, int K,
                                                         long rows_per_block) {
  __shared__ float red[4][8][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long r0 = blockIdx.x * rows_per_block, r1 = min(P, r0 + rows_per_block);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if constexpr (VEC) {
    const int cv = blockIdx.y * 64 + lane;  // channel vector
    if (cv < (K >> 3)) {
      const bf16_t* base = x + cv * 8;
      long r = r0 + w;
      for (; r + 12 < r1; r += 16) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *(const uint4*)(base + (r + 4 * u) * K);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float f[8];
          unpack8(v[u], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] += f[j];
        }
      }
      for (; r < r1; r += 4) {
        float f[8];
        unpack8(*(const uint4*)(base + r * K), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
      }
    }
  } else {
    const int c = blockIdx.y * 64 + lane;  // one channel per lane
    if (c < K)
      for (long r = r0 + w; r < r1; r += 4) s[0] += bf2f(x[r * K + c]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[w][j][lane] = s[j];
  __syncthreads();
  if (w == 0) {
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = red[0][j][lane] + red[1][j][lane] + red[2][j][lane] + red[3][j][lane];
    float* dst = part + blockIdx.x * (long)K;
    if constexpr (VEC) {
      const int cv = blockIdx.y * 64 + lane;
      if (cv < (K >> 3)) {
        *(float4*)(dst + cv * 8) = make_float4(t[0], t[1], t[2], t[3]);
        *(float4*)(dst + cv * 8 + 4) = make_float4(t[4], t[5], t[6], t[7]);
      }
    } else {
      const int c = blockIdx.y * 64 + lane;
      if (c < K) dst[c] = t[0];
    }
  }
}

// out[c] (+)= Σ_b part[b][c]: 64 channels per workgroup, the 4 waves split the partial rows
__global__ void __launch_bounds__(256) colsum_reduce_kernel(const float* __restrict__ part,
                                                           float* __restrict__ out, int nb, int K,
                                                           int accumulate) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float t = 0.f;
  if (c < K)
    for (int b = w; b < nb; b += 4) t += part[(long)b * K + c];
  red[w][lane] = t;
  __syncthreads();
  if (w == 0 && c < K) {
    const float s = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    out[c] = accumulate ? out[c] + s : s;
  }
}

template <int MODE, int BM, int BN, bool AL, bool ST, bool BI, bool AF = false>
void launch_t(const ConvArgs& a, int blocks, hipStream_t st) {
  hipLaunchKernelGGL((conv_gemm_kernel<MODE, BM, BN, AL, ST, BI, AF>), dim3(blocks), dim3(NT), 0, st, a);
}

template <int MODE, bool AL, bool ST, bool BI = false, bool AF = false>
void launch_cfg(const ConvArgs& a, int bm, int bn, int blocks, hipStream_t st) {
  if (bm == 128 && bn == 128)
    launch_t<MODE, 128, 128, AL, ST, BI, AF>(a, blocks, st);
  else if (bm == 128 && bn == 64)
    launch_t<MODE, 128, 64, AL, ST, BI, AF>(a, blocks, st);
  else if (bm == 64 && bn == 128)
    launch_t<MODE, 64, 128, AL, ST, BI, AF>(a, blocks, st);
  else
    launch_t<MODE, 64, 64, AL, ST, BI, AF>(a, blocks, st);
}

}  // namespace

static int gemm_dbg() {
  static const int v = [] { const char* e = getenv("TDL_GEMM_DBG"); return e ? atoi(e) : 0; }();
  return v;
}

static void pick_tile(long M, int Ng, int& bm, int& bn) {
  bn = Ng <= 64 ? 64 : 128;
  bm = M <= 64 ? 64 : 128;
  // small problems: prefer more workgroups
  if (bm == 128 && bn == 128 && (long)cdiv(M, 128) * cdiv(Ng, 128) < 256) bn = 64;
  if (bm == 128 && (long)cdiv(M, bm) * cdiv(Ng, bn) < 256) bm = 64;
}

// tiles per workgroup: keep ≥ ~2 workgroups per CU, and ≥ ~8 K-steps per workgroup
static int pick_tpb(long tiles, int nkt) {
  const char* env = getenv("TDL_CONV_TPB");
  if (env) return std::max(1, atoi(env));
  const long want_steps = 8;
  long tpb = (want_steps + nkt - 1) / std::max(nkt, 1);
  const long cap = std::max<long>(1, tiles / 512);
  tpb = std::max<long>(1, std::min(tpb, cap));
  return (int)tpb;
}

[[noreturn]] static void route_fail(int op, const RouteProblem& p) {
  const int f = route_forced(op);
  std::string msg = std::string(op == 0 ? "conv_fwd" : op == 1 ? "conv_dgrad" : "conv_wgrad") +
                    ": no conv route ran the problem (taps " + std::to_string(p.taps) +
                    ", stride " + std::to_string(p.stride) + ", C " + std::to_string(p.cin) +
                    ", K " + std::to_string(p.cout) + ", rows " + std::to_string(p.rows) +
                    ", flags " + std::to_string(p.flags) + ")";
  if (f >= 0) msg += std::string(" — forced route '") + route_rule(f).name + "' does not take it";
  throw std::runtime_error(msg);
}

static void conv_fwd_gemm(const ConvArgs& a0, hipStream_t st);

// the forward through the route table (conv_route.hip): false when no row took it (a residual
// problem outside the LDS-DMA kernel: the caller adds the residual itself)
static bool conv_fwd_route(const ConvArgs& a0, hipStream_t st) {
  const int flags = (a0.stats ? RF_STATS : 0) | (a0.aff ? RF_AFF : 0) | (a0.res ? RF_RES : 0) |
                    (a0.bias ? RF_BIAS : 0);
  const RouteProblem p = route_problem(0, a0, flags);
  for (int i = route_next(p, -1); i >= 0; i = route_next(p, i)) {
    bool ran = false;
    switch (route_rule(i).impl) {
      case RT_HALO: ran = route_cfg(i) == 1 ? conv_fwd_rw(a0, st) : conv_fwd_halo(a0, st); break;
      case RT_PC: ran = conv_fwd_pc_run(a0, st); break;
      case RT_GLDS: ran = conv_fwd_glds(a0, route_cfg(i), st); break;
      case RT_GEMM: conv_fwd_gemm(a0, st); ran = true; break;
      default: break;
    }
    if (ran) {
      route_record(0, i);
      return true;
    }
  }
  if (route_forced(0) >= 0) route_fail(0, p);
  return false;
}

void conv_fwd_launch(const ConvArgs& a0, hipStream_t st) {
  if (a0.aff && (a0.C % 8 || a0.K % 8 || a0.bias || a0.res))
    throw std::runtime_error("folded-BN conv: C % 8 == 0, K % 8 == 0, no bias / residual");
  if (!conv_fwd_route(a0, st)) route_fail(0, route_problem(0, a0, 0));
}

bool conv_fwd_res_launch(const ConvArgs& a, hipStream_t st) { return conv_fwd_route(a, st); }

static void conv_fwd_gemm(const ConvArgs& a0, hipStream_t st) {
  const bool aff = a0.aff != nullptr;
  ConvArgs a = a0;
  convk::set_fastdivs(a);
  a.dbg = gemm_dbg();
  int bm, bn;
  pick_tile(a.M, a.Ng, bm, bn);
  const long ntm = cdiv(a.M, bm), ntn = cdiv(a.Ng, bn);
  a.ncls = 1;
  a.tpb = pick_tpb(ntm * ntn, cdiv(a.Kg, BK));
  // row groups of tpb tiles × column tiles (see tile_of: FWD ordering)
  const long groups = (ntm + a.tpb - 1) / a.tpb;
  const int blocks = (int)(groups * ntn);
  a.cls_tile0[0] = 0;
  a.cls_tile0[1] = (int)(groups * ntn * a.tpb);
  a.splits = 1;
  const bool al = (a.C % 8 == 0) && (a.K % 8 == 0);
  const bool stats = a.stats != nullptr;
  const bool bias = a.bias != nullptr;
  if (aff) {
    if (stats) launch_cfg<FWD, true, true, false, true>(a, bm, bn, blocks, st);
    else launch_cfg<FWD, true, false, false, true>(a, bm, bn, blocks, st);
  } else if (al) {
    if (bias) {
      if (stats) launch_cfg<FWD, true, true, true>(a, bm, bn, blocks, st);
      else launch_cfg<FWD, true, false, true>(a, bm, bn, blocks, st);
    } else {
      if (stats) launch_cfg<FWD, true, true>(a, bm, bn, blocks, st);
      else launch_cfg<FWD, true, false>(a, bm, bn, blocks, st);
    }
  } else {
    if (bias) {
      if (stats) launch_cfg<FWD, false, true, true>(a, bm, bn, blocks, st);
      else launch_cfg<FWD, false, false, true>(a, bm, bn, blocks, st);
    } else {
      if (stats) launch_cfg<FWD, false, true>(a, bm, bn, blocks, st);
      else launch_cfg<FWD, false, false>(a, bm, bn, blocks, st);
    }
  }
}

// zero a byte range (multiple of 4) with a kernel rather than hipMemsetAsync: an ordinary kernel
// node under HIP-graph capture, ordered on `st` like every other launch of the step
__global__ void zero_fill_kernel(uint32_t* __restrict__ p, long n4) {
  const long n16 = n4 >> 2;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256)
    ((uint4*)p)[i] = make_uint4(0, 0, 0, 0);
  if (blockIdx.x == 0 && threadIdx.x < (n4 & 3)) p[n16 * 4 + threadIdx.x] = 0u;
}

void conv_zero_fill(void* p, uint32_t bytes, hipStream_t st);
static void zero_fill(void* p, uint32_t bytes, hipStream_t st) { conv_zero_fill(p, bytes, st); }
void conv_zero_fill(void* p, uint32_t bytes, hipStream_t st) {
  const long n4 = bytes / 4;
  const int blocks = (int)std::min<long>(2048, std::max<long>(1, (n4 / 4 + 255) / 256));
  hipLaunchKernelGGL(zero_fill_kernel, dim3(blocks), dim3(256), 0, st, (uint32_t*)p, n4);
}

static void conv_dgrad_gemm(const ConvArgs& a0, bool masked, long Mmax, hipStream_t st);

bool conv_dgrad_launch(const ConvArgs& a0, hipStream_t st) {
  ConvArgs a = a0;
  const bool masked = (a.sh > 1 && a.dh > 1) || (a.sw > 1 && a.dw > 1) ||
                      a.sh * a.sw > MAX_DG_CLASSES;
  a.dg_masked = masked ? 1 : 0;
  const ConvArgs a_s1 = a;  // (stride-1 executors: their own geometry, no parity classes)
  // build parity classes
  int ncls = 0;
  long Mmax = 0;
  const int sh = masked ? 1 : a.sh, sw = masked ? 1 : a.sw;
  for (int ca = 0; ca < sh; ++ca)
    for (int cb = 0; cb < sw; ++cb) {
      const int c = ncls++;
      a.cls_a[c] = ca;
      a.cls_b[c] = cb;
      a.cls_Hc[c] = ca < a.H ? (a.H - ca + sh - 1) / sh : 0;
      a.cls_Wc[c] = cb < a.W ? (a.W - cb + sw - 1) / sw : 0;
      if (masked || a.sh == 1) {
        a.cls_r0[c] = 0;
        a.cls_Th[c] = a.R;
      } else {
        const int r0 = ((ca + a.ph) % a.sh + a.sh) % a.sh;
        a.cls_r0[c] = r0;
        a.cls_Th[c] = r0 < a.R ? (a.R - r0 + a.sh - 1) / a.sh : 0;
      }
      if (masked || a.sw == 1) {
        a.cls_s0[c] = 0;
        a.cls_Tw[c] = a.S;
      } else {
        const int s0 = ((cb + a.pw) % a.sw + a.sw) % a.sw;
        a.cls_s0[c] = s0;
        a.cls_Tw[c] = s0 < a.S ? (a.S - s0 + a.sw - 1) / a.sw : 0;
      }
      Mmax = std::max<long>(Mmax, (long)a.N * a.cls_Hc[c] * a.cls_Wc[c]);
    }
  // heaviest classes first (longest-processing-time order: no heavy tail at the end of the grid)
  for (int i = 0; i < ncls; ++i)
    for (int j = i + 1; j < ncls; ++j)
      if (a.cls_Th[j] * a.cls_Tw[j] > a.cls_Th[i] * a.cls_Tw[i]) {
        std::swap(a.cls_a[i], a.cls_a[j]);
        std::swap(a.cls_b[i], a.cls_b[j]);
        std::swap(a.cls_Hc[i], a.cls_Hc[j]);
        std::swap(a.cls_Wc[i], a.cls_Wc[j]);
        std::swap(a.cls_r0[i], a.cls_r0[j]);
        std::swap(a.cls_Th[i], a.cls_Th[j]);
        std::swap(a.cls_s0[i], a.cls_s0[j]);
        std::swap(a.cls_Tw[i], a.cls_Tw[j]);
      }
  if (masked) {  // single class with original (masked) stride semantics
    a.cls_Hc[0] = a.H;
    a.cls_Wc[0] = a.W;
    Mmax = (long)a.N * a.H * a.W;
  }
  // classes with no contributing taps (e.g. 3 of 4 for a 1×1/s2 conv) are zero: one memset
  // instead of GEMM tiles (they are last after the LPT sort)
  int nz = ncls;
  while (nz > 0 && a.cls_Th[nz - 1] * a.cls_Tw[nz - 1] == 0) --nz;
  a.ncls = nz;
  // the route problem: dx rows per parity class with taps; fused statistics only where the
  // LDS-DMA epilogue can take them (dgrad_stats_fusable)
  const bool s1 = !masked && a.sh == 1 && a.sw == 1;
  const bool stats = nz > 0 && dgrad_stats_fusable(a);
  const int flags = (stats ? RF_STATS : 0) | (a.beta ? RF_JOIN : 0) |
                    (stats && a.beta ? RF_STATS_JOIN : 0) | (a.aff ? RF_AFF : 0) |
                    (a.fp8 ? RF_FP8 : 0) | (!masked && a.w_flip ? RF_WFLIP : 0) |
                    (!s1 && !masked ? RF_STRIDED : 0);
  RouteProblem p = route_problem(1, a, flags);
  p.ncls = nz;
  p.rows = 0;
  for (int c = 0; c < nz; ++c) {
    p.cls_rows[c] = (long)a.N * a.cls_Hc[c] * a.cls_Wc[c];
    p.rows += p.cls_rows[c];
  }
  if (nz == 0) {  // no pixel of dx receives a tap
    if (!a.beta) zero_fill(a.out, a.out_bytes, st);
    return false;
  }
  bool zeroed = false;
  for (int i = route_next(p, -1); i >= 0; i = route_next(p, i)) {
    const RouteRule& r = route_rule(i);
    bool fused = false, ran = false;
    if (r.impl == RT_ASFWD) {  // (strided: per-class forward convs, conv_glds.hip)
      ran = !masked && conv_dgrad_as_fwd(a_s1, a.w_flip, a.w_flip_bytes, route_cfg(i), st, &fused);
    } else if (r.impl == RT_HALO) {
      ran = s1 && conv_dgrad_halo(a_s1, st, &fused);
    } else {
      // (when accumulating into an existing dx the zero classes simply keep their values)
      if (!zeroed && nz < ncls && !a.beta) zero_fill(a.out, a.out_bytes, st);
      zeroed = true;
      if (r.impl == RT_GLDS) {
        ran = conv_dgrad_glds(a, route_cfg(i), st, &fused);
      } else if (r.impl == RT_GEMM) {
        conv_dgrad_gemm(a, masked, Mmax, st);
        ran = true;
      }
    }
    if (ran) {
      route_record(1, i);
      return fused;
    }
  }
  if (a.fp8) throw std::runtime_error("fp8 dgrad: LDS-DMA kernel not eligible (K % 128, C % 8, "
                                      "stride with dilation)");
  route_fail(1, p);
}

static void conv_dgrad_gemm(const ConvArgs& a0, bool masked, long Mmax, hipStream_t st) {
  ConvArgs a = a0;
  const int ncls = a.ncls;
  convk::set_fastdivs(a);
  a.dbg = gemm_dbg();
  int bm, bn;
  pick_tile(Mmax * ncls, a.Ng, bm, bn);
  a.cls_tile0[0] = 0;
  int maxkt = 1;
  for (int c = 0; c < ncls; ++c) {
    const long Mc = (long)a.N * a.cls_Hc[c] * a.cls_Wc[c];
    a.cls_tile0[c + 1] = a.cls_tile0[c] + (int)(cdiv(Mc, bm) * (long)cdiv(a.Ng, bn));
    maxkt = std::max(maxkt, cdiv((long)a.cls_Th[c] * a.cls_Tw[c] * a.K, BK));
  }
  const long tiles = a.cls_tile0[ncls];
  if (tiles == 0) return;
  a.tpb = pick_tpb(tiles, maxkt);
  a.splits = 1;
  const int blocks = (int)((tiles + a.tpb - 1) / a.tpb);
  const bool al = (a.C % 8 == 0) && (a.K % 8 == 0) && !masked;
  if (al) launch_cfg<DGRAD, true, false>(a, bm, bn, blocks, st);
  else launch_cfg<DGRAD, false, false>(a, bm, bn, blocks, st);
  // (the register-staged kernel does not fuse BN-backward statistics)
}

static void conv_wgrad_gemm_plan(const ConvArgs& a, WgradPlan* p);

// a folded BN on x (ConvArgs::aff): the register-staged kernel (it transforms the staged B rows)
void conv_wgrad_plan(const ConvArgs& a, WgradPlan* p) {
  RouteProblem q = route_problem(2, a, (a.aff ? RF_AFF : 0) | (a.fp8 ? RF_FP8 : 0));
  for (int i = route_next(q, -1); i >= 0; i = route_next(q, i)) {
    bool ran = false;
    switch (route_rule(i).impl) {
      case RT_HALO: ran = conv_wgrad_halo_plan(a, p); break;
      case RT_GLDS: ran = conv_wgrad_glds_plan(a, route_cfg(i), p); break;
      case RT_GEMM:
        if (a.fp8) break;  // (fp8 operands: the LDS-DMA kernel only)
        conv_wgrad_gemm_plan(a, p);
        ran = true;
        break;
      default: break;
    }
    if (ran) {
      route_record(2, i);
      return;
    }
  }
  route_fail(2, q);
}

static void conv_wgrad_gemm_plan(const ConvArgs& a, WgradPlan* p) {
  p->impl = 0;
  p->cfg = 0;
  p->bm = a.M <= 64 ? 64 : 128;
  p->bn = a.Ng <= 64 ? 64 : 128;
  const int tiles = cdiv(a.M, p->bm) * cdiv(a.Ng, p->bn);
  const int nkt = cdiv(a.Kg, BK);
  const char* env = getenv("TDL_WGRAD_TARGET");
  const int target = env ? atoi(env) : 768;  // ≈3 workgroups per CU over 256 CUs
  int s = std::max(1, std::min(nkt, target / std::max(tiles, 1)));
  int per = cdiv(nkt, s);
  per = std::max(per, 8);  // at least 8 K-steps per split
  p->kps = per;
  p->splits = cdiv(nkt, per);
}

void conv_wgrad_launch(const ConvArgs& a0, const WgradPlan& p, float* out, bool accumulate,
                       hipStream_t st) {
  ConvArgs a = a0;
  const int splits = p.splits;
  if (p.impl == 2) {
    conv_wgrad_halo_launch(a, p, st);
  } else if (p.impl == 1) {
    conv_wgrad_glds_kernel_launch(a, p, st);
  } else {
    const long tiles = (long)cdiv(a.M, p.bm) * cdiv(a.Ng, p.bn) * splits;
    a.ncls = 1;
    a.cls_tile0[0] = 0;
    a.cls_tile0[1] = (int)tiles;
    a.tpb = 1;
    a.splits = splits;
    a.kps = p.kps;
    convk::set_fastdivs(a);
    const bool al = (a.C % 8 == 0) && (a.K % 8 == 0);
    if (a.aff) {
      if (!al) throw std::runtime_error("folded-BN weight gradient: C % 8 == 0, K % 8 == 0");
      launch_cfg<WGRAD, true, false, false, true>(a, p.bm, p.bn, (int)tiles, st);
    } else if (al) launch_cfg<WGRAD, true, false>(a, p.bm, p.bn, (int)tiles, st);
    else launch_cfg<WGRAD, false, false>(a, p.bm, p.bn, (int)tiles, st);
  }
  splitk_reduce_launch((const float*)a.out, out, (long)a.M * a.Ng, splits, accumulate, st);
}

void splitk_reduce_launch(const float* slab, float* out, long n, int splits, bool accumulate,
                          hipStream_t st) {
  const long n4 = std::max<long>(1, n / 4);
  if (splits >= 64) {
    hipLaunchKernelGGL(splitk_reduce_kernel<16>, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, st,
                       slab, out, n, splits, accumulate ? 1 : 0);
  } else if (splits >= 8) {
    hipLaunchKernelGGL(splitk_reduce_kernel<4>, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, st,
                       slab, out, n, splits, accumulate ? 1 : 0);
  } else {
    hipLaunchKernelGGL(splitk_reduce_kernel<1>, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st,
                       slab, out, n, splits, accumulate ? 1 : 0);
  }
}

int colsum_blocks(long P, int K) {
  // row blocks of ≥ 64 rows, at most 64 of them (≈ one workgroup per CU across the channel
  // chunks, and a short serial sum per thread in colsum_reduce_kernel)
  const int ychunks = (K % 8 == 0) ? cdiv(K / 8, 64) : cdiv(K, 64);
  const long want = std::max<long>(8, std::min<long>(64, 256 / ychunks));
  return (int)std::max<long>(1, std::min<long>(want, (P + 63) / 64));
}

void colsum_launch(const bf16_t* x, float* out, float* part, long P, int K, bool accumulate,
                   hipStream_t st) {
  const int nb = colsum_blocks(P, K);
  const long rpb = (P + nb - 1) / nb;
  if (K % 8 == 0) {
    dim3 grid(nb, cdiv(K / 8, 64));
    hipLaunchKernelGGL(colsum_part_kernel<true>, grid, dim3(256), 0, st, x, part, P, K, rpb);
  } else {
    dim3 grid(nb, cdiv(K, 64));
    hipLaunchKernelGGL(colsum_part_kernel<false>, grid, dim3(256), 0, st, x, part, P, K, rpb);
  }
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3(cdiv(K, 64)), dim3(256), 0, st, part, out, nb, K,
                     accumulate ? 1 : 0);
}

}  // namespace tdl
