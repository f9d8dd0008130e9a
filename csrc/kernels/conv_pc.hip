// Producer/consumer (wave-specialised) LDS-DMA forward convolution for gfx950 — FASTK forward
// (a K-step is one filter tap × 64 channels; 1×1 with ragged channel counts too).  Routed by
// conv_fwd_glds (TDL_CONV_PC): by default the 3×3 convs with ≥ 256 input channels take the
// 4-producer form, 14–20 % faster than conv_glds there; on 1×1 convs (1–16 K-steps per tile, the
// producers' per-tile address setup on the critical path) it is slower
// (profiles/r04_conv_pc_ab.txt).
//
// In conv_glds_kernel every wave both feeds the ring (per-piece DMA address math, validity
// selects, the counted vmcnt that also covers its own epilogue stores) and computes (fragment
// reads + MFMAs): per 64-deep K-step a wave issued ≈35 VALU and ≈50 SALU besides its 32 MFMAs and
// 16 ds_reads (hipcc -S of the 256×128 forward), a third of its cycles waited on the ring and
// another third were issue-stalled (profiles/r03_conv_kloop_interleave_ab.txt).  Here:
//
//  * NP producer waves own the whole ring: all DMA address math, all vmcnt waits; their state is
//    rebuilt once per tile in an outer loop (no tile switch inside the issue path — hipcc demotes
//    the per-lane state arrays to scratch when it is);
//  * NW consumer waves run barrier → ds_read → MFMA only, and never wait for their epilogue
//    stores inside the loop (a wave's vmcnt only counts its own memory operations);
//  * one s_barrier per K-step orders both roles: at barrier t the producers have retired step t's
//    DMAs and the consumers have retired their reads of step t−1's slot, which the producers then
//    refill with step t+ST−1.
//
// Same LDS images (KC, source-side swizzle), fragment layout and epilogue (conv_common.h
// store_tile_bf16: bias, ReLU, BN statistics) as conv_glds.hip, so outputs are bit-identical.
#include "conv_common.h"

namespace tdl {

namespace {
using namespace convk;

typedef __attribute__((address_space(3))) void pc_lds_void_t;
typedef __attribute__((address_space(3))) char pc_lds_char_t;

template <int N>
__device__ __forceinline__ void pc_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void pc_barrier() { asm volatile("s_barrier" ::: "memory"); }
__device__ __forceinline__ void pc_dma16(rsrc_t r, char* lds_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (pc_lds_void_t*)lds_base, 16, voff, 0, 0, 0);
}
template <int N, int I = 0>
__device__ __forceinline__ void pc_rows(bf16x8 (&f)[N], uint32_t base) {
  if constexpr (I < N) {
    uint4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(I * 2048) : "memory");
    f[I] = __builtin_bit_cast(bf16x8, v);
    pc_rows<N, I + 1>(f, base);
  }
}

// AFF: a training BN + ReLU folded into this conv (ConvArgs::aff, ops/bnconv.py) — the producers
// stage the A tile through registers instead of LDS-DMA: buffer_load → u = relu(a·z + b) (bf16,
// exactly as the BN apply pass rounds it; padding taps / rows past M stay 0) → ds_write_b128 to
// the same swizzled LDS image.  Step j's loads are issued one step ahead (two register sets), so
// they land under the consumers' MFMAs of step j−1; the consumers are unchanged.
// DEPI: the DGRAD epilogue (mask / join / BN-backward statistics) on this forward K loop — a
// stride-1 input gradient as the forward conv of dy with the flipped filter (conv_glds.hip
// conv_dgrad_as_fwd); NJ: no join (the statistics form)
template <int BM, int BN, int WM, int WN, int ST, int NP, bool STATS, bool BIAS, int FK,
          bool AFF = false, bool DEPI = false, bool NJ = false>
__global__ void __launch_bounds__(64 * (WM * WN + NP), 1) conv_pc_kernel(ConvArgs a) {
  static_assert(!DEPI || (!AFF && !BIAS), "dgrad epilogue: plain operands");
  static_assert(FK == 1 || FK == 2, "FASTK forward only");
  static_assert(!AFF || (FK == 1 && NP % 2 == 0), "folded BN: FASTK, even producer count");
  constexpr bool RAG = FK == 2;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, RM = TM / 16, RN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PA = BM / 8, PB = BN / 8;  // 1-KiB DMA pieces per stage (8 rows × 128 B each)
  static_assert(PA % NP == 0 && PB % NP == 0, "pieces split evenly over the producers");
  constexpr int QA = PA / NP, QB = PB / NP, PP = QA + QB;  // pieces per producer per K-step
  static_assert(PP * (ST - 2) <= 63, "vmcnt field");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_begin = blk * a.tpb;
  const int tile_end = min(a.cls_tile0[a.ncls], tile_begin + a.tpb);
  if (tile_begin >= tile_end) return;
  const Tile T0 = tile_of<FWD, BM, BN, BK, true>(a, tile_begin);
  if (T0.bm0 >= T0.Mc) return;
  // this workgroup's tiles: consecutive row tiles of one column tile (FWD tile order)
  const int ntiles = min(tile_end - tile_begin, (T0.Mc - T0.bm0 + BM - 1) / BM);
  const int nk = T0.kt1;  // K-steps per tile (every FWD tile has the same K)
  const int total = ntiles * nk;
  float* red = (float*)(smem + ST * STAGE);

  if (wid >= NW) {
    // ================================ producers ================================
    __builtin_amdgcn_s_setprio(2);  // ring refills are latency-critical
    const int pid = wid - NW;
    const bool pointwise = a.R == 1 && a.S == 1 && a.ph == 0 && a.pw == 0;
    const rsrc_t rx = make_rsrc(a.x, a.x_bytes), rw = make_rsrc(a.w, a.w_bytes);
    const int HoWo = a.Ho * a.Wo;
    int a_row[QA], a_p0[QA], a_p1[QA], b_row[QB];
    int a_ch[QA], b_ch[QB];  // this lane's (swizzled) channel chunk of each piece row, ×8
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int r = (q * NP + pid) * 8 + (lane >> 3);
      a_ch[q] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int r = (q * NP + pid) * 8 + (lane >> 3);
      b_ch[q] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
      const int n = T0.bn0 + r;
      b_row[q] = n < a.Ng ? n * a.Kg + b_ch[q] : -1;
    }
    if constexpr (AFF) {
      // ---- register-staged producers with the folded BN + ReLU ----
      // this lane's channel chunk is the same in every piece: row r = (q·NP + pid)·8 + lane/8,
      // (r/2) mod 8 = (pid & 1)·4 + lane/16 for even NP
      const int ach = a_ch[0];
      float* tbl = (float*)(smem + ST * STAGE + 2 * BN * 4);  // a[C] then b[C]
      // every producer wave writes the whole coefficient table itself (identical values, its 64
      // lanes cover all 8 chunks of every 64 channels): no cross-wave ordering before its reads
      for (int c0 = 0; c0 < a.C; c0 += BK) {
        float ta[8], tb[8];
        aff_load8(a.aff, a.aff_ld, c0 + ach, ta, tb);
        *(float4*)(tbl + c0 + ach) = make_float4(ta[0], ta[1], ta[2], ta[3]);
        *(float4*)(tbl + c0 + ach + 4) = make_float4(ta[4], ta[5], ta[6], ta[7]);
        *(float4*)(tbl + a.C + c0 + ach) = make_float4(tb[0], tb[1], tb[2], tb[3]);
        *(float4*)(tbl + a.C + c0 + ach + 4) = make_float4(tb[4], tb[5], tb[6], tb[7]);
      }
      uint4 ra0[QA], ra1[QA];
      uint32_t av0 = 0, av1 = 0;
      int fc0 = 0, fc1 = 0;  // channel offset (pc0) of the step held in ra0 / ra1
      int islot = 0, fslot = 0, par = 0;
      bool have = false;
      const uint4 zero = make_uint4(0, 0, 0, 0);
      const uint32_t lds0 = (uint32_t)(size_t)(pc_lds_char_t*)smem;
      const uint32_t tbl_lds = lds0 + (uint32_t)(ST * STAGE + 2 * BN * 4);
      // issue step (tile state, pr/ps/pc0, k) into RA: A loads to registers, B LDS-DMA into its slot
#define TDL_PC_ISSUE(RA, AV, FC)                                                                \
  do {                                                                                        \
    const int rdh_ = pr * a.dh, sdw_ = ps * a.dw;                                             \
    const int tuni_ = (rdh_ * a.W + sdw_) * a.C + pc0;                                        \
    uint32_t vb_ = 0;                                                                         \
    _Pragma("unroll") for (int q = 0; q < QA; ++q) {                                          \
      /* branch-free validity (a short-circuit && compiles to exec-mask branches per piece) */ \
      const bool in_ = ((unsigned)(a_p0[q] + rdh_) < (unsigned)a.H) &                         \
                       ((unsigned)(a_p1[q] + sdw_) < (unsigned)a.W);                           \
      const bool v_ = pointwise ? a_p0[q] >= 0 : in_;                                         \
      RA[q] = bload16(rx, v_ ? (uint32_t)(a_row[q] + tuni_) * 2u : OOB);                      \
      vb_ |= (uint32_t)v_ << q;                                                               \
    }                                                                                         \
    AV = vb_;                                                                                 \
    FC = pc0;                                                                                 \
    char* Bs_ = smem + islot * STAGE + A_BYTES;                                               \
    const int kb_ = k * BK;                                                                   \
    _Pragma("unroll") for (int q = 0; q < QB; ++q)                                            \
      pc_dma16(rw, Bs_ + (q * NP + pid) * 1024, b_row[q] >= 0 ? (uint32_t)(b_row[q] + kb_) * 2u : OOB); \
    islot = islot + 1 == ST ? 0 : islot + 1;                                                  \
  } while (0)
      // transform + write the A tile of the step held in RA into its slot, publish the step.
      // Every LDS access here is inline asm: a compiler-visible ds_read / ds_write after an
      // LDS-DMA issue makes hipcc wait vmcnt(0) first (a possible alias of the DMA's LDS
      // writes), which would drain the next step's loads just issued.
#define TDL_PC_FINISH(RA, AV, FC)                                                               \
  do {                                                                                        \
    uint4 ca0_, ca1_, cb0_, cb1_;                                                             \
    const uint32_t ta_ = tbl_lds + (uint32_t)((FC) + ach) * 4u;                               \
    const uint32_t tb_ = ta_ + (uint32_t)a.C * 4u;                                            \
    asm volatile("ds_read_b128 %0, %1" : "=v"(ca0_) : "v"(ta_) : "memory");                   \
    asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(ca1_) : "v"(ta_) : "memory");         \
    asm volatile("ds_read_b128 %0, %1" : "=v"(cb0_) : "v"(tb_) : "memory");                   \
    asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(cb1_) : "v"(tb_) : "memory");         \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    const float ca_[8] = {__uint_as_float(ca0_.x), __uint_as_float(ca0_.y),                   \
                          __uint_as_float(ca0_.z), __uint_as_float(ca0_.w),                   \
                          __uint_as_float(ca1_.x), __uint_as_float(ca1_.y),                   \
                          __uint_as_float(ca1_.z), __uint_as_float(ca1_.w)};                  \
    const float cb_[8] = {__uint_as_float(cb0_.x), __uint_as_float(cb0_.y),                   \
                          __uint_as_float(cb0_.z), __uint_as_float(cb0_.w),                   \
                          __uint_as_float(cb1_.x), __uint_as_float(cb1_.y),                   \
                          __uint_as_float(cb1_.z), __uint_as_float(cb1_.w)};                  \
    const uint32_t as_ = lds0 + (uint32_t)(fslot * STAGE + pid * 1024 + lane * 16);           \
    _Pragma("unroll") for (int q = 0; q < QA; ++q) {                                          \
      uint4 u_ = aff_relu8(RA[q], ca_, cb_);                                                  \
      const uint32_t m_ = 0u - (((AV) >> q) & 1u); /* padding / rows past M stay 0 */         \
      u_.x &= m_; u_.y &= m_; u_.z &= m_; u_.w &= m_;                                         \
      const v4u32 w_ = {u_.x, u_.y, u_.z, u_.w};                                             \
      asm volatile("ds_write_b128 %0, %1" ::"v"(as_ + (uint32_t)(q * NP * 1024)), "v"(w_)      \
                   : "memory");                                                               \
    }                                                                                         \
    fslot = fslot + 1 == ST ? 0 : fslot + 1;                                                  \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                        \
    pc_barrier();                                                                             \
  } while (0)
      (void)lds0;
      for (int ti = 0; ti < ntiles; ++ti) {
        const int bm0 = T0.bm0 + ti * BM;
#pragma unroll
        for (int q = 0; q < QA; ++q) {
          const int m = bm0 + (q * NP + pid) * 8 + (lane >> 3);
          if (m < T0.Mc) {
            const int n = fdiv(m, a.fd_HoWo), rem = m - n * HoWo;
            const int ho = fdiv(rem, a.fd_Wo), wo = rem - ho * a.Wo;
            a_p0[q] = ho * a.sh - a.ph;
            a_p1[q] = wo * a.sw - a.pw;
            a_row[q] = n * a.H * a.W * a.C + (a_p0[q] * a.W + a_p1[q]) * a.C + ach;
          } else {
            a_p0[q] = -(1 << 28);
            a_p1[q] = 0;
            a_row[q] = 0;
          }
        }
        int pr = 0, ps = 0, pc0 = 0;
        for (int k = 0; k < nk; ++k) {
          // step j's loads go into one register set while step j−1 (the other set) is
          // transformed and published once its loads have retired (QA + QB younger ops)
          if (par == 0) {
            TDL_PC_ISSUE(ra0, av0, fc0);
            if (have) {
              pc_vmwait<QA + QB>();
              TDL_PC_FINISH(ra1, av1, fc1);
            }
          } else {
            TDL_PC_ISSUE(ra1, av1, fc1);
            if (have) {
              pc_vmwait<QA + QB>();
              TDL_PC_FINISH(ra0, av0, fc0);
            }
          }
          par ^= 1;
          have = true;
          pc0 += BK;
          if (pc0 >= a.C) {
            pc0 = 0;
            if (++ps == a.S) {
              ps = 0;
              ++pr;
            }
          }
        }
      }
      pc_vmwait<0>();
      if (par == 1) TDL_PC_FINISH(ra0, av0, fc0);  // the last issued step
      else TDL_PC_FINISH(ra1, av1, fc1);
#undef TDL_PC_ISSUE
#undef TDL_PC_FINISH
      if constexpr (STATS) {
        __syncthreads();
        __syncthreads();
      }
      return;
    }
    int issued = 0, bar = 0, slot = 0;
    for (int ti = 0; ti < ntiles; ++ti) {
      const int bm0 = T0.bm0 + ti * BM;
#pragma unroll
      for (int q = 0; q < QA; ++q) {
        const int m = bm0 + (q * NP + pid) * 8 + (lane >> 3);
        if (m < T0.Mc) {
          const int n = fdiv(m, a.fd_HoWo), rem = m - n * HoWo;
          const int ho = fdiv(rem, a.fd_Wo), wo = rem - ho * a.Wo;
          a_p0[q] = ho * a.sh - a.ph;
          a_p1[q] = wo * a.sw - a.pw;
          a_row[q] = n * a.H * a.W * a.C + (a_p0[q] * a.W + a_p1[q]) * a.C + a_ch[q];
        } else {
          a_p0[q] = -(1 << 28);
          a_p1[q] = 0;
          a_row[q] = 0;
        }
      }
      int pr = 0, ps = 0, pc0 = 0;
      for (int k = 0; k < nk; ++k) {
        if (issued >= ST - 1) {
          // steady state: retire step `bar` (ST−2 younger steps stay in flight), then the
          // consumers' reads of the slot refilled below are done too
          pc_vmwait<PP * (ST - 2)>();
          pc_barrier();
          ++bar;
        }
        char* As = smem + slot * STAGE;
        char* Bs = As + A_BYTES;
        const int rdh = pr * a.dh, sdw = ps * a.dw;
        const int tuni = (rdh * a.W + sdw) * a.C + pc0;
#pragma unroll
        for (int q = 0; q < QA; ++q) {
          bool v = pointwise ? a_p0[q] >= 0
                             : ((unsigned)(a_p0[q] + rdh) < (unsigned)a.H &&
                                (unsigned)(a_p1[q] + sdw) < (unsigned)a.W);
          if constexpr (RAG) v = v && pc0 + a_ch[q] < a.C;
          pc_dma16(rx, As + (q * NP + pid) * 1024, v ? (uint32_t)(a_row[q] + tuni) * 2u : OOB);
        }
        const int kb = k * BK;
#pragma unroll
        for (int q = 0; q < QB; ++q) {
          bool v = b_row[q] >= 0;
          if constexpr (RAG) v = v && kb + b_ch[q] < a.Kg;
          pc_dma16(rw, Bs + (q * NP + pid) * 1024, v ? (uint32_t)(b_row[q] + kb) * 2u : OOB);
        }
        slot = slot + 1 == ST ? 0 : slot + 1;
        ++issued;
        pc0 += BK;
        if (pc0 >= a.C) {
          pc0 = 0;
          if (++ps == a.S) {
            ps = 0;
            ++pr;
          }
        }
      }
    }
    // drain: the last ST−1 (or fewer) steps
    for (; bar < total; ++bar) {
      const int ahead = issued - bar - 1;
      if constexpr (ST >= 4) {
        if (ahead >= 2) pc_vmwait<PP * 2>();
        else if (ahead == 1) pc_vmwait<PP>();
        else pc_vmwait<0>();
      } else {
        if (ahead >= 1) pc_vmwait<PP>();
        else pc_vmwait<0>();
      }
      pc_barrier();
    }
    if constexpr (STATS) {
      __syncthreads();  // consumers' partial sums in LDS
      __syncthreads();  // reduced
    }
    return;
  }

  // ================================ consumers ================================
  const int wm = wid / WN, wn = wid % WN;
  if (wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const rsrc_t rout = make_rsrc(a.out, a.out_bytes);
  const uint32_t smem_lds = (uint32_t)(size_t)(pc_lds_char_t*)smem;
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (STATS) {
    // per-column (Σ, Σ²) of this workgroup's tiles: LDS-atomic partials, flushed once at the
    // end (ordered before any add by the first K-step's barrier) — no sums held in registers
    // across the K loop
    for (int t = tid; t < 2 * BN; t += 64 * NW) red[t] = 0.f;
  }
  const uint32_t a_off0 = (uint32_t)kc_off(wm * TM + (lane & 15), lane >> 4);
  const uint32_t b_off0 = (uint32_t)kc_off(wn * TN + (lane & 15), lane >> 4);
  const uint32_t a_off1 = (uint32_t)kc_off(wm * TM + (lane & 15), 4 + (lane >> 4));
  const uint32_t b_off1 = (uint32_t)kc_off(wn * TN + (lane & 15), 4 + (lane >> 4));
  Tile CT = T0;
  int slot = 0;
  // software pipeline (as conv_glds.hip): the first half-step's fragments of step t+1 are read
  // right after barrier t+1, under the second half-step's MFMAs of step t
  bf16x8 fa[RM], fb[RN], ga[RM], gb[RN];
  pc_barrier();
  pc_rows<RM>(fa, smem_lds + a_off0);
  pc_rows<RN>(fb, smem_lds + A_BYTES + b_off0);
  int t = 0;
  for (int ti = 0; ti < ntiles; ++ti) {
    for (int k = 0; k < nk; ++k, ++t) {
      const uint32_t As = smem_lds + (uint32_t)(slot * STAGE), Bs = As + A_BYTES;
      pc_rows<RM>(ga, As + a_off1);
      pc_rows<RN>(gb, Bs + b_off1);
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RM + RN) : "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rm = 0; rm < RM; ++rm)
#pragma unroll
        for (int rn = 0; rn < RN; ++rn)
          acc[rm][rn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[rn], fa[rm], acc[rm][rn], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot t fully read
      __builtin_amdgcn_sched_barrier(0);
      slot = slot + 1 == ST ? 0 : slot + 1;
      if (t + 1 < total) {
        pc_barrier();
        const uint32_t An = smem_lds + (uint32_t)(slot * STAGE), Bn = An + A_BYTES;
        pc_rows<RM>(fa, An + a_off0);
        pc_rows<RN>(fb, Bn + b_off0);
      }
#pragma unroll
      for (int rm = 0; rm < RM; ++rm)
#pragma unroll
        for (int rn = 0; rn < RN; ++rn)
          acc[rm][rn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gb[rn], ga[rm], acc[rm][rn], 0, 0, 0);
    }
    CT.bm0 = T0.bm0 + ti * BM;
    float s_sum[RN][4], s_sq[RN][4];
#pragma unroll
    for (int rn = 0; rn < RN; ++rn)
#pragma unroll
      for (int i = 0; i < 4; ++i) s_sum[rn][i] = s_sq[rn][i] = 0.f;
    store_tile_bf16<DEPI ? DGRAD : FWD, RM, RN, TM, TN, BIAS, STATS, false, false, NJ, false>(
        a, CT, acc, wm, wn, lane, rout, 1.f, false, s_sum, s_sq);
    if constexpr (STATS) {
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
      if ((lane & 15) == 0) {
#pragma unroll
        for (int rn = 0; rn < RN; ++rn)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int nl = wn * TN + rn * 16 + (lane >> 4) * 4 + i;
            atomicAdd(red + nl, s_sum[rn][i]);
            atomicAdd(red + BN + nl, s_sq[rn][i]);
          }
      }
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (STATS) {
    __syncthreads();
    for (int t = tid; t < 2 * BN; t += 64 * NW) {
      const int which = t / BN, nl = t - which * BN;
      const int n = T0.bn0 + nl;
      if (n < a.Ng) atomicAdd(a.stats + which * a.Ng + n, red[which * BN + nl]);
    }
    __syncthreads();
  }
}

// largest folded-BN channel count whose coefficient table fits beside the ring (256×128 tiles)
constexpr int PC_LDS_MAX = 160 * 1024;
constexpr int pc_lds(int bm, int bn, int st) { return st * (bm + bn) * BK * 2 + 2 * bn * 4; }

template <int BM, int BN, int WM, int WN, int ST, int NP, bool STATS, bool BIAS, int FK,
          bool AFF = false, bool DEPI = false, bool NJ = false>
void launch_pc(const ConvArgs& a, int blocks, hipStream_t st) {
  auto k = conv_pc_kernel<BM, BN, WM, WN, ST, NP, STATS, BIAS, FK, AFF, DEPI, NJ>;
  const int lds = pc_lds(BM, BN, ST) + (AFF ? 2 * a.C * 4 : 0);
  static int attr = 0;  // the largest size set so far
  if (lds > attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              AFF ? PC_LDS_MAX : lds);
    attr = AFF ? PC_LDS_MAX : lds;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * (WM * WN + NP)), lds, st, a);
}

}  // namespace

// the 256×128 forward of conv_fwd_glds (arguments prepared there: fast divisors, tiles per
// workgroup, FWD tile order); fk 1 = C % 64 == 0, 2 = ragged 1×1
// (mode 1: 2 producer waves, 2: 4)
bool conv_fwd_pc_launch(const ConvArgs& a, int blocks, int fk, int mode, hipStream_t st, bool depi) {
  if (a.res || a.dbg) return false;
  const bool stats = a.stats != nullptr, bias = a.bias != nullptr;
  if (depi) {
    // input gradient as a forward conv: DGRAD epilogue; statistics only without a join
    // (no statistics form: its BN-input registers spill at the 12-wave register budget — the
    // LDS-DMA kernel takes those)
    if (fk != 1 || bias || a.aff || stats) return false;
    launch_pc<256, 128, 4, 2, 3, 4, false, false, 1, false, true, false>(a, blocks, st);
    return true;
  }
  if (a.aff) {
    // folded BN + ReLU: 4 register-staging producers, FASTK, no bias, coefficient table in LDS
    if (fk != 1 || bias || pc_lds(256, 128, 3) + 2 * a.C * 4 > PC_LDS_MAX) return false;
    if (stats) launch_pc<256, 128, 4, 2, 3, 4, true, false, 1, true>(a, blocks, st);
    else launch_pc<256, 128, 4, 2, 3, 4, false, false, 1, true>(a, blocks, st);
    return true;
  }
  const bool np4 = mode == 2;
#define TDL_PC(NP, FK)                                                              \
  do {                                                                              \
    if (bias) {                                                                     \
      if (stats) launch_pc<256, 128, 4, 2, 3, NP, true, true, FK>(a, blocks, st);   \
      else launch_pc<256, 128, 4, 2, 3, NP, false, true, FK>(a, blocks, st);        \
    } else {                                                                        \
      if (stats) launch_pc<256, 128, 4, 2, 3, NP, true, false, FK>(a, blocks, st);  \
      else launch_pc<256, 128, 4, 2, 3, NP, false, false, FK>(a, blocks, st);       \
    }                                                                               \
  } while (0)
  if (fk == 1) { if (np4) TDL_PC(4, 1); else TDL_PC(2, 1); }
  else if (fk == 2) { if (np4) TDL_PC(4, 2); else TDL_PC(2, 2); }
  else return false;
#undef TDL_PC
  return true;
}

}  // namespace tdl
