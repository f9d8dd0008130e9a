// Halo-tiled direct convolution for stride-1 R×S filters (the 3×3 bodies of ResNet-18/50/152 and
// of the reference DeepLab net, /root/reference/core/resnet.py:137-138) on gfx950 — forward and
// input gradient.
//
// Why: the implicit-GEMM LDS-DMA kernel (conv_glds.hip) re-gathers the activation operand from
// L2 for every filter tap — a 3×3 conv DMAs its A tile nine times per 64-channel chunk (32 KiB per
// K-step of a 256×128 tile, 48 KiB with the weights), with per-lane bounds checks on every piece.
// That footprint caps the ring at 3 stages and the DMA issue + tap arithmetic made the K-loop
// vector-issue bound (≈30–40 % MFMA-busy on the ResNet-50 3×3 convs).  Here:
//
//  * a tile is TR complete output rows (of one or several images) × BN output channels; its
//    input rows plus the filter halo — every input pixel the tile's taps touch, zero-padded — go
//    to LDS ONCE per 64-channel chunk (`buffer_load … lds`, range-checked: padding taps read
//    zeros, no per-tap checks), double-buffered so the next chunk / tile streams in under the
//    current chunk's R·S K-steps;
//  * a K-step is one tap × 64 channels: only the weight tile (BN × 64) is DMA'd per step, so the
//    weight ring is 16 KiB per stage; the A fragment of a tap is the same halo image read at a
//    wave-uniform slot offset (per-lane slot + tap delta, one swizzle per fragment);
//  * persistent workgroups walk their tiles as one flat (tile, chunk, tap) sequence; the counted
//    `s_waitcnt vmcnt` covers weight pieces, halo fills and epilogue stores in issue order;
//  * epilogue shared with the implicit-GEMM kernels (conv_common.h store_tile_bf16, rows given):
//    bias / ReLU / BN Σ, Σ² (forward), residual join / ReLU bit mask / BN-backward Σg, Σg·x (input
//    gradient).
//
// The input gradient of a stride-1 conv is the same direct conv on dy with the taps mirrored and
// the weights read as W[k][r][s][c] with k the reduction (a transposed, "MC" LDS image read with
// ds_read_b64_tr_b16).
#include "conv_common.h"

#include <type_traits>

namespace tdl {

namespace {
using namespace convk;

constexpr int HALO_MAXTAP = 16;

// geometry of one halo conv (host-prepared)
struct HaloGeom {
  int N, Hi, Wi, Ci;     // direct-conv input: FWD x [N,H,W,C]; DGRAD dy [N,Ho,Wo,K]
  int Ho, Wo, Co;        // output: FWD y; DGRAD dx
  int ntap, nchunk;      // R·S taps; Ci / 64 channel chunks
  int tap_d[HALO_MAXTAP];  // per tap: halo slot delta (oy_t − oy_min)·HP + (ox_t − ox_min)
  int tap_b[HALO_MAXTAP];  // per tap: weight element offset
  int oy_min, ox_min, ext_h, ext_w;
  int ldb;               // FWD: weight row (output channel) stride; DGRAD: k-row stride
  int TR, HP;            // output rows per tile; halo pitch (slots per halo row)
  int nrb, ncb, tpb;     // row blocks, column blocks, tiles per workgroup
  FastDiv fd_HP, fd_Wo, fd_Ho, fd_seg;  // fd_seg: halo rows of a full image segment (Ho + ext_h)
};

template <int N>
__device__ __forceinline__ void hwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void hbarrier() { asm volatile("s_barrier" ::: "memory"); }
constexpr int vmc(int v) { return v < 63 ? v : 63; }

// s_waitcnt vmcnt(IB·ahead + HL·nh + E·ne): the younger VMEM ops of the step being waited for
// (weight pieces of `ahead` later steps, `nh` halo fills among them, `ne` epilogues' stores).
// Counting fewer than are outstanding only waits longer, so nh / ne are clamped to 1.
template <int IB, int HL, int E, int ST, int A = 0>
__device__ __forceinline__ void wait_halo(int ahead, int nh, int ne) {
  if constexpr (A <= ST - 2) {
    if (ahead == A) {
      if (nh == 0) {
        if (ne == 0) hwait<vmc(IB * A)>(); else hwait<vmc(IB * A + E)>();
      } else {
        if (ne == 0) hwait<vmc(IB * A + HL)>(); else hwait<vmc(IB * A + HL + E)>();
      }
      return;
    }
    wait_halo<IB, HL, E, ST, A + 1>(ahead, nh, ne);
  } else {
    hwait<0>();
  }
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) char lds_char_t;

__device__ __forceinline__ void hdma16(rsrc_t r, char* lds_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_base, 16, voff, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 hread(uint32_t addr) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return __builtin_bit_cast(bf16x8, v);
}
template <int N, int I = 0>
__device__ __forceinline__ void hread_rows(bf16x8 (&f)[N], uint32_t base) {
  if constexpr (I < N) {
    uint4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(I * 2048) : "memory");
    f[I] = __builtin_bit_cast(bf16x8, v);
    hread_rows<N, I + 1>(f, base);
  }
}
template <int COLS, int KK>
__device__ __forceinline__ bf16x8 hread_mc(uint32_t addr) {
  v2u32 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(addr), "n"(KK * 64 * COLS) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(addr), "n"(KK * 64 * COLS + 8 * COLS) : "memory");
  uint4 v = make_uint4(lo[0], lo[1], hi[0], hi[1]);
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ void hlgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// an invalid DMA source: past any operand buffer even after a chunk / tap offset is added
// (hosts keep operand buffers below 1.75 GiB)
constexpr uint32_t HOOB = 0x80000000u;

// Tile placement: workgroup b owns column block cb and row blocks [grp·tpb, +tpb) (its tiles
// share the weight column block, so BN statistics flush once); the ncb workgroups of a row
// group run together and read the same halo rows from L2.
struct HTile {
  int rho0, rows;   // first global output row (n·Ho + h), rows in the tile
  int n_first, h_first;
};

__device__ __forceinline__ HTile htile(const HaloGeom& g, int rb) {
  HTile t;
  t.rho0 = rb * g.TR;
  t.rows = min(g.TR, g.N * g.Ho - t.rho0);
  t.n_first = (int)fdiv((uint32_t)t.rho0, g.fd_Ho);
  t.h_first = t.rho0 - t.n_first * g.Ho;
  return t;
}

// DEPI (FWD loader): the DGRAD epilogue — a stride-1 input gradient as the forward conv of dy
// with the flipped filter (conv_glds.hip conv_dgrad_as_fwd)
template <int MODE, int BN, int WM, int WN, int RM, int ST, int HL, bool BIAS, bool STATS, bool NJ,
          bool DEPI = false>
__global__ void __launch_bounds__(512, 1) conv_halo_kernel(ConvArgs a, HaloGeom g) {
  static_assert(!DEPI || (MODE == FWD && !BIAS), "dgrad epilogue on the forward loader");
  constexpr int NW = 8;
  static_assert(WM * WN == NW, "8 waves");
  constexpr int TN = BN / WN, RN = TN / 16, TM = RM * 16;
  constexpr int B_BYTES = BN * 128;
  constexpr int IB = B_BYTES / (1024 * NW);  // weight DMA instructions per wave per step
  static_assert(IB >= 1 && IB * 1024 * NW == B_BYTES, "weight tile / wave mismatch");
  constexpr int HB = HL * NW * 1024;          // halo buffer bytes
  constexpr int HSLOTS = HB / 128;
  constexpr bool B_MC = (MODE == DGRAD);
  constexpr int E = RM * RN / 2;              // epilogue 16-B stores per lane
  static_assert(RN % 2 == 0, "paired 16-B stores");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  if (wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = blk / g.ncb, cb = blk - grp * g.ncb;
  const int rb0 = grp * g.tpb;
  const int ntile = min(g.tpb, g.nrb - rb0);
  if (ntile <= 0) return;
  const int n0 = cb * BN;
  const int spt = g.nchunk * g.ntap;  // K-steps per tile
  const int T = ntile * spt;

  const rsrc_t rin = make_rsrc(MODE == FWD ? (const void*)a.x : (const void*)a.dy,
                               MODE == FWD ? a.x_bytes : a.dy_bytes);
  const rsrc_t rw = make_rsrc(a.w, a.w_bytes);
  const rsrc_t rout = make_rsrc(a.out, a.out_bytes);
  const uint32_t smem_lds = (uint32_t)(size_t)(lds_char_t*)smem;

  // ---------------- load side: halo fill + weight DMA offsets of the load tile ----------------
  uint32_t foff[HL];   // per fill instruction: byte offset of this lane's 16-B piece (chunk 0)
  auto prep_fill = [&](const HTile& t) {
    const int seg = g.Ho + g.ext_h;
    const int rows0 = min(t.rows, g.Ho - t.h_first);
    const int cnt0 = rows0 + g.ext_h;
    const int rest = t.rows - rows0;
    const int hr_total = cnt0 + rest + ((rest + g.Ho - 1) / g.Ho) * g.ext_h;
#pragma unroll
    for (int j = 0; j < HL; ++j) {
      const int s = (j * NW + wid) * 8 + (lane >> 3);
      const int hr = (int)fdiv((uint32_t)s, g.fd_HP);
      const int hc = s - hr * g.HP;
      int k, hi;
      if (hr < cnt0) {
        k = 0;
        hi = t.h_first + g.oy_min + hr;
      } else {
        const int u = hr - cnt0;
        const int kk = (int)fdiv((uint32_t)u, g.fd_seg);
        k = 1 + kk;
        hi = u - kk * seg + g.oy_min;
      }
      const int wi = g.ox_min + hc;
      const bool v = hr < hr_total && hc < g.Wo + g.ext_w && (unsigned)hi < (unsigned)g.Hi &&
                     (unsigned)wi < (unsigned)g.Wi;
      const int lc = (lane & 7) ^ (s & 7);  // slot swizzle: see load_frags
      const int n = t.n_first + k;
      foff[j] = v ? (uint32_t)((((n * g.Hi + hi) * g.Wi + wi) * g.Ci + lc * 8) * 2) : HOOB;
    }
  };
  uint32_t bsrc[IB];   // per weight DMA instruction: byte offset at tap 0, chunk 0
  {
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      if constexpr (!B_MC) {
        const int row = (j * NW + wid) * 8 + (lane >> 3);
        const int co = n0 + row;
        const int lc = (lane & 7) ^ ((row >> 1) & 7);
        bsrc[j] = co < g.Co ? (uint32_t)((co * g.ldb + lc * 8) * 2) : HOOB;
      } else {
        // MC image [64 k-rows][BN cols]: k-row krow, 8-column piece col (swizzled as conv_glds)
        const int krow = (j * NW + wid) * (512 / BN) + lane / (BN / 8);
        const int q = lane % (BN / 8);
        const int swz = mc_swz<BN>(krow);
        const int col = (((q >> 1) ^ swz) << 4) + ((q & 1) << 3);
        const int c = n0 + col;
        bsrc[j] = c < g.Co ? (uint32_t)((krow * g.ldb + c) * 2) : HOOB;
      }
    }
  }

  // ---------------- cursors ----------------
  // load cursor: next step to issue (tile li, chunk lch, tap ltp); halo parity counter
  int sl = 0, li = 0, lch = 0, ltp = 0, lhalo = 0;
  uint32_t hhist = 0;  // bit i: the i-th most recent issued step had a halo fill
  HTile LT = htile(g, rb0);
  prep_fill(LT);
  auto issue = [&]() {
    char* ring = smem + 2 * HB + (sl % ST) * B_BYTES;
    bool fill = ltp == 0;
    if (fill) {
      char* hbuf = smem + (lhalo & 1) * HB;
      const uint32_t cadd = (uint32_t)(lch * 64 * 2);
#pragma unroll
      for (int j = 0; j < HL; ++j) hdma16(rin, hbuf + (j * NW + wid) * 1024, foff[j] + cadd);
      ++lhalo;
    }
    const uint32_t badd = B_MC ? (uint32_t)((lch * 64 * g.ldb + g.tap_b[ltp]) * 2)
                               : (uint32_t)((g.tap_b[ltp] + lch * 64) * 2);
#pragma unroll
    for (int j = 0; j < IB; ++j) hdma16(rw, ring + (j * NW + wid) * 1024, bsrc[j] + badd);
    hhist = (hhist << 1) | (fill ? 1u : 0u);
    ++sl;
    if (++ltp == g.ntap) {
      ltp = 0;
      if (++lch == g.nchunk) {
        lch = 0;
        if (++li < ntile) {
          LT = htile(g, rb0 + li);
          prep_fill(LT);
        }
      }
    }
  };

  // read cursor (fragment reads run half a step ahead of the MFMAs): tile ri, chunk rch, tap rtp
  int ri = 0, rch = 0, rtp = 0, rhalo = 0;
  uint32_t slot0[RM];  // per fragment: this lane's halo slot at tap delta 0 (0 for no pixel)
  auto prep_read = [&](int i) {
    const HTile t = htile(g, rb0 + i);
    const int rows0 = min(t.rows, g.Ho - t.h_first);
    const int cnt0 = rows0 + g.ext_h;
#pragma unroll
    for (int rm = 0; rm < RM; ++rm) {
      const int q = (wm * RM + rm) * 16 + (lane & 15);
      const int r = (int)fdiv((uint32_t)q, g.fd_Wo);
      const int w = q - r * g.Wo;
      int hrow;
      if (r < rows0) {
        hrow = r;
      } else {
        const int u = r - rows0;
        const int kk = (int)fdiv((uint32_t)u, g.fd_Ho);
        hrow = cnt0 + kk * (g.Ho + g.ext_h) + (u - kk * g.Ho);
      }
      slot0[rm] = r < t.rows ? (uint32_t)(hrow * g.HP + w) : 0u;
    }
  };
  prep_read(0);
  const int lane_ch = lane >> 4;
  auto load_frags = [&](int kk, bf16x8 (&af)[RM], bf16x8 (&bfg)[RN], int step_slot) {
    const uint32_t hbase = smem_lds + (uint32_t)((rhalo & 1) * HB);
    const uint32_t d = (uint32_t)g.tap_d[rtp];
#pragma unroll
    for (int rm = 0; rm < RM; ++rm) {
      // 16-B chunk c of slot s sits at position c ^ (s & 7): a ds_read_b128 lane group reads 16
      // consecutive slots (two chunks), conflict-free while a halo row's pitch HP ≡ Wo (mod 8)
      // keeps the slots consecutive mod 8 across the row wraps (halo_common pads HP to that;
      // the former (s >> 1) swizzle left 70 % of these reads 2-way conflicted)
      const uint32_t s = slot0[rm] + d;
      const uint32_t x = (s & 7u) ^ (uint32_t)(kk * 4 + lane_ch);
      af[rm] = hread(hbase + (s << 7) + (x << 4));
    }
    const uint32_t Bs = smem_lds + (uint32_t)(2 * HB + step_slot * B_BYTES);
    if constexpr (!B_MC) {
      hread_rows<RN>(bfg, Bs + (uint32_t)kc_off(wn * TN + (lane & 15), kk * 4 + lane_ch));
    } else {
      const int mck = 8 * (lane >> 4) + ((lane >> 2) & 3);
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) {
        const uint32_t ad = Bs + (uint32_t)mc_off<BN>(mck, wn * TN + rn * 16 + 4 * (lane & 3));
        bfg[rn] = kk == 0 ? hread_mc<BN, 0>(ad) : hread_mc<BN, 1>(ad);
      }
    }
  };
  auto advance_read = [&]() {
    if (++rtp == g.ntap) {
      rtp = 0;
      ++rhalo;
      if (++rch == g.nchunk) {
        rch = 0;
        if (++ri < ntile) prep_read(ri);
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
  auto mfmas = [&](const bf16x8 (&af)[RM], const bf16x8 (&bfg)[RN]) {
#pragma unroll
    for (int rm = 0; rm < RM; ++rm)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn)
        acc[rm][rn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[rn], af[rm], acc[rm][rn], 0, 0, 0);
  };

  float s_sum[RN][4], s_sq[RN][4];
#pragma unroll
  for (int rn = 0; rn < RN; ++rn)
#pragma unroll
    for (int i = 0; i < 4; ++i) s_sum[rn][i] = s_sq[rn][i] = 0.f;

  Tile Tep;  // the shared epilogue reads bn0 (mask slab column) only; rows come from rows_in
  Tep.bm0 = 0;
  Tep.bn0 = n0;
  Tep.cls = 0;
  Tep.Mc = 0;
  Tep.Kgc = 0;
  Tep.kt0 = Tep.kt1 = 0;
  Tep.split = 0;
  auto epilogue = [&](int i) {
    const HTile t = htile(g, rb0 + i);
    uint32_t rows_in[RM];
#pragma unroll
    for (int rm = 0; rm < RM; ++rm) {
      const int q = (wm * RM + rm) * 16 + (lane & 15);
      const int r = (int)fdiv((uint32_t)q, g.fd_Wo);
      const int w = q - r * g.Wo;
      rows_in[rm] = r < t.rows ? (uint32_t)(((t.rho0 + r) * g.Wo + w) * a.ldc) * 2u : ROW_OOB;
    }
    store_tile_bf16<DEPI ? DGRAD : MODE, RM, RN, TM, TN, BIAS, STATS, false, false, NJ, false,
                    true>(
        a, Tep, acc, wm, wn, lane, rout, 1.f, false, s_sum, s_sq, rows_in);
  };

  // ---------------- pipeline ----------------
  int sc = 0;          // step being computed
  int ct = 0, ck = 0;  // its tile, step within the tile
  uint32_t ehist = 0;  // bit i: the epilogue of the i-th previous step issued its stores
  for (int s = 0; s < ST - 1 && sl < T; ++s) issue();
  zero_acc();
  bf16x8 f0a[RM], f0b[RN], f1a[RM], f1b[RN];
  {
    const int ahead = sl - 1;
    wait_halo<IB, HL, E, ST>(ahead, min(1, __builtin_popcount(hhist & ((1u << ahead) - 1u))), 0);
    hbarrier();
  }
  if (sl < T) issue();
  load_frags(0, f0a, f0b, 0);
  hlgkm0();
  while (sc < T) {
    load_frags(1, f1a, f1b, sc % ST);
    mfmas(f0a, f0b);
    hlgkm0();
    advance_read();
    const bool has_next = sc + 1 < T;
    if (has_next) {
      const int ahead = sl - 1 - (sc + 1);
      const int nh = min(1, __builtin_popcount(hhist & ((1u << ahead) - 1u)));
      const int ne = min(1, __builtin_popcount(ehist & ((1u << (ST - 1)) - 1u)));
      wait_halo<IB, HL, E, ST>(ahead, nh, ne);
      hbarrier();
      if (sl < T) issue();
      load_frags(0, f0a, f0b, (sc + 1) % ST);
    }
    mfmas(f1a, f1b);
    ehist <<= 1;
    if (++ck == spt) {
      epilogue(ct);
      ehist |= 1u;
      zero_acc();
      ck = 0;
      ++ct;
    }
    if (has_next) hlgkm0();
    ++sc;
  }

  // ---------------- BN statistics flush (one per workgroup: its tiles share the columns) -----
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
    float* red = (float*)(smem + 2 * HB + ST * B_BYTES);
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
    for (int t = tid; t < 2 * BN; t += 64 * NW) {
      const int which = t / BN, nl = t - which * BN;
      const int n = n0 + nl;
      if (n < g.Co) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) v += red[(w * 2 + which) * BN + nl];
        atomicAdd(a.stats + which * g.Co + n, v);
      }
    }
  }
  (void)HSLOTS;
}

// ------------------------------------------------------------------------------------------
// weight gradient: dW[co][t][ci] = Σ_p dy[p][co] · x[p + off_t][ci]  (stride 1, 3×3 taps)
// ------------------------------------------------------------------------------------------
// A workgroup owns (co block of BM, ci chunk of 64, all 9 taps) and a split of the pixel tiles;
// per pixel tile (TRW complete output rows, ≤ 128 pixels) it stages the dy tile (an MC image:
// pixel k-rows × BM co columns) and the x halo of the ci chunk once, double-buffered, and runs
// 4 k-blocks × 9 taps of MFMAs from them — the 9 taps re-read the same halo at slot offsets, so
// x is fetched once per tile instead of once per tap (the implicit-GEMM wgrad gathers it 9×).
// Both operands are pixel-major in memory: the fragments are transposed reads
// (ds_read_b64_tr_b16) — dy from its MC image, x from the halo's slot rows.  Waves: 2 along co
// (RM = BM/32 fragments each) × 4 along ci (16 channels each); accumulators RM × 9 taps.
// Output: this split's fp32 slab rows [co][t·C + ci] (splitk_reduce sums the splits in order).
template <int KK>
__device__ __forceinline__ bf16x8 hread_tr_pair(uint32_t a0, uint32_t a1) {
  v2u32 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a1) : "memory");
  (void)KK;
  uint4 v = make_uint4(lo[0], lo[1], hi[0], hi[1]);
  return __builtin_bit_cast(bf16x8, v);
}

// 16-B chunk swizzle of the weight gradient's x-halo slot rows (chunk c of slot s at c ^ swz(s)),
// shared by the fill and the transposed reads.  TDL_HALO_WG_SWZ1 selects it at compile time:
// 1 = s & 7 (what the forward halo uses), 0 = (s >> 1) & 7 (round 5; PMC 36 % LDS bank conflicts
// in the step, profiles/r06_resnet50_b1024_pmc.txt)
#ifndef TDL_HALO_WG_SWZ1
#define TDL_HALO_WG_SWZ1 1
#endif
__device__ __forceinline__ int halo_wg_swz(int s) { return TDL_HALO_WG_SWZ1 ? (s & 7) : ((s >> 1) & 7); }

struct HaloWg {
  int nsplit, ncb, nch;  // splits, co blocks, ci chunks
  int rb_per_split;      // pixel tiles (row blocks) per split
};

// BURST: the x fragments of all 9 taps read up front, MFMAs in two bursts (0: one LDS wait per tap,
// the round-5 loop — A/B, TDL_HALO_WG_BURST=0)
template <int BM, int HL, bool BURST = true>
__global__ void __launch_bounds__(512, 1) conv_halo_wgrad_kernel(ConvArgs a, HaloGeom g, HaloWg q) {
  constexpr int NW = 8, NTAP = 9, RM = BM / 32;
  constexpr int PX = 128;                      // pixels per tile (k-rows of the dy image)
  constexpr int A_BYTES = PX * BM * 2;         // dy MC image
  constexpr int IA = A_BYTES / (1024 * NW);    // dy DMA instructions per wave
  constexpr int HB = HL * NW * 1024;           // halo buffer
  constexpr int STAGE = A_BYTES + HB;
  static_assert(IA * 1024 * NW == A_BYTES, "dy image / wave mismatch");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wco = wid >> 2, wci = wid & 3;  // 2 waves along co, 4 along ci
  if (wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int ch = blk % q.nch;
  const int cb = (blk / q.nch) % q.ncb;
  const int split = blk / (q.nch * q.ncb);
  const int rb0 = split * q.rb_per_split;
  const int ntile = min(q.rb_per_split, g.nrb - rb0);
  const int m0 = cb * BM, c0 = ch * 64;
  const rsrc_t rx = make_rsrc(a.x, a.x_bytes);
  const rsrc_t rdy = make_rsrc(a.dy, a.dy_bytes);
  const rsrc_t rout = make_rsrc(a.out, a.out_bytes);
  const uint32_t smem_lds = (uint32_t)(size_t)(lds_char_t*)smem;

  f32x4 acc[RM][NTAP];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int t = 0; t < NTAP; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (ntile > 0) {
    // ---- per-tile DMA (dy MC image + x halo of chunk c0) into stage `b` ----
    auto issue = [&](int i, int b) {
      const HTile t = htile(g, rb0 + i);
      char* As = smem + b * STAGE;
      char* Hs = As + A_BYTES;
      const int npx = t.rows * g.Wo;
      const uint32_t p0 = (uint32_t)(t.rho0 * g.Wo);
#pragma unroll
      for (int j = 0; j < IA; ++j) {
        const int krow = (j * NW + wid) * (512 / BM) + lane / (BM / 8);
        const int qq = lane % (BM / 8);
        const int col = (((qq >> 1) ^ mc_swz<BM>(krow)) << 4) + ((qq & 1) << 3);
        const int co = m0 + col;
        const bool v = krow < npx && co < g.Co;
        hdma16(rdy, As + (j * NW + wid) * 1024,
               v ? ((p0 + (uint32_t)krow) * (uint32_t)g.Co + (uint32_t)co) * 2u : HOOB);
      }
      const int seg = g.Ho + g.ext_h;
      const int rows0 = min(t.rows, g.Ho - t.h_first);
      const int cnt0 = rows0 + g.ext_h;
      const int rest = t.rows - rows0;
      const int hr_total = cnt0 + rest + ((rest + g.Ho - 1) / g.Ho) * g.ext_h;
#pragma unroll
      for (int j = 0; j < HL; ++j) {
        const int s = (j * NW + wid) * 8 + (lane >> 3);
        const int hr = (int)fdiv((uint32_t)s, g.fd_HP);
        const int hc = s - hr * g.HP;
        int k, hi;
        if (hr < cnt0) {
          k = 0;
          hi = t.h_first + g.oy_min + hr;
        } else {
          const int u = hr - cnt0;
          const int kk = (int)fdiv((uint32_t)u, g.fd_seg);
          k = 1 + kk;
          hi = u - kk * seg + g.oy_min;
        }
        const int wi = g.ox_min + hc;
        const bool v = hr < hr_total && hc < g.Wo + g.ext_w && (unsigned)hi < (unsigned)g.Hi &&
                       (unsigned)wi < (unsigned)g.Wi;
        const int lc = (lane & 7) ^ halo_wg_swz(s);
        const int n = t.n_first + k;
        hdma16(rx, Hs + (j * NW + wid) * 1024,
               v ? (uint32_t)((((n * g.Hi + hi) * g.Wi + wi) * g.Ci + c0 + lc * 8) * 2) : HOOB);
      }
    };
    // per-lane halo slots of this lane's two transposed-read pixel rows in each k-block
    const int krow_l = 8 * (lane >> 4) + ((lane >> 2) & 3);
    uint32_t sl[4][2];
    auto prep = [&](int i) {
      const HTile t = htile(g, rb0 + i);
      const int npx = t.rows * g.Wo;
      const int rows0 = min(t.rows, g.Ho - t.h_first);
      const int cnt0 = rows0 + g.ext_h;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int qp = kb * 32 + krow_l + 4 * h;
          const int r = (int)fdiv((uint32_t)qp, g.fd_Wo);
          const int w = qp - r * g.Wo;
          int hrow;
          if (r < rows0) {
            hrow = r;
          } else {
            const int u = r - rows0;
            const int kk = (int)fdiv((uint32_t)u, g.fd_Ho);
            hrow = cnt0 + kk * (g.Ho + g.ext_h) + (u - kk * g.Ho);
          }
          sl[kb][h] = qp < npx ? (uint32_t)(hrow * g.HP + w) : 0u;  // dy rows there are 0
        }
    };
    // dy fragments: MC image column base per co fragment (k-row krow_l; +4 rows: +8·BM bytes)
    uint32_t aoff[RM];
#pragma unroll
    for (int f = 0; f < RM; ++f)
      aoff[f] = (uint32_t)mc_off<BM>(krow_l, wco * (BM / 2) + f * 16 + 4 * (lane & 3));
    const uint32_t cq = (uint32_t)((wci * 16 + 4 * (lane & 3)) >> 3);  // x chunk of this lane
    const uint32_t cbyte = (uint32_t)((lane & 1) * 8);

    issue(0, 0);
    for (int i = 0; i < ntile; ++i) {
      const int b = i & 1;
      if (i + 1 < ntile) {
        issue(i + 1, b ^ 1);  // its stage was last read in step i−1 (barrier below)
        hwait<vmc(IA + HL)>();
      } else {
        hwait<0>();
      }
      hbarrier();
      prep(i);
      const uint32_t As = smem_lds + (uint32_t)(b * STAGE);
      const uint32_t Hs = As + (uint32_t)A_BYTES;
      if constexpr (!BURST) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        bf16x8 af[RM];
#pragma unroll
        for (int f = 0; f < RM; ++f) {
          const uint32_t ad = As + aoff[f] + (uint32_t)(kb * 32 * BM * 2);
          af[f] = hread_tr_pair<0>(ad, ad + 8 * BM);
        }
        auto xaddr = [&](uint32_t s0) {
          return Hs + (s0 << 7) + ((cq ^ (uint32_t)halo_wg_swz((int)s0)) << 4) + cbyte;
        };
        bf16x8 xf = hread_tr_pair<0>(xaddr(sl[kb][0] + (uint32_t)g.tap_d[0]),
                                     xaddr(sl[kb][1] + (uint32_t)g.tap_d[0]));
        hlgkm0();
#pragma unroll
        for (int t = 0; t < NTAP; ++t) {
          bf16x8 xn;
          if (t + 1 < NTAP)
            xn = hread_tr_pair<0>(xaddr(sl[kb][0] + (uint32_t)g.tap_d[t + 1]),
                                  xaddr(sl[kb][1] + (uint32_t)g.tap_d[t + 1]));
#pragma unroll
          for (int f = 0; f < RM; ++f)
            acc[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, af[f], acc[f][t], 0, 0, 0);
          hlgkm0();
          if (t + 1 < NTAP) xf = xn;
        }
      }
      } else {
      // per 32-pixel k-block: the dy fragments (RM) and the x fragments of all 9 taps are read up
      // front and the 9·RM MFMAs run in two bursts (taps 0–4, 5–8) with the reads of the next
      // block's dy and first 5 taps under the second — one LDS wait per burst, not per tap
      auto xaddr = [&](uint32_t s0) {
        return Hs + (s0 << 7) + ((cq ^ (uint32_t)halo_wg_swz((int)s0)) << 4) + cbyte;
      };
      bf16x8 af[2][RM], xf[NTAP];
      auto read_a = [&](int kb, bf16x8 (&a)[RM]) {
#pragma unroll
        for (int f = 0; f < RM; ++f) {
          const uint32_t ad = As + aoff[f] + (uint32_t)(kb * 32 * BM * 2);
          a[f] = hread_tr_pair<0>(ad, ad + 8 * BM);
        }
      };
      auto read_x = [&](int kb, int t0, int t1) {
#pragma unroll
        for (int t = 0; t < NTAP; ++t)
          if (t >= t0 && t < t1)
            xf[t] = hread_tr_pair<0>(xaddr(sl[kb][0] + (uint32_t)g.tap_d[t]),
                                     xaddr(sl[kb][1] + (uint32_t)g.tap_d[t]));
      };
      auto mfma_taps = [&](const bf16x8 (&a)[RM], int t0, int t1) {
#pragma unroll
        for (int t = 0; t < NTAP; ++t)
          if (t >= t0 && t < t1)
#pragma unroll
            for (int f = 0; f < RM; ++f)
              acc[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[t], a[f], acc[f][t], 0, 0, 0);
      };
      // (BM = 128: 36 accumulator fragments — the next block's dy is read only once this
      // block's MFMAs are issued, a second dy buffer would spill)
      constexpr bool DBA = RM <= 2;
      read_a(0, af[0]);
      read_x(0, 0, 5);
      hlgkm0();
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int ab = DBA ? (kb & 1) : 0;
        read_x(kb, 5, NTAP);
        mfma_taps(af[ab], 0, 5);
        hlgkm0();
        if (kb + 1 < 4) {
          if constexpr (DBA) read_a(kb + 1, af[(kb + 1) & 1]);
          read_x(kb + 1, 0, 5);
        }
        mfma_taps(af[ab], 5, NTAP);
        if constexpr (!DBA) {
          if (kb + 1 < 4) read_a(kb + 1, af[0]);
        }
        hlgkm0();
      }
      }
      hbarrier();  // every wave is done with stage b before step i+1 refills it
    }
  }
  // ---- this split's slab rows: lane holds dW[co = m0 + wco·BM/2 + f·16 + (lane&15)]
  //      [tap t][ci = c0 + wci·16 + (lane>>4)·4 + 0..3] (an empty split writes zeros) ----
  const uint32_t RSC = (uint32_t)(NTAP * g.Ci);
  const uint32_t slab0 = (uint32_t)split * (uint32_t)g.Co * RSC;
#pragma unroll
  for (int f = 0; f < RM; ++f) {
    const int co = m0 + wco * (BM / 2) + f * 16 + (lane & 15);
    const uint32_t ci = (uint32_t)(c0 + wci * 16 + (lane >> 4) * 4);
#pragma unroll
    for (int t = 0; t < NTAP; ++t) {
      const uint32_t off = (slab0 + (uint32_t)co * RSC + (uint32_t)t * (uint32_t)g.Ci + ci) * 4u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, acc[f][t]), rout,
                                             co < g.Co ? off : OOB, 0, 0);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Resident-weight halo conv: stride-1 3×3, 64 → 64 channels — the ResNet layer-1 body conv
// (/root/reference/core/resnet.py:137-138) and its input gradient run as a forward conv.
//
// conv_halo_kernel above streams the weight tile of every (tap, chunk) K-step through a ring and
// synchronises the workgroup once per 16 MFMAs per wave: on 56×56×64 it kept the MFMA pipes 19.5 %
// busy with 38 % of wave cycles in s_waitcnt and one SALU + one VALU instruction per MFMA of
// cursor / ring / address arithmetic (profiles/r05_halo_narrow_pmc.txt).  With 64 input channels
// the whole filter (9 taps × 64 × 64 bf16 = 72 KiB) fits in LDS beside two 40 KiB halo buffers, so
// here:
//  * the filter is DMA'd to LDS once per (persistent) workgroup and stays resident;
//  * a tile is 8 output rows × ≤ 30 columns (a 256-lane virtual 8 × 32 grid); its 10 × 32-slot
//    input halo is DMA'd once, double-buffered: the next tile's halo streams in while the 18
//    K-steps (9 taps × 2 × 32 channels) of this one run — ONE barrier per tile, none per K-step;
//  * the halo pitch (32 slots) and the tile grid are compile-time, so every fragment address is
//    one of 6 per-lane base registers (tap column s × K half) plus a compile-time ds_read offset
//    (tap row r, fragment row): the K loop has no address arithmetic at all;
//  * epilogue shared with the other conv kernels (store_tile_bf16, rows given): bias / ReLU / BN
//    Σ, Σ² (forward), ReLU bit mask / residual join / BN-backward Σg, Σg·x (input gradient).
// ------------------------------------------------------------------------------------------
struct RwGeom {
  int N, H, W, Ho, Wo;  // direct-conv input / output (DEPI: dy → dx)
  int ph, pw;           // top / left padding: tap (0, 0) of output (h, w) reads input (h−ph, w−pw)
  int TW;               // valid output columns per tile (≤ RW_HP − 2)
  int nrt, nct;         // row / column tiles per image
  int ntiles, tpb;      // tiles in all, tiles per workgroup
  int ldb;              // weight row (output channel) stride in elements: 9·64
};

constexpr int RW_TR = 8, RW_HP = 32;             // tile rows; halo pitch = virtual tile width
constexpr int RW_HB = (RW_TR + 2) * RW_HP * 128;  // 40 KiB halo buffer (64 channels per slot)
constexpr int RW_WOFF = 2 * RW_HB;               // resident filter: 9 taps × [64 rows][64 ch]
constexpr int RW_REDOFF = RW_WOFF + 9 * 8192;    // BN statistics reduction rows
constexpr int RW_LDS = RW_REDOFF + 2 * 4 * 64 * 4;
static_assert(RW_LDS <= 160 * 1024, "LDS budget");
constexpr int RW_HF = RW_HB / (8 * 1024);  // halo DMA instructions per wave (5)

template <int IMM>
__device__ __forceinline__ bf16x8 rw_read(uint32_t base) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(IMM) : "memory");
  return __builtin_bit_cast(bf16x8, v);
}

// fragments of K-step k = tap·2 + kk: A (pixels) rows 2wm + (rm >> 1), column halves rm & 1
// (ve / vo: the lane's slot in an even / odd fragment at tap column s); B (output channels
// wn·32 + rn·16 + …) from the resident filter, tap blocks 8 KiB apart (vb4: taps 4–8, keeping the
// offsets inside ds_read's 16-bit field)
template <int K>
__device__ __forceinline__ void rw_frags(const uint32_t (&ve)[3][2], const uint32_t (&vo)[3][2],
                                         const uint32_t (&vb)[2], const uint32_t (&vb4)[2],
                                         bf16x8 (&af)[4], bf16x8 (&bfg)[2]) {
  constexpr int t = K >> 1, kk = K & 1, r = t / 3, s = t % 3;
  constexpr int RO = RW_HP * 128;  // one halo row
  af[0] = rw_read<r * RO>(ve[s][kk]);
  af[1] = rw_read<r * RO>(vo[s][kk]);
  af[2] = rw_read<(r + 1) * RO>(ve[s][kk]);
  af[3] = rw_read<(r + 1) * RO>(vo[s][kk]);
  constexpr int tb = t < 4 ? t : t - 4;
  const uint32_t b = t < 4 ? vb[kk] : vb4[kk];
  bfg[0] = rw_read<tb * 8192>(b);
  bfg[1] = rw_read<tb * 8192 + 2048>(b);
}

template <int K, int N, typename F>
__device__ __forceinline__ void rw_static_for(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    rw_static_for<K + 1, N>(f);
  }
}

template <bool DEPI, bool BIAS, bool STATS, bool NJ>
__global__ void __launch_bounds__(512, 1) conv_rw_kernel(ConvArgs a, RwGeom g) {
  static_assert(!(DEPI && BIAS), "no bias on an input gradient");
  constexpr int NW = 8, RM = 4, RN = 2, TM = 64, TN = 32, NSTEP = 18;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  if (wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int t0 = blk * g.tpb;
  const int ntile = min(g.tpb, g.ntiles - t0);
  if (ntile <= 0) return;
  const rsrc_t rin = make_rsrc(a.x, a.x_bytes);
  const rsrc_t rw = make_rsrc(a.w, a.w_bytes);
  const rsrc_t rout = make_rsrc(a.out, a.out_bytes);
  const uint32_t lds0 = (uint32_t)(size_t)(lds_char_t*)smem;
  const int l15 = lane & 15, lch = lane >> 4;

  // ---- resident filter: tap t, output channel row, 64 input channels as a KC row (kc_off) ----
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int q = j * NW + wid;  // 1-KiB piece: tap q >> 3, rows (q & 7)·8 … +7
    const int tap = q >> 3, row = (q & 7) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    hdma16(rw, smem + RW_WOFF + q * 1024, (uint32_t)((row * g.ldb + tap * 64 + lc * 8) * 2));
  }

  struct RT {
    int n, h0, w0;
  };
  auto tile_at = [&](int t) {
    RT r;
    const int tc = t % g.nct, rest = t / g.nct;
    const int tr = rest % g.nrt;
    r.n = rest / g.nrt;
    r.h0 = tr * RW_TR;
    r.w0 = tc * g.TW;
    return r;
  };
  // halo slot (hr, hc) = input pixel (h0 − ph + hr, w0 − pw + hc); 16-B chunk c of slot s sits at
  // position c ^ (s & 7) (conflict-free ds_read_b128 groups: a group reads 16 consecutive slots)
  auto fill = [&](const RT& T, int buf) {
    char* hb = smem + buf * RW_HB;
#pragma unroll
    for (int j = 0; j < RW_HF; ++j) {
      const int q = j * NW + wid;
      const int s = q * 8 + (lane >> 3);
      const int hr = s / RW_HP, hc = s % RW_HP;
      const int hi = T.h0 - g.ph + hr, wi = T.w0 - g.pw + hc;
      const bool v = hc < g.TW + 2 && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      const int lc = (lane & 7) ^ (s & 7);
      hdma16(rin, hb + q * 1024,
             v ? (uint32_t)((((T.n * g.H + hi) * g.W + wi) * 64 + lc * 8) * 2) : HOOB);
    }
  };

  // per-lane fragment bases.  A: slot of (row 2wm, column l15 + s) — an odd fragment adds 16
  // columns, except in lanes whose column would pass the tile width: they read column l15 (finite
  // halo data) and their output rows are dropped.  B: filter row wn·32 + l15, K half kk.
  const uint32_t d16 = 16 + l15 < g.TW ? 16u * 128u : 0u;
  uint32_t vb[2], vb4[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    vb[kk] = lds0 + (uint32_t)(RW_WOFF + (wn * 32 + l15) * 128 +
                               ((((kk * 4 + lch) ^ ((l15 >> 1) & 7))) << 4));
    vb4[kk] = vb[kk] + 4u * 8192u;
  }
  uint32_t va[3][2];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      va[s][kk] = (uint32_t)((2 * wm * RW_HP + l15 + s) * 128 +
                             ((((l15 + s) & 7) ^ (kk * 4 + lch)) << 4));

  f32x4 acc[RM][RN];
  float s_sum[RN][4], s_sq[RN][4];
#pragma unroll
  for (int rn = 0; rn < RN; ++rn)
#pragma unroll
    for (int i = 0; i < 4; ++i) s_sum[rn][i] = s_sq[rn][i] = 0.f;
  Tile Tep;  // the shared epilogue reads bn0 (mask slab column) only; rows come from rows_in
  Tep.bm0 = 0;
  Tep.bn0 = 0;
  Tep.cls = 0;
  Tep.Mc = 0;
  Tep.Kgc = 0;
  Tep.kt0 = Tep.kt1 = 0;
  Tep.split = 0;
  constexpr int E = RM * RN / 2;  // epilogue 16-B stores per lane (64 = WN·TN columns: wide)

  RT cur = tile_at(t0);
  fill(cur, 0);
  hwait<0>();
  hbarrier();
  for (int i = 0; i < ntile; ++i) {
    const int buf = i & 1;
    RT nxt = cur;
    if (i + 1 < ntile) {
      nxt = tile_at(t0 + i + 1);
      fill(nxt, buf ^ 1);  // last read in tile i − 1 (barrier below)
    }
    // the output rows of this tile's lanes: (2wm + (rm >> 1), (rm & 1)·16 + l15)
    uint32_t rows_in[RM];
#pragma unroll
    for (int rm = 0; rm < RM; ++rm) {
      const int h = cur.h0 + 2 * wm + (rm >> 1), col = (rm & 1) * 16 + l15, w = cur.w0 + col;
      rows_in[rm] = h < g.Ho && col < g.TW && w < g.Wo
                        ? (uint32_t)(((cur.n * g.Ho + h) * g.Wo + w) * a.ldc) * 2u
                        : ROW_OOB;
    }
    // input gradient: its epilogue's loads (BN input, mask words, previous dx) go out now and
    // land under the K loop
    EpiPre<RM, RN> pre;
    if constexpr (DEPI) epi_preload_dgrad<RM, RN, TN, STATS, NJ>(a, Tep, wn, lane, rout, rows_in, pre);
    const uint32_t hb = lds0 + (uint32_t)(buf * RW_HB);
    uint32_t ve[3][2], vo[3][2];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        ve[s][kk] = hb + va[s][kk];
        vo[s][kk] = ve[s][kk] + d16;
      }
#pragma unroll
    for (int rm = 0; rm < RM; ++rm)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) acc[rm][rn] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa[2][RM], fb[2][RN];
    rw_frags<0>(ve, vo, vb, vb4, fa[0], fb[0]);
    hlgkm0();
    rw_static_for<0, NSTEP>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if constexpr (k + 1 < NSTEP) rw_frags<k + 1>(ve, vo, vb, vb4, fa[(k + 1) & 1], fb[(k + 1) & 1]);
#pragma unroll
      for (int rm = 0; rm < RM; ++rm)
#pragma unroll
        for (int rn = 0; rn < RN; ++rn)
          acc[rm][rn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[k & 1][rn], fa[k & 1][rm],
                                                                acc[rm][rn], 0, 0, 0);
      hlgkm0();
    });
    // ---- epilogue ----
    store_tile_bf16<DEPI ? DGRAD : FWD, RM, RN, TM, TN, BIAS, STATS, false, false, NJ, false,
                    true, false, DEPI>(a, Tep, acc, wm, wn, lane, rout, 1.f, false, s_sum, s_sq,
                                       rows_in, &pre);
    // the next tile's halo has landed (only this epilogue's stores may still be in flight) and
    // every wave is done with this tile's buffer
    hwait<E>();
    hbarrier();
    cur = nxt;
  }

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
    float* red = (float*)(smem + RW_REDOFF);
    if ((lane & 15) == 0) {
#pragma unroll
      for (int rn = 0; rn < RN; ++rn)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int nl = wn * TN + rn * 16 + (lane >> 4) * 4 + i;
          red[(wm * 2 + 0) * 64 + nl] = s_sum[rn][i];
          red[(wm * 2 + 1) * 64 + nl] = s_sq[rn][i];
        }
    }
    __syncthreads();
    for (int t = tid; t < 2 * 64; t += 64 * NW) {
      const int which = t / 64, nl = t - which * 64;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += red[(w * 2 + which) * 64 + nl];
      atomicAdd(a.stats + which * 64 + nl, v);
    }
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
struct HCfg {
  int bn, st, hl;
};

constexpr int halo_lds(int bn, int st, int hl) {
  return 2 * hl * 8 * 1024 + st * bn * 128 + 2 * 4 * bn * 4;
}

int henv(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

template <int MODE, int BN, int ST, int HL, bool BIAS, bool STATS, bool NJ, bool DEPI = false>
void launch_h(const ConvArgs& a, const HaloGeom& g, int blocks, hipStream_t st) {
  auto k = conv_halo_kernel<MODE, BN, 4, 2, 4, ST, HL, BIAS, STATS, NJ, DEPI>;
  constexpr int lds = halo_lds(BN, ST, HL);
  static_assert(lds <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), lds, st, a, g);
}

// worst-case halo rows of a tile of TR output rows (images of Ho rows, ext_h halo rows each)
int halo_rows(int TR, int Ho, int ext_h) {
  int segs;
  if (Ho % TR == 0) segs = 1;
  else if (TR % Ho == 0) segs = TR / Ho;
  else segs = (TR - 1 + Ho - 1) / Ho + 1;
  return TR + segs * ext_h;
}

// Fill the geometry for a direct conv with output Ho×Wo, taps (oy_t, ox_t) and weight offsets;
// pick TR / BN / HL.  Returns false when no configuration fits.
bool plan_halo(HaloGeom& g, int bn, HCfg& cfg) {
  const int hl_max = bn == 128 ? 6 : 8;
  const int st = bn == 128 ? 3 : (hl_max == 8 ? 3 : 4);
  int best_tr = 0, best_hl = 0;
  for (int TR = std::max(1, 256 / g.Wo); TR >= 1; --TR) {
    if (TR * g.Wo > 256) continue;
    const int hr = halo_rows(TR, g.Ho, g.ext_h);
    const int slots = hr * g.HP;
    const int hl = (slots + 63) / 64;
    if (hl > hl_max) continue;
    best_tr = TR;
    best_hl = hl <= 6 ? 6 : 8;
    break;
  }
  if (!best_tr) return false;
  g.TR = best_tr;
  cfg.bn = bn;
  cfg.hl = best_hl;
  cfg.st = bn == 128 ? 3 : (best_hl == 8 ? 3 : 4);
  (void)st;
  return true;
}

template <int MODE, bool BIAS, bool STATS, bool NJ, bool DEPI = false>
void launch_hcfg(const ConvArgs& a, const HaloGeom& g, const HCfg& c, int blocks, hipStream_t st) {
  if (c.bn == 128) {
    launch_h<MODE, 128, 3, 6, BIAS, STATS, NJ, DEPI>(a, g, blocks, st);
  } else if (c.hl == 8) {
    launch_h<MODE, 64, 3, 8, BIAS, STATS, NJ, DEPI>(a, g, blocks, st);
  } else {
    launch_h<MODE, 64, 4, 6, BIAS, STATS, NJ, DEPI>(a, g, blocks, st);
  }
}

bool halo_common(const ConvArgs& a, HaloGeom& g, int R, int S, const int* oy, const int* ox,
                 int bn, HCfg& cfg, int& blocks) {
  g.ntap = R * S;
  g.nchunk = g.Ci / 64;
  int oy_min = 1 << 30, oy_max = -(1 << 30), ox_min = 1 << 30, ox_max = -(1 << 30);
  for (int t = 0; t < g.ntap; ++t) {
    oy_min = std::min(oy_min, oy[t]);
    oy_max = std::max(oy_max, oy[t]);
    ox_min = std::min(ox_min, ox[t]);
    ox_max = std::max(ox_max, ox[t]);
  }
  g.oy_min = oy_min;
  g.ox_min = ox_min;
  g.ext_h = oy_max - oy_min;
  g.ext_w = ox_max - ox_min;
  // halo pitch: padded to HP ≡ Wo (mod 8) for conflict-free fragment reads (load_frags), unless
  // the padding costs output rows per tile
  g.HP = g.Wo + ((g.ext_w + 7) & ~7);
  HCfg cp;
  const bool padded = plan_halo(g, bn, cp);
  const int tr_padded = padded ? g.TR : 0;
  g.HP = g.Wo + g.ext_w;
  if (!plan_halo(g, bn, cfg)) return false;
  if (padded && tr_padded >= g.TR) {
    g.HP = g.Wo + ((g.ext_w + 7) & ~7);
    g.TR = tr_padded;
    cfg = cp;
  }
  for (int t = 0; t < g.ntap; ++t) g.tap_d[t] = (oy[t] - oy_min) * g.HP + (ox[t] - ox_min);
  g.nrb = cdiv((long)g.N * g.Ho, g.TR);
  g.ncb = cdiv(g.Co, cfg.bn);
  const int cus = henv("TDL_HALO_SLOTS", 256);
  const long tiles = (long)g.nrb * g.ncb;
  g.tpb = (int)std::max<long>(1, (tiles + cus - 1) / cus);
  blocks = cdiv(g.nrb, g.tpb) * g.ncb;
  g.fd_HP = make_fastdiv((uint32_t)g.HP);
  g.fd_Wo = make_fastdiv((uint32_t)g.Wo);
  g.fd_Ho = make_fastdiv((uint32_t)g.Ho);
  g.fd_seg = make_fastdiv((uint32_t)(g.Ho + g.ext_h));
  return true;
}

template <int BM>
void launch_hw(const ConvArgs& a, const HaloGeom& g, const HaloWg& q, hipStream_t st) {
  static const bool burst = henv("TDL_HALO_WG_BURST", 1) != 0;
  auto k = burst ? conv_halo_wgrad_kernel<BM, 4, true> : conv_halo_wgrad_kernel<BM, 4, false>;
  constexpr int lds = 2 * (128 * BM * 2 + 4 * 8 * 1024);
  static_assert(lds <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const int blocks = q.nsplit * q.ncb * q.nch;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), lds, st, a, g, q);
}

// geometry of a stride-1 3×3 weight gradient on the halo kernel (pixel tiles of ≤ 128 pixels, a
// 4-instruction-per-wave halo); false when not eligible
bool plan_halo_wgrad(const ConvArgs& a, HaloGeom& g, HaloWg& q, int& bm) {
  if (a.sh != 1 || a.sw != 1 || a.R != 3 || a.S != 3 || a.C % 64 || a.K % 8) return false;
  if (a.x_bytes >= 0x70000000u || a.dy_bytes >= 0x70000000u) return false;
  g = HaloGeom{};
  g.N = a.N; g.Hi = a.H; g.Wi = a.W; g.Ci = a.C;
  g.Ho = a.Ho; g.Wo = a.Wo; g.Co = a.K;
  g.ntap = 9;
  g.nchunk = a.C / 64;
  int oy[9], ox[9];
  for (int r = 0; r < 3; ++r)
    for (int s = 0; s < 3; ++s) {
      oy[r * 3 + s] = r * a.dh - a.ph;
      ox[r * 3 + s] = s * a.dw - a.pw;
    }
  int oy_min = 1 << 30, oy_max = -(1 << 30), ox_min = 1 << 30, ox_max = -(1 << 30);
  for (int t = 0; t < 9; ++t) {
    oy_min = std::min(oy_min, oy[t]);
    oy_max = std::max(oy_max, oy[t]);
    ox_min = std::min(ox_min, ox[t]);
    ox_max = std::max(ox_max, ox[t]);
  }
  g.oy_min = oy_min; g.ox_min = ox_min;
  g.ext_h = oy_max - oy_min; g.ext_w = ox_max - ox_min;
  g.HP = g.Wo + g.ext_w;
  for (int t = 0; t < 9; ++t) g.tap_d[t] = (oy[t] - oy_min) * g.HP + (ox[t] - ox_min);
  int TR = 0;
  for (int tr = std::max(1, 128 / g.Wo); tr >= 1; --tr) {
    if (tr * g.Wo > 128) continue;
    if (halo_rows(tr, g.Ho, g.ext_h) * g.HP <= 4 * 64) {
      TR = tr;
      break;
    }
  }
  if (!TR) return false;
  g.TR = TR;
  g.nrb = cdiv((long)g.N * g.Ho, TR);
  bm = henv("TDL_HALO_WG_BM", a.K >= 128 ? 128 : 64);
  q.ncb = cdiv(a.K, bm);
  q.nch = a.C / 64;
  // ≈ 2 workgroups per CU slot in all, ≥ 8 pixel tiles per split
  const int target = henv("TDL_HALO_WG_TARGET", 512);
  int ns = std::max(1, target / (q.ncb * q.nch));
  ns = std::min(ns, std::max(1, g.nrb / 8));
  q.rb_per_split = cdiv(g.nrb, ns);
  q.nsplit = cdiv(g.nrb, q.rb_per_split);
  g.fd_HP = make_fastdiv((uint32_t)g.HP);
  g.fd_Wo = make_fastdiv((uint32_t)g.Wo);
  g.fd_Ho = make_fastdiv((uint32_t)g.Ho);
  g.fd_seg = make_fastdiv((uint32_t)(g.Ho + g.ext_h));
  return true;
}

// the resident-weight conv's geometry; false when the kernel does not take the problem
bool plan_rw(const ConvArgs& a, RwGeom& g, int& blocks) {
  if (a.R != 3 || a.S != 3 || a.sh != 1 || a.sw != 1 || a.dh != 1 || a.dw != 1) return false;
  if (a.C != 64 || a.K != 64 || a.ldc < 64 || a.ldc % 8) return false;
  if (a.aff || a.fp8 || a.res) return false;
  if (a.mask && a.ldc % 64) return false;  // mask slabs: 64-column rows
  if (a.x_bytes >= 0x70000000u || a.w_bytes >= 0x70000000u || a.out_bytes >= ROW_OOB) return false;
  if (a.Ho < 1 || a.Wo < 1 || a.Ho > a.H + 2 || a.Wo > a.W + 2) return false;
  g = RwGeom{};
  g.N = a.N; g.H = a.H; g.W = a.W; g.Ho = a.Ho; g.Wo = a.Wo;
  g.ph = a.ph; g.pw = a.pw;
  g.nct = cdiv(a.Wo, RW_HP - 2);
  g.TW = cdiv(a.Wo, g.nct);
  g.nrt = cdiv(a.Ho, RW_TR);
  const long tiles = (long)a.N * g.nrt * g.nct;
  if (tiles >= (1L << 30)) return false;
  g.ntiles = (int)tiles;
  const int cus = henv("TDL_RW_SLOTS", 256);
  g.tpb = std::max(1, cdiv(g.ntiles, cus));
  blocks = cdiv(g.ntiles, g.tpb);
  g.ldb = 9 * 64;
  return true;
}

template <bool DEPI, bool BIAS, bool STATS, bool NJ>
void launch_rw(const ConvArgs& a, const RwGeom& g, int blocks, hipStream_t st) {
  auto k = conv_rw_kernel<DEPI, BIAS, STATS, NJ>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, RW_LDS);
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), RW_LDS, st, a, g);
}

}  // namespace

// route row fwd.halo.rw64: the resident-weight 3×3 64 → 64 forward (false: not eligible)
bool conv_fwd_rw(const ConvArgs& a, hipStream_t st) {
  RwGeom g;
  int blocks;
  if (!plan_rw(a, g, blocks)) return false;
  const bool stats = a.stats != nullptr, bias = a.bias != nullptr;
  if (bias) {
    if (stats) launch_rw<false, true, true, true>(a, g, blocks, st);
    else launch_rw<false, true, false, true>(a, g, blocks, st);
  } else {
    if (stats) launch_rw<false, false, true, true>(a, g, blocks, st);
    else launch_rw<false, false, false, true>(a, g, blocks, st);
  }
  return true;
}

// route row dgrad.asfwd.rw64: a stride-1 3×3 64 → 64 input gradient already rewritten as the
// forward conv of dy with the flipped filter (conv_dgrad_as_fwd), DGRAD epilogue (ReLU bit mask,
// residual join, BN-backward sums); *fused: a.stats was filled
bool conv_fwd_rw_depi(const ConvArgs& a, hipStream_t st, bool* fused) {
  if (fused) *fused = false;
  RwGeom g;
  int blocks;
  if (a.bias || !plan_rw(a, g, blocks)) return false;
  const bool stats = a.stats != nullptr && a.bn_x != nullptr;
  ConvArgs b = a;
  if (!stats) b.stats = nullptr;
  b.Ng = 64;
  if (stats) {
    if (a.beta) launch_rw<true, false, true, false>(b, g, blocks, st);
    else launch_rw<true, false, true, true>(b, g, blocks, st);
  } else {
    if (a.beta) launch_rw<true, false, false, false>(b, g, blocks, st);
    else launch_rw<true, false, false, true>(b, g, blocks, st);
  }
  if (fused) *fused = stats;
  return true;
}

// route rows wgrad.halo.*: false when the kernel does not take the problem
bool conv_wgrad_halo_plan(const ConvArgs& a, WgradPlan* p) {
  if (a.aff || a.fp8) return false;
  HaloGeom g;
  HaloWg q;
  int bm;
  if (!plan_halo_wgrad(a, g, q, bm)) return false;
  p->impl = 2;
  p->cfg = bm;
  p->bm = bm;
  p->bn = 64;
  p->splits = q.nsplit;
  p->kps = q.rb_per_split;
  return true;
}

void conv_wgrad_halo_launch(const ConvArgs& a, const WgradPlan& p, hipStream_t st) {
  HaloGeom g;
  HaloWg q;
  int bm;
  if (!plan_halo_wgrad(a, g, q, bm) || q.nsplit != p.splits)
    throw std::runtime_error("conv_wgrad_halo_launch: plan mismatch");
  if (bm == 128) launch_hw<128>(a, g, q, st);
  else launch_hw<64>(a, g, q, st);
}

static int g_halo_override = -1;
int conv_halo_mode() {
  static int m = henv("TDL_HALO", 1);
  return g_halo_override >= 0 ? g_halo_override : m;
}
void conv_set_halo_mode(int mode) { g_halo_override = mode; }

// FWD, stride 1: true when the halo kernel ran
bool conv_fwd_halo(const ConvArgs& a, hipStream_t st) {
  if (a.aff) return false;  // no folded-BN staging
  if (a.sh != 1 || a.sw != 1 || a.res || a.fp8) return false;
  const int ntap = a.R * a.S;
  if (ntap < 3 || ntap > HALO_MAXTAP || a.C % 64 || a.K % 8 || a.ldc % 8) return false;
  if (a.x_bytes >= 0x70000000u || a.w_bytes >= 0x70000000u || a.out_bytes >= ROW_OOB) return false;
  HaloGeom g{};
  g.N = a.N; g.Hi = a.H; g.Wi = a.W; g.Ci = a.C;
  g.Ho = a.Ho; g.Wo = a.Wo; g.Co = a.K;
  g.ldb = ntap * a.C;
  int oy[HALO_MAXTAP], ox[HALO_MAXTAP];
  for (int r = 0; r < a.R; ++r)
    for (int s = 0; s < a.S; ++s) {
      const int t = r * a.S + s;
      oy[t] = r * a.dh - a.ph;
      ox[t] = s * a.dw - a.pw;
      g.tap_b[t] = t * a.C;
    }
  HCfg c;
  int blocks;
  const int bn = henv("TDL_HALO_BN", a.K >= 128 ? 128 : 64);
  if (!halo_common(a, g, a.R, a.S, oy, ox, bn, c, blocks)) return false;
  const bool stats = a.stats != nullptr, bias = a.bias != nullptr;
  if (bias) {
    if (stats) launch_hcfg<FWD, true, true, true>(a, g, c, blocks, st);
    else launch_hcfg<FWD, true, false, true>(a, g, c, blocks, st);
  } else {
    if (stats) launch_hcfg<FWD, false, true, true>(a, g, c, blocks, st);
    else launch_hcfg<FWD, false, false, true>(a, g, c, blocks, st);
  }
  return true;
}

// A stride-1 input gradient prepared as a forward conv (conv_dgrad_as_fwd: x = dy, w = the
// flipped filter, C / K swapped) on the halo forward loader with the DGRAD epilogue — where the
// halo forward wins (≤ 64 output channels, 3×3: ResNet layer1, 698 → 503 µs at b1024,
// bench/dgrad_paths.py).  *fused: the BN-backward statistics were written.
bool conv_fwd_halo_depi(const ConvArgs& a, hipStream_t st, bool* fused) {
  if (fused) *fused = false;
  if (a.aff || a.fp8 || a.sh != 1 || a.sw != 1) return false;
  const int ntap = a.R * a.S;
  if (ntap < 3 || ntap > HALO_MAXTAP || a.C % 64 || a.K % 8 || a.ldc % 8) return false;
  if (a.mask && a.ldc % 64) return false;
  if (a.x_bytes >= 0x70000000u || a.w_bytes >= 0x70000000u || a.out_bytes >= ROW_OOB) return false;
  const bool stats = a.stats != nullptr && a.bn_x != nullptr;
  // the statistics form lost to the DGRAD kernel's 256×64 tiles (ResNet layer1 3×3, b1024: 700
  // vs 607 µs — profiles/r05_dgrad_as_fwd.txt): plain / join only
  if (stats) return false;
  HaloGeom g{};
  g.N = a.N; g.Hi = a.H; g.Wi = a.W; g.Ci = a.C;
  g.Ho = a.Ho; g.Wo = a.Wo; g.Co = a.K;
  g.ldb = ntap * a.C;
  int oy[HALO_MAXTAP], ox[HALO_MAXTAP];
  for (int r = 0; r < a.R; ++r)
    for (int s = 0; s < a.S; ++s) {
      const int t = r * a.S + s;
      oy[t] = r * a.dh - a.ph;
      ox[t] = s * a.dw - a.pw;
      g.tap_b[t] = t * a.C;
    }
  HCfg c;
  int blocks;
  const int bn = henv("TDL_HALO_BN", a.K >= 128 ? 128 : 64);
  if (!halo_common(a, g, a.R, a.S, oy, ox, bn, c, blocks)) return false;
  ConvArgs b = a;
  b.stats = nullptr;
  launch_hcfg<FWD, false, false, false, true>(b, g, c, blocks, st);
  return true;
}

// DGRAD, stride 1 (one parity class): true when the halo kernel ran; *fused: a.stats filled
bool conv_dgrad_halo(const ConvArgs& a, hipStream_t st, bool* fused) {
  if (fused) *fused = false;
  if (a.aff) return false;  // the folded-BN mask: LDS-DMA statistics epilogue only
  if (a.sh != 1 || a.sw != 1 || a.fp8 || a.dg_masked) return false;
  const int ntap = a.R * a.S;
  if (ntap < 3 || ntap > HALO_MAXTAP || a.K % 64 || a.C % 8 || a.ldc % 8) return false;
  if (a.dy_bytes >= 0x70000000u || a.w_bytes >= 0x70000000u || a.out_bytes >= ROW_OOB) return false;
  const bool stats = a.stats && a.bn_x;
  if (a.mask && a.ldc % 64) return false;  // mask slabs: 64-column rows
  HaloGeom g{};
  g.N = a.N; g.Hi = a.Ho; g.Wi = a.Wo; g.Ci = a.K;
  g.Ho = a.H; g.Wo = a.W; g.Co = a.C;
  g.ldb = ntap * a.C;
  int oy[HALO_MAXTAP], ox[HALO_MAXTAP];
  for (int r = 0; r < a.R; ++r)
    for (int s = 0; s < a.S; ++s) {
      const int t = r * a.S + s;
      oy[t] = a.ph - r * a.dh;
      ox[t] = a.pw - s * a.dw;
      g.tap_b[t] = t * a.C;
    }
  HCfg c;
  int blocks;
  // 128-wide dx tiles with both the join's previous-dx and the BN-statistics x registers spill:
  // 64-wide there
  const int bn = henv("TDL_HALO_BN", a.C >= 128 && !(stats && a.beta) ? 128 : 64);
  if (!halo_common(a, g, a.R, a.S, oy, ox, bn, c, blocks)) return false;
  ConvArgs b = a;
  b.Ng = a.C;  // the shared epilogue's column count
  if (!stats) b.stats = nullptr;
  const bool nj = !a.beta;
  if (stats) {
    if (nj) launch_hcfg<DGRAD, false, true, true>(b, g, c, blocks, st);
    else launch_hcfg<DGRAD, false, true, false>(b, g, c, blocks, st);
  } else {
    if (nj) launch_hcfg<DGRAD, false, false, true>(b, g, c, blocks, st);
    else launch_hcfg<DGRAD, false, false, false>(b, g, c, blocks, st);
  }
  if (fused) *fused = stats;
  return true;
}

}  // namespace tdl
