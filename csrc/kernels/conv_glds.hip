// LDS-DMA pipelined implicit-GEMM convolution for gfx950 (MI355X / CDNA4) — the large-problem
// path of FWD / DGRAD / WGRAD (conv_gemm.hip keeps the register-staged kernel for small or
// unaligned problems).
//
// Why a second kernel: the register-staged 128×128 kernel issues the loads of K-step s+1, runs
// the 16 MFMAs of step s (≈256 cycles) and then waits for those loads — far shorter than an
// HBM/L2 round trip, so every step exposes most of the memory latency (300–550 TF/s measured on
// the ResNet-50 shapes).  Here:
//
//  * operands go global → LDS directly with `buffer_load_dwordx4 … lds` (LDS-DMA, 16 B per lane).
//    The buffer form keeps the range-checked descriptors of conv_gemm.hip: a padding tap / ragged
//    edge gets offset OOB and the DMA writes zeros — the implicit-GEMM gather needs no branches.
//    The LDS image is lane-linear per wave instruction (1 KiB), so the bank swizzles of
//    conv_common.h are applied on the SOURCE side (each lane fetches the logical chunk that
//    belongs at its physical slot) and again on the ds_read side (guide rule 21).
//  * a STAGES-deep ring (3–4 × up to 48 KiB), one raw `s_barrier` per K-step and a counted
//    `s_waitcnt vmcnt(N)` that leaves the younger stages in flight across the barrier
//    (`__syncthreads()` would emit vmcnt(0) and drain the ring).
//  * 256-row tiles on 8 (or 4) waves, each wave a 64×64 sub-tile (RM = RN = 4 16×16×32 MFMA
//    fragments): 32 FLOP per LDS byte read.
//  * persistent workgroups: one workgroup per CU walks ⌈tiles/256⌉ tiles as one flat
//    (tile, K-step) sequence, so the ring stays full across tile boundaries and the pipeline
//    fill is paid once per CU, not once per tile.
//
// Epilogue (bias, ReLU, BN Σ/Σ² statistics of the stored bf16 values, DGRAD class scatter, WGRAD
// fp32 split-K slabs) is the same as conv_gemm.hip's.
#include "conv_common.h"
#include "conv_route.h"

namespace tdl {

namespace {
using namespace convk;

typedef __attribute__((address_space(3))) void lds_void_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

constexpr int vm63(int v) { return v < 63 ? v : 63; }  // 6-bit vmcnt field: a smaller count only waits longer

// s_waitcnt vmcnt(LPS·ahead + E·ne) with the immediates the ring can need.  The steady states
// come first — long-K tiles (ahead = ST−2, no epilogue in the window) and one-K-step tiles (an
// epilogue every step) — so the usual wait is two scalar compares, not a branch tree.
template <int LPS, int E, int ST>
__device__ __forceinline__ void wait_ring(int ahead, int ne) {
  if (ahead == ST - 2) {
    if (ne == 0) { wait_vmcnt<vm63(LPS * (ST - 2))>(); return; }
    if (ne == ST - 1) { wait_vmcnt<vm63(LPS * (ST - 2) + E * (ST - 1))>(); return; }
  }
#define TDL_W(A, NE)                                  \
  if (ahead == A && ne == NE) {                       \
    wait_vmcnt<vm63(LPS * A + E * NE)>();             \
    return;                                           \
  }
  TDL_W(0, 0) TDL_W(0, 1)
  if constexpr (ST >= 3) { TDL_W(0, 2) TDL_W(1, 1) }
  if constexpr (ST >= 4) { TDL_W(0, 3) TDL_W(1, 0) TDL_W(1, 2) TDL_W(1, 3) TDL_W(2, 1) TDL_W(2, 2) }
#undef TDL_W
  wait_vmcnt<0>();
}

typedef __attribute__((address_space(3))) char lds_char_t;

// Fragment reads are inline asm: hipcc cannot order LDS reads against in-flight LDS-DMA and
// otherwise emits `s_waitcnt vmcnt(0)` before the first ds_read of every K-step, draining the
// ring.  Visibility of the DMA'd data is established explicitly (counted vmcnt + s_barrier), and
// the reads are retired with an explicit lgkmcnt wait followed by sched_barrier(0) so no MFMA is
// hoisted above it (guide rule 18).
__device__ __forceinline__ bf16x8 lds_read_kc(uint32_t tile, int row, int chunk) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(tile + (uint32_t)kc_off(row, chunk)) : "memory");
  return __builtin_bit_cast(bf16x8, v);
}
// I-th .. N-1-th 16-row fragment of a KC image column block: rows 16 apart are 2048 B apart
// and share the swizzle ((row >> 1) & 7 only sees the low 4 row bits), so one base address per
// block serves every fragment with ds_read immediate offsets (no per-fragment v_add)
template <int N, int I = 0>
__device__ __forceinline__ void lds_read_kc_rows(bf16x8 (&f)[N], uint32_t base) {
  if constexpr (I < N) {
    uint4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(I * 2048) : "memory");
    f[I] = __builtin_bit_cast(bf16x8, v);
    lds_read_kc_rows<N, I + 1>(f, base);
  }
}
// MC fragment at (kk, col block): addr = tile + mc_off<COLS>(krow of kk = 0, col).  The k-rows
// +4 (the fragment's second half) and +32 (kk = 1) keep the swizzle (krow's bits 0-1 and 3 are
// unchanged), so both are immediate offsets of one base address per column block
template <int COLS, int KK>
__device__ __forceinline__ bf16x8 lds_read_mc_imm(uint32_t addr) {
  v2u32 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(addr), "n"(KK * 64 * COLS) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(addr), "n"(KK * 64 * COLS + 8 * COLS) : "memory");
  uint4 v = make_uint4(lo[0], lo[1], hi[0], hi[1]);
  return __builtin_bit_cast(bf16x8, v);
}
template <int COLS>
__device__ __forceinline__ bf16x8 lds_read_mc(uint32_t tile, int krow, int col) {
  v2u32 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(tile + (uint32_t)mc_off<COLS>(krow, col)) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(tile + (uint32_t)mc_off<COLS>(krow + 4, col)) : "memory");
  uint4 v = make_uint4(lo[0], lo[1], hi[0], hi[1]);
  return __builtin_bit_cast(bf16x8, v);
}
typedef int i32x8 __attribute__((ext_vector_type(8)));
// fp8 A/B fragment of v_mfma_scale_f32_16x16x128_f8f6f4: lane l holds bytes k = 32·(l>>4) … +31 of
// row l&15 (any k permutation applied to both operands is exact; dev/tools/mfma_fp8_layout.hip)
__device__ __forceinline__ i32x8 lds_read_kc_f8(uint32_t tile, int row, int g) {
  uint4 lo, hi;
  asm volatile("ds_read_b128 %0, %1" : "=v"(lo) : "v"(tile + (uint32_t)kc_off(row, 2 * g)) : "memory");
  asm volatile("ds_read_b128 %0, %1" : "=v"(hi) : "v"(tile + (uint32_t)kc_off(row, 2 * g + 1)) : "memory");
  i32x8 v;
  v[0] = (int)lo.x; v[1] = (int)lo.y; v[2] = (int)lo.z; v[3] = (int)lo.w;
  v[4] = (int)hi.x; v[5] = (int)hi.y; v[6] = (int)hi.z; v[7] = (int)hi.w;
  return v;
}

// fp8 MC image (weight gradients: [128 k-rows = pixels][COLS bytes]): 16-B chunk c of k-row r
// is stored at chunk c ^ mc8_swz(r), so the 16 k-rows a 32-lane half reads with one
// ds_read_b64_tr_b8 (two 8-row blocks 32 rows apart, one chunk column) sit on distinct banks
template <int COLS>
__device__ __forceinline__ int mc8_swz(int r) {
  static_assert(COLS == 256 || COLS == 128, "fp8 MC images: 128- or 256-byte rows");
  if constexpr (COLS == 256)
    return (r & 7) | (((r >> 5) & 1) << 3);
  else
    return ((r >> 1) & 3) | (((r >> 5) & 1) << 2);
}
template <int COLS>
__device__ __forceinline__ int mc8_off(int r, int chunk) {
  return r * COLS + ((chunk ^ mc8_swz<COLS>(r)) << 4);
}
// fp8 fragment of v_mfma_scale_f32_16x16x128_f8f6f4 from an MC image: four ds_read_b64_tr_b8
// (per 16-lane group a block of 8 k-rows × 16 columns, delivered column-major: lane i of the group
// gets column i of the 8 rows; lane 2q+p supplies row q, bytes 8p … 8p+7).  Lane l (group
// g = l>>4) holds column col0 + (l&15) of k-rows 32g + 8j + 0..7, j = 0..3 — one k order shared
// by both operands, which is all the product needs (lds_read_kc_f8).  The swizzle of the rows a
// lane reads does not change with j, so one base address serves the four reads.
template <int COLS>
__device__ __forceinline__ i32x8 lds_read_mc_f8(uint32_t tile, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const uint32_t base = tile + (uint32_t)(mc8_off<COLS>(32 * g + (i >> 1), col0 >> 4) + 8 * (i & 1));
  v2u32 x0, x1, x2, x3;
  asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(x0) : "v"(base) : "memory");
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(x1) : "v"(base), "n"(8 * COLS) : "memory");
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(x2) : "v"(base), "n"(16 * COLS) : "memory");
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(x3) : "v"(base), "n"(24 * COLS) : "memory");
  i32x8 v;
  v[0] = (int)x0[0]; v[1] = (int)x0[1]; v[2] = (int)x1[0]; v[3] = (int)x1[1];
  v[4] = (int)x2[0]; v[5] = (int)x2[1]; v[6] = (int)x3[0]; v[7] = (int)x3[1];
  return v;
}

__device__ __forceinline__ void lgkm_wait0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// one wave instruction: 64 lanes × 16 B from per-lane buffer offsets into LDS [base, base+1 KiB)
__device__ __forceinline__ void dma16(rsrc_t r, char* lds_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_base, 16, voff, 0, 0, 0);
}

// 32×32 accumulator blocks (v_mfma_f32_32x32x16_bf16, operands swapped like the 16×16 form:
// row = output column n, col = output row m) → the 16×16 layout the shared epilogue takes.
// Lane l of a 32×32 block holds m = l&31, n = 8g + 4(l>>5) + i in register 4g + i; the 16×16
// sub-block (mm, nn) wants lane 16q + p to hold m = 16mm + p, n = 16nn + 4q + i, i.e. register
// 8nn + 4(q>>1) + i of lane 32(q&1) + 16mm + p.  Per register pair (8nn + i, 8nn + 4 + i) one
// v_permlane32_swap then one v_permlane16_swap produce the two target fragments (mm = 0, 1).
template <int QM, int QN>
__device__ __forceinline__ void acc32_to_16(const f32x16 (&c)[QM][QN], f32x4 (&acc)[2 * QM][2 * QN]) {
#pragma unroll
  for (int qm = 0; qm < QM; ++qm)
#pragma unroll
    for (int qn = 0; qn < QN; ++qn)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(c[qm][qn][8 * nn + i]),
                                                          __float_as_uint(c[qm][qn][8 * nn + 4 + i]),
                                                          false, false);
          const auto u = __builtin_amdgcn_permlane16_swap(t[0], t[1], false, false);
          acc[2 * qm][2 * qn + nn][i] = __uint_as_float(u[0]);
          acc[2 * qm + 1][2 * qn + nn][i] = __uint_as_float(u[1]);
        }
}

// DEPI (FWD K loop): the DGRAD epilogue — a stride-1 input gradient computed as the forward conv
// of dy with the flipped, transposed filter (conv_dgrad_as_fwd below): mask, residual join and
// BN-backward statistics exactly as the DGRAD kernels store them
template <int MODE, int BM, int BN, int WM, int WN, int STAGES, bool STATS, bool BIAS, int FK,
          bool FP8 = false, bool NJ = false, bool FRES = false, bool M32 = false, bool AFM = false,
          bool DEPI = false>
__global__ void __launch_bounds__(64 * WM * WN, 1) conv_glds_kernel(ConvArgs a) {
  static_assert(!DEPI || (MODE == FWD && !FRES && !BIAS), "dgrad epilogue on the FWD loop");
  // AFM: DGRAD statistics epilogue masking by a folded BN's a·x + b > 0 (conv_common.h)
  // M32: the K loop runs v_mfma_f32_32x32x16_bf16 on 32×32 blocks (half the MFMA instructions
  // and half the vector-issue hold per FLOP of the 16×16×32 form); accumulators are re-laid to
  // the 16×16 fragment layout (acc32_to_16) before the shared epilogue.  Both operands must be
  // K-contiguous (KC) LDS images: FWD, and DGRAD with transposed weights.
  // FRES (FWD): residual a.res added in the epilogue before the ReLU (conv_common.h)
  // NJ (DGRAD): no residual join (a.beta == 0) — the epilogue's previous-dx registers are not
  // allocated (the fused-statistics dgrad needs them for the BN input x instead)
  // FK: 0 = generic K decomposition; 1 = FASTK (a K-step is one filter tap × 64 (fp8: 128)
  // channels); 2 = FASTK on a 1×1 filter whose channel count is not a multiple of 64 — the row's
  // last channel chunk is range-checked (compile time: a runtime test per DMA cost 10–20 %)
  // FK 3 (DGRAD, bf16): FASTK with the weights given transposed ([R][S][C][K], a.w_t) so both
  // operands are K-contiguous rows read with ds_read_b128, as in the forward and the fp8 dgrad
  constexpr bool FASTK = FK != 0, RAG = FK == 2, WT = FP8 || FK == 3;
  // STATS: FWD — BN Σy, Σy² of the output; DGRAD — BN-backward Σg, Σg·x of dx (a.bn_x), tiles in
  // column-grouped order (one class) so a workgroup's sums flush once
  static_assert(!STATS || MODE != WGRAD, "no statistics for weight gradients");
  constexpr bool COLG = MODE == FWD || (MODE == DGRAD && STATS);
  // FP8: operands are OCP fp8 bytes, a K-step is 128 deep (one 128-B LDS row per tile row, as
  // for bf16), fragments are 32 B and feed v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0
  // block scales; the per-tensor scales are applied in the epilogue.  FWD: x e4m3 × W e4m3.
  // DGRAD: dy e5m2 (gradients: wider range) × W^T e4m3 — the weight copy is stored transposed
  // ([R][S][C][K], ops/fp8.py) so both operands are K-contiguous rows (KC LDS images, no
  // transposed LDS reads); FASTK only (K % 128 == 0: a K-step is one tap, 128 output channels).
  // WGRAD (fp8): dy e5m2 × x e4m3, both as MC images of 128 pixels per K-step (fp8 MC layout
  // mc8_off, fragments by transposed 8-bit reads lds_read_mc_f8), fp32 split-K slabs × the scales
  static_assert(!FP8 || MODE != WGRAD || ((BM == 256 || BM == 128) && BN == 128),
                "fp8 weight gradients: 256x128 / 128x128 tiles");
  static_assert(!FP8 || MODE != DGRAD || FASTK, "fp8 dgrad needs K % 128 == 0");
  constexpr int ESZ = FP8 ? 1 : 2;         // bytes per element
  constexpr int EPC = 16 / ESZ;            // elements per 16-B chunk
  constexpr int KSTEP = 128 / ESZ;         // GEMM K per step (one 128-B LDS row)
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int TM = BM / WM, TN = BN / WN, RM = TM / 16, RN = TN / 16;
  constexpr bool A_MC = (MODE == WGRAD), B_MC = (MODE == WGRAD) || (MODE == DGRAD && !WT);
  static_assert(!M32 || (!A_MC && !B_MC && !FP8), "32x32 blocks: KC operands, bf16");
  constexpr int QM = (BM / WM) / 32 > 0 ? (BM / WM) / 32 : 1, QN = (BN / WN) / 32 > 0 ? (BN / WN) / 32 : 1;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int IA = A_BYTES / (1024 * NW), IB = B_BYTES / (1024 * NW);
  static_assert(IA * 1024 * NW == A_BYTES && IB * 1024 * NW == B_BYTES, "tile / wave mismatch");
  constexpr int LPS = IA + IB;  // DMA instructions per wave per K-step
  static_assert(STAGES >= 2 && STAGES <= 4, "ring depth");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // timing-only ablation flags (TDL_CONV_DBG) exist in TDL_CONV_ABLATION builds only: a runtime
  // test per flag per K-step costs scalar issue slots in the production loop
#if TDL_CONV_ABLATION
  const int DBG = a.dbg;
#else
  constexpr int DBG = 0;
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  // static priority 1 for the second-dispatched half of the waves, the arbitration loser of every
  // segment (MI355X_MICROARCH.md, two waves per SIMD, item 4): 0–5 % (dev/tools/fwd_ablate.py, dbg
  // 512 turns it off)
  if (!(DBG & 512) && wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const int tile_begin = blk * a.tpb;
  const int tile_end = min(a.cls_tile0[a.ncls], tile_begin + a.tpb);
  if (tile_begin >= tile_end) return;
  const int HoWo = a.Ho * a.Wo;
  // 1×1 filter without padding (wave-uniform): the FASTK A-operand DMAs need only the row check
  const bool pointwise = a.R == 1 && a.S == 1 && a.ph == 0 && a.pw == 0;
  const bool no_loads = DBG & 1;
  const rsrc_t rx = make_rsrc(a.x, no_loads ? 0u : a.x_bytes);
  const rsrc_t rw = make_rsrc(a.w, no_loads ? 0u : a.w_bytes);
  const rsrc_t rdy = make_rsrc(a.dy, no_loads ? 0u : a.dy_bytes);
  const rsrc_t rout = make_rsrc(a.out, a.out_bytes);
  const rsrc_t ra_src = (MODE == FWD) ? rx : rdy;
  const rsrc_t rb_src = (MODE == WGRAD) ? rx : rw;

  // ---- per-lane slot geometry (tile independent) ----
  // KC image [rows][64]: instruction j of this wave fills rows (j·NW + wid)·8 … +8
  // MC image [64][COLS]: instruction j fills k-rows (j·NW + wid)·RPI … +RPI
  auto kc_row = [&](int j) { return (j * NW + wid) * 8 + (lane >> 3); };
  const bool lin_src = DBG & 8;  // timing-only: natural source order (wrong LDS image)
  auto kc_lchunk = [&](int j) { return lin_src ? (lane & 7) : ((lane & 7) ^ ((kc_row(j) >> 1) & 7)); };
  auto mc_krow = [&](int j, int cols) { return (j * NW + wid) * (512 / cols) + lane / (cols / 8); };
  auto mc_col = [&](int j, int cols, int krow) {
    const int q = lane % (cols / 8);
    const int swz = cols >= 128 ? ((krow & 3) | (((krow >> 3) & 1) << 2))
                                : (((krow >> 1) & 1) | (((krow >> 3) & 1) << 1));
    return lin_src ? (q << 3) : ((((q >> 1) ^ swz) << 4) + ((q & 1) << 3));
  };

  // fp8 MC image [128][COLS bytes]: instruction j fills k-rows (j·NW + wid)·(1024/COLS) … ; the
  // lane fetches the logical 16-column chunk that belongs at its physical (swizzled) slot
  auto mc8_row = [&](int j, int cols) { return (j * NW + wid) * (1024 / cols) + lane / (cols / 16); };
  auto mc8_col = [&](int j, int cols) {
    const int r = mc8_row(j, cols), q = lane % (cols / 16);
    return 16 * (q ^ (cols == 256 ? mc8_swz<256>(r) : mc8_swz<128>(r)));
  };

  // ---- per-tile load state ----
  int a_base[IA], a_p0[IA], a_p1[IA];  // KC A: pixel base / spatial origin; MC A: column
  int a_row[IA];                       // FASTK FWD / DGRAD: row offset at tap (0, 0)
  int b_base[IB], b_f2[IB], b_f3[IB];  // KC B: row base; MC B: column / tap offsets
  // load-cursor position inside the filter (FWD: tap r, s and channel c0; DGRAD: class tap
  // th, tw and output channel c0) — FWD / DGRAD tiles always start at K-step 0
  int pos_r = 0, pos_s = 0, pos_c0 = 0;

  auto prep_tile = [&](const Tile& T) {
    if constexpr (MODE == FWD) {
#pragma unroll
      for (int j = 0; j < IA; ++j) {
        const int m = T.bm0 + kc_row(j);
        if (m < T.Mc) {
          const int n = fdiv(m, a.fd_HoWo), rem = m - n * HoWo;
          const int ho = fdiv(rem, a.fd_Wo), wo = rem - ho * a.Wo;
          a_base[j] = n * a.H * a.W * a.C;
          a_p0[j] = ho * a.sh - a.ph;
          a_p1[j] = wo * a.sw - a.pw;
        } else {
          a_base[j] = 0;
          a_p0[j] = -(1 << 28);
          a_p1[j] = 0;
        }
        // FASTK: the row's element offset at tap (0, 0), channel chunk included — a K-step then
        // adds one wave-uniform term (no per-DMA multiplies)
        if constexpr (FASTK) a_row[j] = m < T.Mc ? a_base[j] + (a_p0[j] * a.W + a_p1[j]) * a.C + kc_lchunk(j) * EPC : 0;
      }
#pragma unroll
      for (int j = 0; j < IB; ++j) {
        const int n = T.bn0 + kc_row(j);
        b_base[j] = n < a.Ng ? n * a.Kg : -1;
        if constexpr (FASTK) b_f2[j] = b_base[j] + kc_lchunk(j) * EPC;
      }
    } else if constexpr (MODE == DGRAD) {
      const int c = T.cls;
      const int Hc = a.cls_Hc[c], Wc = a.cls_Wc[c], HWc = Hc * Wc;
      const int ca = a.cls_a[c], cb = a.cls_b[c], r0 = a.cls_r0[c], s0 = a.cls_s0[c];
#pragma unroll
      for (int j = 0; j < IA; ++j) {
        const int m = T.bm0 + kc_row(j);
        if (m < T.Mc) {
          const int n = fdiv(m, a.cls_fdHW[c]), rem = m - n * HWc;
          const int ii = fdiv(rem, a.cls_fdW[c]), jj = rem - ii * Wc;
          const int h = ca + a.sh * ii, w = cb + a.sw * jj;
          a_base[j] = n * HoWo * a.K;
          // exact and non-negative for the class's first tap (r0 ≡ h + ph mod sh)
          a_p0[j] = fdiv(h + a.ph - r0 * a.dh, a.fd_sh);
          a_p1[j] = fdiv(w + a.pw - s0 * a.dw, a.fd_sw);
        } else {
          a_base[j] = 0;
          a_p0[j] = -(1 << 28);
          a_p1[j] = -(1 << 28);
        }
        if constexpr (FASTK) a_row[j] = m < T.Mc ? a_base[j] + (a_p0[j] * a.Wo + a_p1[j]) * a.K + kc_lchunk(j) * EPC : 0;
      }
#pragma unroll
      for (int j = 0; j < IB; ++j) {
        if constexpr (WT) {  // KC rows of W^T [R][S][C][K]: row ci of tap (r, s) at (r·S+s)·C·K + ci·K
          const int ci = T.bn0 + kc_row(j);
          b_base[j] = ci < a.Ng ? ci * a.K : -1;
        } else {
          const int ci = T.bn0 + mc_col(j, BN, mc_krow(j, BN));
          b_base[j] = ci < a.Ng ? ci : -1;
          // FASTK: W [K][R][S][C] row co0 + krow of tap (r, s) = this part + a wave-uniform part
          if constexpr (FASTK) b_f2[j] = mc_krow(j, BN) * a.R * a.S * a.C + b_base[j];
        }
      }
    } else {  // WGRAD
#pragma unroll
      for (int j = 0; j < IA; ++j) {
        const int co = T.bm0 + (FP8 ? mc8_col(j, BM) : mc_col(j, BM, mc_krow(j, BM)));
        a_base[j] = co < a.M ? co : -1;
      }
#pragma unroll
      for (int j = 0; j < IB; ++j) {
        const int nn = T.bn0 + (FP8 ? mc8_col(j, BN) : mc_col(j, BN, mc_krow(j, BN)));
        if (nn < a.Ng) {
          const int rs = fdiv(nn, a.fd_C), ci = nn - rs * a.C;
          const int r = fdiv(rs, a.fd_S), s = rs - r * a.S;
          b_base[j] = ci;
          b_f2[j] = r * a.dh - a.ph;
          b_f3[j] = s * a.dw - a.pw;
        } else {
          b_base[j] = -1;
          b_f2[j] = -(1 << 28);
          b_f3[j] = 0;
        }
      }
    }
  };

  // ---- issue the DMAs of one K-step into ring slot `slot` ----
  auto issue_step = [&](const Tile& T, int kt, int slot) {
    char* As = smem + slot * STAGE;
    char* Bs = As + A_BYTES;
    const int kb = kt * KSTEP;
    if constexpr (MODE == FWD) {
      // FASTK (C % 64 == 0): the K-step is one filter tap (pos_r, pos_s) and channels
      // pos_c0 … +63, advanced incrementally by advance_load (no division in the loop)
      const int tap_r = pos_r, tap_s = pos_s, c0 = pos_c0;
      const int kbase = kb;
      if constexpr (FASTK) {
        const int rdh = tap_r * a.dh, sdw = tap_s * a.dw;
        const int tuni = (rdh * a.W + sdw) * a.C + c0;  // wave-uniform
        if (pointwise) {
          // 1×1 filter, no padding: every tap of a valid row is in range (row validity only —
          // loop-invariant, so the per-DMA cost is the offset add and the select)
#pragma unroll
          for (int j = 0; j < IA; ++j) {
            bool v = a_p0[j] >= 0;
            if constexpr (RAG) v = v && c0 + kc_lchunk(j) * EPC < a.C;
            dma16(ra_src, As + (j * NW + wid) * 1024, v ? (uint32_t)(a_row[j] + tuni) * (uint32_t)ESZ : OOB);
          }
        } else {
#pragma unroll
          for (int j = 0; j < IA; ++j) {
            bool v = (unsigned)(a_p0[j] + rdh) < (unsigned)a.H && (unsigned)(a_p1[j] + sdw) < (unsigned)a.W;
            if constexpr (RAG) v = v && c0 + kc_lchunk(j) * EPC < a.C;
            dma16(ra_src, As + (j * NW + wid) * 1024, v ? (uint32_t)(a_row[j] + tuni) * (uint32_t)ESZ : OOB);
          }
        }
      } else
#pragma unroll
      for (int j = 0; j < IA; ++j) {
        const int lc = kc_lchunk(j);
        int r = tap_r, s = tap_s, c = c0 + lc * EPC;
        bool kv = kb < a.Kg;
        if constexpr (!FASTK) {
          const int k = kb + lc * EPC;
          kv = k < a.Kg;
          const int rs = fdiv(k, a.fd_C);
          c = k - rs * a.C;
          r = fdiv(rs, a.fd_S);
          s = rs - r * a.S;
        }
        const int hi = a_p0[j] + r * a.dh, wi = a_p1[j] + s * a.dw;
        const bool v = kv && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
        const uint32_t off = (uint32_t)(a_base[j] + (hi * a.W + wi) * a.C + c) * (uint32_t)ESZ;
        dma16(ra_src, As + (j * NW + wid) * 1024, v ? off : OOB);
      }
      if constexpr (FASTK) {  // every K-step of a FASTK tile is inside Kg (ragged: its chunks)
#pragma unroll
        for (int j = 0; j < IB; ++j) {
          bool v = b_base[j] >= 0;
          if constexpr (RAG) v = v && kbase + kc_lchunk(j) * EPC < a.Kg;
          dma16(rb_src, Bs + (j * NW + wid) * 1024, v ? (uint32_t)(b_f2[j] + kbase) * (uint32_t)ESZ : OOB);
        }
      } else
#pragma unroll
      for (int j = 0; j < IB; ++j) {
        const int k = kbase + kc_lchunk(j) * EPC;
        const bool v = k < a.Kg && b_base[j] >= 0;
        dma16(rb_src, Bs + (j * NW + wid) * 1024, v ? (uint32_t)(b_base[j] + k) * (uint32_t)ESZ : OOB);
      }
    } else if constexpr (MODE == DGRAD) {
      const int c = T.cls;
      const int Tw = a.cls_Tw[c];
      const int step_h = a.sh == 1 ? a.dh : 1, step_w = a.sw == 1 ? a.dw : 1;
      // FASTK (K % 64 == 0): one tap (pos_r = th, pos_s = tw) per K-step, channels pos_c0 … +63
      const int co0 = pos_c0;
      if constexpr (FASTK) {
        const int dth = pos_r * step_h, dtw = pos_s * step_w;
        const int tuni = co0 - (dth * a.Wo + dtw) * a.K;  // wave-uniform
        if (pointwise) {  // as in FWD: a valid row's only tap is in range
#pragma unroll
          for (int j = 0; j < IA; ++j) {
            bool v = a_p0[j] >= 0;
            if constexpr (RAG) v = v && co0 + kc_lchunk(j) * EPC < a.K;
            dma16(ra_src, As + (j * NW + wid) * 1024, v ? (uint32_t)(a_row[j] + tuni) * (uint32_t)ESZ : OOB);
          }
        } else {
#pragma unroll
          for (int j = 0; j < IA; ++j) {
            bool v = (unsigned)(a_p0[j] - dth) < (unsigned)a.Ho && (unsigned)(a_p1[j] - dtw) < (unsigned)a.Wo;
            if constexpr (RAG) v = v && co0 + kc_lchunk(j) * EPC < a.K;
            dma16(ra_src, As + (j * NW + wid) * 1024, v ? (uint32_t)(a_row[j] + tuni) * (uint32_t)ESZ : OOB);
          }
        }
      } else
#pragma unroll
      for (int j = 0; j < IA; ++j) {
        const int lc = kc_lchunk(j);
        int th = pos_r, tw = pos_s, co = co0 + lc * EPC;
        bool kv = kb < T.Kgc;
        if constexpr (!FASTK) {
          const int k = kb + lc * 8;
          kv = k < T.Kgc;
          co = k % a.K;
          const int t = k / a.K;
          th = t / Tw;
          tw = t - th * Tw;
        }
        const int ho = a_p0[j] - th * step_h, wo = a_p1[j] - tw * step_w;
        const bool v = kv && (unsigned)ho < (unsigned)a.Ho && (unsigned)wo < (unsigned)a.Wo;
        const uint32_t off = (uint32_t)(a_base[j] + (ho * a.Wo + wo) * a.K + co) * (uint32_t)ESZ;
        dma16(ra_src, As + (j * NW + wid) * 1024, v ? off : OOB);
      }
      const int r0 = a.cls_r0[c], s0 = a.cls_s0[c];
      if constexpr (WT) {  // W^T rows: tap (r, s) of this class, output channels co0 … +KSTEP−1
        const int r = r0 + a.sh * pos_r, s = s0 + a.sw * pos_s;
        const int toff = (r * a.S + s) * a.C * a.K + co0;
#pragma unroll
        for (int j = 0; j < IB; ++j) {
          const bool v = kb < T.Kgc && b_base[j] >= 0;
          dma16(rb_src, Bs + (j * NW + wid) * 1024,
                v ? (uint32_t)(b_base[j] + toff + kc_lchunk(j) * EPC) * (uint32_t)ESZ : OOB);
        }
      } else if constexpr (FASTK) {
        const int r = r0 + a.sh * pos_r, s = s0 + a.sw * pos_s;
        const int buni = (co0 * a.R * a.S + r * a.S + s) * a.C;  // wave-uniform
#pragma unroll
        for (int j = 0; j < IB; ++j) {
          bool v = b_base[j] >= 0;
          if constexpr (RAG) v = v && co0 + mc_krow(j, BN) < a.K;
          dma16(rb_src, Bs + (j * NW + wid) * 1024, v ? (uint32_t)(b_f2[j] + buni) * 2u : OOB);
        }
      } else
#pragma unroll
      for (int j = 0; j < IB; ++j) {
        const int kk = kb + mc_krow(j, BN);
        int co2, th2, tw2;
        if constexpr (FASTK) {
          th2 = pos_r;
          tw2 = pos_s;
          co2 = co0 + mc_krow(j, BN);
        } else {
          co2 = kk % a.K;
          const int t2 = kk / a.K;
          th2 = t2 / Tw;
          tw2 = t2 - th2 * Tw;
        }
        const int r = r0 + a.sh * th2, s = s0 + a.sw * tw2;
        const bool v = kk < T.Kgc && b_base[j] >= 0;
        const uint32_t off = (uint32_t)(((co2 * a.R + r) * a.S + s) * a.C + b_base[j]) * 2u;
        dma16(rb_src, Bs + (j * NW + wid) * 1024, v ? off : OOB);
      }
    } else {  // WGRAD
#pragma unroll
      for (int j = 0; j < IA; ++j) {
        const int p = kb + (FP8 ? mc8_row(j, BM) : mc_krow(j, BM));
        const bool v = p < a.Kg && a_base[j] >= 0;
        dma16(ra_src, As + (j * NW + wid) * 1024, v ? (uint32_t)(p * a.K + a_base[j]) * (uint32_t)ESZ : OOB);
      }
      if (pointwise && a.sh == 1 && a.sw == 1) {
        // 1×1, stride 1, no padding: x pixel = output pixel p (no per-DMA pixel divisions)
#pragma unroll
        for (int j = 0; j < IB; ++j) {
          const int p = kb + (FP8 ? mc8_row(j, BN) : mc_krow(j, BN));
          const bool v = p < a.Kg && b_base[j] >= 0;
          dma16(rb_src, Bs + (j * NW + wid) * 1024, v ? (uint32_t)(p * a.C + b_base[j]) * (uint32_t)ESZ : OOB);
        }
      } else {
#pragma unroll
        for (int j = 0; j < IB; ++j) {
          const int p = kb + (FP8 ? mc8_row(j, BN) : mc_krow(j, BN));
          const int ni = fdiv(p, a.fd_HoWo), rem = p - ni * HoWo;
          const int ho = fdiv(rem, a.fd_Wo), wo = rem - ho * a.Wo;
          const int hi = ho * a.sh + b_f2[j], wi = wo * a.sw + b_f3[j];
          const bool v = p < a.Kg && b_base[j] >= 0 && (unsigned)hi < (unsigned)a.H &&
                         (unsigned)wi < (unsigned)a.W;
          const uint32_t off = (uint32_t)(((ni * a.H + hi) * a.W + wi) * a.C + b_base[j]) * (uint32_t)ESZ;
          dma16(rb_src, Bs + (j * NW + wid) * 1024, v ? off : OOB);
        }
      }
    }
  };

  f32x4 acc[RM][RN];
  f32x16 acc32[QM][QN];
  auto zero_acc = [&]() {
    if constexpr (M32) {
#pragma unroll
      for (int i = 0; i < QM; ++i)
#pragma unroll
        for (int j = 0; j < QN; ++j)
#pragma unroll
          for (int v = 0; v < 16; ++v) acc32[i][j][v] = 0.f;
    } else {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  const uint32_t smem_lds = (uint32_t)(size_t)(lds_char_t*)smem;
  const bool no_reads = DBG & 16, no_barrier = DBG & 32, no_dma = DBG & 64;
  auto load_frags = [&](uint32_t As, uint32_t Bs, int kk, bf16x8(&af)[RM], bf16x8(&bfg)[RN]) {
    if (no_reads) return;
    if constexpr (M32) {
      // half-step kk = 16-deep slices 2kk, 2kk+1; lane l reads k-chunk 4kk + 2s + (l>>5) of row
      // l&31 (A and B alike: any k permutation shared by both operands is exact)
#pragma unroll
      for (int q = 0; q < QM; ++q)
#pragma unroll
        for (int sl = 0; sl < 2; ++sl)
          af[2 * q + sl] = lds_read_kc(As, wm * TM + q * 32 + (lane & 31), kk * 4 + sl * 2 + (lane >> 5));
#pragma unroll
      for (int q = 0; q < QN; ++q)
#pragma unroll
        for (int sl = 0; sl < 2; ++sl)
          bfg[2 * q + sl] = lds_read_kc(Bs, wn * TN + q * 32 + (lane & 31), kk * 4 + sl * 2 + (lane >> 5));
      return;
    }
    static_assert(TM % 16 == 0 && TN % 16 == 0, "16-row fragment blocks");
    const int mck = 8 * (lane >> 4) + ((lane >> 2) & 3);  // MC fragment k-row at kk = 0
    if constexpr (A_MC) {
#pragma unroll
      for (int rm = 0; rm < RM; ++rm) {
        const uint32_t ad = As + (uint32_t)mc_off<BM>(mck, wm * TM + rm * 16 + 4 * (lane & 3));
        af[rm] = kk == 0 ? lds_read_mc_imm<BM, 0>(ad) : lds_read_mc_imm<BM, 1>(ad);
      }
    } else {
      lds_read_kc_rows<RM>(af, As + (uint32_t)kc_off(wm * TM + (lane & 15), kk * 4 + (lane >> 4)));
    }
    if constexpr (B_MC) {
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) {
        const uint32_t ad = Bs + (uint32_t)mc_off<BN>(mck, wn * TN + rn * 16 + 4 * (lane & 3));
        bfg[rn] = kk == 0 ? lds_read_mc_imm<BN, 0>(ad) : lds_read_mc_imm<BN, 1>(ad);
      }
    } else {
      lds_read_kc_rows<RN>(bfg, Bs + (uint32_t)kc_off(wn * TN + (lane & 15), kk * 4 + (lane >> 4)));
    }
  };
  const bool no_mfma = DBG & 2;
  const bool no_epi_mem = DBG & 128;  // timing-only: epilogue issues no global loads / stores
  auto mfmas = [&](const bf16x8(&af)[RM], const bf16x8(&bfg)[RN]) {
    if (no_mfma) {
#pragma unroll
      for (int rm = 0; rm < RM; ++rm) asm volatile("" ::"v"(af[rm]));
#pragma unroll
      for (int rn = 0; rn < RN; ++rn) asm volatile("" ::"v"(bfg[rn]));
      return;
    }
    if constexpr (M32) {
#pragma unroll
      for (int sl = 0; sl < 2; ++sl)
#pragma unroll
        for (int qm = 0; qm < QM; ++qm)
#pragma unroll
          for (int qn = 0; qn < QN; ++qn)
            acc32[qm][qn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfg[2 * qn + sl], af[2 * qm + sl],
                                                                    acc32[qm][qn], 0, 0, 0);
      return;
    }
#pragma unroll
    for (int rm = 0; rm < RM; ++rm)
#pragma unroll
      for (int rn = 0; rn < RN; ++rn)
        acc[rm][rn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[rn], af[rm], acc[rm][rn], 0, 0, 0);
  };
  static_assert(BK == 64, "two 32-deep fragment sets per K-step");

  float s_sum[RN][4], s_sq[RN][4];
#pragma unroll
  for (int rn = 0; rn < RN; ++rn)
#pragma unroll
    for (int i = 0; i < 4; ++i) s_sum[rn][i] = s_sq[rn][i] = 0.f;

  // lane holds C[m = bm0 + wm*TM + rm*16 + (lane&15)][n = bn0 + wn*TN + rn*16 + (lane>>4)*4 + i]
  const float out_scale = FP8 ? (*a.scale_x) * (*a.scale_w) : 1.f;
  auto epilogue = [&](const Tile& T) {
    if constexpr (MODE == WGRAD) {
      const uint32_t slab0 = (uint32_t)T.split * (uint32_t)(a.M * a.Ng);
#pragma unroll
      for (int rm = 0; rm < RM; ++rm) {
        const int m = T.bm0 + wm * TM + rm * 16 + (lane & 15);
#pragma unroll
        for (int rn = 0; rn < RN; ++rn) {
          const int n0 = T.bn0 + wn * TN + rn * 16 + (lane >> 4) * 4;
          const bool v = m < a.M && n0 < a.Ng;
          const uint32_t off = (slab0 + (uint32_t)(m * a.Ng + n0)) * 4u;
          f32x4 o = acc[rm][rn];
          if constexpr (FP8) o *= out_scale;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, o), rout, v ? off : OOB, 0, 0);
        }
      }
    } else {
      if constexpr (M32) acc32_to_16<QM, QN>(acc32, acc);
      // (statistics + join of the dgrad-as-forward: operands in two halves, else they spill)
      constexpr int RG = DEPI && STATS && !NJ && RM >= 4 ? RM / 2 : RM;
      store_tile_bf16<DEPI ? DGRAD : MODE, RM, RN, TM, TN, BIAS, STATS, FP8, false, NJ, FRES,
                      false, AFM, false, RG>(
          a, T, acc, wm, wn, lane, rout, out_scale, no_epi_mem, s_sum, s_sq);
    }
  };

  auto flush_stats = [&](int bn0) {
    if constexpr (STATS && MODE != WGRAD) {
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
      float* red = (float*)(smem + STAGES * STAGE);
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
  };

  // Next tile of this workgroup without the divisions of tile_of: FWD workgroups walk one
  // column's consecutive row tiles; DGRAD / WGRAD walk row-major (n fastest) inside a class /
  // split, and fall back to tile_of at a class or split boundary.
  const int ntn_c = (a.Ng + BN - 1) / BN;
  auto next_tile = [&](Tile& T, int t) {
    if constexpr (COLG) {
      T.bm0 += BM;
    } else {
      T.bn0 += BN;
      if (T.bn0 >= a.Ng) {
        T.bn0 = 0;
        T.bm0 += BM;
        if (T.bm0 >= T.Mc) T = tile_of<MODE, BM, BN, KSTEP, COLG>(a, t);
      }
    }
    (void)ntn_c;
  };

  // ---- flat (tile, K-step) pipeline over this workgroup's tiles ----
  int lt = tile_begin;
  Tile LT = tile_of<MODE, BM, BN, KSTEP, COLG>(a, lt);
  int lkt = LT.kt0;
  bool lmore = LT.bm0 < LT.Mc;
  if (!lmore) return;
  prep_tile(LT);
  const int pos_C = MODE == FWD ? a.C : a.K;
  auto advance_load = [&]() {
    if (lkt + 1 < LT.kt1) {
      ++lkt;
      if constexpr (FASTK && MODE != WGRAD) {
        pos_c0 += KSTEP;
        if (pos_c0 >= pos_C) {
          pos_c0 = 0;
          const int Sl = MODE == FWD ? a.S : a.cls_Tw[LT.cls];
          if (++pos_s == Sl) {
            pos_s = 0;
            ++pos_r;
          }
        }
      }
    } else if (lt + 1 < tile_end) {
      ++lt;
      next_tile(LT, lt);
      lkt = LT.kt0;
      pos_r = pos_s = pos_c0 = 0;
      if (LT.bm0 < LT.Mc)
        prep_tile(LT);
      else
        lmore = false;  // FWD row groups: trailing empty tiles
    } else {
      lmore = false;
    }
  };

  int ct = tile_begin;
  Tile CT = LT;
  int ckt = CT.kt0;
  int inflight = 0;  // steps issued and not yet fully computed
  // epilogue stores per lane: RM·RN/2 16-B stores (FWD / DGRAD; a ragged column tile issues
  // RM·RN 8-B ones — more than counted, so its stores are only waited for sooner), RM·RN (WGRAD)
  constexpr int E = MODE == WGRAD ? RM * RN : RM * RN / 2;
  // bit i: the epilogue of the i-th previous K-step issued its stores
  uint32_t ehist = 0;
  int slot_load = 0, slot_comp = 0;
  auto issue_next = [&]() {
    if (!no_dma) issue_step(LT, lkt, slot_load);
    slot_load = slot_load + 1 == STAGES ? 0 : slot_load + 1;
    ++inflight;
    advance_load();
  };
  // Retire the DMAs of the step about to be read while `ahead` younger steps stay in flight,
  // then make them visible to every wave.  vmcnt retires in issue order, so the count must
  // include every younger VMEM op: the `ahead` DMA steps and the stores of each epilogue since
  // the awaited step was issued (STAGES − 1 K-steps ago).  Counting only the last epilogue's
  // stores forced the previous tile's stores to complete one K-step after they were issued —
  // store-completion latency then paced the memory-bound (one-K-step) tiles.
  auto ring_wait_barrier = [&](int ahead) {
    const int ne = __builtin_popcount(ehist & ((1u << (STAGES - 1)) - 1u));
    wait_ring<LPS, E, STAGES>(ahead, ne);
    if (!no_barrier) raw_barrier();
  };

  if constexpr (FP8) {
    // fp8: one 128-deep MFMA per fragment pair; straight ring loop (wait → barrier → refill the
    // slot every wave has finished → read fragments → MFMAs)
    for (int s = 0; s < STAGES - 1; ++s)
      if (lmore) issue_next();
    zero_acc();
    // as in the bf16 loop below: an in-tile fast step (loop-invariant load state) and the general one
#define TDL_GLDS_STEP8(FAST)                                                                   \
    do {                                                                                       \
      ring_wait_barrier(inflight - 1);                                                         \
      ehist <<= 1;                                                                             \
      if constexpr ((FAST)) {                                                                  \
        if (!no_dma) issue_step(LT, lkt, slot_load);                                           \
        slot_load = slot_load + 1 == STAGES ? 0 : slot_load + 1;                               \
        ++inflight;                                                                            \
        ++lkt; /* advance_load in-tile branch */                                               \
        if constexpr (FASTK && MODE != WGRAD) {                                                \
          pos_c0 += KSTEP;                                                                     \
          if (pos_c0 >= pos_C) {                                                               \
            pos_c0 = 0;                                                                        \
            const int Sl = MODE == FWD ? a.S : a.cls_Tw[LT.cls];                               \
            if (++pos_s == Sl) {                                                               \
              pos_s = 0;                                                                       \
              ++pos_r;                                                                         \
            }                                                                                  \
          }                                                                                    \
        }                                                                                      \
      } else {                                                                                 \
        if (lmore) issue_next();                                                               \
      }                                                                                        \
      const uint32_t As = smem_lds + (uint32_t)(slot_comp * STAGE), Bs = As + A_BYTES;         \
      i32x8 a8[RM], b8[RN];                                                                    \
      if constexpr (MODE == WGRAD) {                                                           \
_Pragma("unroll")                                                                             \
        for (int rm = 0; rm < RM; ++rm) a8[rm] = lds_read_mc_f8<BM>(As, wm * TM + rm * 16, lane);\
_Pragma("unroll")                                                                             \
        for (int rn = 0; rn < RN; ++rn) b8[rn] = lds_read_mc_f8<BN>(Bs, wn * TN + rn * 16, lane);\
      } else {                                                                                 \
_Pragma("unroll")                                                                             \
        for (int rm = 0; rm < RM; ++rm) a8[rm] = lds_read_kc_f8(As, wm * TM + rm * 16 + (lane & 15), lane >> 4);\
_Pragma("unroll")                                                                             \
        for (int rn = 0; rn < RN; ++rn) b8[rn] = lds_read_kc_f8(Bs, wn * TN + rn * 16 + (lane & 15), lane >> 4);\
      }                                                                                        \
      lgkm_wait0();                                                                            \
_Pragma("unroll")                                                                             \
      for (int rm = 0; rm < RM; ++rm)                                                          \
_Pragma("unroll")                                                                             \
        for (int rn = 0; rn < RN; ++rn)                                                        \
/* operand formats: first (B tile: weights / WGRAD activations) e4m3 = 0; second (A tile) */  \
/* e4m3 = 0 for FWD activations, e5m2 (bf8) = 1 for DGRAD / WGRAD output gradients and for */  \
/* the dy of a dgrad run as the forward conv (DEPI) */                                          \
          acc[rm][rn] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(                      \
              b8[rn], a8[rm], acc[rm][rn], 0, (MODE == FWD && !DEPI) ? 0 : 1, 0, 127, 0, 127); \
      slot_comp = slot_comp + 1 == STAGES ? 0 : slot_comp + 1;                                 \
      --inflight;                                                                              \
      if (ckt + 1 >= CT.kt1) {                                                                 \
        epilogue(CT);                                                                          \
        ehist |= 1u;                                                                           \
        zero_acc();                                                                            \
        if (inflight > 0) {                                                                    \
          ++ct;                                                                                \
          next_tile(CT, ct);                                                                   \
          ckt = CT.kt0;                                                                        \
        }                                                                                      \
      } else {                                                                                 \
        ++ckt;                                                                                 \
      }                                                                                        \
    } while (0)
    while (inflight > 0) {
      while (inflight > 1 && lmore && lkt + 1 < LT.kt1) TDL_GLDS_STEP8(true);
      TDL_GLDS_STEP8(false);
    }
#undef TDL_GLDS_STEP8
    flush_stats(CT.bn0);
    return;
  }
  // Software pipeline across K-steps (one barrier per step):
  //   reads(t, k0..31) ready → issue reads(t, k32..63) → MFMA(t, first half) → lgkm(0) →
  //   [wait DMA(t+1), barrier, DMA(t+S) into the slot just drained, reads(t+1, k0..31)] →
  //   MFMA(t, second half) → epilogue if the tile ends → lgkm(0)
  // so the barrier, the DMA address math and the next step's first fragment reads all sit under
  // 16 MFMAs instead of in front of an idle MFMA pipe.
  for (int s = 0; s < STAGES - 1; ++s)
    if (lmore) issue_next();
  zero_acc();
  bf16x8 f0a[RM], f0b[RN], f1a[RM], f1b[RN];
  ring_wait_barrier(inflight - 1);
  if (lmore) issue_next();
  load_frags(smem_lds + (uint32_t)(slot_comp * STAGE), smem_lds + (uint32_t)(slot_comp * STAGE + A_BYTES), 0, f0a, f0b);
  lgkm_wait0();
  // One pipeline step.  FAST: the DMA issued in this step keeps the load cursor inside its tile
  // (no prep_tile), so the per-lane load state is invariant across the inner loop below.  With a
  // single loop whose issue might switch tiles, the compiler carried that state through phi
  // copies: ≈28 v_mov per K-step on the vector-issue-bound path.
#define TDL_GLDS_STEP(FAST)                                                                    \
  do {                                                                                         \
    const uint32_t As = smem_lds + (uint32_t)(slot_comp * STAGE), Bs = As + A_BYTES;           \
    load_frags(As, Bs, 1, f1a, f1b);                                                           \
    mfmas(f0a, f0b);                                                                           \
    lgkm_wait0();                                                                              \
    const bool has_next = (FAST) || inflight > 1;                                              \
    slot_comp = slot_comp + 1 == STAGES ? 0 : slot_comp + 1;                                   \
    if (has_next) {                                                                            \
      ring_wait_barrier(inflight - 2);                                                         \
      if constexpr ((FAST)) {                                                                  \
        if (!no_dma) issue_step(LT, lkt, slot_load);                                           \
        slot_load = slot_load + 1 == STAGES ? 0 : slot_load + 1;                               \
        ++inflight;                                                                            \
        ++lkt; /* advance_load in-tile branch */                                              \
        if constexpr (FASTK && MODE != WGRAD) {                                                \
          pos_c0 += KSTEP;                                                                     \
          if (pos_c0 >= pos_C) {                                                               \
            pos_c0 = 0;                                                                        \
            const int Sl = MODE == FWD ? a.S : a.cls_Tw[LT.cls];                               \
            if (++pos_s == Sl) {                                                               \
              pos_s = 0;                                                                       \
              ++pos_r;                                                                         \
            }                                                                                  \
          }                                                                                    \
        }                                                                                      \
      } else {                                                                                 \
        if (lmore) issue_next();                                                               \
      }                                                                                        \
      const uint32_t An = smem_lds + (uint32_t)(slot_comp * STAGE), Bn = An + A_BYTES;         \
      load_frags(An, Bn, 0, f0a, f0b);                                                         \
    }                                                                                          \
    mfmas(f1a, f1b);                                                                           \
    --inflight;                                                                                \
    ehist <<= 1;                                                                               \
    if (ckt + 1 >= CT.kt1) {                                                                   \
      epilogue(CT);                                                                            \
      ehist |= 1u;                                                                             \
      zero_acc();                                                                              \
      if (inflight > 0) {                                                                      \
        ++ct;                                                                                  \
        next_tile(CT, ct);                                                                     \
        ckt = CT.kt0;                                                                          \
      }                                                                                        \
    } else {                                                                                   \
      ++ckt;                                                                                   \
    }                                                                                          \
    if (has_next) lgkm_wait0();                                                                \
  } while (0)
  while (inflight > 0) {
    while (inflight > 1 && lmore && lkt + 1 < LT.kt1) TDL_GLDS_STEP(true);
    TDL_GLDS_STEP(false);
  }
#undef TDL_GLDS_STEP
  flush_stats(CT.bn0);
}

// ------------------------------------------------------------------------------------------
// configurations
// ------------------------------------------------------------------------------------------
struct GCfg {
  int bm, bn, wm, wn, stages;
};
constexpr GCfg G256x128{256, 128, 4, 2, 3};
constexpr GCfg G256x64{256, 64, 4, 1, 3};
constexpr GCfg G128x128{128, 128, 2, 2, 4};
constexpr GCfg G128x128s2{128, 128, 2, 2, 2};  // 66 KB LDS: two workgroups per CU
constexpr GCfg G256x64w8{256, 64, 8, 1, 3};    // 64-wide N with 8 waves (32-row wave tiles)
constexpr GCfg G128x64{128, 64, 4, 1, 4};      // 64-wide N, 4 stages, 96 KB LDS
constexpr GCfg G128x128w8{128, 128, 4, 2, 4};  // 8 waves of 32×64 (half the accumulators)
constexpr GCfg G64x256{64, 256, 1, 4, 3};      // WGRAD, ≤ 64 output channels, 129–256 columns

constexpr int lds_bytes(int bm, int bn, int wm, int stages) {
  return stages * (bm + bn) * BK * 2 + 2 * wm * bn * 4;
}

template <int MODE, int BM, int BN, int WM, int WN, int ST, bool STATS, bool BIAS, int FK,
          bool F8 = false, bool NJ = false, bool FRES = false, bool M32 = false, bool AFM = false,
          bool DEPI = false>
void launch_g(const ConvArgs& a, int blocks, hipStream_t st) {
  auto k = conv_glds_kernel<MODE, BM, BN, WM, WN, ST, STATS, BIAS, FK, F8, NJ, FRES, M32, AFM, DEPI>;
  constexpr int lds = lds_bytes(BM, BN, WM, ST);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * WM * WN), lds, st, a);
}

// the tile configs launch_gcfg instantiates: 0–5 (5 = the 128×64 default), 6 for fused-statistics
// dgrads, 7 for weight gradients — route_cfg_instantiated (conv_route.hip) is the table of record;
// a config the launcher does not have would leave output tiles unwritten
template <int MODE, bool STATS, bool BIAS, int FK, bool NJ = false>
void launch_gcfg(const ConvArgs& a, int cfg, int blocks, hipStream_t st) {
  if (cfg == 0)
    launch_g<MODE, 256, 128, 4, 2, 3, STATS, BIAS, FK, false, NJ>(a, blocks, st);
  else if (cfg == 1)
    launch_g<MODE, 256, 64, 4, 1, 3, STATS, BIAS, FK, false, NJ>(a, blocks, st);
  else if (cfg == 2)
    launch_g<MODE, 128, 128, 2, 2, 4, STATS, BIAS, FK, false, NJ>(a, blocks, st);
  else if (cfg == 3)
    launch_g<MODE, 128, 128, 2, 2, 2, STATS, BIAS, FK, false, NJ>(a, blocks, st);
  else if (cfg == 4)
    launch_g<MODE, 256, 64, 8, 1, 3, STATS, BIAS, FK, false, NJ>(a, blocks, st);
  else if (cfg == 6 && MODE == DGRAD && STATS)  // fused-statistics dgrads only
    launch_g<MODE, 128, 128, 4, 2, 4, STATS, BIAS, FK, false, NJ>(a, blocks, st);
  else if (cfg == 7 && MODE == WGRAD) {  // few-output-channel weight gradients (the ResNet stem)
    if constexpr (MODE == WGRAD) launch_g<MODE, 64, 256, 1, 4, 3, STATS, BIAS, FK, false, NJ>(a, blocks, st);
  } else if (cfg == 5)
    launch_g<MODE, 128, 64, 4, 1, 4, STATS, BIAS, FK, false, NJ>(a, blocks, st);
  else
    throw std::runtime_error("LDS-DMA conv: tile config " + std::to_string(cfg) +
                             " not instantiated for this problem");
}

const GCfg& cfg_of(int c) {
  switch (c) {
    case 0: return G256x128;
    case 1: return G256x64;
    case 2: return G128x128;
    case 3: return G128x128s2;
    case 4: return G256x64w8;
    case 6: return G128x128w8;
    case 7: return G64x256;
    default: return G128x64;
  }
}


int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// persistent grid: ⌈tiles / CUs⌉ consecutive tiles per workgroup
int persistent_tpb(long tiles) {
  const int cus = env_int("TDL_GLDS_SLOTS", 256);
  return (int)std::max<long>(1, (tiles + cus - 1) / cus);
}

// the same for a column-grouped grid (every workgroup walks tpb row tiles of ONE column tile;
// class c contributes ⌈ntm[c] / tpb⌉ groups per column): raised until the grid fits the slots.
// ⌈tiles / CUs⌉ alone can round the groups up past them — Xception-41's 38×38×728 pointwise
// convs got 43 groups × 6 columns = 258 workgroups for 256 CUs, and the two extra ran as a
// second wave of whole groups: 613 instead of ~330 µs (profiles/r06_grouped_tiling.txt)
int grouped_tpb(const long* ntm, int ncls, long ntn) {
  const long slots = env_int("TDL_GLDS_SLOTS", 256);
  long tiles = 0, ntm_max = 1;
  for (int c = 0; c < ncls; ++c) {
    tiles += ntm[c];
    ntm_max = std::max(ntm_max, ntm[c]);
  }
  long tpb = std::min<long>(std::max(1, persistent_tpb(tiles * ntn)), ntm_max);
  auto blocks = [&](long t) {
    long g = 0;
    for (int c = 0; c < ncls; ++c) g += (ntm[c] + t - 1) / t;
    return g * ntn;
  };
  static const bool fit = env_int("TDL_GROUPED_FIT", 1) != 0;  // (0: the old rounding, A/B)
  while (fit && tpb < ntm_max && blocks(tpb) > slots) ++tpb;
  return (int)tpb;
}

}  // namespace

// fp8 forward: LDS-DMA kernel only (C % 16 == 0: a 16-B chunk never crosses a filter tap); the
// tile config from the route table (fwd.glds.fp8 / fwd.glds.fp8.n64)
void conv_fwd_fp8_launch(const ConvArgs& a0, hipStream_t st) {
  const RouteProblem p = route_problem(FWD, a0, RF_FP8 | (a0.stats ? RF_STATS : 0));
  const int ri = route_next(p, -1);
  if (ri < 0) throw std::runtime_error("fp8 forward: no conv route takes this problem");
  const int cfg = route_cfg(ri);
  if (cfg != 0 && cfg != 1)
    throw std::runtime_error(std::string("fp8 forward: route ") + route_rule(ri).name +
                             " is not an fp8 tile config");
  route_record(FWD, ri);
  ConvArgs a = a0;
  a.dbg = 0;
  set_fastdivs(a);
  const GCfg& g = cfg_of(cfg);
  const long ntm = cdiv(a.M, g.bm), ntn = cdiv(a.Ng, g.bn);
  a.ncls = 1;
  a.splits = 1;
  a.tpb = grouped_tpb(&ntm, 1, ntn);
  const long groups = (ntm + a.tpb - 1) / a.tpb;
  const int blocks = (int)(groups * ntn);
  a.cls_tile0[0] = 0;
  a.cls_tile0[1] = (int)(groups * ntn * a.tpb);
  const bool fk = a.C % 128 == 0, stats = a.stats != nullptr;
#define TDL_F8(ST, FK)                                                              \
  do {                                                                              \
    if (cfg == 0) launch_g<FWD, 256, 128, 4, 2, 3, ST, false, FK, true>(a, blocks, st); \
    else launch_g<FWD, 256, 64, 4, 1, 3, ST, false, FK, true>(a, blocks, st);       \
  } while (0)
  if (fk) {
    if (stats) TDL_F8(true, 1); else TDL_F8(false, 1);
  } else {
    if (stats) TDL_F8(true, 0); else TDL_F8(false, 0);
  }
#undef TDL_F8
}

// Mode selection: 0 = register-staged kernel only, 1 = glds for eligible problems (default),
// 2 = glds whenever aligned (testing).
static int g_glds_override = -1;
int conv_glds_mode() {
  static int m = env_int("TDL_CONV_GLDS", 1);
  return g_glds_override >= 0 ? g_glds_override : m;
}
void conv_set_glds_mode(int mode) { g_glds_override = mode; }
static int g_m32_override = -1;
int conv_m32() {
  static int m = env_int("TDL_M32", 0);
  return g_m32_override >= 0 ? g_m32_override : m;
}
void conv_set_m32(int on) { g_m32_override = on; }
// producer/consumer forward (conv_pc.hip): TDL_CONV_PC unset = the route table's rows
// (fwd.pc.*), 0 = those rows off, 1 / 2 = 2 / 4 producer waves on every FASTK 256×128 forward;
// conv_set_pc(-1) = env
static int g_pc_override = -1;
int conv_pc() {
  static int m = env_int("TDL_CONV_PC", -1);
  return g_pc_override >= 0 ? g_pc_override : m;
}
void conv_set_pc(int on) { g_pc_override = on; }

// FWD tile order (tile_of): a workgroup owns one column tile and tpb consecutive row tiles
static int fwd_tiling(ConvArgs& a, const GCfg& g) {
  const long ntm = cdiv(a.M, g.bm), ntn = cdiv(a.Ng, g.bn);
  a.ncls = 1;
  a.splits = 1;
  a.tpb = grouped_tpb(&ntm, 1, ntn);
  const long groups = (ntm + a.tpb - 1) / a.tpb;
  a.cls_tile0[0] = 0;
  a.cls_tile0[1] = (int)(groups * ntn * a.tpb);
  return (int)(groups * ntn);
}

// route rows fwd.pc.*: the wave-specialised producer/consumer forward on 256×128 FASTK tiles; a
// folded BN (a.aff) only here — its producers stage the transformed operand
bool conv_fwd_pc_run(const ConvArgs& a0, hipStream_t st) {
  if (a0.C % 8 || a0.K % 8 || a0.res) return false;
  if (a0.aff && (a0.C % 64 || a0.bias)) return false;
  const int fk = a0.C % 64 == 0 ? 1 : (a0.R * a0.S == 1 ? 2 : 0);
  if (fk == 0) return false;
  ConvArgs a = a0;
  a.dbg = env_int("TDL_CONV_DBG", 0);
  set_fastdivs(a);
  const int blocks = fwd_tiling(a, G256x128);
  const int waves = a.aff ? 2 : (conv_pc() > 0 ? conv_pc() : 2);
  return conv_fwd_pc_launch(a, blocks, fk, waves, st);
}

// route rows fwd.glds.*: the LDS-DMA forward with tile config `cfg` (false: not eligible /
// not instantiated — nothing launched)
bool conv_fwd_glds(const ConvArgs& a0, int cfg, hipStream_t st) {
  if (a0.C % 8 || a0.K % 8 || a0.aff) return false;
  if (a0.res && !a0.bias) return false;  // residual epilogue instantiated with bias only
  if (!route_cfg_instantiated(RT_GLDS, FWD, cfg, a0.res ? RF_RES : 0)) return false;
  ConvArgs a = a0;
  a.dbg = env_int("TDL_CONV_DBG", 0);
  set_fastdivs(a);
  const int blocks = fwd_tiling(a, cfg_of(cfg));
  // FASTK (FK 1): a K-step is one filter tap × 64 channels; 1×1 filters with C % 64 != 0 take
  // it with the row's last channel chunk range-checked (FK 2: Xception's 728-channel pointwise
  // convs); otherwise the generic K decomposition (FK 0)
  const int fk = a.C % 64 == 0 ? 1 : (a.R * a.S == 1 ? 2 : 0);
  const bool stats = a.stats != nullptr, bias = a.bias != nullptr;
#define TDL_G(FK)                                                            \
  do {                                                                       \
    if (bias) {                                                              \
      if (stats) launch_gcfg<FWD, true, true, FK>(a, cfg, blocks, st);       \
      else launch_gcfg<FWD, false, true, FK>(a, cfg, blocks, st);            \
    } else {                                                                 \
      if (stats) launch_gcfg<FWD, true, false, FK>(a, cfg, blocks, st);      \
      else launch_gcfg<FWD, false, false, FK>(a, cfg, blocks, st);           \
    }                                                                        \
  } while (0)
  if (a.res) {
    // residual epilogue (DeepLab units): the default FWD tile configs, bias, ± statistics
#define TDL_R(FK)                                                                            \
  do {                                                                                       \
    if (cfg == 4) {                                                                          \
      if (stats) launch_g<FWD, 256, 64, 8, 1, 3, true, true, FK, false, false, true>(a, blocks, st);   \
      else launch_g<FWD, 256, 64, 8, 1, 3, false, true, FK, false, false, true>(a, blocks, st);        \
    } else {                                                                                 \
      if (stats) launch_g<FWD, 256, 128, 4, 2, 3, true, true, FK, false, false, true>(a, blocks, st);  \
      else launch_g<FWD, 256, 128, 4, 2, 3, false, true, FK, false, false, true>(a, blocks, st);       \
    }                                                                                        \
  } while (0)
    if (cfg != 0 && cfg != 4) return false;
    if (fk == 1) TDL_R(1);
    else if (fk == 2) TDL_R(2);
    else TDL_R(0);
#undef TDL_R
    return true;
  }
  // TDL_M32=1: the 256×128 FASTK forward on 32×32×16 MFMA blocks (A/B: dev/tools/m32_ab.py)
  if (conv_m32() && fk == 1 && cfg == 0) {
    if (bias) {
      if (stats) launch_g<FWD, 256, 128, 4, 2, 3, true, true, 1, false, false, false, true>(a, blocks, st);
      else launch_g<FWD, 256, 128, 4, 2, 3, false, true, 1, false, false, false, true>(a, blocks, st);
    } else {
      if (stats) launch_g<FWD, 256, 128, 4, 2, 3, true, false, 1, false, false, false, true>(a, blocks, st);
      else launch_g<FWD, 256, 128, 4, 2, 3, false, false, 1, false, false, false, true>(a, blocks, st);
    }
    return true;
  }
  // TDL_CONV_PC=1 / 2: the producer/consumer forward on every FASTK 256×128 problem (A/B)
  if (conv_pc() > 0 && fk != 0 && cfg == 0 && conv_fwd_pc_launch(a, blocks, fk, conv_pc(), st))
    return true;
  if (fk == 1) TDL_G(1);
  else if (fk == 2) TDL_G(2);
  else TDL_G(0);
#undef TDL_G
  return true;
}

// Stride-1 input gradient as the FORWARD conv of dy with the flipped, transposed filter:
// dx[n,h,w,c] = Σ_{r',s',k} dy[n, h − ph' + r'·dh, w − pw' + s'·dw, k] · w_flip[c][r'][s'][k],
// ph' = dh·(R−1) − ph — the forward kernels' K loop (LDS-DMA / producer-consumer; both operands
// K-contiguous, no transposed LDS reads, no parity-class bookkeeping) with the DGRAD epilogue
// (DEPI: ReLU bit mask, residual join, BN-backward statistics).  bench/dgrad_paths.py, ResNet-50
// b1024: 3×3 dgrads 22–31 % faster than the DGRAD kernel, 1×1 3–15 %.
// Strided (sh, sw > 1, no dilation): one forward conv of dy per parity class (a, b) of dx.  Class
// (a, b) — pixels h = a + sh·i, w = b + sw·j — receives only the taps r ≡ a + ph (mod sh),
// s ≡ b + pw (mod sw): Th × Tw of them, so it is a stride-1 Th × Tw forward conv over dy with
// padding Th − 1 − (a + ph − r0)/sh, whose filter is that class's flipped sub-filter
// (w_flip: the classes' [C][Th][Tw][K] sub-filters concatenated a-major, empty classes skipped —
// ops/conv.py flip_classes), and whose DGRAD epilogue scatters class row (n, i, j) to dx pixel
// (n, a + sh·i, b + sw·j) (ConvArgs::esh / esw / eH / eW).  Classes without taps are zero-filled
// first unless the dgrad accumulates.  bench/dgrad_strided.py, ResNet-50 b1024: 3×3 / s2 dgrads
// 1.2–1.8×, 1×1 / s2 1.9–2.2× (before the zero fill).
static bool dgrad_as_fwd_strided(const ConvArgs& a0, const bf16_t* wf, int cfg, hipStream_t st,
                                 bool* fused) {
  if (a0.dh != 1 || a0.dw != 1 || (cfg != 0 && cfg != 4)) return false;
  const int sh = a0.sh, sw = a0.sw;
  if (sh > 16 || sw > 16) return false;
  struct Cls { int a, r0, T, p, Hc; };
  Cls rows[16], cols[16];
  auto classes = [](int s, int R, int pad, int H, Cls* out) {
    for (int a = 0; a < s; ++a) {
      const int r0 = ((a + pad) % s + s) % s;
      const int T = r0 < R ? (R - r0 + s - 1) / s : 0;
      const int e = (a + pad - r0) / s;  // exact: r0 ≡ a + pad (mod s)
      out[a] = Cls{a, r0, T, T - 1 - e, a < H ? (H - a + s - 1) / s : 0};
    }
  };
  classes(sh, a0.R, a0.ph, a0.H, rows);
  classes(sw, a0.S, a0.pw, a0.W, cols);
  // (a class's padding Th − 1 − e may be negative — stride > kernel reach, e.g. 3×3 / s3: the
  // forward K loop's gather is plain arithmetic on ho − ph, range-checked against dy)
  bool any_empty = false;
  for (int i = 0; i < sh; ++i)
    for (int j = 0; j < sw; ++j) {
      const Cls &r = rows[i], &c = cols[j];
      if (r.T == 0 || c.T == 0 || r.Hc == 0 || c.Hc == 0) any_empty = true;
    }
  const bool stats = a0.stats != nullptr && a0.bn_x != nullptr;
  if (stats && a0.beta) return false;
  if (any_empty && !a0.beta) conv_zero_fill(a0.out, a0.out_bytes, st);
  long off = 0;
  for (int i = 0; i < sh; ++i)
    for (int j = 0; j < sw; ++j) {
      const Cls &r = rows[i], &c = cols[j];
      if (r.T == 0 || c.T == 0) continue;
      const long nsub = (long)a0.C * r.T * c.T * a0.K;
      if (r.Hc == 0 || c.Hc == 0) {
        off += nsub;
        continue;
      }
      ConvArgs a = a0;
      a.x = a0.dy;
      a.x_bytes = a0.dy_bytes;
      a.w = wf + off;
      a.w_bytes = (uint32_t)(nsub * 2);
      a.w_t = nullptr;
      a.C = a0.K;  // input channels of the forward conv: dy's
      a.K = a0.C;  // its output channels: dx's
      a.R = r.T;
      a.S = c.T;
      a.sh = a.sw = 1;
      a.ph = r.p;
      a.pw = c.p;
      a.H = a0.Ho;  // the forward's input: dy
      a.W = a0.Wo;
      a.Ho = r.Hc;  // its output: the class grid
      a.Wo = c.Hc;
      a.M = a.N * a.Ho * a.Wo;
      a.Ng = a.K;
      a.Kg = a.R * a.S * a.C;
      a.relu = 0;
      a.ncls = 1;
      a.cls_a[0] = r.a;
      a.cls_b[0] = c.a;
      a.cls_Hc[0] = r.Hc;
      a.cls_Wc[0] = c.Hc;
      a.cls_r0[0] = a.cls_s0[0] = 0;
      a.cls_Th[0] = a.R;
      a.cls_Tw[0] = a.S;
      a.eH = a0.H;  // the epilogue's scatter into dx
      a.eW = a0.W;
      a.esh = sh;
      a.esw = sw;
      a.dbg = 0;
      a.splits = 1;
      a.stats = stats ? a0.stats : nullptr;
      set_fastdivs(a);
      const int blocks = fwd_tiling(a, cfg_of(cfg));
      if (cfg == 4) {
        if (stats) launch_g<FWD, 256, 64, 8, 1, 3, true, false, 1, false, true, false, false, false, true>(a, blocks, st);
        else launch_g<FWD, 256, 64, 8, 1, 3, false, false, 1, false, false, false, false, false, true>(a, blocks, st);
      } else {
        if (stats) launch_g<FWD, 256, 128, 4, 2, 3, true, false, 1, false, true, false, false, false, true>(a, blocks, st);
        else launch_g<FWD, 256, 128, 4, 2, 3, false, false, 1, false, false, false, false, false, true>(a, blocks, st);
      }
      off += nsub;
    }
  if (fused) *fused = stats;
  return true;
}

// cfg (the route row's): 0 / 4 the LDS-DMA K loop with 256×128 / 8-wave 256×64 tiles, 100 the
// halo forward loader, 102 the producer/consumer kernel.
// fp8 (stride 1): e5m2 dy × the e4m3 flipped filter [C][R][S][K] on the forward fp8 K loop
// (A-operand format e5m2) with the scaled DGRAD epilogue; K % 128 == 0, cfg 0 (256×128)
static bool dgrad_as_fwd_fp8(const ConvArgs& a0, const bf16_t* wf, uint32_t wf_bytes, int cfg,
                             hipStream_t st, bool* fused) {
  if (cfg != 0 || a0.sh != 1 || a0.sw != 1 || a0.K % 128 || a0.C % 8 || a0.ldc != a0.C ||
      a0.aff || a0.dg_masked || a0.Ho != a0.H || a0.Wo != a0.W)
    return false;
  const int ph = a0.dh * (a0.R - 1) - a0.ph, pw = a0.dw * (a0.S - 1) - a0.pw;
  if (ph < 0 || pw < 0) return false;
  ConvArgs a = a0;
  a.x = a0.dy;
  a.x_bytes = a0.dy_bytes;
  a.w = wf;
  a.w_bytes = wf_bytes;
  a.w_t = nullptr;
  a.C = a0.K;
  a.K = a0.C;
  a.ph = ph;
  a.pw = pw;
  a.M = a.N * a.Ho * a.Wo;
  a.Ng = a.K;
  a.Kg = a.R * a.S * a.C;
  a.relu = 0;
  a.ncls = 1;
  a.cls_a[0] = a.cls_b[0] = 0;
  a.cls_Hc[0] = a.H;
  a.cls_Wc[0] = a.W;
  a.cls_r0[0] = a.cls_s0[0] = 0;
  a.cls_Th[0] = a.R;
  a.cls_Tw[0] = a.S;
  a.dbg = 0;
  a.splits = 1;
  set_fastdivs(a);
  const bool stats = a.stats != nullptr && a.bn_x != nullptr;
  if (!stats) a.stats = nullptr;
  const int blocks = fwd_tiling(a, cfg_of(0));
  if (stats && a.beta)
    launch_g<FWD, 256, 128, 4, 2, 3, true, false, 1, true, false, false, false, false, true>(a, blocks, st);
  else if (stats)
    launch_g<FWD, 256, 128, 4, 2, 3, true, false, 1, true, true, false, false, false, true>(a, blocks, st);
  else
    launch_g<FWD, 256, 128, 4, 2, 3, false, false, 1, true, false, false, false, false, true>(a, blocks, st);
  if (fused) *fused = stats;
  return true;
}

bool conv_dgrad_as_fwd(const ConvArgs& a0, const bf16_t* wf, uint32_t wf_bytes, int cfg,
                       hipStream_t st, bool* fused) {
  if (fused) *fused = false;
  if (a0.fp8) return wf != nullptr && dgrad_as_fwd_fp8(a0, wf, wf_bytes, cfg, st, fused);
  if (wf != nullptr && (a0.sh > 1 || a0.sw > 1) && !a0.fp8 && !a0.aff && !a0.dg_masked &&
      a0.K % 64 == 0 && a0.C % 8 == 0 && a0.ldc == a0.C)
    return dgrad_as_fwd_strided(a0, wf, cfg, st, fused);
  if (wf == nullptr || a0.fp8 || a0.aff || a0.dg_masked) return false;
  if (a0.sh != 1 || a0.sw != 1 || a0.K % 64 || a0.C % 8 || a0.ldc != a0.C) return false;
  // the DGRAD epilogue indexes dx through dy's geometry: same spatial size ("same" padding)
  if (a0.Ho != a0.H || a0.Wo != a0.W) return false;
  const int ph = a0.dh * (a0.R - 1) - a0.ph, pw = a0.dw * (a0.S - 1) - a0.pw;
  if (ph < 0 || pw < 0) return false;
  ConvArgs a = a0;
  a.x = a0.dy;
  a.x_bytes = a0.dy_bytes;
  a.w = wf;
  a.w_bytes = wf_bytes;
  a.w_t = nullptr;
  a.C = a0.K;  // input channels of the forward conv: dy's
  a.K = a0.C;  // its output channels: dx's
  a.ph = ph;
  a.pw = pw;
  a.M = a.N * a.Ho * a.Wo;
  a.Ng = a.K;
  a.Kg = a.R * a.S * a.C;
  a.relu = 0;
  // one identity parity class for the epilogue's row mapping (out_row_fast<DGRAD>)
  a.ncls = 1;
  a.cls_a[0] = a.cls_b[0] = 0;
  a.cls_Hc[0] = a.H;
  a.cls_Wc[0] = a.W;
  a.cls_r0[0] = a.cls_s0[0] = 0;
  a.cls_Th[0] = a.R;
  a.cls_Tw[0] = a.S;
  a.dbg = 0;
  a.splits = 1;
  set_fastdivs(a);
  const bool stats = a.stats != nullptr && a.bn_x != nullptr;
  if (!stats) a.stats = nullptr;
  if (cfg == 101) return conv_fwd_rw_depi(a, st, fused);  // (statistics and join both fit)
  // statistics + join: the LDS-DMA tiles (cfg 0 / 4; the 256×128 epilogue loads its operands in
  // two halves) — not the halo or producer/consumer loaders
  if (stats && a.beta && cfg != 4 && cfg != 0) return false;
  if (cfg == 100) return conv_fwd_halo_depi(a, st, fused);
  if (cfg == 102) {
    // (not with the statistics epilogue: its x registers spill at the 12-wave register budget)
    if (stats) return false;
    const int blocks = fwd_tiling(a, G256x128);
    return conv_fwd_pc_launch(a, blocks, 1, 2, st, true);
  }
  if (cfg != 0 && cfg != 4) return false;
  const int blocks = fwd_tiling(a, cfg_of(cfg));
  if (cfg == 4) {
    if (stats && a.beta)  // statistics + join: the 8-wave tiles hold both the x and previous-dx loads
      launch_g<FWD, 256, 64, 8, 1, 3, true, false, 1, false, false, false, false, false, true>(a, blocks, st);
    else if (stats) launch_g<FWD, 256, 64, 8, 1, 3, true, false, 1, false, true, false, false, false, true>(a, blocks, st);
    else launch_g<FWD, 256, 64, 8, 1, 3, false, false, 1, false, false, false, false, false, true>(a, blocks, st);
  } else {
    if (stats && a.beta) launch_g<FWD, 256, 128, 4, 2, 3, true, false, 1, false, false, false, false, false, true>(a, blocks, st);
    else if (stats) launch_g<FWD, 256, 128, 4, 2, 3, true, false, 1, false, true, false, false, false, true>(a, blocks, st);
    else launch_g<FWD, 256, 128, 4, 2, 3, false, false, 1, false, false, false, false, false, true>(a, blocks, st);
  }
  if (fused) *fused = stats;
  return true;
}

// the per-parity-class flipped sub-filters of a strided conv in one launch (was a flip, a
// permute copy and a concatenation per class in ATen): element e of class i (offset off[i],
// [C][Th][Tw][K]) = w[k][r0 + sh·(Th−1−t)][s0 + sw·(Tw−1−u)][c]
struct FlipCls {
  int n;
  int r0[16], th[16], s0[16], tw[16];
  long off[17];
};
__global__ void __launch_bounds__(256) flip_classes_kernel(const bf16_t* __restrict__ w,
                                                           bf16_t* __restrict__ out, int K, int R,
                                                           int S, int C, int sh, int sw,
                                                           FlipCls fc) {
  const long total = fc.off[fc.n];
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    int i = 0;
    while (i + 1 < fc.n && e >= fc.off[i + 1]) ++i;
    long q = e - fc.off[i];
    const int k = (int)(q % K);
    q /= K;
    const int u = (int)(q % fc.tw[i]);
    q /= fc.tw[i];
    const int t = (int)(q % fc.th[i]);
    const int c = (int)(q / fc.th[i]);
    const int r = fc.r0[i] + sh * (fc.th[i] - 1 - t), s2 = fc.s0[i] + sw * (fc.tw[i] - 1 - u);
    out[e] = w[(((long)k * R + r) * S + s2) * C + c];
  }
}

// w_flip[c][r][s][k] = w[k][R−1−r][S−1−s][c]: a 32×32-element tiled transpose per filter tap
__global__ void __launch_bounds__(256) flip_weight_kernel(const bf16_t* __restrict__ w,
                                                          bf16_t* __restrict__ wf, int K, int R,
                                                          int S, int C) {
  __shared__ bf16_t t[32][33];
  const int tap = blockIdx.z;  // r·S + s of the output
  const int r = tap / S, s = tap - r * S;
  const int src_tap = (R - 1 - r) * S + (S - 1 - s);
  const int k0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 × 8
  for (int i = ty; i < 32; i += 8) {
    const int k = k0 + i, c = c0 + tx;
    t[i][tx] = (k < K && c < C) ? w[((long)k * R * S + src_tap) * C + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, k = k0 + tx;
    if (c < C && k < K) wf[((long)c * R * S + tap) * K + k] = t[tx][i];
  }
}

void conv_flip_weight_launch(const bf16_t* w, bf16_t* wf, int K, int R, int S, int C,
                             hipStream_t st) {
  dim3 grid((unsigned)cdiv(C, 32), (unsigned)cdiv(K, 32), (unsigned)(R * S));
  hipLaunchKernelGGL(flip_weight_kernel, grid, dim3(256), 0, st, w, wf, K, R, S, C);
}

// every flipped filter of a model in ONE launch (after each optimizer step): the bf16 weights live
// in one flat buffer (models/params.py), their flips at the same offsets of a parallel buffer.
// Work row (8 × int64): element offset, K, R, S, C, output tap, k tile, c tile — one 32×32 tile
// per workgroup, the same transpose as flip_weight_kernel.
__global__ void __launch_bounds__(256) multi_flip_kernel(const bf16_t* __restrict__ src,
                                                         bf16_t* __restrict__ dst,
                                                         const long* __restrict__ rows) {
  __shared__ bf16_t t[32][33];
  const long* q = rows + 8 * (long)blockIdx.x;
  const long off = q[0];
  const int K = (int)q[1], R = (int)q[2], S = (int)q[3], C = (int)q[4], tap = (int)q[5];
  const int k0 = (int)q[6] * 32, c0 = (int)q[7] * 32;
  const bf16_t* w = src + off;
  bf16_t* wf = dst + off;
  const int r = tap / S, s = tap - r * S;
  const int src_tap = (R - 1 - r) * S + (S - 1 - s);
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int k = k0 + i, c = c0 + tx;
    t[i][tx] = (k < K && c < C) ? w[((long)k * R * S + src_tap) * C + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, k = k0 + tx;
    if (c < C && k < K) wf[((long)c * R * S + tap) * K + k] = t[tx][i];
  }
}

long conv_flip_classes_numel(int K, int R, int S, int C, int sh, int sw, int ph, int pw) {
  if (sh < 1 || sw < 1 || sh > 4 || sw > 4)
    throw std::runtime_error("conv_flip_classes: 1 <= stride <= 4");
  long total = 0;
  for (int a = 0; a < sh; ++a) {
    const int r0 = ((a + ph) % sh + sh) % sh, th = r0 < R ? (R - r0 + sh - 1) / sh : 0;
    for (int b = 0; b < sw; ++b) {
      const int s0 = ((b + pw) % sw + sw) % sw, tw = s0 < S ? (S - s0 + sw - 1) / sw : 0;
      total += (long)C * th * tw * K;
    }
  }
  return total;
}

void conv_flip_classes_launch(const bf16_t* w, bf16_t* out, int K, int R, int S, int C, int sh,
                              int sw, int ph, int pw, hipStream_t st) {
  if (sh < 1 || sw < 1 || sh > 4 || sw > 4)
    throw std::runtime_error("conv_flip_classes: 1 <= stride <= 4");
  FlipCls fc{};
  long off = 0;
  for (int a = 0; a < sh; ++a) {
    const int r0 = ((a + ph) % sh + sh) % sh, th = r0 < R ? (R - r0 + sh - 1) / sh : 0;
    for (int b = 0; b < sw; ++b) {
      const int s0 = ((b + pw) % sw + sw) % sw, tw = s0 < S ? (S - s0 + sw - 1) / sw : 0;
      if (!th || !tw) continue;
      fc.r0[fc.n] = r0;
      fc.th[fc.n] = th;
      fc.s0[fc.n] = s0;
      fc.tw[fc.n] = tw;
      fc.off[fc.n] = off;
      off += (long)C * th * tw * K;
      ++fc.n;
    }
  }
  fc.off[fc.n] = off;
  if (off == 0) return;
  const int blocks = (int)std::min<long>(4096, (off + 255) / 256);
  hipLaunchKernelGGL(flip_classes_kernel, dim3(blocks), dim3(256), 0, st, w, out, K, R, S, C, sh, sw,
                     fc);
}

void conv_flip_weights_multi_launch(const bf16_t* src, bf16_t* dst, const long* rows, int nrows,
                                    hipStream_t st) {
  if (nrows <= 0) return;
  hipLaunchKernelGGL(multi_flip_kernel, dim3(nrows), dim3(256), 0, st, src, dst, rows);
}

// fused BN-backward statistics in the LDS-DMA DGRAD epilogue (a.stats, a.bn_x): FASTK (K % 64 == 0,
// or the ragged form of a one-class 1×1); joins need stride 1 — an accumulate leaves the pixels of
// a class without taps unmasked; a folded BN's mask (a.aff) rides on the single-consumer form
bool dgrad_stats_fusable(const ConvArgs& a) {
  if (!a.stats || !a.bn_x || a.dg_masked) return false;
  // fp8 (e5m2 dy × e4m3 Wᵀ, K % 128 == 0): the statistics epilogue, no folded BN; a join only at
  // stride 1 (as below)
  if (a.fp8)
    return a.K % 128 == 0 && !a.aff && (!a.beta || (a.ncls == 1 && a.sh == 1 && a.sw == 1));
  const bool rag = a.K % 64 != 0 && a.R * a.S == 1 && a.ncls == 1 && a.K % 8 == 0;
  if (a.K % 64 != 0 && !rag) return false;
  if (a.beta && !(a.ncls == 1 && a.sh == 1 && a.sw == 1)) return false;
  return !a.aff || (a.K % 64 == 0 && !a.beta);
}

// DGRAD with prepared parity classes (conv_dgrad_launch builds them) on tile config `cfg` (the
// route row's); false when the kernel does not take the problem or config — nothing launched
bool conv_dgrad_glds(const ConvArgs& a0, int cfg, hipStream_t st, bool* fused) {
  if (fused) *fused = false;
  if (a0.dg_masked || a0.C % 8) return false;
  if (a0.fp8 ? (a0.K % 128 || (cfg != 0 && cfg != 1)) : a0.K % 8) return false;
  const bool bn_stats = dgrad_stats_fusable(a0);
  if (!a0.fp8) {
    const int flags = (bn_stats ? RF_STATS : 0) | (bn_stats && a0.aff ? RF_AFF : 0);
    if (!route_cfg_instantiated(RT_GLDS, DGRAD, cfg, flags)) return false;
  }
  ConvArgs a = a0;
  a.dbg = env_int("TDL_CONV_DBG", 0);
  set_fastdivs(a);
  const GCfg& g = cfg_of(cfg);
  a.cls_tile0[0] = 0;
  for (int c = 0; c < a.ncls; ++c) {
    const long Mc = (long)a.N * a.cls_Hc[c] * a.cls_Wc[c];
    a.cls_tile0[c + 1] = a.cls_tile0[c] + (int)(cdiv(Mc, g.bm) * (long)cdiv(a.Ng, g.bn));
  }
  const long tiles = a.cls_tile0[a.ncls];
  if (tiles == 0) return true;
  // BN-backward statistics: tiles in the forward's column-grouped order (tile_of COLG) so each
  // workgroup flushes its column sums once (strided dgrads: every parity class in the same order,
  // each class's tiles padded to whole workgroups so none straddles two classes; a class without
  // taps was zero-filled and adds 0).  Tile configs (dev/tools/dgrad_bnstat_ab.py, ResNet-50
  // b256): without a join 256×128 (NJ: no previous-dx registers); with the join's previous-dx
  // loads as well those spill — 8 waves of 32×64 (cfg 6); a folded BN's coefficients likewise
  const bool rag_stats = a.K % 64 != 0;
  if (bn_stats) {
    const long ntn = cdiv(a.Ng, g.bn);
    long ntm_c[MAX_DG_CLASSES];
    for (int c = 0; c < a.ncls; ++c) ntm_c[c] = cdiv((long)a.N * a.cls_Hc[c] * a.cls_Wc[c], g.bm);
    a.tpb = grouped_tpb(ntm_c, a.ncls, ntn);
    a.cls_tile0[0] = 0;
    for (int c = 0; c < a.ncls; ++c) {
      const long groups_c = cdiv(cdiv((long)a.N * a.cls_Hc[c] * a.cls_Wc[c], g.bm), a.tpb);
      a.cls_tile0[c + 1] = a.cls_tile0[c] + (int)(groups_c * ntn * a.tpb);
    }
    const int blocks = a.cls_tile0[a.ncls] / a.tpb;
    a.splits = 1;
    if (a.fp8) {
      if (a.beta) {  // + the join's previous-dx loads
        if (cfg == 1)
          launch_g<DGRAD, 256, 64, 4, 1, 3, true, false, 1, true, false>(a, blocks, st);
        else
          launch_g<DGRAD, 256, 128, 4, 2, 3, true, false, 1, true, false>(a, blocks, st);
      } else if (cfg == 1) {
        launch_g<DGRAD, 256, 64, 4, 1, 3, true, false, 1, true, true>(a, blocks, st);
      } else {
        launch_g<DGRAD, 256, 128, 4, 2, 3, true, false, 1, true, true>(a, blocks, st);
      }
    } else if (a.aff) {  // (K % 64 == 0, no join; cfg 4 or 6)
      if (cfg == 4)
        launch_g<DGRAD, 256, 64, 8, 1, 3, true, false, 1, false, true, false, false, true>(a, blocks, st);
      else  // (8 waves of 32×64: the 256×128 tiles spill with the coefficient registers)
        launch_g<DGRAD, 128, 128, 4, 2, 4, true, false, 1, false, true, false, false, true>(a, blocks, st);
    } else if (rag_stats) {
      if (a.beta)
        launch_gcfg<DGRAD, true, false, 2>(a, cfg, blocks, st);
      else
        launch_gcfg<DGRAD, true, false, 2, true>(a, cfg, blocks, st);
    } else if (a.beta) {
      launch_gcfg<DGRAD, true, false, 1>(a, cfg, blocks, st);
    } else {
      launch_gcfg<DGRAD, true, false, 1, true>(a, cfg, blocks, st);
    }
    if (fused) *fused = true;
    return true;
  }
  a.stats = nullptr;
  a.tpb = persistent_tpb(tiles);
  a.splits = 1;
  const int blocks = (int)((tiles + a.tpb - 1) / a.tpb);
  if (a.fp8) {
    if (cfg == 1)
      launch_g<DGRAD, 256, 64, 4, 1, 3, false, false, 1, true>(a, blocks, st);
    else
      launch_g<DGRAD, 256, 128, 4, 2, 3, false, false, 1, true>(a, blocks, st);
  } else if (a.K % 64 == 0 && a.w_t) {  // transposed weights: KC B operand
    a.w = a.w_t;
    if (conv_m32() && cfg == 0)
      launch_g<DGRAD, 256, 128, 4, 2, 3, false, false, 3, false, false, false, true>(a, blocks, st);
    else
      launch_gcfg<DGRAD, false, false, 3>(a, cfg, blocks, st);
  } else if (a.K % 64 == 0) {
    launch_gcfg<DGRAD, false, false, 1>(a, cfg, blocks, st);
  } else if (a.R * a.S == 1 && a.ncls == 1) {  // ragged FASTK (see conv_fwd_glds)
    launch_gcfg<DGRAD, false, false, 2>(a, cfg, blocks, st);
  } else {
    launch_gcfg<DGRAD, false, false, 0>(a, cfg, blocks, st);
  }
  return true;
}

// WGRAD split-K plan for the LDS-DMA kernel on tile config `cfg` (the route row's: 0 / 2 the
// usual tiles, 7 the 64×256 column of the row-packed stem): ≈ one tile-split per CU slot,
// ≥ 16 K-steps each
bool conv_wgrad_glds_plan(const ConvArgs& a, int cfg, WgradPlan* p) {
  if (a.fp8) return conv_wgrad_fp8_plan(a, cfg, p);
  if (a.C % 8 || a.K % 8 || a.aff) return false;
  if (!route_cfg_instantiated(RT_GLDS, WGRAD, cfg, 0)) return false;
  const GCfg& g = cfg_of(cfg);
  const long tiles = (long)cdiv(a.M, g.bm) * cdiv(a.Ng, g.bn);
  const int nkt = cdiv(a.Kg, BK);
  // ≈ tile-splits per launch (TDL_GLDS_WGRAD_TARGET): 128 (half a wave of CUs; fewer fp32 slabs to
  // write and reduce) vs 256 / 512: Xception-41 b128 3,260 / 3,223 / 3,193 img/s, ResNet-50 b1024
  // 13,316 / 13,273 / 13,084 (same box)
  const int target = env_int("TDL_GLDS_WGRAD_TARGET", 128);
  int s = (int)std::max<long>(1, std::min<long>(nkt, (target + tiles - 1) / tiles));
  int per = std::max(cdiv(nkt, s), env_int("TDL_GLDS_WGRAD_MINSTEPS", 16));
  s = cdiv(nkt, per);
  p->impl = 1;
  p->cfg = cfg;
  p->bm = g.bm;
  p->bn = g.bn;
  p->splits = s;
  p->kps = per;
  return true;
}

// fp8 weight gradient (route rows wgrad.glds.fp8*: dy e5m2 × x e4m3, a.scale_x / a.scale_w the
// per-tensor scales): cfg 0 = 256×128, 2 = 128×128 tiles; K-steps of 128 pixels
bool conv_wgrad_fp8_plan(const ConvArgs& a, int cfg, WgradPlan* p) {
  if (!a.fp8 || a.C % 16 || a.K % 16 || a.aff || (cfg != 0 && cfg != 2)) return false;
  const GCfg& g = cfg_of(cfg);
  const long tiles = (long)cdiv(a.M, g.bm) * cdiv(a.Ng, g.bn);
  const int nkt = cdiv(a.Kg, 128);
  const int target = env_int("TDL_GLDS_WGRAD_TARGET", 128);
  int s = (int)std::max<long>(1, std::min<long>(nkt, (target + tiles - 1) / tiles));
  int per = std::max(cdiv(nkt, s), std::max(1, env_int("TDL_GLDS_WGRAD_MINSTEPS", 16) / 2));
  s = cdiv(nkt, per);
  p->impl = 1;
  p->cfg = cfg;
  p->bm = g.bm;
  p->bn = g.bn;
  p->splits = s;
  p->kps = per;
  return true;
}

void conv_wgrad_glds_kernel_launch(const ConvArgs& a0, const WgradPlan& p, hipStream_t st) {
  ConvArgs a = a0;
  a.dbg = env_int("TDL_CONV_DBG", 0);
  set_fastdivs(a);
  const long tiles = (long)cdiv(a.M, p.bm) * cdiv(a.Ng, p.bn) * p.splits;
  a.kps = p.kps;
  a.splits = p.splits;
  a.ncls = 1;
  a.cls_tile0[0] = 0;
  a.cls_tile0[1] = (int)tiles;
  a.tpb = persistent_tpb(tiles);
  const int blocks = (int)((tiles + a.tpb - 1) / a.tpb);
  if (a.fp8) {
    if (p.cfg == 0)
      launch_g<WGRAD, 256, 128, 4, 2, 3, false, false, 1, true>(a, blocks, st);
    else if (p.cfg == 2)
      launch_g<WGRAD, 128, 128, 2, 2, 4, false, false, 1, true>(a, blocks, st);
    else
      throw std::runtime_error("fp8 weight gradient: tile config not instantiated");
    return;
  }
  launch_gcfg<WGRAD, false, false, 1>(a, p.cfg, blocks, st);
}

}  // namespace tdl
