// Host-side declarations of the gfx950 kernel launchers (raw pointers + hipStream_t; no torch).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <cstdlib>

namespace tdl {

typedef uint16_t bf16_t;  // storage type of bf16 tensors (raw bits)

// fp8 amax "slot": AMAX_SPREAD partial maxima AMAX_STRIDE floats apart (common.h amax_publish);
// a delayed-scaling ring is 3 slots
constexpr int AMAX_SPREAD = 16, AMAX_STRIDE = 64, AMAX_SLOT = AMAX_SPREAD * AMAX_STRIDE;

struct FastDiv {
  uint32_t m, s;
};
// Division by a runtime constant d via a host-computed magic number: n / d = (n·m) >> s, exact for
// 0 ≤ n < 2^31 (m = ⌈2^(31+l)/d⌉, l = ⌈log2 d⌉; checked exhaustively in tests/test_ops_cpu.py).
// Replaces the ~40-instruction v_rcp/readfirstlane sequences hipcc emits for `/` in hot loops.
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint32_t sh = 31 + l;
  const uint64_t m = ((1ull << sh) + d - 1) / d;
  return FastDiv{(uint32_t)m, sh};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) {
  return (uint32_t)(((uint64_t)n * f.m) >> f.s);
}


struct ConvArgs {
  const bf16_t* x;   // FWD / WGRAD: input activations [N,H,W,C]
  const bf16_t* w;   // FWD / DGRAD: weights [K,R,S,C]
  const bf16_t* dy;  // DGRAD / WGRAD: output gradient [N,Ho,Wo,K]
  void* out;         // FWD: y bf16 [M][ldc]; DGRAD: dx bf16 [M][ldc]; WGRAD: fp32 split slabs
  const float* bias; // FWD: optional bias [K]
  float* stats;      // FWD: optional BN statistics [2][K] (Σy, Σy²), accumulated.
                     // DGRAD: BN-backward statistics of the BN whose output is this conv's input
                     // ((Σg, Σg·x) with g the stored dx and x = a.bn_x, the BN's input; LDS-DMA
                     // kernel, stride-1 only) — the BN backward then needs no reduce pass
  const bf16_t* bn_x;  // DGRAD with stats: the BN input [N,H,W,C] (same layout as dx)
  const bf16_t* res;   // FWD (LDS-DMA kernel, with bias): residual added before the ReLU, laid
                       // out like the output
  int N, H, W, C, K, R, S, Ho, Wo;
  int sh, sw, ph, pw, dh, dw;
  int M, Ng, Kg;     // GEMM dims
  int ldc;
  int relu;
  const float* scale_x;  // fp8 FWD: per-tensor scales of x and w (device scalars)
  const float* scale_w;
  int beta;          // DGRAD: 1 = accumulate into the existing dx (residual-gradient join)
  int fp8;           // DGRAD: dy is e5m2 (a.dy), the weight e4m3 transposed [R][S][C][K] (a.w),
                     // per-tensor scales a.scale_x (dy) and a.scale_w (LDS-DMA kernel, K % 128 == 0)
  const bf16_t* w_t;    // DGRAD (bf16): optional copy of the weights transposed to [R][S][C][K];
                        // the LDS-DMA kernel then reads both operands as K-contiguous rows
  const uint8_t* mask;  // DGRAD: optional ReLU bit mask of dx (1 bit per element, NHWC order):
                        // dx = ([dx +] dgrad)·[bit] — the consumers of a block output apply the
                        // mask of its ReLU, so the producer BN's backward reads no mask
  uint32_t x_bytes, w_bytes, dy_bytes, out_bytes;  // buffer-descriptor ranges (OOB -> 0 / dropped)
  int kps;           // WGRAD: K-steps per split
  int splits;        // WGRAD: number of K splits
  int tpb;           // tiles per workgroup (FWD / DGRAD multi-tile pipelining)
  FastDiv fd_HoWo, fd_Wo, fd_C, fd_S, fd_sh, fd_sw;  // magic divisors (LDS-DMA launchers)
  FastDiv cls_fdHW[16], cls_fdW[16];                 // DGRAD per-class pixel decomposition
  int dbg;           // ablation flags (TDL_CONV_DBG, diagnostics only): 1 drop operand loads, 2 skip MFMA
  // DGRAD parity classes (stride s: s_h·s_w classes of input pixels, each with its exact taps)
  int ncls;
  int dg_masked;     // 1: stride>1 with dilation>1 — single class, divisibility-masked taps
  // DGRAD epilogue scatter geometry (out_row_fast<DGRAD>): dx pixel of class row (n, i, j) =
  // (n, cls_a + esh·i, cls_b + esw·j) in an eH × eW image — the conv's own H, W, sh, sw
  // (conv_args), except for a strided input gradient run as per-class forward convs of dy
  // (conv_dgrad_as_fwd), whose K loop sees stride 1 over dy's Ho × Wo
  int eH, eW, esh, esw;
  int cls_tile0[17]; // prefix sum of tiles per class
  int cls_a[16], cls_b[16], cls_Hc[16], cls_Wc[16];
  int cls_r0[16], cls_Th[16], cls_s0[16], cls_Tw[16];
  // Training BN + ReLU of the conv's input folded into this conv (ops/bnconv.py): the input is
  // u = relu(a·x + b), a = aff[c], b = aff[aff_ld + c] (bn_finalize's fp32 coefficient rows),
  // rounded to bf16 exactly as the BN apply pass stores it; padding taps stay 0.
  //   FWD    the A operand (conv_pc producers, conv_gemm staging)
  //   WGRAD  the B operand (conv_gemm staging)
  //   DGRAD  the ReLU mask of dx is a·bn_x + b > 0 (only together with the fused BN-backward
  //          statistics, a.stats / a.bn_x — the launcher's return value says whether it ran)
  // Launchers that cannot apply it must not run the problem (conv_aff_fwd_ok / the routing).
  const float* aff;
  int aff_ld;
  // DGRAD (bf16, stride 1): optional flipped, transposed weights w_flip[c][r][s][k] =
  // w[k][R−1−r][S−1−s][c] — the input gradient then runs as the forward conv of dy (the forward
  // kernels' K loop with the DGRAD epilogue, conv_dgrad_as_fwd)
  const bf16_t* w_flip;
  uint32_t w_flip_bytes;
};
constexpr int MAX_DG_CLASSES = 16;

// deterministic mode (det.hip): fixed-order slab reductions instead of fp32 atomics
int deterministic();
void det_set(int on);  // -1: environment (TDL_DETERMINISTIC)
float* det_slab(size_t floats, hipStream_t st);  // per-stream scratch, grows on demand
void slab_sum_launch(const float* slab, float* out, int rows, long n, long row_stride,
                     hipStream_t st);  // out[i] += Σ_r slab[r·row_stride + i], rows in order

void conv_fwd_launch(const ConvArgs& a, hipStream_t st);
// FWD with a.res: false (nothing launched) when the LDS-DMA kernel does not take the problem
bool conv_fwd_res_launch(const ConvArgs& a, hipStream_t st);
// returns true when a.stats was filled (DGRAD BN-backward statistics fused into the epilogue);
// a.stats is ignored (false) when the problem does not run on the LDS-DMA kernel
bool conv_dgrad_launch(const ConvArgs& a, hipStream_t st);
// WGRAD plan: impl 0 = register-staged kernel (bm × bn tiles), 1 = LDS-DMA kernel (config cfg);
// the caller allocates splits·M·Ng fp32 slab floats and passes them in a.out.
struct WgradPlan {
  int impl, cfg, bm, bn, splits, kps;
};
void conv_wgrad_plan(const ConvArgs& a, WgradPlan* p);
void conv_wgrad_launch(const ConvArgs& a, const WgradPlan& p, float* out, bool accumulate,
                       hipStream_t st);
// LDS-DMA pipelined kernels (conv_glds.hip); false / 0 = not eligible, use the register-staged one
int conv_glds_mode();
void conv_set_glds_mode(int mode);  // -1: environment / default
// 32×32×16-MFMA K loop for the KC-operand LDS-DMA convs (FWD FASTK, DGRAD with W^T): TDL_M32 /
// override (-1: environment)
int conv_m32();
void conv_set_m32(int on);
// training BN folded into its 1×1 consumer (bnfold.hip)
void bn_fold_weight_launch(const void* w, bool bf16, const float* coef, int K, int C, int ldcoef,
                           void* wout, const float* bias_in, float* bias_out, hipStream_t st);
void scale_cols_launch(float* dw, const float* a, long n, int C, hipStream_t st);
int conv_pc();
bool conv_fwd_pc_launch(const ConvArgs& a, int blocks, int fk, int mode, hipStream_t st,
                        bool depi = false);
// stride-1 input gradient as the forward conv of dy with the flipped filter w_flip [C][R][S][K]
// (conv_glds.hip): true when it ran (*fused: the BN-backward statistics were written); false =
// not eligible, nothing launched
bool conv_dgrad_as_fwd(const ConvArgs& a, const bf16_t* w_flip, uint32_t w_flip_bytes, int cfg,
                       hipStream_t st, bool* fused);
// zero a byte range (multiple of 4) with a kernel (graph-capturable, stream-ordered)
void conv_zero_fill(void* p, uint32_t bytes, hipStream_t st);
// w_flip[c][r][s][k] = w[k][R−1−r][S−1−s][c] (bf16)
void conv_flip_weight_launch(const bf16_t* w, bf16_t* wf, int K, int R, int S, int C,
                             hipStream_t st);
// many flips in one launch: rows int64 [n][8] = (offset, K, R, S, C, tap, k tile, c tile), the
// flip of the [K,R,S,C] filter at src + offset written at dst + offset
// strided dgrad-as-forward sub-filters (ops/conv.flip_classes): for every stride parity class
// with taps (a-major, then b), [C][Th][Tw][K] with tap t ↦ r0 + sh·(Th−1−t), concatenated
// elements conv_flip_classes_launch writes (every parity class's sub-filter, back to back)
long conv_flip_classes_numel(int K, int R, int S, int C, int sh, int sw, int ph, int pw);
void conv_flip_classes_launch(const bf16_t* w, bf16_t* out, int K, int R, int S, int C, int sh,
                              int sw, int ph, int pw, hipStream_t st);
void conv_flip_weights_multi_launch(const bf16_t* src, bf16_t* dst, const long* rows, int nrows,
                                    hipStream_t st);
void conv_set_pc(int on);
// route executors (conv_route.h): true when they ran, false = not eligible, nothing launched
bool conv_fwd_glds(const ConvArgs& a, int cfg, hipStream_t st);
bool conv_fwd_pc_run(const ConvArgs& a, hipStream_t st);
// halo-tiled direct conv (conv_halo.hip) for stride-1 R×S filters, Cin % 64 == 0: true when it
// ran (TDL_HALO=0 turns its route rows off); the dgrad sets *fused when a.stats was filled
int conv_halo_mode();
void conv_set_halo_mode(int mode);  // -1: environment; 2: every eligible problem (tests)
bool conv_fwd_halo(const ConvArgs& a, hipStream_t st);
bool conv_dgrad_halo(const ConvArgs& a, hipStream_t st, bool* fused);
// a stride-1 dgrad already rewritten as a forward conv (conv_dgrad_as_fwd) on the halo forward
// loader with the DGRAD epilogue
bool conv_fwd_halo_depi(const ConvArgs& a, hipStream_t st, bool* fused);
// resident-weight halo conv (conv_halo.hip): stride-1 3×3, 64 → 64 channels — the forward and a
// dgrad already rewritten as a forward conv (DGRAD epilogue); false: not eligible
bool conv_fwd_rw(const ConvArgs& a, hipStream_t st);
bool conv_fwd_rw_depi(const ConvArgs& a, hipStream_t st, bool* fused);
// stride-1 3×3 weight gradient on the halo kernel: plan impl 2 (fp32 split slabs as usual)
bool conv_wgrad_halo_plan(const ConvArgs& a, WgradPlan* p);
void conv_wgrad_halo_launch(const ConvArgs& a, const WgradPlan& p, hipStream_t st);
// *fused: set to whether a.stats was filled (stride-1 FASTK problems only)
bool conv_dgrad_glds(const ConvArgs& a, int cfg, hipStream_t st, bool* fused = nullptr);
// can the LDS-DMA DGRAD epilogue fuse this problem's BN-backward statistics (classes built)?
bool dgrad_stats_fusable(const ConvArgs& a);
bool conv_wgrad_glds_plan(const ConvArgs& a, int cfg, WgradPlan* p);  // (a.fp8: the fp8 plan)
bool conv_wgrad_fp8_plan(const ConvArgs& a, int cfg, WgradPlan* p);
void conv_wgrad_glds_kernel_launch(const ConvArgs& a, const WgradPlan& p, hipStream_t st);
// fp8 (OCP e4m3) forward conv: a.x / a.w point at e4m3 bytes, a.scale_x / a.scale_w at their fp32 scales
void conv_fwd_fp8_launch(const ConvArgs& a, hipStream_t st);
void fp8_amax_launch(const bf16_t* x, long n, float* slot, hipStream_t st);
// end-of-step roll of n amax rings (device pointer table): slot0 ← slot1, slot1 ← 0
void fp8_roll_launch(const unsigned long long* rings, int n, hipStream_t st);
// delayed-scaling policy: scale = margin · amax / fp8_max (e4m3 activations and weights; e5m2
// gradients), amax slot 0 ← max(this step's, decay · previous) at each roll
struct Fp8Policy {
  float margin_e4m3, margin_e5m2, decay;
};
Fp8Policy fp8_policy();
void fp8_set_policy(float margin_e4m3, float margin_e5m2, float decay);  // < 0: environment
// prev: amax slot giving the scale; meas (optional): slot accumulating |x|max; clr (optional):
// slot cleared for the next call
void fp8_quantize_launch(const bf16_t* x, long n, const float* prev, float* meas, float* clr,
                         float* scale_out, uint8_t* y, hipStream_t st);
// chunks: int64 [nchunks][4] = (segment, start element, length (% 16 == 0), first-of-segment)
void fp8_multi_quantize_launch(const bf16_t* src, uint8_t* dst, const long* chunks, int nchunks,
                               float* rings, float* scales, int phase, bool prime, hipStream_t st);
void fp8_dequantize_launch(const uint8_t* y, long n, const float* scale, float* out, hipStream_t st);
// OCP e5m2 (bf8) flavour of fp8_quantize_launch (scale = amax / 57344) — output gradients
void fp8_quantize_e5m2_launch(const bf16_t* x, long n, const float* prev, float* meas, float* clr,
                              float* scale_out, uint8_t* y, hipStream_t st);
void fp8_dequantize_e5m2_launch(const uint8_t* y, long n, const float* scale, float* out,
                                hipStream_t st);
// byte-matrix transposes in one launch: tiles int64 [ntiles][4] = (offset, rows, cols, tile id);
// dst[offset + c·rows + r] = src[offset + r·cols + c] (rows, cols % 16 == 0) — the fp8 dgrad's
// transposed weight copies [R][S][C][K] of every fp8 conv weight [K][R·S·C]
void fp8_multi_transpose_launch(const uint8_t* src, uint8_t* dst, const long* tiles, int ntiles,
                                hipStream_t st);
// bias gradient: out[K] (+)= column sums of x[P][K]; part = fp32 scratch of colsum_blocks(P, K)·K
int colsum_blocks(long P, int K);
void colsum_launch(const bf16_t* x, float* out, float* part, long P, int K, bool accumulate,
                   hipStream_t st);

// batch norm ---------------------------------------------------------------------------------
void bn_stats_launch(const bf16_t* x, float* stats, long M, int C, hipStream_t st);
void bn_finalize_launch(const float* stats, float* coef, const float* gamma, const float* beta,
                        float* rmean, float* rvar, int C, int c_run, float count, float decay,
                        float eps, bool training, hipStream_t st);
void bn_apply_launch(const bf16_t* x, const float* coef, const bf16_t* res, bf16_t* y, long M,
                     int C, bool relu, hipStream_t st, uint8_t* y8 = nullptr,
                     const float* amax_prev = nullptr, float* scale_out = nullptr,
                     float* amax_out = nullptr, float* amax_zero = nullptr,
                     uint8_t* mask = nullptr,  // mask: 1 bit per element of y > 0 (C % 8 == 0)
                     long ldy = 0);  // y row stride (elements; 0 = C): y a channel slice of a concat buffer
void bn_bwd_reduce_launch(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* coef,
                          float* red, long M, int C, int relu, hipStream_t st,
                          long ldd = 0);  // ldd: dy row stride (0 = C; C % 8 == 0, C <= 2048) relu: 0 none, 1 mask y>0, 2 mask x·scale+shift>0, 3 bit mask (y = uint8 mask, C % 8 == 0, C <= 2048)
// two BNs fed the same (unmasked) gradient dy: red = (Σdy, Σdy·x̂) of x (coef), red2 = (Σdy,
// Σdy·x2) raw; false (nothing launched) unless C % 8 == 0 and C <= 2048
bool bn_bwd_reduce2_launch(const bf16_t* dy, const bf16_t* x, const bf16_t* x2, const float* coef,
                           float* red, float* red2, long M, int C, hipStream_t st);
// optional e5m2 side output of dx (fp8 dgrad of the producing conv), delayed scaling as
// bn_apply's e4m3 one: dx8 = e5m2(sat(dx·57344/amax_prev)), scale_out = amax_prev/57344,
// this call's |dx|max into amax_out, amax_zero cleared (C % 8 == 0 only)
void bn_bwd_apply_launch(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* coef,
                         const float* red, const float* gamma, bf16_t* dx, bf16_t* dres,
                         float* dgamma, float* dbeta, long M, int C, float count, int relu,
                         hipStream_t st, uint8_t* dx8 = nullptr, const float* amax_prev = nullptr,
                         float* scale_out = nullptr, float* amax_out = nullptr,
                         float* amax_zero = nullptr,
                         bool red_raw = false,  // red = (Σg, Σg·x) from a fused dgrad epilogue
                         long ldd = 0,  // dy row stride (elements; 0 = C)
                         const bf16_t* dadd = nullptr);  // added to dx (C % 8 == 0)

// elementwise --------------------------------------------------------------------------------
// t [N][H][Wo][Cp] = row-packed x [N][H][W][Cx] for a k×k stem conv (first Cr channels, S taps of
// stride sw from column wo·sw − pl; zeros past the row / after S·Cr); Cp % 8 == 0
void row_pack_launch(const bf16_t* x, bf16_t* t, int N, int H, int W, int Cx, int Cr, int S,
                     int sw, int pl, int Wo, int Cp, hipStream_t st);
void relu_bwd_launch(const bf16_t* dy, const bf16_t* y, bf16_t* dx, long n, hipStream_t st);
void add_act_launch(const bf16_t* a, const bf16_t* b, bf16_t* y, long n, bool relu,
                    hipStream_t st);
void scale_by_scalar_launch(const void* x, const float* s, void* y, long n, bool bf16,
                            hipStream_t st);
// fp32 → bf16 (RNE) or bf16 → fp32 of n contiguous elements (16-B aligned buffers)
void convert_launch(const void* x, bool x_bf16, void* y, long n, hipStream_t st);
void sigmoid_threshold_launch(const void* x, bool x_bf16, float* prob, float* pred, long n,
                              float thr, hipStream_t st);

// pooling ------------------------------------------------------------------------------------
void maxpool_fwd_launch(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C,
                        int Ho, int Wo, int k, int s, int pt, int pl, hipStream_t st);
// maxpool backward that also applies the producing BN's ReLU bit mask to dx and accumulates the
// BN-backward sums (Σg, Σg·x) of the stored dx into red [2][C] (x = bx, the BN input); false (and
// nothing launched) unless C % 8 == 0 and 256 % (C / 8) == 0
bool maxpool_bwd_stats_launch(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, const bf16_t* bx,
                              const uint8_t* mask, float* red, int N, int H, int W, int C, int Ho,
                              int Wo, int k, int s, int pt, int pl, hipStream_t st);
// the stem's BN + ReLU + max-pool in one pass (ReLU bit in idx bit 7; C % 8 == 0, else false) and
// the matching backward gather without statistics (deterministic mode)
bool bn_maxpool_fwd_launch(const bf16_t* x, const float* coef, bf16_t* y, uint8_t* idx,
                           bf16_t* zarg, int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                           int pt, int pl, hipStream_t st);
// the fused backward of bn_maxpool_fwd (with zarg): BN sums per pool output, then the gather +
// BN backward apply per input pixel; red [2, C] zeroed by the caller; false: C does not fit
bool maxpool_bn_bwd_launch(const bf16_t* dy, const uint8_t* idx, const bf16_t* zarg,
                           const bf16_t* x, const float* coef, float* red, const float* gamma,
                           bf16_t* dx, float* dgamma, float* dbeta, int N, int H, int W, int C,
                           int Ho, int Wo, int k, int s, int pt, int pl, float inv_count,
                           hipStream_t st);
void maxpool_bwd_rb_launch(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W,
                           int C, int Ho, int Wo, int k, int s, int pt, int pl, hipStream_t st);
void maxpool_bwd_launch(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W,
                        int C, int Ho, int Wo, int k, int s, int pt, int pl, hipStream_t st);
void avgpool_fwd_launch(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t st);
// dadd (optional, C % 8 == 0, may alias dx): dx = dy/HW + dadd (residual-gradient join)
void avgpool_bwd_launch(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st,
                        const bf16_t* dadd = nullptr);

// losses -------------------------------------------------------------------------------------
void softmax_xent_launch(const void* logits, bool bf16, const int64_t* labels, float* loss,
                         void* grad, int N, int K, float smoothing, hipStream_t st);
// evaluation head: probs (optional) = softmax rows (fp32); with labels, loss_sum += Σ row CE and
// correct += Σ [argmax == label] (either may be null)
void softmax_eval_launch(const void* logits, bool bf16, const int64_t* labels, float* loss_sum,
                         float* correct, float* probs, int N, int K, hipStream_t st);
void lovasz_hinge_launch(const void* logits, bool logits_bf16, const void* labels, int label_kind,
                         float* loss, float* grad, int B, int P, hipStream_t st);
// P > 16384 pixels per image: multi-pass global bitonic sort; key / idx hold B × padded_len(P)
int lovasz_padded_len(int P);
void lovasz_hinge_large_launch(const void* logits, bool logits_bf16, const void* labels,
                               int label_kind, float* loss, float* grad, float* key, int* idx, int B,
                               int P, hipStream_t st);
void seg_metrics_launch(const void* labels, int label_kind, const float* pred, float* score,
                        float* acc, int B, int P, bool kaggle, hipStream_t st);

// optimizers ---------------------------------------------------------------------------------
// lr_scale (optional device scalar) multiplies lr / lr_t inside the kernel (HIP-graph replays)
void sgd_momentum_launch(float* p, const float* g, float* mom, bf16_t* lowp, const uint8_t* flags,
                         long n, float lr, const float* lr_scale, float mu, float wd, float gscale,
                         bool nesterov, hipStream_t st);
void adam_launch(float* p, const float* g, float* m, float* v, bf16_t* lowp, const uint8_t* flags,
                 long n, float lr_t, const float* lr_scale, float b1, float b2, float eps, float wd,
                 float gscale, hipStream_t st);

// depthwise conv -----------------------------------------------------------------------------
struct DwArgs {
  const bf16_t* x;
  const bf16_t* w;     // [R,S,C]
  const float* bias;   // [C] or null
  const bf16_t* dy;
  bf16_t* out;
  float* dw;           // fp32 [R,S,C]
  float* db;           // fp32 [C]
  int N, H, W, C, R, S, Ho, Wo, sh, sw, ph, pw, dh, dwl;
  int relu;
  // fused pre-activation ReLU of the input (Xception's relu → separable conv): fwd / wgrad read
  // max(x, 0); dgrad zeroes dx where mask_x ≤ 0 (mask_x = the un-rectified x).  3×3, C % 8 == 0.
  int relu_in = 0;
  // optional fused BN sums (fp32 [2][C], accumulated; stride-1 3×3 tile kernels only — the
  // launchers return whether they were written): fwd (Σy, Σy²); dgrad (Σg, Σg·bn_x)
  float* stats = nullptr;
  const bf16_t* bn_x = nullptr;
  const bf16_t* mask_x = nullptr;
  int accum = 1;  // wgrad: 1 = add into a.dw / a.db, 0 = overwrite them
  // dgrad: dx = (masked) dgrad + dadd (shaped like dx; may alias a.out) — the residual-gradient
  // join of a tensor whose other consumer's gradient is already in the buffer (ops/gradjoin.py)
  const bf16_t* dadd = nullptr;
  // input BN + ReLU folded in (ops/dwfold.py): the conv's input is u = relu(a·x + b) with
  // a = aff[c], b = aff[aff_ld + c] (fp32 BN coefficients) — fwd: applied to the staged tile;
  // dgrad: the ReLU mask is a·bn_x + b > 0 (bn_x = x); wgrad: applied to the x loads.
  // Stride-1 3×3 tile / sliding kernels only (dwconv_aff_ok)
  const float* aff = nullptr;
  int aff_ld = 0;
};
bool dwconv_aff_ok(const DwArgs& a);
bool dwconv_fwd_launch(const DwArgs& a, hipStream_t st);  // true: a.stats written
bool dwconv_dgrad_launch(const DwArgs& a, hipStream_t st);  // true: a.stats written
int dwconv_wgrad_slabs(const DwArgs& a);  // row-slab count of the fast wgrad (0: generic)
// adds dW / db into a.dw / a.db (a.accum = 0: overwrites them); ws: slabs·(R·S + 1)·C floats when
// dwconv_wgrad_slabs(a) > 0
void dwconv_wgrad_launch(const DwArgs& a, float* ws, hipStream_t st);
// out[i] (+)= Σ_z slab[z·n + i]  (split-K / slab reduction, conv_gemm.hip)
void splitk_reduce_launch(const float* slab, float* out, long n, int splits, bool accumulate,
                          hipStream_t st);

// upsample (TF1 legacy bilinear with symmetric pad) -----------------------------------------
// ldy / ldd: pixel stride (elements) of y / dy — C, or wider for a channel slice of a concat
// buffer (concat-free ASPP / decoder); <= 0 means C
void upsample_fwd_launch(const bf16_t* x, bf16_t* y, const int* ih, const float* wh,
                         const int* iw, const float* ww, int N, int H, int W, int C, int Ho,
                         int Wo, hipStream_t st, int ldy = 0);
void upsample_bwd_launch(const bf16_t* dy, bf16_t* dx, const int* ih, const float* wh,
                         const int* iw, const float* ww, int N, int H, int W, int C, int Ho,
                         int Wo, hipStream_t st, int ldd = 0);

// fp32 path (f32.hip; the reference's own precision) --------------------------------------------
// NHWC fp32 activations, KRSC fp32 weights; every channel count (C, K) % 4 == 0 (host-checked)
struct ConvF32Args {
  const float* x;      // FWD / WGRAD input [N,H,W,C]
  const float* w;      // FWD / DGRAD weights [K,R,S,C]
  const float* dy;     // DGRAD / WGRAD output gradient [N,Ho,Wo,K]
  float* out;          // FWD y [N,Ho,Wo,K]; DGRAD dx [N,H,W,C]; WGRAD dW [K,R,S,C]
  const float* bias;   // FWD optional [K]
  float* stats;        // FWD optional BN sums [2][K] (Σy, Σy² of the stored y), accumulated
  const float* res;    // FWD optional residual shaped like y, added before the ReLU
  int N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw;
  int relu;            // FWD
  int accumulate;      // DGRAD: dx += …; WGRAD: dW += … (else overwritten)
  float* slab;         // WGRAD with conv_f32_wgrad_splits(a) > 1: fp32 scratch of splits·K·R·S·C
  FastDiv fd_HoWo, fd_Wo;  // (launcher) magic divisors of the WGRAD pixel decomposition
};
void conv_f32_fwd_launch(const ConvF32Args& a, hipStream_t st);
// FWD / DGRAD workgroup tile override (64 or 128 each; anything else: automatic choice)
void conv_f32_set_tile(int tbm, int tbn);
void conv_f32_dgrad_launch(const ConvF32Args& a, hipStream_t st);
// WGRAD splits the pixel reduction: each split writes its partial dW slab (plain stores), one
// reduction pass sums the slabs into dW (no memset, no atomics)
int conv_f32_wgrad_splits(const ConvF32Args& a);
void conv_f32_wgrad_launch(const ConvF32Args& a, hipStream_t st);
// out[c] += Σ_m x[m·ldx + c] (the caller zeroes out for an overwrite)
void colsum_f32_launch(const float* x, float* out, long M, int C, long ldx, hipStream_t st);
void bn_stats_f32_launch(const float* x, float* stats, long M, int C, hipStream_t st);
// relu: 0 none, 1 mask y > 0, 2 mask x·scale + shift > 0; ldd: dy row stride
void bn_bwd_reduce_f32_launch(const float* dy, const float* y, const float* x, const float* coef,
                              float* red, long M, int C, int relu, long ldd, hipStream_t st);
void bn_apply_f32_launch(const float* x, const float* coef, const float* res, float* y, long M,
                         int C, bool relu, long ldy, hipStream_t st);
void bn_bwd_apply_f32_launch(const float* dy, const float* y, const float* x, const float* coef,
                             const float* red, const float* gamma, float* dx, float* dres,
                             float* dgamma, float* dbeta, const float* dadd, long M, int C,
                             float count, int relu, long ldd, hipStream_t st);
void row_pack_f32_launch(const float* x, float* t, int N, int H, int W, int Cx, int Cr, int S,
                         int sw, int pl, int Wo, int Cp, hipStream_t st);
void relu_bwd_f32_launch(const float* dy, const float* y, float* dx, long n, hipStream_t st);
void add_act_f32_launch(const float* a, const float* b, float* y, long n, bool relu,
                        hipStream_t st);
struct DwF32Args {
  const float* x;
  const float* w;      // [R,S,C]
  const float* bias;   // [C] or null
  const float* dy;
  float* out;
  float* dwt;          // fp32 [R,S,C], accumulated
  float* db;           // fp32 [C], accumulated (optional)
  int N, H, W, C, R, S, Ho, Wo, sh, sw, ph, pw, dh, dwl;
  int relu;
  const float* dadd;   // dgrad: added to dx (residual-gradient join; may alias out)
};
void dwconv_f32_fwd_launch(const DwF32Args& a, hipStream_t st);
void dwconv_f32_dgrad_launch(const DwF32Args& a, hipStream_t st);
void dwconv_f32_wgrad_launch(const DwF32Args& a, hipStream_t st);  // R·S ≤ 9
// fp32 instantiations of the type-generic pooling / upsample kernels
void maxpool_fwd_launch(const float* x, float* y, uint8_t* idx, int N, int H, int W, int C,
                        int Ho, int Wo, int k, int s, int pt, int pl, hipStream_t st);
void maxpool_bwd_launch(const float* dy, const uint8_t* idx, float* dx, int N, int H, int W,
                        int C, int Ho, int Wo, int k, int s, int pt, int pl, hipStream_t st);
void avgpool_fwd_launch(const float* x, float* y, int N, int HW, int C, hipStream_t st);
void avgpool_bwd_launch(const float* dy, float* dx, int N, int HW, int C, hipStream_t st,
                        const float* dadd = nullptr);
void upsample_fwd_launch(const float* x, float* y, const int* ih, const float* wh,
                         const int* iw, const float* ww, int N, int H, int W, int C, int Ho,
                         int Wo, hipStream_t st, int ldy = 0);
void upsample_bwd_launch(const float* dy, float* dx, const int* ih, const float* wh,
                         const int* iw, const float* ww, int N, int H, int W, int C, int Ho,
                         int Wo, hipStream_t st, int ldd = 0);

// fault injection: a 1-lane kernel that spins `ms` milliseconds (≤ 60 s) on stream st
void debug_spin_launch(double ms, hipStream_t st);

}  // namespace tdl
