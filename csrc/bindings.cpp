// Python bindings of the gfx950 kernels (torch tensors in, launches on the current HIP stream).
// Kernels themselves live in csrc/kernels/*.hip and see only raw pointers (no torch headers there).
#include <torch/extension.h>

#include <cstring>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPCachingAllocator.h>

#include "kernels/kernels.h"
#include "kernels/conv_route.h"
#include "runtime/loader.h"
#include "runtime/comm.h"

using torch::Tensor;
using namespace tdl;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_T(t, dt)                                                                        \
  TORCH_CHECK((t).is_cuda(), #t " must be a HIP tensor");                                     \
  TORCH_CHECK((t).is_contiguous(), #t " must be contiguous");                                 \
  TORCH_CHECK((t).scalar_type() == (dt), #t " has wrong dtype ", (t).scalar_type())

#define BF(t) reinterpret_cast<const bf16_t*>((t).data_ptr())
// NHWC bf16 tensor that is contiguous or a channel slice [..., c0:c0+C] of a contiguous NHWC
// buffer (the concat-free ASPP / decoder): returns the pixel stride in elements
static int64_t nhwc_ld(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kBFloat16, what, ": bf16 HIP tensor");
  if (t.is_contiguous()) return t.size(-1);
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1 && t.stride(2) >= t.size(3) &&
                  t.stride(1) == t.stride(2) * t.size(2) && t.stride(0) == t.stride(1) * t.size(1),
              what, ": must be contiguous NHWC or a channel slice of a contiguous NHWC buffer");
  return t.stride(2);
}
#define BFW(t) reinterpret_cast<bf16_t*>((t).data_ptr())
// row stride of a strided operand of the vector BN kernels (8-element vectors, 16-byte aligned)
static int64_t bn_vec_ld(const at::Tensor& t, int64_t C, const char* what) {
  const int64_t ld = nhwc_ld(t, what);
  if (ld != C)
    TORCH_CHECK(C % 8 == 0 && C <= 2048 && ld % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
                what, ": a channel slice needs C % 8 == 0, C <= 2048, 8-aligned offset and stride");
  return ld;
}

const float* optf(const c10::optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->is_contiguous(), "expected fp32 contiguous");
  return t->data_ptr<float>();
}
float* optfw(const c10::optional<Tensor>& t) { return const_cast<float*>(optf(t)); }
const bf16_t* optb(const c10::optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == torch::kBFloat16 && t->is_contiguous(), "expected bf16 contiguous");
  return BF(*t);
}
bf16_t* optbw(const c10::optional<Tensor>& t) { return const_cast<bf16_t*>(optb(t)); }

uint32_t nbytes32(const Tensor& t) {
  const int64_t n = t.numel() * t.element_size();
  // < 3.75 GiB: the conv epilogues push invalid rows to byte offset 0xF0000000 (ROW_OOB)
  TORCH_CHECK(n < int64_t(0xF0000000), "tensor too large for 32-bit buffer addressing");
  return (uint32_t)n;
}

ConvArgs conv_args(const Tensor& x_like, const Tensor& w_like, int64_t N, int64_t H, int64_t W,
                   int64_t C, int64_t K, int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t ph,
                   int64_t pw, int64_t dh, int64_t dw, int64_t Ho, int64_t Wo) {
  ConvArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.K = K; a.R = R; a.S = S;
  a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dw = dw;
  a.Ho = Ho; a.Wo = Wo;
  a.eH = H; a.eW = W; a.esh = sh; a.esw = sw;
  (void)x_like; (void)w_like;
  return a;
}

// folded BN + ReLU of a conv's input (ConvArgs::aff): bn_finalize's fp32 coefficient rows
// [≥2, C] (row 0 the scale a, row 1 the shift b)
static void set_conv_aff(ConvArgs& a, const c10::optional<Tensor>& aff, int64_t C, const char* who) {
  a.aff = nullptr;
  a.aff_ld = 0;
  if (!aff.has_value() || !aff->defined()) return;
  TORCH_CHECK(aff->is_cuda() && aff->scalar_type() == torch::kFloat32 && aff->is_contiguous() &&
                  aff->dim() == 2 && aff->size(0) >= 2 && aff->size(1) == C && C % 8 == 0,
              who, " aff: fp32 [>=2, C] BN coefficients, C % 8 == 0");
  a.aff = aff->data_ptr<float>();
  a.aff_ld = (int)C;
}

// ------------------------------------------------------------------------------- fp32 path (f32.hip)
// Every entry point below dispatches on the activation dtype: fp32 tensors run the fp32 kernels
// (the reference's precision), bf16 the fused bf16 kernels.  The fp32 path has no fused ReLU bit
// masks, BN-backward-statistics epilogues or fp8 side outputs: requests for them return "not
// fused" (the caller then runs the plain pass) or fail loudly.
#define F32(t) ((t).data_ptr<float>())
static bool is_f32(const Tensor& t) { return t.scalar_type() == torch::kFloat32; }

static void check_c4(int64_t c, const char* what) {
  TORCH_CHECK(c % 4 == 0, what, ": the fp32 kernels need channel counts % 4 == 0 (got ", c, ")");
}

// fp32 NHWC tensor, contiguous or a channel slice of a contiguous NHWC buffer: pixel stride
static int64_t nhwc_ld_f32(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && is_f32(t), what, ": fp32 HIP tensor");
  if (t.is_contiguous()) return t.size(-1);
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1 && t.stride(2) >= t.size(3) &&
                  t.stride(1) == t.stride(2) * t.size(2) && t.stride(0) == t.stride(1) * t.size(1) &&
                  t.stride(2) % 4 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              what, ": must be contiguous NHWC or a 4-aligned channel slice of one");
  return t.stride(2);
}

static const float* opt_f32_like(const c10::optional<Tensor>& t, const Tensor& like,
                                 const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_T(*t, torch::kFloat32);
  TORCH_CHECK(t->sizes() == like.sizes(), what, ": shaped like ", like.sizes());
  return F32(*t);
}

static ConvF32Args conv_f32_args(int64_t N, int64_t H, int64_t W, int64_t C, int64_t K, int64_t R,
                                 int64_t S, int64_t Ho, int64_t Wo, int64_t sh, int64_t sw,
                                 int64_t ph, int64_t pw, int64_t dh, int64_t dw) {
  check_c4(C, "conv input channels");  // (any output channel count)
  TORCH_CHECK(N * std::max(H * W, Ho * Wo) < (1LL << 31) && K * R * S * C < (1LL << 31),
              "fp32 conv: problem too large for 32-bit GEMM indices");
  ConvF32Args a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.K = K; a.R = R; a.S = S; a.Ho = Ho; a.Wo = Wo;
  a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dw = dw;
  return a;
}

bool conv_fwd_f32(Tensor x, Tensor w, Tensor y, c10::optional<Tensor> bias,
                  c10::optional<Tensor> stats, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                  int64_t dh, int64_t dw, bool relu, c10::optional<Tensor> res) {
  CHECK_T(x, torch::kFloat32);
  CHECK_T(w, torch::kFloat32);
  CHECK_T(y, torch::kFloat32);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && y.dim() == 4 && x.size(3) == w.size(3) &&
                  y.size(0) == x.size(0) && y.size(3) == w.size(0), "conv_fwd fp32 shapes");
  ConvF32Args a = conv_f32_args(x.size(0), x.size(1), x.size(2), x.size(3), w.size(0), w.size(1),
                                w.size(2), y.size(1), y.size(2), sh, sw, ph, pw, dh, dw);
  a.x = F32(x); a.w = F32(w); a.out = F32(y);
  a.bias = optf(bias);
  if (a.bias) TORCH_CHECK(bias->numel() == a.K, "conv_fwd bias: [K]");
  a.stats = optfw(stats);
  if (a.stats) TORCH_CHECK(stats->numel() == 2 * a.K, "stats must be [2, K]");
  a.res = opt_f32_like(res, y, "conv_fwd res");
  a.relu = relu;
  conv_f32_fwd_launch(a, stream());
  return true;
}

bool conv_dgrad_f32(Tensor dy, Tensor w, Tensor dx, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                    int64_t dh, int64_t dw, bool accumulate, c10::optional<Tensor> mask) {
  CHECK_T(dy, torch::kFloat32);
  CHECK_T(w, torch::kFloat32);
  CHECK_T(dx, torch::kFloat32);
  TORCH_CHECK(!(mask.has_value() && mask->defined()), "fp32 conv_dgrad: no fused ReLU mask");
  TORCH_CHECK(dx.size(3) == w.size(3) && dy.size(3) == w.size(0) && dx.size(0) == dy.size(0),
              "conv_dgrad fp32 shapes");
  ConvF32Args a = conv_f32_args(dx.size(0), dx.size(1), dx.size(2), dx.size(3), w.size(0), w.size(1),
                                w.size(2), dy.size(1), dy.size(2), sh, sw, ph, pw, dh, dw);
  a.dy = F32(dy); a.w = F32(w); a.out = F32(dx);
  a.accumulate = accumulate;
  conv_f32_dgrad_launch(a, stream());
  return false;  // BN-backward statistics never fused on this path
}

void conv_wgrad_f32(Tensor dy, Tensor x, Tensor out, c10::optional<Tensor> bias_grad, int64_t sh,
                    int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw, bool accumulate) {
  CHECK_T(dy, torch::kFloat32);
  CHECK_T(x, torch::kFloat32);
  CHECK_T(out, torch::kFloat32);
  TORCH_CHECK(out.dim() == 4 && out.size(3) == x.size(3) && dy.size(3) == out.size(0) &&
                  dy.size(0) == x.size(0), "conv_wgrad fp32 shapes (dW KRSC)");
  ConvF32Args a = conv_f32_args(x.size(0), x.size(1), x.size(2), x.size(3), out.size(0),
                                out.size(1), out.size(2), dy.size(1), dy.size(2), sh, sw, ph, pw,
                                dh, dw);
  a.dy = F32(dy); a.x = F32(x); a.out = F32(out);
  a.accumulate = accumulate;
  auto st = stream();
  const int splits = conv_f32_wgrad_splits(a);
  Tensor slab;
  if (splits > 1) {
    slab = torch::empty({(int64_t)splits * out.numel()}, out.options());
    a.slab = F32(slab);
  }
  conv_f32_wgrad_launch(a, st);
  if (bias_grad.has_value() && bias_grad->defined()) {
    CHECK_T(*bias_grad, torch::kFloat32);
    TORCH_CHECK(bias_grad->numel() == a.K, "bias_grad must have K elements");
    (void)hipMemsetAsync(bias_grad->data_ptr(), 0, a.K * sizeof(float), st);
    colsum_f32_launch(F32(dy), F32(*bias_grad), (long)dy.numel() / a.K, a.K, a.K, st);
  }
}

// ------------------------------------------------------------------------------------------ conv
// res (optional, shaped like y): y = act(conv + bias + res) in the LDS-DMA epilogue; returns
// false — nothing launched — when that kernel does not take the problem (the caller then adds
// the residual itself)
// aff (optional): the input is relu(aff[0]·x + aff[1]) — a training BN + ReLU folded into this
// conv (ops/bnconv.py); no bias / residual with it
bool conv_fwd(Tensor x, Tensor w, Tensor y, c10::optional<Tensor> bias, c10::optional<Tensor> stats,
              int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw, bool relu,
              c10::optional<Tensor> res, c10::optional<Tensor> aff) {
  if (is_f32(x)) {
    TORCH_CHECK(!(aff.has_value() && aff->defined()), "fp32 conv: no folded BN");
    return conv_fwd_f32(x, w, y, bias, stats, sh, sw, ph, pw, dh, dw, relu, res);
  }
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(w, torch::kBFloat16);
  CHECK_T(y, torch::kBFloat16);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && y.dim() == 4, "NHWC / KRSC expected");
  TORCH_CHECK(x.size(3) == w.size(3), "C mismatch");
  ConvArgs a = conv_args(x, w, x.size(0), x.size(1), x.size(2), x.size(3), w.size(0), w.size(1),
                         w.size(2), sh, sw, ph, pw, dh, dw, y.size(1), y.size(2));
  TORCH_CHECK(y.size(0) == a.N && y.size(3) == a.K, "output shape mismatch");
  a.x = BF(x); a.w = BF(w); a.out = y.data_ptr();
  a.x_bytes = nbytes32(x); a.w_bytes = nbytes32(w); a.out_bytes = nbytes32(y);
  a.bias = optf(bias);
  a.stats = optfw(stats);
  if (a.stats) TORCH_CHECK(stats->numel() == 2 * a.K, "stats must be [2, K]");
  a.M = a.N * a.Ho * a.Wo; a.Ng = a.K; a.Kg = a.R * a.S * a.C; a.ldc = a.K; a.relu = relu;
  set_conv_aff(a, aff, a.C, "conv_fwd");
  if (a.aff) TORCH_CHECK(!a.bias && !(res.has_value() && res->defined()) && a.K % 8 == 0,
                         "conv_fwd aff: no bias / residual, K % 8 == 0");
  if (res.has_value() && res->defined()) {
    CHECK_T(*res, torch::kBFloat16);
    TORCH_CHECK(res->sizes() == y.sizes(), "conv_fwd res: shaped like y");
    a.res = BF(*res);
    if (a.M == 0) return true;
    float* det_stats = nullptr;
    if (a.stats && deterministic()) {
      det_stats = a.stats;
      a.stats = nullptr;
    }
    const bool ran = conv_fwd_res_launch(a, stream());  // false: nothing launched
    if (ran && det_stats) bn_stats_launch(BF(y), det_stats, a.M, a.K, stream());
    return ran;
  }
  if (a.M == 0) return true;
  float* det_stats = nullptr;
  if (a.stats && deterministic()) {  // fixed-order statistics pass instead of epilogue atomics
    det_stats = a.stats;
    a.stats = nullptr;
  }
  conv_fwd_launch(a, stream());
  if (det_stats) bn_stats_launch(BF(y), det_stats, a.M, a.K, stream());
  return true;
}

// fp8 (e4m3) forward conv: x8 [N,H,W,C] and w8 [K,R,S,C] as 1-byte tensors, sx / sw fp32 [1]
void conv_fwd_fp8(Tensor x8, Tensor w8, Tensor y, c10::optional<Tensor> stats, Tensor sx, Tensor sw_,
                  int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw, bool relu) {
  TORCH_CHECK(x8.is_cuda() && w8.is_cuda() && x8.element_size() == 1 && w8.element_size() == 1,
              "fp8 operands expected");
  TORCH_CHECK(x8.is_contiguous() && w8.is_contiguous(), "contiguous operands expected");
  CHECK_T(y, torch::kBFloat16);
  CHECK_T(sx, torch::kFloat32);
  CHECK_T(sw_, torch::kFloat32);
  TORCH_CHECK(x8.size(3) == w8.size(3) && x8.size(3) % 16 == 0, "fp8 conv needs C % 16 == 0");
  ConvArgs a = conv_args(x8, w8, x8.size(0), x8.size(1), x8.size(2), x8.size(3), w8.size(0),
                         w8.size(1), w8.size(2), sh, sw, ph, pw, dh, dw, y.size(1), y.size(2));
  TORCH_CHECK(y.size(0) == a.N && y.size(3) == a.K && a.K % 8 == 0, "output shape mismatch");
  a.x = (const bf16_t*)x8.data_ptr(); a.w = (const bf16_t*)w8.data_ptr(); a.out = y.data_ptr();
  a.x_bytes = (uint32_t)x8.numel(); a.w_bytes = (uint32_t)w8.numel(); a.out_bytes = nbytes32(y);
  TORCH_CHECK(x8.numel() < (1LL << 32) && w8.numel() < (1LL << 32), "tensor too large");
  a.stats = optfw(stats);
  if (a.stats) TORCH_CHECK(stats->numel() == 2 * a.K, "stats must be [2, K]");
  a.scale_x = sx.data_ptr<float>(); a.scale_w = sw_.data_ptr<float>();
  a.M = a.N * a.Ho * a.Wo; a.Ng = a.K; a.Kg = a.R * a.S * a.C; a.ldc = a.K; a.relu = relu;
  if (a.M == 0) return;
  float* det_stats = nullptr;
  if (a.stats && deterministic()) {
    det_stats = a.stats;
    a.stats = nullptr;
  }
  conv_fwd_fp8_launch(a, stream());
  if (det_stats) bn_stats_launch(BF(y), det_stats, a.M, a.K, stream());
}

// amax rings are fp32 [3, AMAX_SLOT] (kernels.h); slot indices 0..2
float* ring_slot(const Tensor& ring, int64_t k) {
  CHECK_T(ring, torch::kFloat32);
  TORCH_CHECK(ring.numel() == 3 * AMAX_SLOT && ring.is_contiguous(), "amax ring: fp32[3, AMAX_SLOT]");
  return ring.data_ptr<float>() + ((k % 3) + 3) % 3 * AMAX_SLOT;
}

// ptrs: int64 [n] device table of ring base addresses
void fp8_roll(Tensor ptrs) {
  TORCH_CHECK(ptrs.is_cuda() && ptrs.scalar_type() == torch::kInt64 && ptrs.is_contiguous(),
              "fp8_roll: int64 device pointer table");
  fp8_roll_launch((const unsigned long long*)ptrs.data_ptr<int64_t>(), (int)ptrs.numel(), stream());
}

void fp8_amax(Tensor x, Tensor ring, int64_t slot) {
  CHECK_T(x, torch::kBFloat16);
  TORCH_CHECK(x.numel() % 8 == 0, "numel % 8");
  fp8_amax_launch(BF(x), x.numel(), ring_slot(ring, slot), stream());
}

// scale from ring[phase]; measure: |x|max into ring[phase+1], ring[phase+2] cleared
void fp8_quantize(Tensor x, Tensor ring, int64_t phase, bool measure, Tensor scale, Tensor y8) {
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(scale, torch::kFloat32);
  TORCH_CHECK(y8.is_cuda() && y8.element_size() == 1 && y8.is_contiguous() && y8.numel() == x.numel());
  TORCH_CHECK(x.numel() % 16 == 0, "numel % 16");
  fp8_quantize_launch(BF(x), x.numel(), ring_slot(ring, phase),
                      measure ? ring_slot(ring, phase + 1) : nullptr,
                      measure ? ring_slot(ring, phase + 2) : nullptr, scale.data_ptr<float>(),
                      (uint8_t*)y8.data_ptr(), stream());
}

// src: flat bf16 buffer; dst: flat 1-byte buffer of the same numel; chunks int64 [n,4];
// rings fp32 [S,3,AMAX_SLOT]; scales fp32 [S]
void fp8_multi_quantize(Tensor src, Tensor dst, Tensor chunks, Tensor rings, Tensor scales,
                        int64_t phase, bool prime) {
  CHECK_T(src, torch::kBFloat16);
  CHECK_T(rings, torch::kFloat32);
  CHECK_T(scales, torch::kFloat32);
  TORCH_CHECK(dst.is_cuda() && dst.element_size() == 1 && dst.is_contiguous() &&
              dst.numel() == src.numel(), "dst: flat 1-byte buffer like src");
  TORCH_CHECK(chunks.is_cuda() && chunks.scalar_type() == torch::kInt64 && chunks.dim() == 2 &&
              chunks.size(1) == 4 && chunks.is_contiguous(), "chunks: int64 [n,4]");
  TORCH_CHECK(rings.dim() == 3 && rings.size(1) == 3 && rings.size(2) == AMAX_SLOT &&
              rings.is_contiguous() && scales.numel() == rings.size(0), "rings [S,3,AMAX_SLOT]");
  TORCH_CHECK(phase >= 0 && phase < 3);
  fp8_multi_quantize_launch(BF(src), (uint8_t*)dst.data_ptr(), chunks.data_ptr<int64_t>(),
                            (int)chunks.size(0), rings.data_ptr<float>(), scales.data_ptr<float>(),
                            (int)phase, prime, stream());
}

void fp8_dequantize(Tensor y8, Tensor scale, Tensor out) {
  TORCH_CHECK(y8.is_cuda() && y8.element_size() == 1 && y8.is_contiguous());
  CHECK_T(out, torch::kFloat32);
  fp8_dequantize_launch((const uint8_t*)y8.data_ptr(), y8.numel(), scale.data_ptr<float>(),
                        out.data_ptr<float>(), stream());
}

// bn_x / bn_red (optional, together): also accumulate the BN-backward sums (Σg, Σg·x) of the
// stored dx into bn_red fp32 [2, C] (zeroed by the caller), x = bn_x the input of the BN whose
// output this conv consumed.  Returns whether they were computed (stride-1 problems on the
// LDS-DMA kernel); otherwise bn_red is untouched and the BN backward reduces itself.
// aff (optional, with bn_x / bn_red): the ReLU mask of a folded BN — dx · [aff[0]·bn_x + aff[1]
// > 0] — applied together with the fused statistics; the return value says whether both ran
// (otherwise dx is unmasked and the BN backward masks: relu mode 2)
// w_flip (optional, stride 1): the flipped, transposed weights [C][R][S][K] (conv_flip_weight) —
// the input gradient may then run as the forward conv of dy (conv_dgrad_as_fwd)
bool conv_dgrad(Tensor dy, Tensor w, Tensor dx, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                int64_t dh, int64_t dw, bool accumulate, c10::optional<Tensor> mask,
                c10::optional<Tensor> w_t, c10::optional<Tensor> bn_x,
                c10::optional<Tensor> bn_red, c10::optional<Tensor> aff,
                c10::optional<Tensor> w_flip) {
  if (is_f32(dy)) {
    TORCH_CHECK(!(aff.has_value() && aff->defined()), "fp32 conv_dgrad: no folded BN");
    return conv_dgrad_f32(dy, w, dx, sh, sw, ph, pw, dh, dw, accumulate, mask);
  }
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(w, torch::kBFloat16);
  CHECK_T(dx, torch::kBFloat16);
  ConvArgs a = conv_args(dx, w, dx.size(0), dx.size(1), dx.size(2), dx.size(3), w.size(0), w.size(1),
                         w.size(2), sh, sw, ph, pw, dh, dw, dy.size(1), dy.size(2));
  TORCH_CHECK(dx.size(3) == w.size(3) && dy.size(3) == w.size(0), "shape mismatch");
  a.dy = BF(dy); a.w = BF(w); a.out = dx.data_ptr();
  a.dy_bytes = nbytes32(dy); a.w_bytes = nbytes32(w); a.out_bytes = nbytes32(dx);
  a.M = a.N * a.H * a.W; a.Ng = a.C; a.Kg = a.R * a.S * a.K; a.ldc = a.C; a.relu = 0;
  a.beta = accumulate ? 1 : 0;
  a.mask = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == torch::kUInt8 && mask->is_contiguous() &&
                mask->numel() * 8 == dx.numel() && dx.size(3) % 64 == 0,
                "conv_dgrad mask: uint8 [numel(dx)/8], C % 64 == 0");
    a.mask = (const uint8_t*)mask->data_ptr();
  }
  a.w_t = nullptr;
  if (w_t.has_value() && w_t->defined()) {  // [R,S,C,K] copy of w (the LDS-DMA kernel's KC path)
    CHECK_T(*w_t, torch::kBFloat16);
    TORCH_CHECK(w_t->dim() == 4 && w_t->size(0) == a.R && w_t->size(1) == a.S &&
                w_t->size(2) == a.C && w_t->size(3) == a.K && w_t->is_contiguous(),
                "conv_dgrad w_t must be the [R,S,C,K] transpose of w");
    a.w_t = BF(*w_t);
  }
  a.w_flip = nullptr;
  a.w_flip_bytes = 0;
  if (w_flip.has_value() && w_flip->defined()) {
    CHECK_T(*w_flip, torch::kBFloat16);
    if (sh == 1 && sw == 1) {
      TORCH_CHECK(w_flip->dim() == 4 && w_flip->size(0) == a.C && w_flip->size(1) == a.R &&
                  w_flip->size(2) == a.S && w_flip->size(3) == a.K && w_flip->is_contiguous(),
                  "conv_dgrad w_flip must be the [C,R,S,K] flipped transpose of w");
    } else {  // strided: the per-parity-class flipped sub-filters, concatenated (ops/conv.py)
      TORCH_CHECK(w_flip->is_contiguous() && w_flip->numel() == a.C * a.R * a.S * a.K,
                  "conv_dgrad w_flip (strided): the class sub-filters, C*R*S*K elements");
    }
    a.w_flip = BF(*w_flip);
    a.w_flip_bytes = nbytes32(*w_flip);
  }
  a.stats = nullptr;
  a.bn_x = nullptr;
  if (bn_x.has_value() && bn_x->defined()) {
    TORCH_CHECK(bn_red.has_value() && bn_red->defined(), "conv_dgrad: bn_x needs bn_red");
    CHECK_T(*bn_x, torch::kBFloat16);
    CHECK_T(*bn_red, torch::kFloat32);
    TORCH_CHECK(bn_x->sizes() == dx.sizes() && bn_red->numel() == 2 * dx.size(3) &&
                bn_red->is_contiguous(), "conv_dgrad bn_x: shape of dx, bn_red fp32 [2, C]");
    // deterministic mode: no fused BN-backward sums (epilogue atomics); the BN reduces itself
    if (!deterministic()) {
      a.bn_x = BF(*bn_x);
      a.stats = bn_red->data_ptr<float>();
      set_conv_aff(a, aff, a.C, "conv_dgrad");
      TORCH_CHECK(!a.aff || (!a.mask && !accumulate), "conv_dgrad aff: no bit mask / join");
    }
  } else {
    TORCH_CHECK(!(aff.has_value() && aff->defined()), "conv_dgrad aff needs bn_x / bn_red");
  }
  if (a.M == 0) return false;
  return conv_dgrad_launch(a, stream());
}

// fp8 dgrad: dy8 e5m2 [N,Ho,Wo,K], w8t e4m3 transposed weights [R,S,C,K] (ops/fp8.py), dx bf16
// [N,H,W,C]; per-tensor scales sdy, sw (device scalars); join accumulate / ReLU mask as conv_dgrad
// bn_x / bn_red (optional): the BN-backward statistics (Σg, Σg·x) of the stored dx in the epilogue,
// as conv_dgrad (a join: stride 1 only); returns whether they were fused
bool conv_dgrad_fp8(Tensor dy8, Tensor w8t, Tensor dx, Tensor sdy, Tensor sw_, int64_t sh, int64_t sw,
                    int64_t ph, int64_t pw, int64_t dh, int64_t dw, bool accumulate,
                    c10::optional<Tensor> mask, c10::optional<Tensor> bn_x,
                    c10::optional<Tensor> bn_red, c10::optional<Tensor> w_flip) {
  TORCH_CHECK(dy8.is_cuda() && w8t.is_cuda() && dy8.element_size() == 1 && w8t.element_size() == 1,
              "fp8 operands expected");
  TORCH_CHECK(dy8.is_contiguous() && w8t.is_contiguous(), "contiguous operands expected");
  CHECK_T(dx, torch::kBFloat16);
  CHECK_T(sdy, torch::kFloat32);
  CHECK_T(sw_, torch::kFloat32);
  // logical weight shape K×R×S×C from the transposed copy R×S×C×K
  const int64_t K = w8t.size(3), R = w8t.size(0), S = w8t.size(1), C = w8t.size(2);
  TORCH_CHECK(dx.size(3) == C && dy8.size(3) == K && K % 128 == 0 && C % 8 == 0,
              "fp8 dgrad shapes: K % 128 == 0, C % 8 == 0");
  ConvArgs a = conv_args(dx, dx, dx.size(0), dx.size(1), dx.size(2), C, K, R, S, sh, sw, ph, pw, dh,
                         dw, dy8.size(1), dy8.size(2));
  a.dy = (const bf16_t*)dy8.data_ptr(); a.w = (const bf16_t*)w8t.data_ptr(); a.out = dx.data_ptr();
  TORCH_CHECK(dy8.numel() < (1LL << 32) && w8t.numel() < (1LL << 32), "tensor too large");
  a.dy_bytes = (uint32_t)dy8.numel(); a.w_bytes = (uint32_t)w8t.numel(); a.out_bytes = nbytes32(dx);
  a.M = a.N * a.H * a.W; a.Ng = a.C; a.Kg = a.R * a.S * a.K; a.ldc = a.C; a.relu = 0;
  a.beta = accumulate ? 1 : 0;
  a.fp8 = 1;
  a.scale_x = sdy.data_ptr<float>(); a.scale_w = sw_.data_ptr<float>();
  a.mask = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == torch::kUInt8 && mask->is_contiguous() &&
                mask->numel() * 8 == dx.numel() && dx.size(3) % 64 == 0,
                "conv_dgrad mask: uint8 [numel(dx)/8], C % 64 == 0");
    a.mask = (const uint8_t*)mask->data_ptr();
  }
  // w_flip (optional, stride 1): the e4m3 flipped filter [C, R, S, K] — the route row
  // dgrad.asfwd.fp8 runs the dgrad as the forward conv of dy with it (for a 1x1 conv it is w8t)
  a.w_flip = nullptr;
  a.w_flip_bytes = 0;
  if (w_flip.has_value() && w_flip->defined()) {
    TORCH_CHECK(w_flip->is_cuda() && w_flip->element_size() == 1 && w_flip->is_contiguous() &&
                    w_flip->numel() == w8t.numel() && sh == 1 && sw == 1,
                "conv_dgrad_fp8 w_flip: the e4m3 [C,R,S,K] flipped filter, stride 1");
    a.w_flip = (const bf16_t*)w_flip->data_ptr();
    a.w_flip_bytes = (uint32_t)w_flip->numel();
  }
  a.stats = nullptr;
  a.bn_x = nullptr;
  if (bn_x.has_value() && bn_x->defined()) {
    TORCH_CHECK(bn_red.has_value() && bn_red->defined(), "conv_dgrad_fp8: bn_x needs bn_red");
    CHECK_T(*bn_x, torch::kBFloat16);
    CHECK_T(*bn_red, torch::kFloat32);
    TORCH_CHECK(bn_x->sizes() == dx.sizes() && bn_red->numel() == 2 * dx.size(3) &&
                bn_red->is_contiguous(), "conv_dgrad_fp8 bn_x: shape of dx, bn_red fp32 [2, C]");
    if (!deterministic()) {  // (deterministic mode: the BN reduces itself, no epilogue atomics)
      a.bn_x = BF(*bn_x);
      a.stats = bn_red->data_ptr<float>();
    }
  }
  if (a.M == 0) return false;
  try {
    return conv_dgrad_launch(a, stream());
  } catch (const std::exception& e) {
    TORCH_CHECK(false, e.what());
  }
  return false;
}

// aff (optional): x is the pre-BN tensor of a folded BN + ReLU (dW = dyᵀ · relu(aff[0]·x + aff[1]))
void conv_wgrad(Tensor dy, Tensor x, Tensor out, c10::optional<Tensor> bias_grad, int64_t sh,
                int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw, bool accumulate,
                c10::optional<Tensor> aff) {
  if (is_f32(dy)) {
    TORCH_CHECK(!(aff.has_value() && aff->defined()), "fp32 conv_wgrad: no folded BN");
    return conv_wgrad_f32(dy, x, out, bias_grad, sh, sw, ph, pw, dh, dw, accumulate);
  }
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(out, torch::kFloat32);
  TORCH_CHECK(out.dim() == 4, "dW must be KRSC");
  ConvArgs a = conv_args(x, out, x.size(0), x.size(1), x.size(2), x.size(3), out.size(0),
                         out.size(1), out.size(2), sh, sw, ph, pw, dh, dw, dy.size(1), dy.size(2));
  TORCH_CHECK(out.size(3) == a.C && dy.size(3) == a.K && dy.size(0) == a.N, "shape mismatch");
  a.dy = BF(dy); a.x = BF(x);
  a.dy_bytes = nbytes32(dy); a.x_bytes = nbytes32(x);
  a.M = a.K; a.Ng = a.R * a.S * a.C; a.Kg = a.N * a.Ho * a.Wo;
  set_conv_aff(a, aff, a.C, "conv_wgrad");
  if (a.aff) TORCH_CHECK(a.K % 8 == 0, "conv_wgrad aff: K % 8 == 0");
  WgradPlan plan;
  conv_wgrad_plan(a, &plan);
  a.kps = plan.kps;
  auto ws = torch::empty({(int64_t)plan.splits * a.M * a.Ng}, out.options());
  a.out = ws.data_ptr();
  a.out_bytes = nbytes32(ws);
  auto st = stream();
  conv_wgrad_launch(a, plan, out.data_ptr<float>(), accumulate, st);
  if (bias_grad.has_value() && bias_grad->defined()) {
    CHECK_T((*bias_grad), torch::kFloat32);
    TORCH_CHECK(bias_grad->numel() == a.K, "bias_grad must have K elements");
    auto part = torch::empty({(int64_t)colsum_blocks((long)a.Kg, a.K) * a.K}, out.options());
    colsum_launch(BF(dy), bias_grad->data_ptr<float>(), part.data_ptr<float>(), (long)a.Kg, a.K,
                  false, st);
  }
}

// fp8 weight gradient: dy8 e5m2 [N,Ho,Wo,K], x8 e4m3 [N,H,W,C] (1-byte tensors), per-tensor
// device scales sdy / sx; dW fp32 [K,R,S,C] (accumulate: +=).  C % 16, K % 16 (a 16-B chunk never
// crosses a filter tap)
void conv_wgrad_fp8(Tensor dy8, Tensor x8, Tensor out, Tensor sdy, Tensor sx, int64_t sh, int64_t sw,
                    int64_t ph, int64_t pw, int64_t dh, int64_t dw, bool accumulate) {
  TORCH_CHECK(dy8.is_cuda() && x8.is_cuda() && dy8.element_size() == 1 && x8.element_size() == 1 &&
              dy8.is_contiguous() && x8.is_contiguous(), "fp8 operands expected");
  CHECK_T(out, torch::kFloat32);
  CHECK_T(sdy, torch::kFloat32);
  CHECK_T(sx, torch::kFloat32);
  TORCH_CHECK(out.dim() == 4 && out.is_contiguous(), "dW must be contiguous KRSC");
  ConvArgs a = conv_args(x8, out, x8.size(0), x8.size(1), x8.size(2), x8.size(3), out.size(0),
                         out.size(1), out.size(2), sh, sw, ph, pw, dh, dw, dy8.size(1), dy8.size(2));
  TORCH_CHECK(out.size(3) == a.C && dy8.size(3) == a.K && dy8.size(0) == a.N && a.C % 16 == 0 &&
              a.K % 16 == 0, "fp8 weight gradient shapes: C % 16 == 0, K % 16 == 0");
  TORCH_CHECK(x8.numel() < (1LL << 32) && dy8.numel() < (1LL << 32), "tensor too large");
  a.dy = (const bf16_t*)dy8.data_ptr(); a.x = (const bf16_t*)x8.data_ptr();
  a.dy_bytes = (uint32_t)dy8.numel(); a.x_bytes = (uint32_t)x8.numel();
  a.M = a.K; a.Ng = a.R * a.S * a.C; a.Kg = a.N * a.Ho * a.Wo;
  a.fp8 = 1;
  a.scale_x = sdy.data_ptr<float>(); a.scale_w = sx.data_ptr<float>();
  if (a.Kg == 0) {
    if (!accumulate) out.zero_();
    return;
  }
  WgradPlan plan;
  try {
    conv_wgrad_plan(a, &plan);
  } catch (const std::exception& e) {
    TORCH_CHECK(false, e.what());
  }
  a.kps = plan.kps;
  auto ws = torch::empty({(int64_t)plan.splits * a.M * a.Ng}, out.options());
  a.out = ws.data_ptr();
  a.out_bytes = nbytes32(ws);
  conv_wgrad_launch(a, plan, out.data_ptr<float>(), accumulate, stream());
}

// ------------------------------------------------------------------------------------------- bn
void bn_stats(Tensor x, Tensor stats) {
  if (is_f32(x)) {
    CHECK_T(x, torch::kFloat32);
    CHECK_T(stats, torch::kFloat32);
    check_c4(x.size(-1), "bn_stats");
    bn_stats_f32_launch(F32(x), F32(stats), x.numel() / x.size(-1), x.size(-1), stream());
    return;
  }
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(stats, torch::kFloat32);
  const int64_t C = x.size(-1);
  bn_stats_launch(BF(x), stats.data_ptr<float>(), x.numel() / C, C, stream());
}

void bn_finalize(c10::optional<Tensor> stats, Tensor coef, c10::optional<Tensor> gamma, Tensor beta,
                 Tensor rmean, Tensor rvar, double count, double decay, double eps, bool training) {
  CHECK_T(coef, torch::kFloat32);
  CHECK_T(beta, torch::kFloat32);
  CHECK_T(rmean, torch::kFloat32);
  CHECK_T(rvar, torch::kFloat32);
  TORCH_CHECK(!training || optf(stats) != nullptr, "training BN needs stats");
  // beta may be the channel-padded view (physical C); the moving statistics cover the logical
  // channels only
  TORCH_CHECK(rmean.numel() == rvar.numel() && rmean.numel() <= beta.numel(), "bn_finalize shapes");
  TORCH_CHECK(coef.numel() >= 4 * beta.numel(), "bn_finalize coef size");
  if (gamma.has_value() && gamma->defined())
    TORCH_CHECK(gamma->numel() == beta.numel(), "bn_finalize gamma / beta size");
  bn_finalize_launch(optf(stats), coef.data_ptr<float>(), optf(gamma), beta.data_ptr<float>(),
                     rmean.data_ptr<float>(), rvar.data_ptr<float>(), beta.numel(),
                     (int)rmean.numel(), (float)count, (float)decay, (float)eps, training,
                     stream());
}

// fp8 side output (delayed scaling): amax_ring is fp32[3, AMAX_SLOT]; slot `phase` holds the previous
// step's |y|max (scale source), slot phase+1 accumulates this step's, slot phase+2 is cleared
// for the next step — no separate memset launch.
// training BN folded into its 1×1 consumer conv (ops/bnfold.py): W' = W·diag(coef[0]) and
// bias = W·coef[1] (+ bias_in) in one launch
void bn_fold_weight(Tensor w, Tensor coef, Tensor wout, c10::optional<Tensor> bias_in,
                    Tensor bias_out) {
  TORCH_CHECK(w.is_cuda() && w.is_contiguous() && wout.is_contiguous() &&
                  w.scalar_type() == wout.scalar_type() && w.numel() == wout.numel(),
              "bn_fold_weight: w / wout");
  const bool bf16 = w.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf16 || w.scalar_type() == torch::kFloat32, "bn_fold_weight: bf16 or fp32 weight");
  CHECK_T(coef, torch::kFloat32);
  CHECK_T(bias_out, torch::kFloat32);
  const int64_t K = w.size(0), C = w.size(-1);
  TORCH_CHECK(w.numel() == K * C, "bn_fold_weight: a 1x1 weight [K, 1, 1, C]");
  TORCH_CHECK(coef.dim() == 2 && coef.size(0) >= 2 && coef.size(1) >= C, "bn_fold_weight: coef");
  TORCH_CHECK(bias_out.numel() == K, "bn_fold_weight: bias_out [K]");
  const float* bi = nullptr;
  if (bias_in.has_value() && bias_in->defined()) {
    CHECK_T(*bias_in, torch::kFloat32);
    TORCH_CHECK(bias_in->numel() == K, "bn_fold_weight: bias_in [K]");
    bi = bias_in->data_ptr<float>();
  }
  bn_fold_weight_launch(w.data_ptr(), bf16, coef.data_ptr<float>(), (int)K, (int)C,
                        (int)coef.size(1), wout.data_ptr(), bi, bias_out.data_ptr<float>(),
                        stream());
}

// dw[k][c] *= a[c] (fp32, in place)
void scale_cols(Tensor dw, Tensor a) {
  CHECK_T(dw, torch::kFloat32);
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == torch::kFloat32 && a.stride(-1) == 1,
              "scale_cols: a fp32 HIP vector");
  const int64_t C = dw.size(-1);
  TORCH_CHECK(a.numel() >= C, "scale_cols: a shorter than the columns");
  scale_cols_launch(dw.data_ptr<float>(), a.data_ptr<float>(), dw.numel(), (int)C, stream());
}

void bn_apply(Tensor x, Tensor coef, c10::optional<Tensor> res, Tensor y, bool relu,
              c10::optional<Tensor> y8, c10::optional<Tensor> amax_ring, int64_t phase,
              c10::optional<Tensor> scale_out, c10::optional<Tensor> mask, bool store_y) {
  if (is_f32(x)) {
    CHECK_T(x, torch::kFloat32);
    CHECK_T(coef, torch::kFloat32);
    TORCH_CHECK(!(y8.has_value() && y8->defined()) && !(amax_ring.has_value() && amax_ring->defined()) &&
                    !(mask.has_value() && mask->defined()),
                "fp32 bn_apply: no fp8 side output / ReLU bit mask");
    const int64_t C = x.size(-1);
    check_c4(C, "bn_apply");
    const int64_t ldy = nhwc_ld_f32(y, "bn_apply y");
    TORCH_CHECK(y.numel() == x.numel(), "bn_apply: y and x sizes");
    bn_apply_f32_launch(F32(x), F32(coef), opt_f32_like(res, x, "bn_apply res"), F32(y),
                        x.numel() / C, C, relu, ldy, stream());
    return;
  }
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(coef, torch::kFloat32);
  const int64_t C = x.size(-1);
  // y may be a channel slice of a wider NHWC buffer (concat-free ASPP / decoder)
  const int64_t ldy = bn_vec_ld(y, C, "bn_apply y");
  TORCH_CHECK(y.numel() == x.numel(), "bn_apply: y and x sizes");
  uint8_t* y8p = nullptr;
  float *prev = nullptr, *out = nullptr, *zero = nullptr;
  if (amax_ring.has_value() && amax_ring->defined()) {
    TORCH_CHECK(C % 8 == 0, "fp8 side output needs C % 8 == 0");
    CHECK_T(*amax_ring, torch::kFloat32);
    TORCH_CHECK(amax_ring->numel() == 3 * AMAX_SLOT && phase >= 0 && phase < 3,
                "amax_ring: fp32[3, AMAX_SLOT], phase 0..2");
    float* r = amax_ring->data_ptr<float>();
    prev = r + phase * AMAX_SLOT;
    out = r + (phase + 1) % 3 * AMAX_SLOT;
    zero = r + (phase + 2) % 3 * AMAX_SLOT;
    if (y8.has_value() && y8->defined()) {
      TORCH_CHECK(y8->element_size() == 1 && y8->numel() == x.numel() && y8->is_contiguous());
      y8p = (uint8_t*)y8->data_ptr();
    }
  }
  uint8_t* maskp = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(C % 8 == 0 && mask->is_cuda() && mask->element_size() == 1 &&
                mask->is_contiguous() && mask->numel() * 8 == x.numel(),
                "relu bit mask: uint8 [numel/8], C % 8 == 0");
    maskp = (uint8_t*)mask->data_ptr();
  }
  // store_y = false: only the e4m3 copy (and mask / amax) — an fp8-only BN output whose every
  // consumer reads the e4m3 tensor (ops/bn.py, models.enable_fp8)
  TORCH_CHECK(store_y || (y8p != nullptr && C % 8 == 0), "bn_apply store_y=False needs the e4m3 copy");
  bn_apply_launch(BF(x), coef.data_ptr<float>(), optb(res), store_y ? BFW(y) : nullptr,
                  x.numel() / C, C, relu, stream(), y8p, prev, optfw(scale_out), out, zero, maskp,
                  ldy);
}

// relu mode 3: `y` is the uint8 bit mask bn_apply wrote (vector kernels only: C % 8 == 0 and
// C / 8 <= 256), passed through the y pointer slot
const bf16_t* mask_or_y(const c10::optional<Tensor>& y, const Tensor& x, int64_t relu) {
  if (relu != 3) return optb(y);
  const int64_t C = x.size(-1);
  TORCH_CHECK(y.has_value() && y->defined() && y->is_cuda() && y->element_size() == 1 &&
              y->is_contiguous() && y->numel() * 8 == x.numel() && C % 8 == 0 && C <= 2048,
              "relu mask mode 3 needs the uint8 bit mask and C % 8 == 0, C <= 2048");
  return (const bf16_t*)y->data_ptr();
}

void bn_bwd_reduce(Tensor dy, c10::optional<Tensor> y, Tensor x, Tensor coef, Tensor red, int64_t relu) {
  if (is_f32(x)) {
    CHECK_T(red, torch::kFloat32);
    CHECK_T(coef, torch::kFloat32);
    const int64_t C = x.size(-1);
    check_c4(C, "bn_bwd_reduce");
    TORCH_CHECK(relu >= 0 && relu <= 2, "fp32 bn_bwd_reduce: relu mode 0, 1 (y) or 2 (x)");
    TORCH_CHECK(relu != 1 || (y.has_value() && y->defined()), "relu mask mode 1 needs y");
    const int64_t ldd = nhwc_ld_f32(dy, "bn_bwd_reduce dy");
    TORCH_CHECK(dy.numel() == x.numel() && x.is_contiguous(), "bn_bwd_reduce: dy and x sizes");
    bn_bwd_reduce_f32_launch(F32(dy), relu == 1 ? opt_f32_like(y, x, "bn_bwd_reduce y") : nullptr,
                             F32(x), F32(coef), F32(red), x.numel() / C, C, (int)relu, ldd,
                             stream());
    return;
  }
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(red, torch::kFloat32);
  const int64_t C = x.size(-1);
  const int64_t ldd = bn_vec_ld(dy, C, "bn_bwd_reduce dy");  // dy: contiguous or channel slice
  TORCH_CHECK(dy.numel() == x.numel(), "bn_bwd_reduce: dy and x sizes");
  TORCH_CHECK(relu != 1 || (y.has_value() && y->defined()), "relu mask mode 1 needs y");
  bn_bwd_reduce_launch(BF(dy), mask_or_y(y, x, relu), BF(x), coef.data_ptr<float>(),
                       red.data_ptr<float>(), x.numel() / C, C, (int)relu, stream(), ldd);
}

bool bn_bwd_reduce2(Tensor dy, Tensor x, Tensor x2, Tensor coef, Tensor red, Tensor red2) {
  if (is_f32(x)) return false;  // fp32: each BN reduces itself
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(x2, torch::kBFloat16);
  CHECK_T(red, torch::kFloat32);
  CHECK_T(red2, torch::kFloat32);
  const int64_t C = x.size(-1);
  TORCH_CHECK(x2.sizes() == x.sizes() && dy.sizes() == x.sizes() && red.numel() == 2 * C &&
              red2.numel() == 2 * C, "bn_bwd_reduce2: dy, x, x2 of one shape, red / red2 [2, C]");
  return bn_bwd_reduce2_launch(BF(dy), BF(x), BF(x2), coef.data_ptr<float>(), red.data_ptr<float>(),
                               red2.data_ptr<float>(), x.numel() / C, C, stream());
}

void bn_bwd_apply(Tensor dy, c10::optional<Tensor> y, Tensor x, Tensor coef, Tensor red,
                  c10::optional<Tensor> gamma, Tensor dx, c10::optional<Tensor> dres,
                  c10::optional<Tensor> dgamma, c10::optional<Tensor> dbeta, double count,
                  int64_t relu, c10::optional<Tensor> dx8, c10::optional<Tensor> amax_ring,
                  int64_t phase, c10::optional<Tensor> scale_out, bool red_raw,
                  c10::optional<Tensor> dadd, bool store_dx) {
  if (is_f32(x)) {
    TORCH_CHECK(store_dx, "fp32 bn_bwd_apply: dx is always stored");
    CHECK_T(x, torch::kFloat32);
    CHECK_T(dx, torch::kFloat32);
    CHECK_T(coef, torch::kFloat32);
    CHECK_T(red, torch::kFloat32);
    TORCH_CHECK(!red_raw && !(amax_ring.has_value() && amax_ring->defined()),
                "fp32 bn_bwd_apply: no fused-dgrad statistics / fp8 side output");
    TORCH_CHECK(relu >= 0 && relu <= 2, "fp32 bn_bwd_apply: relu mode 0, 1 (y) or 2 (x)");
    const int64_t C = x.size(-1);
    check_c4(C, "bn_bwd_apply");
    const int64_t ldd = nhwc_ld_f32(dy, "bn_bwd_apply dy");
    TORCH_CHECK(dy.numel() == x.numel() && dx.numel() == x.numel(), "bn_bwd_apply: dy, x, dx sizes");
    float* dresp = nullptr;
    if (dres.has_value() && dres->defined()) {
      CHECK_T(*dres, torch::kFloat32);
      TORCH_CHECK(dres->numel() == x.numel(), "dres size");
      dresp = F32(*dres);
    }
    bn_bwd_apply_f32_launch(F32(dy), relu == 1 ? opt_f32_like(y, x, "bn_bwd_apply y") : nullptr,
                            F32(x), F32(coef), F32(red), optf(gamma), F32(dx), dresp, optfw(dgamma),
                            optfw(dbeta), opt_f32_like(dadd, x, "bn_bwd_apply dadd"), x.numel() / C,
                            C, (float)count, (int)relu, ldd, stream());
    return;
  }
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(dx, torch::kBFloat16);
  const bf16_t* addp = nullptr;
  if (dadd.has_value() && dadd->defined()) {
    CHECK_T(*dadd, torch::kBFloat16);
    TORCH_CHECK(dadd->sizes() == dx.sizes() && x.size(-1) % 8 == 0,
                "bn_bwd_apply dadd: shaped like dx, C % 8 == 0");
    addp = BF(*dadd);
  }
  const int64_t C = x.size(-1);
  const int64_t ldd = bn_vec_ld(dy, C, "bn_bwd_apply dy");  // dy: contiguous or channel slice
  TORCH_CHECK(dy.numel() == x.numel() && dx.numel() == x.numel(), "bn_bwd_apply: dy, x, dx sizes");
  uint8_t* d8 = nullptr;
  float *prev = nullptr, *out = nullptr, *zero = nullptr;
  if (amax_ring.has_value() && amax_ring->defined()) {  // e5m2 side output (fp8 dgrad)
    TORCH_CHECK(C % 8 == 0, "fp8 side output needs C % 8 == 0");
    prev = ring_slot(*amax_ring, phase);
    out = ring_slot(*amax_ring, phase + 1);
    zero = ring_slot(*amax_ring, phase + 2);
    if (dx8.has_value() && dx8->defined()) {
      TORCH_CHECK(dx8->element_size() == 1 && dx8->numel() == dx.numel() && dx8->is_contiguous());
      d8 = (uint8_t*)dx8->data_ptr();
    }
  }
  // store_dx == false: only the e5m2 copy is written (every reader of this gradient is an fp8
  // dgrad / weight gradient, models.enable_fp8 fp8_bwd_only); dx stays an unwritten placeholder
  TORCH_CHECK(store_dx || (d8 != nullptr && C % 8 == 0),
              "bn_bwd_apply: store_dx=False needs the e5m2 side output (C % 8 == 0)");
  bn_bwd_apply_launch(BF(dy), mask_or_y(y, x, relu), BF(x), coef.data_ptr<float>(), red.data_ptr<float>(),
                      optf(gamma), store_dx ? BFW(dx) : nullptr, optbw(dres), optfw(dgamma),
                      optfw(dbeta), x.numel() / C,
                      C, (float)count, (int)relu, stream(), d8, prev, optfw(scale_out), out, zero,
                      red_raw, ldd, addp);
}

// ---------------------------------------------------------------------------------- elementwise
void row_pack(Tensor x, Tensor t, int64_t creal, int64_t S, int64_t sw, int64_t pl) {
  if (is_f32(x)) {
    CHECK_T(x, torch::kFloat32);
    CHECK_T(t, torch::kFloat32);
    TORCH_CHECK(x.dim() == 4 && t.dim() == 4 && t.size(0) == x.size(0) && t.size(1) == x.size(1) &&
                t.size(3) >= S * creal && creal <= x.size(3), "row_pack: x [N,H,W,Cx], t [N,H,Wo,Cp]");
    row_pack_f32_launch(F32(x), F32(t), x.size(0), x.size(1), x.size(2), x.size(3), creal, S, sw, pl,
                        t.size(2), t.size(3), stream());
    return;
  }
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(t, torch::kBFloat16);
  TORCH_CHECK(x.dim() == 4 && t.dim() == 4 && t.size(0) == x.size(0) && t.size(1) == x.size(1) &&
              t.size(3) % 8 == 0 && t.size(3) >= S * creal && creal <= x.size(3),
              "row_pack: x [N,H,W,Cx], t [N,H,Wo,Cp] with Cp % 8 == 0, Cp >= S*creal");
  row_pack_launch(BF(x), BFW(t), x.size(0), x.size(1), x.size(2), x.size(3), creal, S, sw, pl,
                  t.size(2), t.size(3), stream());
}

void relu_bwd(Tensor dy, Tensor y, Tensor dx) {
  if (is_f32(dy)) {
    CHECK_T(dy, torch::kFloat32);
    CHECK_T(y, torch::kFloat32);
    CHECK_T(dx, torch::kFloat32);
    TORCH_CHECK(dy.numel() % 4 == 0 && y.numel() == dy.numel() && dx.numel() == dy.numel());
    relu_bwd_f32_launch(F32(dy), F32(y), F32(dx), dy.numel(), stream());
    return;
  }
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(y, torch::kBFloat16);
  CHECK_T(dx, torch::kBFloat16);
  relu_bwd_launch(BF(dy), BF(y), BFW(dx), dy.numel(), stream());
}

void add_act(Tensor a, c10::optional<Tensor> b, Tensor y, bool relu) {
  if (is_f32(a)) {
    CHECK_T(a, torch::kFloat32);
    CHECK_T(y, torch::kFloat32);
    TORCH_CHECK(a.numel() % 4 == 0 && y.numel() == a.numel());
    add_act_f32_launch(F32(a), opt_f32_like(b, a, "add_act b"), F32(y), a.numel(), relu, stream());
    return;
  }
  CHECK_T(a, torch::kBFloat16);
  CHECK_T(y, torch::kBFloat16);
  add_act_launch(BF(a), optb(b), BFW(y), a.numel(), relu, stream());
}

void scale_by_scalar(Tensor x, Tensor s, Tensor y) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && y.is_contiguous());
  const bool bf = x.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf || x.scalar_type() == torch::kFloat32);
  scale_by_scalar_launch(x.data_ptr(), s.data_ptr<float>(), y.data_ptr(), x.numel(), bf, stream());
}

// dtype conversion between a flat fp32 and a flat bf16 buffer (either direction)
void convert(Tensor x, Tensor y) {
  TORCH_CHECK(x.is_cuda() && y.is_cuda() && x.is_contiguous() && y.is_contiguous() &&
              x.numel() == y.numel(), "convert: contiguous GPU tensors of equal numel");
  const bool xb = x.scalar_type() == torch::kBFloat16;
  TORCH_CHECK((xb && y.scalar_type() == torch::kFloat32) ||
              (x.scalar_type() == torch::kFloat32 && y.scalar_type() == torch::kBFloat16),
              "convert: fp32 <-> bf16");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0) &&
              (reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0), "convert: 16-B aligned");
  convert_launch(x.data_ptr(), xb, y.data_ptr(), x.numel(), stream());
}

void sigmoid_threshold(Tensor x, Tensor prob, Tensor pred, double thr) {
  const bool bf = x.scalar_type() == torch::kBFloat16;
  sigmoid_threshold_launch(x.data_ptr(), bf, prob.data_ptr<float>(), pred.data_ptr<float>(),
                           x.numel(), (float)thr, stream());
}

// -------------------------------------------------------------------------------------- pooling
void maxpool_fwd(Tensor x, Tensor y, Tensor idx, int64_t k, int64_t s, int64_t pt, int64_t pl) {
  if (is_f32(x)) {
    CHECK_T(x, torch::kFloat32);
    CHECK_T(y, torch::kFloat32);
    CHECK_T(idx, torch::kUInt8);
    TORCH_CHECK(k * k <= 255, "window too large for uint8 argmax");
    maxpool_fwd_launch(F32(x), F32(y), idx.data_ptr<uint8_t>(), x.size(0), x.size(1), x.size(2),
                       x.size(3), y.size(1), y.size(2), k, s, pt, pl, stream());
    return;
  }
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(y, torch::kBFloat16);
  CHECK_T(idx, torch::kUInt8);
  TORCH_CHECK(k * k <= 255, "window too large for uint8 argmax");
  maxpool_fwd_launch(BF(x), BFW(y), idx.data_ptr<uint8_t>(), x.size(0), x.size(1), x.size(2),
                     x.size(3), y.size(1), y.size(2), k, s, pt, pl, stream());
}

void maxpool_bwd(Tensor dy, Tensor idx, Tensor dx, int64_t k, int64_t s, int64_t pt, int64_t pl) {
  if (is_f32(dy)) {
    CHECK_T(dy, torch::kFloat32);
    CHECK_T(dx, torch::kFloat32);
    maxpool_bwd_launch(F32(dy), idx.data_ptr<uint8_t>(), F32(dx), dx.size(0), dx.size(1), dx.size(2),
                       dx.size(3), dy.size(1), dy.size(2), k, s, pt, pl, stream());
    return;
  }
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(dx, torch::kBFloat16);
  maxpool_bwd_launch(BF(dy), idx.data_ptr<uint8_t>(), BFW(dx), dx.size(0), dx.size(1), dx.size(2),
                     dx.size(3), dy.size(1), dy.size(2), k, s, pt, pl, stream());
}

// maxpool backward with the producing BN's ReLU mask applied and its backward sums (Σg, Σg·x)
// accumulated into bn_red fp32 [2, C] (zeroed by the caller); returns false (nothing launched)
// when the channel count does not fit the kernel
bool maxpool_bwd_stats(Tensor dy, Tensor idx, Tensor dx, int64_t k, int64_t s, int64_t pt,
                       int64_t pl, Tensor bn_x, Tensor mask, Tensor bn_red) {
  if (is_f32(dy)) return false;  // fp32: no fused ReLU mask / BN statistics
  if (deterministic()) return false;  // epilogue atomics: the BN reduces itself (det.hip)
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(dx, torch::kBFloat16);
  CHECK_T(bn_x, torch::kBFloat16);
  CHECK_T(bn_red, torch::kFloat32);
  TORCH_CHECK(bn_x.sizes() == dx.sizes() && mask.is_cuda() && mask.scalar_type() == torch::kUInt8 &&
              mask.numel() * 8 == dx.numel() && bn_red.numel() == 2 * dx.size(3),
              "maxpool_bwd_stats: bn_x like dx, 1-bit mask, bn_red [2, C]");
  return maxpool_bwd_stats_launch(BF(dy), idx.data_ptr<uint8_t>(), BFW(dx), BF(bn_x),
                                  mask.data_ptr<uint8_t>(), bn_red.data_ptr<float>(), dx.size(0),
                                  dx.size(1), dx.size(2), dx.size(3), dy.size(1), dy.size(2), k, s,
                                  pt, pl, stream());
}

// the ResNet stem's training BN + ReLU + max-pool in one pass (pool.hip bn_maxpool_fwd_kernel):
// y = maxpool(relu(x·coef[0] + coef[1])) with the ReLU bit of each window maximum in idx bit 7;
// false: not eligible (C % 8), nothing launched
bool bn_maxpool_fwd(Tensor x, Tensor coef, Tensor y, Tensor idx, int64_t k, int64_t s, int64_t pt,
                    int64_t pl, c10::optional<Tensor> zarg) {
  const bool za = zarg.has_value() && zarg->defined();
  if (za) {
    CHECK_T((*zarg), torch::kBFloat16);
    TORCH_CHECK(zarg->sizes() == y.sizes() && zarg->is_contiguous(), "bn_maxpool_fwd: zarg like y");
  }
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(y, torch::kBFloat16);
  CHECK_T(idx, torch::kUInt8);
  CHECK_T(coef, torch::kFloat32);
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(3) == y.size(3) &&
                  idx.numel() == y.numel() && coef.numel() >= 2 * x.size(3) && k * k <= 127 &&
                  k >= 1 && s >= 1,
              "bn_maxpool_fwd: x [N,H,W,C], y / idx [N,Ho,Wo,C], coef [>=2, C], k*k < 128");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && idx.is_contiguous() && coef.is_contiguous(),
              "bn_maxpool_fwd: contiguous operands");
  return bn_maxpool_fwd_launch(BF(x), coef.data_ptr<float>(), BFW(y), idx.data_ptr<uint8_t>(),
                               za ? BFW((*zarg)) : nullptr, x.size(0), x.size(1), x.size(2),
                               x.size(3), y.size(1), y.size(2), k, s, pt, pl, stream());
}

// fused backward of bn_maxpool_fwd(zarg=…): dx of the BN input from the pool's dy in two passes
// (pool.hip maxpool_bn_sums_kernel + maxpool_bn_apply_kernel); red [2, C] zeroed by the caller
// receives (Σg, Σg·x); dgamma / dbeta [C] fp32 (optional) receive dγ, dβ.  False (nothing
// launched) in deterministic mode (the sums use fp32 atomics) or when C does not fit
bool maxpool_bn_bwd(Tensor dy, Tensor idx, Tensor zarg, Tensor x, Tensor coef, Tensor red,
                    c10::optional<Tensor> gamma, Tensor dx, c10::optional<Tensor> dgamma,
                    c10::optional<Tensor> dbeta, double count, int64_t k, int64_t s, int64_t pt,
                    int64_t pl) {
  if (deterministic()) return false;
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(zarg, torch::kBFloat16);
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(dx, torch::kBFloat16);
  CHECK_T(idx, torch::kUInt8);
  CHECK_T(coef, torch::kFloat32);
  CHECK_T(red, torch::kFloat32);
  const int64_t C = x.size(3);
  TORCH_CHECK(dy.dim() == 4 && x.dim() == 4 && dx.sizes() == x.sizes() && zarg.sizes() == dy.sizes() &&
                  idx.numel() == dy.numel() && dy.size(0) == x.size(0) && dy.size(3) == C &&
                  coef.numel() >= 4 * C && red.numel() == 2 * C,
              "maxpool_bn_bwd: dy / zarg / idx [N,Ho,Wo,C], x / dx [N,H,W,C], coef [4, C], red [2, C]");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dx.is_contiguous() && zarg.is_contiguous() &&
                  idx.is_contiguous() && coef.is_contiguous() && red.is_contiguous(),
              "maxpool_bn_bwd: contiguous operands");
  auto f32opt = [&](const c10::optional<Tensor>& t) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    CHECK_T((*t), torch::kFloat32);
    TORCH_CHECK(t->numel() >= C && t->is_contiguous(), "maxpool_bn_bwd: per-channel fp32 [C]");
    return t->data_ptr<float>();
  };
  return maxpool_bn_bwd_launch(BF(dy), idx.data_ptr<uint8_t>(), BF(zarg), BF(x),
                               coef.data_ptr<float>(), red.data_ptr<float>(), f32opt(gamma),
                               BFW(dx), f32opt(dgamma), f32opt(dbeta), x.size(0), x.size(1),
                               x.size(2), C, dy.size(1), dy.size(2), k, s, pt, pl,
                               (float)(1.0 / count), stream());
}

// backward of bn_maxpool_fwd: dx = the gathered dy where the window maximum was > 0 (idx bit 7);
// with bn_x / bn_red (and outside deterministic mode) also the BN-backward sums (Σg, Σg·x) into
// bn_red [2, C] (zeroed by the caller) — returns whether they were accumulated
bool maxpool_bwd_rb(Tensor dy, Tensor idx, Tensor dx, int64_t k, int64_t s, int64_t pt, int64_t pl,
                    c10::optional<Tensor> bn_x, c10::optional<Tensor> bn_red) {
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(dx, torch::kBFloat16);
  CHECK_T(idx, torch::kUInt8);
  TORCH_CHECK(dy.dim() == 4 && dx.dim() == 4 && dy.size(0) == dx.size(0) &&
                  dy.size(3) == dx.size(3) && dx.size(3) % 8 == 0 && idx.numel() == dy.numel() &&
                  dy.is_contiguous() && dx.is_contiguous() && idx.is_contiguous(),
              "maxpool_bwd_rb: dy / idx [N,Ho,Wo,C], dx [N,H,W,C], C % 8 == 0");
  const bool stats = bn_x.has_value() && bn_x->defined() && bn_red.has_value() &&
                     bn_red->defined() && !deterministic();
  if (stats) {
    CHECK_T((*bn_x), torch::kBFloat16);
    CHECK_T((*bn_red), torch::kFloat32);
    TORCH_CHECK(bn_x->sizes() == dx.sizes() && bn_x->is_contiguous() &&
                    bn_red->numel() == 2 * dx.size(3),
                "maxpool_bwd_rb: bn_x like dx, bn_red [2, C]");
    if (maxpool_bwd_stats_launch(BF(dy), idx.data_ptr<uint8_t>(), BFW(dx), BF((*bn_x)), nullptr,
                                 bn_red->data_ptr<float>(), dx.size(0), dx.size(1), dx.size(2),
                                 dx.size(3), dy.size(1), dy.size(2), k, s, pt, pl, stream()))
      return true;
  }
  maxpool_bwd_rb_launch(BF(dy), idx.data_ptr<uint8_t>(), BFW(dx), dx.size(0), dx.size(1),
                        dx.size(2), dx.size(3), dy.size(1), dy.size(2), k, s, pt, pl, stream());
  return false;
}

void avgpool_fwd(Tensor x, Tensor y) {
  if (is_f32(x)) {
    CHECK_T(x, torch::kFloat32);
    CHECK_T(y, torch::kFloat32);
    avgpool_fwd_launch(F32(x), F32(y), x.size(0), x.size(1) * x.size(2), x.size(3), stream());
    return;
  }
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(y, torch::kBFloat16);
  avgpool_fwd_launch(BF(x), BFW(y), x.size(0), x.size(1) * x.size(2), x.size(3), stream());
}

// dadd (optional, shaped like dx, may be dx itself; C % 8 == 0): dx = dy/HW + dadd
void avgpool_bwd(Tensor dy, Tensor dx, c10::optional<Tensor> dadd) {
  const bool has_add = dadd.has_value() && dadd->defined();
  if (has_add)
    TORCH_CHECK(dadd->sizes() == dx.sizes() && dadd->is_contiguous() &&
                    dadd->scalar_type() == dx.scalar_type() && dx.size(3) % 8 == 0,
                "avgpool_bwd dadd: shaped like dx, C % 8 == 0");
  if (is_f32(dy)) {
    CHECK_T(dy, torch::kFloat32);
    CHECK_T(dx, torch::kFloat32);
    avgpool_bwd_launch(F32(dy), F32(dx), dx.size(0), dx.size(1) * dx.size(2), dx.size(3), stream(),
                       has_add ? F32(*dadd) : nullptr);
    return;
  }
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(dx, torch::kBFloat16);
  avgpool_bwd_launch(BF(dy), BFW(dx), dx.size(0), dx.size(1) * dx.size(2), dx.size(3), stream(),
                     has_add ? BF(*dadd) : nullptr);
}

// --------------------------------------------------------------------------------------- losses
void softmax_xent(Tensor logits, Tensor labels, Tensor loss, Tensor grad, double smoothing) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2);
  const bool bf = logits.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == torch::kFloat32);
  TORCH_CHECK(labels.scalar_type() == torch::kInt64 && labels.is_contiguous());
  TORCH_CHECK(grad.scalar_type() == logits.scalar_type());
  softmax_xent_launch(logits.data_ptr(), bf, labels.data_ptr<int64_t>(), loss.data_ptr<float>(),
                      grad.data_ptr(), logits.size(0), logits.size(1), (float)smoothing, stream());
}

// logits [N, K] bf16 / fp32; labels (optional int64 [N]) with loss_sum / correct (fp32 [1],
// accumulated); probs (optional fp32 [N, K])
void softmax_eval(Tensor logits, c10::optional<Tensor> labels, c10::optional<Tensor> loss_sum,
                  c10::optional<Tensor> correct, c10::optional<Tensor> probs) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2, "softmax_eval logits");
  const bool bf = logits.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == torch::kFloat32, "softmax_eval: bf16 / fp32 logits");
  const int64_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    TORCH_CHECK(labels->scalar_type() == torch::kInt64 && labels->is_contiguous() &&
                labels->numel() == logits.size(0), "softmax_eval labels: int64 [N]");
    lab = labels->data_ptr<int64_t>();
  }
  float* p = optfw(probs);
  if (p) TORCH_CHECK(probs->numel() == logits.numel() && probs->is_contiguous(), "probs: fp32 [N, K]");
  if (logits.size(0) == 0) return;
  softmax_eval_launch(logits.data_ptr(), bf, lab, optfw(loss_sum), optfw(correct), p,
                      logits.size(0), logits.size(1), stream());
}

int label_kind(const Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kFloat32: return 0;
    case torch::kUInt8: return 1;
    case torch::kBool: return 1;
    case torch::kInt64: return 2;
    case torch::kBFloat16: return 3;
    case torch::kInt32: return 4;
    default: TORCH_CHECK(false, "unsupported label dtype");
  }
  return 0;
}

void lovasz_hinge(Tensor logits, Tensor labels, Tensor loss, Tensor grad) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && labels.is_contiguous());
  const bool bf = logits.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == torch::kFloat32);
  const int64_t B = logits.size(0), P = logits.numel() / B;
  TORCH_CHECK(P < (1 << 30), "lovasz: too many pixels per image");
  if (P <= 16384) {  // one workgroup per image, sort in LDS
    lovasz_hinge_launch(logits.data_ptr(), bf, labels.data_ptr(), label_kind(labels),
                        loss.data_ptr<float>(), grad.data_ptr<float>(), B, P, stream());
    return;
  }
  const int64_t Pp = lovasz_padded_len((int)P);
  auto opt = logits.options().dtype(torch::kFloat32);
  Tensor key = torch::empty({B, Pp}, opt), idx = torch::empty({B, Pp}, opt.dtype(torch::kInt32));
  lovasz_hinge_large_launch(logits.data_ptr(), bf, labels.data_ptr(), label_kind(labels),
                            loss.data_ptr<float>(), grad.data_ptr<float>(), key.data_ptr<float>(),
                            idx.data_ptr<int>(), B, P, stream());
}

void seg_metrics(Tensor labels, Tensor pred, Tensor score, Tensor acc, bool kaggle) {
  TORCH_CHECK(pred.scalar_type() == torch::kFloat32 && pred.is_contiguous());
  const int64_t B = pred.size(0), P = pred.numel() / B;
  seg_metrics_launch(labels.data_ptr(), label_kind(labels), pred.data_ptr<float>(),
                     score.data_ptr<float>(), acc.data_ptr<float>(), B, P, kaggle, stream());
}

// ----------------------------------------------------------------------------------- optimizers
void sgd_momentum(Tensor p, Tensor g, Tensor m, c10::optional<Tensor> lowp, Tensor flags, double lr,
                  double mu, double wd, double gs, bool nesterov, c10::optional<Tensor> lr_scale) {
  CHECK_T(p, torch::kFloat32);
  CHECK_T(g, torch::kFloat32);
  CHECK_T(m, torch::kFloat32);
  TORCH_CHECK(p.numel() % 64 == 0, "flat buffer must be 64-aligned");
  sgd_momentum_launch(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), optbw(lowp),
                      flags.data_ptr<uint8_t>(), p.numel(), lr, optf(lr_scale), mu, wd, gs,
                      nesterov, stream());
}

void adam(Tensor p, Tensor g, Tensor m, Tensor v, c10::optional<Tensor> lowp, Tensor flags,
          double lr_t, double b1, double b2, double eps, double wd, double gs,
          c10::optional<Tensor> lr_scale) {
  CHECK_T(p, torch::kFloat32);
  CHECK_T(g, torch::kFloat32);
  TORCH_CHECK(p.numel() % 64 == 0, "flat buffer must be 64-aligned");
  adam_launch(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
              optbw(lowp), flags.data_ptr<uint8_t>(), p.numel(), lr_t, optf(lr_scale), b1, b2, eps,
              wd, gs, stream());
}

// ------------------------------------------------------------------------------- depthwise conv
DwArgs dw_args(const Tensor& x_like, const Tensor& w, int64_t Ho, int64_t Wo, int64_t sh,
               int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw) {
  DwArgs a{};
  a.N = x_like.size(0); a.H = x_like.size(1); a.W = x_like.size(2); a.C = x_like.size(3);
  a.R = w.size(0); a.S = w.size(1); a.Ho = Ho; a.Wo = Wo;
  a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dwl = dw;
  TORCH_CHECK(w.size(2) == a.C, "depthwise weight must be [R,S,C]");
  return a;
}

static DwF32Args dw_f32_args(const Tensor& x_like, const Tensor& w, int64_t Ho, int64_t Wo, int64_t sh,
                             int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw) {
  DwF32Args a{};
  a.N = x_like.size(0); a.H = x_like.size(1); a.W = x_like.size(2); a.C = x_like.size(3);
  a.R = w.size(0); a.S = w.size(1); a.Ho = Ho; a.Wo = Wo;
  a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dwl = dw;
  TORCH_CHECK(w.dim() == 3 && w.size(2) == a.C, "depthwise weight must be [R,S,C]");
  check_c4(a.C, "depthwise conv");
  return a;
}

// aff (optional fp32 [≥2, ld ≥ C]: rows a, b of a BN's coefficients): the conv's input is
// relu(a·x + b) — the BN + ReLU folded in (ops/dwfold.py); only where dwconv_aff_ok
static void set_dw_aff(DwArgs& a, const c10::optional<Tensor>& aff, const char* who) {
  if (!aff.has_value() || !aff->defined()) return;
  CHECK_T(*aff, torch::kFloat32);
  TORCH_CHECK(aff->dim() == 2 && aff->size(0) >= 2 && aff->size(1) >= a.C && aff->is_contiguous() &&
                  aff->size(1) % 4 == 0,
              who, " aff: contiguous fp32 [>=2, ld >= C], ld % 4 == 0");
  TORCH_CHECK(dwconv_aff_ok(a), who, " aff: not supported for this geometry");
  a.aff = aff->data_ptr<float>();
  a.aff_ld = (int)aff->size(1);
}

static bool dwconv_aff_ok_py(Tensor x, Tensor w, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                             int64_t dh, int64_t dw) {
  if (x.dim() != 4 || w.dim() != 3 || w.size(2) != x.size(3)) return false;
  const int64_t R = w.size(0), S = w.size(1);
  const int64_t Ho = (x.size(1) + 2 * ph - dh * (R - 1) - 1) / sh + 1;
  const int64_t Wo = (x.size(2) + 2 * pw - dw * (S - 1) - 1) / sw + 1;
  if (Ho <= 0 || Wo <= 0) return false;
  DwArgs a = dw_args(x, w, Ho, Wo, sh, sw, ph, pw, dh, dw);
  return dwconv_aff_ok(a);
}

// stats (optional fp32 [2, C], zeroed by the caller): BN sums of y fused into the kernel;
// returns whether they were written (stride-1 3×3 tile kernel only)
bool dwconv_fwd(Tensor x, Tensor w, c10::optional<Tensor> bias, Tensor y, int64_t sh, int64_t sw,
                int64_t ph, int64_t pw, int64_t dh, int64_t dw, bool relu, bool relu_in,
                c10::optional<Tensor> stats, c10::optional<Tensor> aff) {
  if (is_f32(x)) {
    CHECK_T(x, torch::kFloat32);
    CHECK_T(w, torch::kFloat32);
    CHECK_T(y, torch::kFloat32);
    TORCH_CHECK(!relu_in, "fp32 depthwise: no fused input ReLU");
    DwF32Args a = dw_f32_args(x, w, y.size(1), y.size(2), sh, sw, ph, pw, dh, dw);
    a.x = F32(x); a.w = F32(w); a.bias = optf(bias); a.out = F32(y); a.relu = relu;
    dwconv_f32_fwd_launch(a, stream());
    return false;  // statistics never fused here: the caller runs bn_stats
  }

  CHECK_T(x, torch::kBFloat16);
  CHECK_T(w, torch::kBFloat16);
  CHECK_T(y, torch::kBFloat16);
  DwArgs a = dw_args(x, w, y.size(1), y.size(2), sh, sw, ph, pw, dh, dw);
  a.x = BF(x); a.w = BF(w); a.bias = optf(bias); a.out = BFW(y); a.relu = relu;
  TORCH_CHECK(!relu_in || (a.C % 8 == 0 && a.R * a.S == 9), "fused input ReLU: 3x3, C % 8 == 0");
  a.relu_in = relu_in;
  // deterministic mode: no fused statistics (epilogue atomics) — the caller's bn_stats pass
  // reduces in a fixed order (det.hip)
  if (stats.has_value() && stats->defined() && !deterministic()) {
    TORCH_CHECK(stats->numel() == 2 * a.C, "dwconv_fwd stats: fp32 [2, C]");
    a.stats = optfw(stats);
  }
  set_dw_aff(a, aff, "dwconv_fwd");
  return dwconv_fwd_launch(a, stream());
}

// bn_x / bn_red (optional, together): also accumulate the BN-backward sums (Σg, Σg·bn_x) of the
// stored dx (stride-1 3×3 tile kernel only; returns whether they were written)
// dadd (optional, shaped like dx, may be dx itself): dx = dgrad + dadd — the residual-gradient
// join (ops/gradjoin.py) of a tensor whose other consumer wrote its gradient first
bool dwconv_dgrad(Tensor dy, Tensor w, Tensor dx, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                  int64_t dh, int64_t dw, c10::optional<Tensor> mask_x,
                  c10::optional<Tensor> bn_x, c10::optional<Tensor> bn_red,
                  c10::optional<Tensor> dadd, c10::optional<Tensor> aff) {
  if (is_f32(dy)) {
    CHECK_T(dy, torch::kFloat32);
    CHECK_T(w, torch::kFloat32);
    CHECK_T(dx, torch::kFloat32);
    TORCH_CHECK(!(mask_x.has_value() && mask_x->defined()), "fp32 depthwise: no fused input ReLU");
    DwF32Args a = dw_f32_args(dx, w, dy.size(1), dy.size(2), sh, sw, ph, pw, dh, dw);
    a.dy = F32(dy); a.w = F32(w); a.out = F32(dx);
    a.dadd = opt_f32_like(dadd, dx, "dwconv_dgrad dadd");
    dwconv_f32_dgrad_launch(a, stream());
    return false;
  }
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(w, torch::kBFloat16);
  CHECK_T(dx, torch::kBFloat16);
  DwArgs a = dw_args(dx, w, dy.size(1), dy.size(2), sh, sw, ph, pw, dh, dw);
  a.dy = BF(dy); a.w = BF(w); a.out = BFW(dx);
  a.mask_x = optb(mask_x);
  if (dadd.has_value() && dadd->defined()) {
    CHECK_T(*dadd, torch::kBFloat16);
    TORCH_CHECK(dadd->sizes() == dx.sizes(), "dwconv_dgrad dadd must be shaped like dx");
    a.dadd = BF(*dadd);
  }
  if (a.mask_x) {
    TORCH_CHECK(mask_x->sizes() == dx.sizes(), "mask_x must be shaped like dx");
    TORCH_CHECK(a.C % 8 == 0 && a.R * a.S == 9, "fused input ReLU: 3x3, C % 8 == 0");
  }
  if (bn_x.has_value() && bn_x->defined()) {
    TORCH_CHECK(bn_red.has_value() && bn_red->defined(), "dwconv_dgrad: bn_x needs bn_red");
    CHECK_T(*bn_x, torch::kBFloat16);
    TORCH_CHECK(bn_x->sizes() == dx.sizes() && bn_red->numel() == 2 * a.C,
                "dwconv_dgrad bn_x: shape of dx, bn_red fp32 [2, C]");
    a.bn_x = BF(*bn_x);  // (the folded BN's mask source even without the sums)
    if (!deterministic()) a.stats = optfw(bn_red);  // else the BN backward reduces itself
  }
  set_dw_aff(a, aff, "dwconv_dgrad");
  TORCH_CHECK(!a.aff || (a.bn_x && !a.mask_x), "dwconv_dgrad aff: the mask comes from bn_x");
  return dwconv_dgrad_launch(a, stream());
}

void dwconv_wgrad(Tensor dy, Tensor x, Tensor dwt, c10::optional<Tensor> db, int64_t sh, int64_t sw,
                  int64_t ph, int64_t pw, int64_t dh, int64_t dw, bool relu_in, bool accumulate,
                  c10::optional<Tensor> aff) {
  if (is_f32(dy)) {
    CHECK_T(dy, torch::kFloat32);
    CHECK_T(x, torch::kFloat32);
    CHECK_T(dwt, torch::kFloat32);
    TORCH_CHECK(!relu_in, "fp32 depthwise: no fused input ReLU");
    TORCH_CHECK(dwt.size(0) * dwt.size(1) <= 9, "fp32 depthwise weight gradient: up to 3x3 taps");
    DwF32Args a = dw_f32_args(x, dwt, dy.size(1), dy.size(2), sh, sw, ph, pw, dh, dw);
    a.dy = F32(dy); a.x = F32(x); a.dwt = F32(dwt); a.db = optfw(db);
    if (!accumulate) {
      (void)hipMemsetAsync(a.dwt, 0, dwt.numel() * sizeof(float), stream());
      if (a.db) (void)hipMemsetAsync(a.db, 0, a.C * sizeof(float), stream());
    }
    dwconv_f32_wgrad_launch(a, stream());
    return;
  }
  CHECK_T(dy, torch::kBFloat16);
  CHECK_T(x, torch::kBFloat16);
  CHECK_T(dwt, torch::kFloat32);
  TORCH_CHECK(dwt.size(0) * dwt.size(1) <= 49, "depthwise kernel up to 7x7");
  DwArgs a = dw_args(x, dwt, dy.size(1), dy.size(2), sh, sw, ph, pw, dh, dw);
  a.dy = BF(dy); a.x = BF(x); a.dw = dwt.data_ptr<float>(); a.db = optfw(db);
  a.accum = accumulate;
  TORCH_CHECK(!relu_in || (a.C % 8 == 0 && a.R * a.S == 9), "fused input ReLU: 3x3, C % 8 == 0");
  a.relu_in = relu_in;
  set_dw_aff(a, aff, "dwconv_wgrad");
  const int slabs = dwconv_wgrad_slabs(a);
  Tensor ws;
  if (slabs > 0) ws = torch::empty({(int64_t)slabs * (a.R * a.S + 1) * a.C}, dwt.options());
  dwconv_wgrad_launch(a, slabs > 0 ? ws.data_ptr<float>() : nullptr, stream());
}

// ------------------------------------------------------------------------------------- upsample
void upsample_fwd(Tensor x, Tensor y, Tensor ih, Tensor wh, Tensor iw, Tensor ww) {
  if (is_f32(x)) {
    CHECK_T(x, torch::kFloat32);
    const int64_t ldy = nhwc_ld_f32(y, "upsample y");
    upsample_fwd_launch(F32(x), F32(y), ih.data_ptr<int>(), wh.data_ptr<float>(), iw.data_ptr<int>(),
                        ww.data_ptr<float>(), x.size(0), x.size(1), x.size(2), x.size(3), y.size(1),
                        y.size(2), stream(), (int)ldy);
    return;
  }
  CHECK_T(x, torch::kBFloat16);
  const int64_t ldy = nhwc_ld(y, "upsample y");
  upsample_fwd_launch(BF(x), BFW(y), ih.data_ptr<int>(), wh.data_ptr<float>(), iw.data_ptr<int>(),
                      ww.data_ptr<float>(), x.size(0), x.size(1), x.size(2), x.size(3), y.size(1),
                      y.size(2), stream(), (int)ldy);
}

void upsample_bwd(Tensor dy, Tensor dx, Tensor ih, Tensor wh, Tensor iw, Tensor ww) {
  if (is_f32(dy)) {
    const int64_t ldd = nhwc_ld_f32(dy, "upsample dy");
    CHECK_T(dx, torch::kFloat32);
    upsample_bwd_launch(F32(dy), F32(dx), ih.data_ptr<int>(), wh.data_ptr<float>(), iw.data_ptr<int>(),
                        ww.data_ptr<float>(), dx.size(0), dx.size(1), dx.size(2), dx.size(3),
                        dy.size(1), dy.size(2), stream(), (int)ldd);
    return;
  }
  const int64_t ldd = nhwc_ld(dy, "upsample dy");
  CHECK_T(dx, torch::kBFloat16);
  upsample_bwd_launch(BF(dy), BFW(dx), ih.data_ptr<int>(), wh.data_ptr<float>(), iw.data_ptr<int>(),
                      ww.data_ptr<float>(), dx.size(0), dx.size(1), dx.size(2), dx.size(3), dy.size(1),
                      dy.size(2), stream(), (int)ldd);
}

// --------------------------------------------------------------------------- native data loader
// ------------------------------------------------------------------------- native RCCL comm
comm::DType comm_dtype(const Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kFloat32: return comm::DType::F32;
    case torch::kBFloat16: return comm::DType::BF16;
    case torch::kFloat16: return comm::DType::F16;
    case torch::kFloat64: return comm::DType::F64;
    case torch::kInt32: return comm::DType::I32;
    case torch::kInt64: return comm::DType::I64;
    case torch::kUInt8: return comm::DType::U8;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL: ", t.scalar_type());
  }
  return comm::DType::F32;
}

comm::Op comm_op(const std::string& op) {
  if (op == "sum") return comm::Op::Sum;
  if (op == "max") return comm::Op::Max;
  if (op == "min") return comm::Op::Min;
  if (op == "prod") return comm::Op::Prod;
  if (op == "avg") return comm::Op::Avg;
  TORCH_CHECK(false, "unknown reduce op ", op);
  return comm::Op::Sum;
}

// Collectives run on a dedicated high-priority stream from torch's pool, ordered after the
// current (compute) stream; the caching allocator is told the comm stream uses each buffer.
struct PyComm {
  std::unique_ptr<comm::Communicator> c;
  c10::hip::HIPStream cs;
  int device;

  PyComm(py::bytes uid, int rank, int world, int dev, double timeout_s)
      : cs(c10::hip::getStreamFromPool(true, dev)), device(dev) {
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)dev));
    py::gil_scoped_release nogil;  // ncclCommInitRank blocks until every rank joined
    c = std::make_unique<comm::Communicator>(std::string(uid), rank, world, dev, timeout_s);
  }
  void use(const Tensor& t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RCCL buffers must be contiguous HIP tensors");
    TORCH_CHECK(t.device().index() == device, "tensor on device ", t.device().index(),
                ", communicator on ", device);
    c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), cs);
  }
  int64_t all_reduce(Tensor t, const std::string& op) {
    use(t);
    return (int64_t)c->all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), comm_dtype(t), comm_op(op),
                                  stream(), cs.stream());
  }
  int64_t broadcast(Tensor t, int root) {
    use(t);
    return (int64_t)c->broadcast(t.data_ptr(), t.data_ptr(), t.numel(), comm_dtype(t), root, stream(),
                                 cs.stream());
  }
  int64_t reduce_scatter(Tensor in, Tensor out, const std::string& op) {
    use(in);
    use(out);
    TORCH_CHECK(in.scalar_type() == out.scalar_type() && in.numel() == out.numel() * c->world(),
                "reduce_scatter: in must hold world x out elements");
    return (int64_t)c->reduce_scatter(in.data_ptr(), out.data_ptr(), out.numel(), comm_dtype(in),
                                      comm_op(op), stream(), cs.stream());
  }
  int64_t all_gather(Tensor in, Tensor out) {
    use(in);
    use(out);
    TORCH_CHECK(in.scalar_type() == out.scalar_type() && out.numel() == in.numel() * c->world(),
                "all_gather: out must hold world x in elements");
    return (int64_t)c->all_gather(in.data_ptr(), out.data_ptr(), in.numel(), comm_dtype(in), stream(),
                                  cs.stream());
  }
  void wait(int64_t ticket) { c->wait((uint64_t)ticket, stream()); }
  void synchronize() {
    py::gil_scoped_release nogil;
    c->synchronize();
  }
  // fault injection: delay the comm stream by `ms` (bounded spin kernel) — watchdog tests
  int64_t debug_delay(double ms, bool track) {
    debug_spin_launch(ms, cs.stream());
    return track ? (int64_t)c->track("debug_delay", cs.stream()) : 0;
  }
  // watch the work queued so far on the current (compute) stream like a collective — a HIP-graph
  // replay whose captured collectives hang is then timed out by the watchdog as well
  int64_t track_current(const std::string& name) { return (int64_t)c->track(name.c_str(), stream()); }
};

struct PyLoader {
  std::unique_ptr<tdl_rt::BatchLoader> impl;
  bool has_masks;
  bool pin;
  PyLoader(std::vector<std::string> images, std::vector<std::string> masks, int batch, bool augment,
           bool shuffle, bool repeat, int64_t seed, int threads, int prefetch, int channels,
           int transformation, bool pin_memory, py::dict aug, bool fp32)
      : has_masks(!masks.empty()), pin(pin_memory) {
    tdl_rt::AugConfig cfg;
    for (auto item : aug) {
      const std::string k = py::str(item.first);
      if (k == "horizontal_flip") cfg.horizontal_flip = item.second.cast<bool>();
      else if (k == "vertical_flip") cfg.vertical_flip = item.second.cast<bool>();
      else if (k == "rotate_range") cfg.rotate_range = item.second.cast<double>();
      else if (k == "crop_probability") cfg.crop_probability = item.second.cast<double>();
      else if (k == "crop_min_percent") cfg.crop_min_percent = item.second.cast<double>();
      else if (k == "crop_max_percent") cfg.crop_max_percent = item.second.cast<double>();
      else if (k == "height_shift_range") cfg.height_shift_range = item.second.cast<double>();
      else if (k == "width_shift_range") cfg.width_shift_range = item.second.cast<double>();
      else if (k == "brightness_range") cfg.brightness_range = item.second.cast<double>();
      else throw std::invalid_argument("unknown augmentation option: " + k);
    }
    impl.reset(new tdl_rt::BatchLoader(images, masks, batch, augment, shuffle, repeat,
                                       (uint64_t)seed, threads, prefetch, channels,
                                       transformation, cfg, fp32));
  }
  // pinned host tensors of one batch (no Python objects: runs without the GIL)
  void to_tensors(const tdl_rt::Batch& b, Tensor& x, Tensor& y, Tensor& ids) {
    const int B = impl->batch(), H = impl->height(), W = impl->width(), C = impl->channels();
    auto opt = torch::TensorOptions().pinned_memory(pin);
    if (impl->fp32()) {
      x = torch::empty({B, H, W, C}, opt.dtype(torch::kFloat32));
      memcpy(x.data_ptr(), b.xf.data(), b.xf.size() * 4);
    } else {
      x = torch::empty({B, H, W, C}, opt.dtype(torch::kBFloat16));
      memcpy(x.data_ptr(), b.x.data(), b.x.size() * 2);
    }
    ids = torch::from_blob((void*)b.ids.data(), {(int64_t)b.ids.size()}, torch::kInt64).clone();
    if (has_masks) {
      y = torch::empty({B, H, W, 1}, opt.dtype(torch::kFloat32));
      memcpy(y.data_ptr(), b.y.data(), b.y.size() * 4);
    }
  }
  py::object next() {
    tdl_rt::Batch b;
    Tensor x, y, ids;
    bool ok;
    {
      // the pinned copies (≈6 MB per DeepLab batch) run without the GIL too, so a prefetch
      // thread (data/prefetch.py) overlaps them with the training thread
      py::gil_scoped_release nogil;
      ok = impl->next(b);
      if (ok) to_tensors(b, x, y, ids);
    }
    if (!ok) return py::none();
    if (has_masks) return py::make_tuple(x, y, ids, b.count);
    return py::make_tuple(x, py::none(), ids, b.count);
  }
};

// CRC32C (Castagnoli) of a byte string — the TFRecord framing of the summary event files
// (engine/summary.py); table-driven, slicing by 8 (the pure-Python loop cost ≈1 ms per 10 KB
// image summary, several ms per summary step on the training thread)
static uint32_t g_crc_tab[8][256];
static void crc32c_init() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1) ? 0x82F63B78u : 0u);
    g_crc_tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t)
      g_crc_tab[t][i] = (g_crc_tab[t - 1][i] >> 8) ^ g_crc_tab[0][g_crc_tab[t - 1][i] & 0xFF];
}
uint32_t crc32c(const std::string& data) {
  static const bool init = (crc32c_init(), true);
  (void)init;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(data.data());
  size_t n = data.size();
  uint32_t crc = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= crc;
    crc = g_crc_tab[7][v & 0xFF] ^ g_crc_tab[6][(v >> 8) & 0xFF] ^ g_crc_tab[5][(v >> 16) & 0xFF] ^
          g_crc_tab[4][(v >> 24) & 0xFF] ^ g_crc_tab[3][(v >> 32) & 0xFF] ^
          g_crc_tab[2][(v >> 40) & 0xFF] ^ g_crc_tab[1][(v >> 48) & 0xFF] ^ g_crc_tab[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) crc = g_crc_tab[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return crc ^ 0xFFFFFFFFu;
}

Tensor png_decode_gray(const std::string& path) {
  tdl_rt::GrayImage g = tdl_rt::load_png_gray(path);
  Tensor t = torch::empty({g.h, g.w}, torch::kFloat32);
  memcpy(t.data_ptr(), g.px.data(), g.px.size() * 4);
  return t;
}

py::tuple augment_one(Tensor img, c10::optional<Tensor> mask, bool transpose, bool hflip, bool vflip,
                      double angle, double tx, double ty, int64_t pad, double brightness,
                      bool crop, double crop_pct, double crop_left, double crop_top) {
  TORCH_CHECK(img.dim() == 2 && img.scalar_type() == torch::kFloat32 && img.is_contiguous());
  tdl_rt::GrayImage gi;
  gi.h = img.size(0);
  gi.w = img.size(1);
  gi.px.assign(img.data_ptr<float>(), img.data_ptr<float>() + img.numel());
  tdl_rt::GrayImage gm;
  const bool hm = mask.has_value() && mask->defined();
  if (hm) {
    gm.h = gi.h;
    gm.w = gi.w;
    gm.px.assign(mask->data_ptr<float>(), mask->data_ptr<float>() + mask->numel());
  }
  tdl_rt::AugParams p;
  p.transpose = transpose; p.hflip = hflip; p.vflip = vflip; p.angle = angle; p.tx = tx; p.ty = ty;
  p.brightness = brightness; p.crop = crop; p.crop_pct = crop_pct; p.crop_left = crop_left;
  p.crop_top = crop_top;
  Tensor oi = torch::empty_like(img), om = torch::empty_like(img);
  tdl_rt::augment_sample(gi, hm ? &gm : nullptr, p, (int)pad, oi.data_ptr<float>(),
                         hm ? om.data_ptr<float>() : nullptr);
  Tensor lap = torch::empty_like(img);
  tdl_rt::laplace(oi.data_ptr<float>(), gi.h, gi.w, lap.data_ptr<float>());
  return py::make_tuple(oi, hm ? py::object(py::cast(om)) : py::none(), lap);
}

std::vector<double> transform_matrix(bool hflip, bool vflip, double angle, double tx, double ty,
                                     int64_t H, int64_t W, bool crop, double crop_pct,
                                     double crop_left, double crop_top) {
  tdl_rt::AugParams p;
  p.hflip = hflip; p.vflip = vflip; p.angle = angle; p.tx = tx; p.ty = ty;
  p.crop = crop; p.crop_pct = crop_pct; p.crop_left = crop_left; p.crop_top = crop_top;
  double t[8];
  tdl_rt::make_transform(p, (int)H, (int)W, t);
  return std::vector<double>(t, t + 8);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "tensorflowdistributedlearning_amd native gfx950 kernels";
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("bias"),
        py::arg("stats"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("dh"), py::arg("dw"), py::arg("relu"), py::arg("res") = py::none(),
        py::arg("aff") = py::none());
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("sh"),
        py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"),
        py::arg("accumulate") = false, py::arg("mask") = py::none(), py::arg("w_t") = py::none(),
        py::arg("bn_x") = py::none(), py::arg("bn_red") = py::none(), py::arg("aff") = py::none(),
        py::arg("w_flip") = py::none());
  m.def("conv_wgrad_fp8", &conv_wgrad_fp8, py::arg("dy8"), py::arg("x8"), py::arg("out"),
        py::arg("sdy"), py::arg("sx"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("dh"), py::arg("dw"), py::arg("accumulate") = false,
        "fp8 weight gradient: e5m2 dy x e4m3 x on the f8f6f4 MFMA, fp32 dW");
  m.def("conv_flip_weights_multi", [](Tensor src, Tensor dst, Tensor rows) {
    CHECK_T(src, torch::kBFloat16);
    CHECK_T(dst, torch::kBFloat16);
    TORCH_CHECK(src.is_contiguous() && dst.is_contiguous() && dst.numel() == src.numel(),
                "conv_flip_weights_multi: contiguous flat buffers of one size");
    TORCH_CHECK(rows.is_cuda() && rows.scalar_type() == torch::kInt64 && rows.dim() == 2 &&
                rows.size(1) == 8 && rows.is_contiguous(), "rows: int64 [n, 8]");
    conv_flip_weights_multi_launch(BF(src), BFW(dst), rows.data_ptr<int64_t>(), (int)rows.size(0),
                                   stream());
  }, "every registered filter flip of a flat weight buffer in one launch (rows: offset, K, R, S, "
     "C, tap, k tile, c tile; validated on the host by ops/conv.FlatFlips)");
  m.def("conv_flip_classes", [](Tensor w, Tensor out, int64_t sh, int64_t sw, int64_t ph,
                                int64_t pw) {
    CHECK_T(w, torch::kBFloat16);
    CHECK_T(out, torch::kBFloat16);
    TORCH_CHECK(w.dim() == 4 && w.is_contiguous() && out.is_contiguous() && sh >= 1 && sw >= 1,
                "conv_flip_classes: w [K,R,S,C], out contiguous, stride >= 1");
    const long need = conv_flip_classes_numel((int)w.size(0), (int)w.size(1), (int)w.size(2),
                                              (int)w.size(3), (int)sh, (int)sw, (int)ph, (int)pw);
    TORCH_CHECK(out.numel() == need, "conv_flip_classes: out has ", out.numel(),
                " elements, the parity-class sub-filters need ", need);
    conv_flip_classes_launch(BF(w), BFW(out), (int)w.size(0), (int)w.size(1), (int)w.size(2),
                             (int)w.size(3), (int)sh, (int)sw, (int)ph, (int)pw, stream());
  });
  m.def("conv_flip_weight", [](Tensor w, Tensor wf) {
    CHECK_T(w, torch::kBFloat16);
    CHECK_T(wf, torch::kBFloat16);
    TORCH_CHECK(w.dim() == 4 && wf.dim() == 4 && w.is_contiguous() && wf.is_contiguous() &&
                wf.size(0) == w.size(3) && wf.size(1) == w.size(1) && wf.size(2) == w.size(2) &&
                wf.size(3) == w.size(0), "conv_flip_weight: w [K,R,S,C] -> wf [C,R,S,K]");
    conv_flip_weight_launch(BF(w), BFW(wf), w.size(0), w.size(1), w.size(2), w.size(3), stream());
  }, "w_flip[c][r][s][k] = w[k][R-1-r][S-1-s][c]");
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("out"),
        py::arg("bias_grad"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("dh"), py::arg("dw"), py::arg("accumulate"), py::arg("aff") = py::none());
  m.def("conv_fwd_fp8", &conv_fwd_fp8);
  m.def("conv_dgrad_fp8", &conv_dgrad_fp8, py::arg("dy8"), py::arg("w8t"), py::arg("dx"),
        py::arg("scale_dy"), py::arg("scale_w"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("dh"), py::arg("dw"), py::arg("accumulate") = false, py::arg("mask") = py::none(),
        py::arg("bn_x") = py::none(), py::arg("bn_red") = py::none(), py::arg("w_flip") = py::none());
  m.attr("AMAX_SLOT") = AMAX_SLOT;
  m.def("fp8_amax", &fp8_amax);
  m.def("fp8_roll", &fp8_roll);
  m.def("fp8_quantize", &fp8_quantize);
  m.def("fp8_multi_quantize", &fp8_multi_quantize);
  m.def("fp8_dequantize", &fp8_dequantize);
  m.def("bn_stats", &bn_stats);
  m.def("bn_finalize", &bn_finalize);
  m.def("bn_apply", &bn_apply, py::arg("x"), py::arg("coef"), py::arg("res"), py::arg("y"),
        py::arg("relu"), py::arg("y8") = py::none(), py::arg("amax_ring") = py::none(),
        py::arg("phase") = 0, py::arg("scale_out") = py::none(), py::arg("mask") = py::none(),
        py::arg("store_y") = true);
  m.def("bn_bwd_reduce", &bn_bwd_reduce);
  m.def("bn_bwd_reduce2", &bn_bwd_reduce2);
  m.def("bn_bwd_apply", &bn_bwd_apply, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("coef"),
        py::arg("red"), py::arg("gamma"), py::arg("dx"), py::arg("dres"), py::arg("dgamma"),
        py::arg("dbeta"), py::arg("count"), py::arg("relu"), py::arg("dx8") = py::none(),
        py::arg("amax_ring") = py::none(), py::arg("phase") = 0, py::arg("scale_out") = py::none(),
        py::arg("red_raw") = false, py::arg("dadd") = py::none(), py::arg("store_dx") = true);
  m.def("fp8_quantize_e5m2", [](Tensor x, Tensor ring, int64_t phase, bool measure, Tensor scale,
                                Tensor y8) {
    CHECK_T(x, torch::kBFloat16);
    CHECK_T(scale, torch::kFloat32);
    TORCH_CHECK(x.numel() % 16 == 0 && y8.element_size() == 1 && y8.numel() == x.numel() &&
                y8.is_contiguous(), "fp8_quantize_e5m2: numel % 16 == 0, byte output");
    fp8_quantize_e5m2_launch(BF(x), x.numel(), ring_slot(ring, phase),
                             measure ? ring_slot(ring, phase + 1) : nullptr,
                             measure ? ring_slot(ring, phase + 2) : nullptr, scale.data_ptr<float>(),
                             (uint8_t*)y8.data_ptr(), stream());
  });
  m.def("fp8_dequantize_e5m2", [](Tensor y8, Tensor scale, Tensor out) {
    TORCH_CHECK(y8.is_cuda() && y8.element_size() == 1 && y8.is_contiguous());
    CHECK_T(out, torch::kFloat32);
    fp8_dequantize_e5m2_launch((const uint8_t*)y8.data_ptr(), y8.numel(), scale.data_ptr<float>(),
                               out.data_ptr<float>(), stream());
  });
  m.def("fp8_multi_transpose", [](Tensor src, Tensor dst, Tensor tiles) {
    TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.element_size() == 1 && dst.element_size() == 1 &&
                src.numel() == dst.numel() && src.is_contiguous() && dst.is_contiguous(),
                "fp8_multi_transpose: flat byte buffers of equal size");
    TORCH_CHECK(tiles.is_cuda() && tiles.scalar_type() == torch::kInt64 && tiles.dim() == 2 &&
                tiles.size(1) == 4 && tiles.is_contiguous(), "tiles: int64 [n,4]");
    fp8_multi_transpose_launch((const uint8_t*)src.data_ptr(), (uint8_t*)dst.data_ptr(),
                               tiles.data_ptr<int64_t>(), (int)tiles.size(0), stream());
  });
  m.def("relu_bwd", &relu_bwd);
  m.def("row_pack", &row_pack);
  m.def("add_act", &add_act);
  m.def("scale_by_scalar", &scale_by_scalar);
  m.def("convert", &convert, "fp32 <-> bf16 flat conversion (RNE)");
  m.def("sigmoid_threshold", &sigmoid_threshold);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("maxpool_bwd_stats", &maxpool_bwd_stats);
  m.def("bn_maxpool_fwd", &bn_maxpool_fwd, py::arg("x"), py::arg("coef"), py::arg("y"),
        py::arg("idx"), py::arg("k"), py::arg("s"), py::arg("pt"), py::arg("pl"),
        py::arg("zarg") = py::none());
  m.def("maxpool_bn_bwd", &maxpool_bn_bwd);
  m.def("maxpool_bwd_rb", &maxpool_bwd_rb, py::arg("dy"), py::arg("idx"), py::arg("dx"),
        py::arg("k"), py::arg("s"), py::arg("pt"), py::arg("pl"), py::arg("bn_x") = py::none(),
        py::arg("bn_red") = py::none());
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd, py::arg("dy"), py::arg("dx"), py::arg("dadd") = py::none());
  m.def("softmax_xent", &softmax_xent);
  m.def("softmax_eval", &softmax_eval, py::arg("logits"), py::arg("labels") = py::none(),
        py::arg("loss_sum") = py::none(), py::arg("correct") = py::none(),
        py::arg("probs") = py::none());
  m.def("lovasz_hinge", &lovasz_hinge);
  m.def("seg_metrics", &seg_metrics);
  m.def("sgd_momentum", &sgd_momentum, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("lowp"),
        py::arg("flags"), py::arg("lr"), py::arg("mu"), py::arg("wd"), py::arg("gs"),
        py::arg("nesterov"), py::arg("lr_scale") = py::none());
  m.def("adam", &adam, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("lowp"),
        py::arg("flags"), py::arg("lr_t"), py::arg("b1"), py::arg("b2"), py::arg("eps"),
        py::arg("wd"), py::arg("gs"), py::arg("lr_scale") = py::none());
  m.def("dwconv_fwd", &dwconv_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"),
        py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"),
        py::arg("relu"), py::arg("relu_in"), py::arg("stats") = py::none(),
        py::arg("aff") = py::none());
  m.def("dwconv_dgrad", &dwconv_dgrad, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("sh"),
        py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"),
        py::arg("mask_x") = py::none(), py::arg("bn_x") = py::none(),
        py::arg("bn_red") = py::none(), py::arg("dadd") = py::none(), py::arg("aff") = py::none());
  m.def("dwconv_wgrad", &dwconv_wgrad, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("db"),
        py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dwl"),
        py::arg("relu_in"), py::arg("accumulate") = true, py::arg("aff") = py::none());
  m.def("dwconv_aff_ok", &dwconv_aff_ok_py, py::arg("x"), py::arg("w"), py::arg("sh"),
        py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"),
        "whether the depthwise kernels for this geometry take a folded input BN + ReLU (aff)");
  m.def("upsample_fwd", &upsample_fwd);
  m.def("upsample_bwd", &upsample_bwd);
  m.def("conv_set_glds_mode", &conv_set_glds_mode,
        "conv kernel selection: 0 register-staged only, 1 LDS-DMA for large problems (default), "
        "2 LDS-DMA whenever aligned, -1 environment (TDL_CONV_GLDS)");
  m.def("conv_glds_mode", &conv_glds_mode);
  m.def("deterministic", &deterministic,
        "deterministic mode on (fixed-order slab reductions instead of fp32 atomics)");
  m.def("det_set", &det_set, "deterministic mode: 1 on, 0 off, -1 environment (TDL_DETERMINISTIC)");
  m.def("conv_set_halo_mode", &conv_set_halo_mode,
        "halo-tiled stride-1 conv: -1 environment (TDL_HALO, default 1), 0 off, 1 default "
        "selection, 2 every eligible problem regardless of size (tests)");
  m.def("bn_fold_weight", &bn_fold_weight, py::arg("w"), py::arg("coef"), py::arg("wout"),
        py::arg("bias_in"), py::arg("bias_out"));
  m.def("scale_cols", &scale_cols, py::arg("dw"), py::arg("a"));
  m.def("fp8_set_policy", &fp8_set_policy, py::arg("margin_e4m3") = -1.0, py::arg("margin_e5m2") = -1.0,
        py::arg("decay") = -1.0,
        "fp8 delayed scaling: scale = margin * amax / fp8_max, amax history slot <- max(step amax, "
        "decay * previous) at each roll; < 0: environment (TDL_FP8_MARGIN, TDL_FP8_MARGIN_E5M2, "
        "TDL_FP8_AMAX_DECAY)");
  m.def("fp8_policy", []() { auto p = fp8_policy(); return py::make_tuple(p.margin_e4m3, p.margin_e5m2, p.decay); });
  m.def("conv_set_pc", &conv_set_pc, "wave-specialised producer/consumer forward (-1: env)");
  // ---- the conv route table (kernels/conv_route.h)
  m.def("conv_route_table", []() {
    py::list out;
    static const char* impls[] = {"gemm", "glds", "pc", "halo", "asfwd"};
    static const char* ops[] = {"fwd", "dgrad", "wgrad"};
    for (int i = 0; i < route_count(); ++i) {
      const RouteRule& r = route_rule(i);
      py::dict d;
      d["name"] = r.name; d["op"] = ops[r.op]; d["impl"] = impls[r.impl];
      d["taps"] = py::make_tuple(r.taps_min, r.taps_max); d["stride1"] = (bool)r.stride1;
      d["cin"] = py::make_tuple(r.cin_min, r.cin_max); d["cout"] = py::make_tuple(r.cout_min, r.cout_max);
      d["rows_min"] = r.rows_min; d["tile"] = py::make_tuple(r.tile_m, r.tile_n);
      d["tiles_min"] = r.tiles_min; d["need"] = r.need; d["forbid"] = r.forbid;
      d["cfg"] = route_cfg(i); d["default_cfg"] = r.cfg; d["on"] = route_on(i);
      d["default_on"] = r.on; d["test"] = r.test; d["evidence"] = r.evidence;
      d["instantiated"] = route_cfg_instantiated(r.impl, r.op, route_cfg(i), r.need);
      d["mode"] = route_family_mode(r);
      out.append(d);
    }
    return out;
  }, "every conv routing row in order, with its current state");
  m.def("conv_route_select", [](int op, int taps, int stride, int cin, int cout, int64_t rows,
                                int flags, std::vector<int64_t> cls_rows) {
    RouteProblem p;
    p.op = op; p.taps = taps; p.stride = stride; p.cin = cin; p.cout = cout; p.rows = rows;
    p.flags = flags;
    TORCH_CHECK(cls_rows.size() <= (size_t)MAX_DG_CLASSES, "too many parity classes");
    p.ncls = (int)cls_rows.size();
    for (size_t c = 0; c < cls_rows.size(); ++c) p.cls_rows[c] = cls_rows[c];
    py::list names;
    for (int i = route_next(p, -1); i >= 0; i = route_next(p, i)) names.append(route_rule(i).name);
    return names;
  }, py::arg("op"), py::arg("taps"), py::arg("stride"), py::arg("cin"), py::arg("cout"),
     py::arg("rows"), py::arg("flags") = 0, py::arg("cls_rows") = std::vector<int64_t>{},
     "the rows a launcher would try for this problem, in order (each launcher then runs the first "
     "whose kernel takes it)");
  m.def("conv_route_force", [](int op, std::string name) { route_force(op, name.c_str()); },
        py::arg("op"), py::arg("name") = "",
        "tests: only this row for op (0 fwd, 1 dgrad, 2 wgrad); a launcher that cannot run it "
        "raises; '' clears");
  m.def("conv_route_set", [](std::string name, int on, int cfg) { route_set(name.c_str(), on, cfg); },
        py::arg("name"), py::arg("on") = -1, py::arg("cfg") = -1,
        "in-process A/B: turn a row on (1) / off (0) and / or set its tile config (validated)");
  m.def("conv_route_reset", &route_reset, "route rows back to the table + environment");
  m.def("conv_last_route", [](int op) -> py::object {
    const int i = route_last(op);
    if (i < 0) return py::none();
    return py::str(route_rule(i).name);
  }, py::arg("op"), "the row the last conv launch of op ran on this thread");
  m.def("conv_route_counts", [](bool reset) {
    py::dict d;
    for (int i = 0; i < route_count(); ++i)
      if (route_count_of(i)) d[py::str(route_rule(i).name)] = route_count_of(i);
    if (reset) route_counts_reset();
    return d;
  }, py::arg("reset") = false, "launches per route row since the last reset (eager launches)");
  m.def("conv_route_cfg_instantiated", &route_cfg_instantiated, py::arg("impl"), py::arg("op"),
        py::arg("cfg"), py::arg("flags") = 0);
  m.def("conv_set_m32", &conv_set_m32, "32x32x16-MFMA K loop for KC-operand LDS-DMA convs (-1: env)");
  m.def("conv_m32", &conv_m32);
  m.def("conv_f32_set_tile", &conv_f32_set_tile, "fp32 conv FWD/DGRAD tile override (0, 0: auto)");
  m.def("fastdiv", [](uint32_t d) { auto f = make_fastdiv(d); return py::make_tuple(f.m, f.s); },
        "magic (m, s) with n / d == (n * m) >> s for 0 <= n < 2^31");
  m.def("rccl_unique_id", []() { return py::bytes(comm::get_unique_id()); });
  m.def("rccl_version", &comm::rccl_version);
  py::class_<PyComm>(m, "RcclComm")
      .def(py::init<py::bytes, int, int, int, double>(), py::arg("uid"), py::arg("rank"),
           py::arg("world"), py::arg("device"), py::arg("timeout_s") = 600.0)
      .def("all_reduce", &PyComm::all_reduce, py::arg("t"), py::arg("op") = "sum")
      .def("broadcast", &PyComm::broadcast, py::arg("t"), py::arg("root") = 0)
      .def("reduce_scatter", &PyComm::reduce_scatter, py::arg("inp"), py::arg("out"),
           py::arg("op") = "sum")
      .def("all_gather", &PyComm::all_gather)
      .def("wait", &PyComm::wait)
      .def("synchronize", &PyComm::synchronize)
      .def("debug_delay", &PyComm::debug_delay, py::arg("ms"), py::arg("track") = false)
      .def("track_current", &PyComm::track_current, py::arg("name") = "graph_replay")
      .def_property_readonly("rccl_count", [](PyComm& p) { return p.c->rccl_count(); })
      .def_property_readonly("rccl_rank", [](PyComm& p) { return p.c->rccl_rank(); })
      .def_property_readonly("rccl_device", [](PyComm& p) { return p.c->rccl_device(); })
      .def("abort", [](PyComm& p, const std::string& why) { p.c->abort(why); })
      .def_property_readonly("error", [](PyComm& p) { return p.c->error(); })
      .def_property_readonly("ok", [](PyComm& p) { return p.c->ok(); })
      .def_property_readonly("outstanding", [](PyComm& p) { return p.c->outstanding(); })
      .def_property_readonly("rank", [](PyComm& p) { return p.c->rank(); })
      .def_property_readonly("world", [](PyComm& p) { return p.c->world(); });
  py::class_<PyLoader>(m, "BatchLoader")
      .def(py::init<std::vector<std::string>, std::vector<std::string>, int, bool, bool, bool,
                    int64_t, int, int, int, int, bool, py::dict, bool>(),
           py::arg("images"), py::arg("masks"), py::arg("batch"), py::arg("augment"),
           py::arg("shuffle"), py::arg("repeat"), py::arg("seed"), py::arg("threads"),
           py::arg("prefetch"), py::arg("channels"), py::arg("transformation"),
           py::arg("pin_memory") = false, py::arg("aug") = py::dict(),
           py::arg("fp32") = false)
      .def("next", &PyLoader::next)
      .def_property_readonly("num_batches", [](PyLoader& l) { return l.impl->num_batches(); })
      .def_property_readonly("height", [](PyLoader& l) { return l.impl->height(); })
      .def_property_readonly("width", [](PyLoader& l) { return l.impl->width(); });
  m.def("png_decode_gray", &png_decode_gray);
  m.def("crc32c", [](py::bytes b) { return crc32c(std::string(b)); });
  m.def("augment_one", &augment_one, py::arg("img"), py::arg("mask"), py::arg("transpose"),
        py::arg("hflip"), py::arg("vflip"), py::arg("angle"), py::arg("tx"), py::arg("ty"),
        py::arg("pad"), py::arg("brightness") = 0.0, py::arg("crop") = false,
        py::arg("crop_pct") = 1.0, py::arg("crop_left") = 0.0, py::arg("crop_top") = 0.0);
  m.def("transform_matrix", &transform_matrix, py::arg("hflip"), py::arg("vflip"),
        py::arg("angle"), py::arg("tx"), py::arg("ty"), py::arg("H"), py::arg("W"),
        py::arg("crop") = false, py::arg("crop_pct") = 1.0, py::arg("crop_left") = 0.0,
        py::arg("crop_top") = 0.0);
}
