"""2-D convolution (dense, strided, dilated) in NHWC with KRSC weights.

GPU path: hand-written gfx950 MFMA implicit-GEMM kernels (``csrc/kernels/conv_gemm.hip``):
``conv_fwd`` (A = gathered input, B = weights, optional bias / ReLU / BN-statistics epilogue),
``conv_dgrad`` (A = gathered output-gradient, B = weights read through the LDS transpose path) and
``conv_wgrad`` (split-K over N·Ho·Wo, both operands through the LDS transpose path, fp32 slab
reduction straight into the flat gradient buffer).

CPU path: ``torch.nn.functional.conv2d`` in fp32 — the numerics oracle.

Reference parity: replaces every ``layers_lib.conv2d`` / ``slim.conv2d`` of the reference
(core/resnet.py:75,79,83,130,134,137,142,164-166,250,449,466,471,482,487; core/layers.py:43;
core/xception.py:111,212) which lowered to cuDNN Conv2D/BackpropInput/BackpropFilter
and, for ``rate>1``, to SpaceToBatchND (N9) — here dilation is native in the address generator.
Padding is explicit (top, bottom, left, right) so TF ``SAME`` (asymmetric at stride 2) is exact.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .common import (on_gpu, fused_gpu, ext, compute_weight, grad_target, deliver_grad, flat_view,
                     export_impl)
from . import workspace
from . import streams
from . import gradjoin


@dataclass(frozen=True)
class ConvGeom:
    stride: tuple = (1, 1)
    padding: tuple = (0, 0, 0, 0)  # top, bottom, left, right
    dilation: tuple = (1, 1)

    def out_hw(self, H, W, R, S):
        sh, sw = self.stride
        pt, pb, pl, pr = self.padding
        dh, dw = self.dilation
        Ho = (H + pt + pb - dh * (R - 1) - 1) // sh + 1
        Wo = (W + pl + pr - dw * (S - 1) - 1) // sw + 1
        return Ho, Wo


def same_padding(size, k, stride, dilation=1):
    """TF 'SAME' padding (before, after) for one spatial dim."""
    keff = k + (k - 1) * (dilation - 1)
    out = -(-size // stride)
    total = max((out - 1) * stride + keff - size, 0)
    return total // 2, total - total // 2


def symmetric_padding(k, dilation=1):
    keff = k + (k - 1) * (dilation - 1)
    p = (keff - 1) // 2
    return p, keff - 1 - p


# ----------------------------------------------------------------------------------------------
# reference (CPU / oracle) implementations, fp32
# ----------------------------------------------------------------------------------------------

def ref_conv_fwd(x, w, geom: ConvGeom, bias=None):
    pt, pb, pl, pr = geom.padding
    xt = F.pad(x.permute(0, 3, 1, 2).float(), (pl, pr, pt, pb))
    y = F.conv2d(xt, w.permute(0, 3, 1, 2).float(), None if bias is None else bias.float(),
                 stride=geom.stride, dilation=geom.dilation)
    return y.permute(0, 2, 3, 1).contiguous()


def ref_conv_dgrad(dy, w, x_shape, geom: ConvGeom):
    N, H, W, C = x_shape
    pt, pb, pl, pr = geom.padding
    Hp, Wp = H + pt + pb, W + pl + pr
    dxp = torch.nn.grad.conv2d_input((N, C, Hp, Wp), w.permute(0, 3, 1, 2).float(),
                                     dy.permute(0, 3, 1, 2).float(), stride=geom.stride,
                                     dilation=geom.dilation)
    dx = dxp[:, :, pt:pt + H, pl:pl + W]
    return dx.permute(0, 2, 3, 1).contiguous()


def ref_conv_wgrad(dy, x, w_shape, geom: ConvGeom):
    K, R, S, C = w_shape
    pt, pb, pl, pr = geom.padding
    xt = F.pad(x.permute(0, 3, 1, 2).float(), (pl, pr, pt, pb))
    dw = torch.nn.grad.conv2d_weight(xt, (K, C, R, S), dy.permute(0, 3, 1, 2).float(),
                                     stride=geom.stride, dilation=geom.dilation)
    return dw.permute(0, 2, 3, 1).contiguous()


# ----------------------------------------------------------------------------------------------
# raw ops (dispatch)
# ----------------------------------------------------------------------------------------------

def conv_fwd(x, w, geom: ConvGeom, bias=None, relu=False, stats=None, out_dtype=None,
             residual=None):
    """y = conv(x, w) (+bias) (+residual) (relu).  If ``stats`` (fp32 [2, K]) is given,
    per-channel sum and sum of squares of the *stored* output are accumulated into it (BN
    statistics epilogue).  ``residual`` (shaped like y) is added in the LDS-DMA kernel's epilogue
    before the ReLU (with a bias); problems that kernel does not take add it in one elementwise
    pass afterwards."""
    ex = export_impl()
    if ex is not None and stats is None and out_dtype is None:
        return ex.conv2d(x, w, geom, bias, relu, residual)
    N, H, W, C = x.shape
    K, R, S, Cw = w.shape
    assert C == Cw, f"channel mismatch {C} vs {Cw}"
    Ho, Wo = geom.out_hw(H, W, R, S)
    if on_gpu(x):
        y = torch.empty((N, Ho, Wo, K), device=x.device, dtype=out_dtype or x.dtype)
        args = (geom.stride[0], geom.stride[1], geom.padding[0], geom.padding[2],
                geom.dilation[0], geom.dilation[1])
        if residual is None:
            ext().conv_fwd(x, w, y, bias, stats, *args, bool(relu))
            return y
        if bias is not None and ext().conv_fwd(x, w, y, bias, stats, *args, bool(relu),
                                               residual.contiguous()):
            return y
        ext().conv_fwd(x, w, y, bias, None, *args, False)
        out = torch.empty_like(y)
        ext().add_act(y, residual.contiguous(), out, bool(relu))
        if stats is not None:
            ext().bn_stats(out, stats)
        return out
    y = ref_conv_fwd(x, w, geom, bias)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    y = y.to(out_dtype or x.dtype)
    if stats is not None:
        yf = y.float().reshape(-1, K)
        stats[0] += yf.sum(0)
        stats[1] += (yf * yf).sum(0)
    return y


def conv_fwd_fp8(x8, sx, w8, sw, geom: ConvGeom, relu=False, stats=None):
    """Forward conv on fp8 e4m3 operands with per-tensor scales (y = Σ x8·w8 · sx·sw), bf16 out.
    GPU: LDS-DMA kernel on v_mfma_scale_f32_16x16x128_f8f6f4.  CPU: fp32 on dequantised data."""
    N, H, W, C = x8.shape
    K, R, S, _ = w8.shape
    Ho, Wo = geom.out_hw(H, W, R, S)
    if on_gpu(x8):
        y = torch.empty((N, Ho, Wo, K), device=x8.device, dtype=torch.bfloat16)
        ext().conv_fwd_fp8(x8, w8, y, stats, sx, sw, geom.stride[0], geom.stride[1],
                           geom.padding[0], geom.padding[2], geom.dilation[0], geom.dilation[1],
                           bool(relu))
        return y
    y = ref_conv_fwd(x8.float() * sx, w8.float() * sw, geom)
    if relu:
        y = torch.relu(y)
    y = y.to(torch.bfloat16)
    if stats is not None:
        yf = y.float().reshape(-1, K)
        stats[0] += yf.sum(0)
        stats[1] += (yf * yf).sum(0)
    return y


def conv_dgrad(dy, w, x_shape, geom: ConvGeom, out_dtype=None, out=None, accumulate=False,
               mask=None, w_t=None, w_flip=None):
    """dx.  With ``out`` the result is written there (``accumulate``: dx += …, fused in the GEMM
    epilogue — used by the residual-gradient join, ops/gradjoin.py).  ``mask`` (uint8, 1 bit per
    element of dx, GPU): dx = ([dx +] dgrad)·[bit] for the elements this dgrad writes.  ``w_t``
    (GPU, optional): the same weights transposed to [R,S,C,K]; the LDS-DMA kernel then reads both
    operands as K-contiguous rows (same result).  ``w_flip`` (GPU, stride 1, optional): the
    flipped transpose [C,R,S,K] (models.layers.Conv2d.flip_weight) — dx is then computed as the
    forward conv of dy on the forward kernels (:func:`dgrad_as_fwd_ok`)."""
    if on_gpu(dy):
        dx = out if out is not None else torch.empty(x_shape, device=dy.device,
                                                     dtype=out_dtype or dy.dtype)
        ext().conv_dgrad(dy, w, dx, geom.stride[0], geom.stride[1], geom.padding[0],
                         geom.padding[2], geom.dilation[0], geom.dilation[1],
                         bool(accumulate and out is not None), mask, w_t, w_flip=w_flip)
        return dx
    r = ref_conv_dgrad(dy, w, x_shape, geom)
    if mask is not None:
        from .bn import unpack_relu_mask
        keep = unpack_relu_mask(mask, r.shape[-1]).reshape(r.shape)
        if accumulate and out is not None:  # pixels this dgrad does not write keep their value
            keep = keep | ~_dgrad_touched(w.shape, x_shape, geom)
        r = r + out.float() if accumulate and out is not None else r
        r = r * keep
    elif accumulate and out is not None:
        r = out.float() + r
    if out is None:
        return r.to(out_dtype or dy.dtype)
    out.copy_(r.to(out.dtype))
    return out


def conv_dgrad_bnstat(dy, w, x_shape, geom: ConvGeom, bn_x, out=None, accumulate=False,
                      mask=None, w_flip=None):
    """:func:`conv_dgrad` that also returns the BN-backward sums of the stored dx: fp32 [2, C] =
    (Σg, Σg·x) with g = dx (as stored, after the join accumulate / ReLU mask) and x = ``bn_x``,
    the input of the BN whose output this conv consumed — the BN backward then skips its reduce
    pass (``bn_bwd_apply(red_raw=True)`` turns Σg·x into Σg·x̂).  Returns ``(dx, red)``; ``red`` is
    None when the kernel could not fuse them (strided dgrads, problems that run on the
    register-staged kernel): the BN then reduces as usual."""
    if on_gpu(dy):
        dx = out if out is not None else torch.empty(x_shape, device=dy.device, dtype=dy.dtype)
        red = workspace.zeros((2, x_shape[-1]), dy.device)
        fused = ext().conv_dgrad(dy, w, dx, geom.stride[0], geom.stride[1], geom.padding[0],
                                 geom.padding[2], geom.dilation[0], geom.dilation[1],
                                 bool(accumulate and out is not None), mask, None, bn_x, red,
                                 w_flip=w_flip)
        return dx, (red if fused else None)
    dx = conv_dgrad(dy, w, x_shape, geom, out=out, accumulate=accumulate, mask=mask)
    if accumulate and out is not None and geom.stride != (1, 1):
        return dx, None  # a strided accumulate leaves untouched pixels unmasked
    C = x_shape[-1]
    g = dx.float().reshape(-1, C)
    red = torch.stack([g.sum(0), (g * bn_x.float().reshape(-1, C)).sum(0)])
    return dx, red


DGRAD_AS_FWD = os.environ.get("TDL_DGRAD_AS_FWD", "1") == "1"


def dgrad_as_fwd_ok(dy, x_shape, geom: ConvGeom) -> bool:
    """Can this input gradient run as the forward conv of dy with the flipped filter?  bf16 on the
    GPU, dy channels % 64 (the forward kernels' FASTK), dx channels % 8; stride 1: dx and dy of
    the same spatial size; strided: no dilation (one forward conv per parity class,
    :func:`flip_classes`).  The kernel still declines problems its forward route would not take."""
    if not (DGRAD_AS_FWD and fused_gpu(dy) and dy.shape[-1] % 64 == 0 and x_shape[-1] % 8 == 0):
        return False
    if geom.stride == (1, 1):
        return tuple(dy.shape[1:3]) == tuple(x_shape[1:3])
    return geom.dilation == (1, 1) and geom.stride[0] <= 16 and geom.stride[1] <= 16


def _classes(s, R, pad):
    """per parity class a of one dimension: the taps it receives, flipped (the forward conv's order)"""
    out = []
    for a in range(s):
        r0 = (a + pad) % s
        T = (R - r0 + s - 1) // s if r0 < R else 0
        out.append([r0 + s * (T - 1 - t) for t in range(T)])
    return out


def flip_classes(w, geom: ConvGeom, out=None):
    """The per-parity-class flipped sub-filters of a strided conv's weight w [K, R, S, C], each
    [C, Th, Tw, K], concatenated a-major over the classes with taps (csrc/kernels/conv_glds.hip
    dgrad_as_fwd_strided reads them in the same order): class (a, b) of dx is the stride-1
    forward conv of dy with its sub-filter.  ``out``: a previous result's buffer to rebuild in
    place (GPU; the persistent per-layer copy — no new buffer and no copy)."""
    (sh, sw), ph, pw = geom.stride, geom.padding[0], geom.padding[2]
    R, S = w.shape[1], w.shape[2]
    if on_gpu(w) and w.dtype == torch.bfloat16 and sh <= 4 and sw <= 4:
        n = sum(len(rr) for rr in _classes(sh, R, ph)) * sum(len(ss) for ss in _classes(sw, S, pw))
        n *= w.shape[0] * w.shape[3]
        if out is None or out.numel() != n or out.dtype != w.dtype or out.device != w.device:
            out = torch.empty(n, device=w.device, dtype=w.dtype)
        ext().conv_flip_classes(w.contiguous(), out, sh, sw, ph, pw)  # one launch
        return out
    parts = []
    # (strided slices + flips only: no index tensors, so the rebuild is HIP-graph capturable)
    for rr in _classes(sh, R, ph):
        for ss in _classes(sw, S, pw):
            if rr and ss:
                sub = w[:, rr[-1]:rr[0] + 1:sh, ss[-1]:ss[0] + 1:sw].flip(1, 2)  # [K, Th, Tw, C]
                parts.append(sub.permute(3, 1, 2, 0).reshape(-1))  # [C, Th, Tw, K]
    return torch.cat(parts)


def _dgrad_touched(w_shape, x_shape, geom: ConvGeom):
    """[N, H, W, 1] bool: input pixels the dgrad writes (a strided conv with taps of fewer than
    ``stride`` rows / columns leaves whole parity classes untouched)."""
    K, R, S, C = w_shape
    N, H, W, _ = x_shape
    Ho, Wo = geom.out_hw(H, W, R, S)
    cover = ref_conv_dgrad(torch.ones(1, Ho, Wo, 1), torch.ones(1, R, S, 1), (1, H, W, 1), geom)
    return cover > 0


def conv_dgrad_fp8(dy8, sdy, w8t, sw, x_shape, geom: ConvGeom, out=None, accumulate=False,
                   mask=None, bn_x=None, w_flip=None):
    """dx from fp8 operands: ``dy8`` e5m2 [N,Ho,Wo,K] with scale ``sdy``, ``w8t`` the e4m3 weight
    transposed to [R,S,C,K] with scale ``sw`` (ops/fp8.py).  GPU: the LDS-DMA dgrad on
    v_mfma_scale_f32_16x16x128_f8f6f4 (K % 128 == 0); join accumulate / ReLU mask as
    :func:`conv_dgrad`.  CPU: fp32 on the dequantised operands.  With ``bn_x`` (no join) returns
    ``(dx, red)`` as :func:`conv_dgrad_bnstat`: the BN-backward sums fused into the epilogue.
    ``w_flip`` (stride 1): the e4m3 flipped filter [C, R, S, K] (:func:`fp8_flip_weight`) — the
    dgrad then runs as the forward fp8 conv of dy (route row dgrad.asfwd.fp8)."""
    if on_gpu(dy8):
        dx = out if out is not None else torch.empty(x_shape, device=dy8.device,
                                                     dtype=torch.bfloat16)
        red = workspace.zeros((2, x_shape[-1]), dy8.device) if bn_x is not None else None
        fused = ext().conv_dgrad_fp8(dy8.view(torch.uint8), w8t.view(torch.uint8), dx, sdy, sw,
                                     geom.stride[0], geom.stride[1], geom.padding[0],
                                     geom.padding[2], geom.dilation[0], geom.dilation[1],
                                     bool(accumulate and out is not None), mask, bn_x, red,
                                     None if w_flip is None else w_flip.view(torch.uint8))
        return dx if bn_x is None else (dx, red if fused else None)
    w = (w8t.float() * sw).permute(3, 0, 1, 2).contiguous()
    dx = conv_dgrad(dy8.float() * sdy, w, x_shape, geom, out=out, accumulate=accumulate,
                    mask=mask, out_dtype=torch.bfloat16)
    return dx if bn_x is None else (dx, None)


def fp8_flip_weight(w8t):
    """The e4m3 flipped filter [C, R, S, K] (w_flip[c][r][s][k] = w[k][R−1−r][S−1−s][c]) from the
    transposed fp8 weight [R, S, C, K]; for a 1×1 conv the same bytes (a view, no copy)."""
    R, S, C, K = w8t.shape
    if R == 1 and S == 1:
        return w8t.reshape(C, 1, 1, K)
    return w8t.view(torch.uint8).flip(0, 1).permute(2, 0, 1, 3).contiguous().view(w8t.dtype)


# the fp8 dgrad as the forward conv of dy: 1 — 1×1 stride-1 convs (the flipped filter is the
# transposed weight itself), 2 (default) — every stride-1 conv (a flip pass per 3×3 weight and
# step), 0 off.  ResNet-152 b256 fp8 graph, same box: 6,167 / 6,171 (2) vs 6,160 / 6,164 (1) vs
# 6,151 / 6,151 img/s (0) — profiles/r05_fp8_dgrad_as_fwd_ab.txt
FP8_DGRAD_AS_FWD = int(os.environ.get("TDL_FP8_DGRAD_AS_FWD", "2"))


def fp8_dgrad_eligible(layer, dy, geom: ConvGeom, w_shape):
    """Can this conv's dgrad run on fp8 operands?  An fp8 layer whose output gradient arrived
    with an e5m2 copy (the BN backward's side output), K % 128 == 0 (one tap per 128-deep K-step)
    and no stride-with-dilation (masked-class dgrad)."""
    if layer is None or not getattr(layer, "fp8_dgrad", False) or \
            getattr(dy, "_tdl_fp8", None) is None:
        return False
    K, R, S, C = w_shape
    (sh, sw), (dh, dw) = geom.stride, geom.dilation
    masked = (sh > 1 and dh > 1) or (sw > 1 and dw > 1)
    return K % 128 == 0 and C % 8 == 0 and not masked and not layer.grad_needs_unpad()


FP8_WGRAD = os.environ.get("TDL_FP8_WGRAD", "1") == "1"
# the BN-backward sums in the fp8 dgrad's epilogue (0: the BN reduces itself, for A/B)
FP8_DGRAD_STATS = os.environ.get("TDL_FP8_DGRAD_STATS", "1") == "1"


def fp8_wgrad_eligible(layer, x, w) -> bool:
    """Does this fp8 conv's weight gradient run on fp8 operands (csrc conv_wgrad_fp8)?  A layer
    enabled for it (models.enable_fp8), unpadded weights, C % 16 and K % 16 (a 16-byte chunk never
    crosses a filter tap), no bias."""
    return (FP8_WGRAD and getattr(layer, "fp8_wgrad", False) and not layer.grad_needs_unpad()
            and layer.bias is None and x.shape[-1] % 16 == 0 and w.shape[0] % 16 == 0)


def dgrad_covers_input(geom: ConvGeom, R, S):
    """Does the dgrad of this conv write every input pixel (no empty stride parity class)?"""
    (sh, sw), (dh, dw) = geom.stride, geom.dilation
    if (sh, sw) == (1, 1):
        return True
    return dh == 1 and dw == 1 and R >= sh and S >= sw


def conv_wgrad(dy, x, w_shape, geom: ConvGeom, out=None, accumulate=False, bias_grad=None):
    """dW (fp32, KRSC).  Writes into ``out`` if given (overwrite, or add when ``accumulate``).
    If ``bias_grad`` (fp32 [K]) is given, the column sums of dy are written into it too."""
    if on_gpu(dy):
        if out is None:
            out = torch.empty(w_shape, device=dy.device, dtype=torch.float32)
            accumulate = False
        ext().conv_wgrad(dy, x, out, bias_grad, geom.stride[0], geom.stride[1], geom.padding[0],
                         geom.padding[2], geom.dilation[0], geom.dilation[1], bool(accumulate))
        return out
    dw = ref_conv_wgrad(dy, x, w_shape, geom)
    if bias_grad is not None:
        bias_grad.copy_(dy.float().reshape(-1, dy.shape[-1]).sum(0))
    if out is None:
        return dw
    if accumulate:
        out.add_(dw.reshape(out.shape))
    else:
        out.copy_(dw.reshape(out.shape))
    return out


class _RowPackFn(torch.autograd.Function):
    """Differentiable :func:`row_pack` (the input gradient — rare for an image — is the
    transposed gather: S strided slice-adds)."""

    @staticmethod
    def forward(ctx, x, creal, S, sw, pl, Wo, Cp):
        ctx.args = (tuple(x.shape), creal, S, sw, pl, Wo)
        return _row_pack(x, creal, S, sw, pl, Wo, Cp)

    @staticmethod
    def backward(ctx, dt):
        (N, H, W, Cx), creal, S, sw, pl, Wo = ctx.args
        g = dt[..., : S * creal].float().reshape(N, H, Wo, S, creal)
        span = (Wo - 1) * sw + S
        dxp = torch.zeros(N, H, max(span, pl + W), creal, device=dt.device)
        for s in range(S):
            dxp[:, :, s: s + (Wo - 1) * sw + 1: sw] += g[:, :, :, s]
        dx = torch.zeros(N, H, W, Cx, device=dt.device, dtype=dt.dtype)
        dx[..., :creal] = dxp[:, :, pl: pl + W].to(dt.dtype)
        return dx, None, None, None, None, None, None


def row_pack(x, creal, S, sw, pl, Wo, Cp):
    """See :func:`_row_pack`; differentiable when ``x`` requires a gradient."""
    ex = export_impl()
    if ex is not None:
        return ex.row_pack(x, creal, S, sw, pl, Wo, Cp)
    if x.requires_grad and torch.is_grad_enabled():
        return _RowPackFn.apply(x, creal, S, sw, pl, Wo, Cp)
    return _row_pack(x, creal, S, sw, pl, Wo, Cp)


def _row_pack(x, creal, S, sw, pl, Wo, Cp):
    """Row packing of a few-channel image for its S-wide stem conv: t [N, H, Wo, Cp] with
    t[n, h, wo, s·creal + c] = x[n, h, wo·sw − pl + s, c] (zero outside the row, zero after
    S·creal).  A k×k conv over x equals a k×1 conv over t with the weight re-laid to
    [K, k, 1, Cp] (models.layers.RowPackedConv2d) — its GEMM K shrinks from k·k·8 (input padded to
    8 channels) to k·Cp (7×7 RGB stem: 392 → 168).  GPU: one HIP gather pass."""
    N, H, W, Cx = x.shape
    if on_gpu(x):
        t = torch.empty((N, H, Wo, Cp), device=x.device, dtype=x.dtype)
        ext().row_pack(x, t, int(creal), int(S), int(sw), int(pl))
        return t
    xp = F.pad(x[..., :creal], (0, 0, pl, max(0, (Wo - 1) * sw + S - W - pl)))
    cols = xp.unfold(2, S, sw)[:, :, :Wo]               # [N, H, Wo, creal, S]
    t = cols.permute(0, 1, 2, 4, 3).reshape(N, H, Wo, S * creal)
    return F.pad(t, (0, Cp - S * creal)).contiguous()


def relu_bwd(dy, y):
    """dy * (y > 0) — GPU: fused elementwise kernel."""
    if on_gpu(dy):
        dx = torch.empty_like(dy)
        ext().relu_bwd(dy, y, dx)
        return dx
    return (dy.float() * (y.float() > 0)).to(dy.dtype)


# ----------------------------------------------------------------------------------------------
# autograd
# ----------------------------------------------------------------------------------------------

class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, geom, relu, want_stats, layer, join, residual=None,
                res_link=None):
        x_in = x
        w = layer.compute_weight(x.dtype) if layer is not None else compute_weight(weight, x.dtype)
        stats = None
        if want_stats:
            stats = workspace.zeros((2, w.shape[0]), x.device)
        b = None if bias is None else (layer.compute_bias() if layer is not None
                                       else bias.detach())
        if layer is not None and getattr(layer, "fp8", False) and b is None and on_gpu(x) \
                and residual is None:
            # fp8 forward (weights + activations e4m3, per-tensor scales); backward stays bf16
            pre = getattr(x, "_tdl_fp8", None)  # e4m3 copy emitted by the producing BN
            x8, sx = pre if pre is not None else layer.fp8_input(x)
            w8, sw = layer.fp8_weight(w)
            y = conv_fwd_fp8(x8, sx, w8, sw, geom, relu=relu, stats=stats)
            if fp8_wgrad_eligible(layer, x, w):
                # the weight gradient runs on this e4m3 copy (ops/conv._conv_param_grads): the
                # bf16 input is not kept for the backward
                ctx.x8 = (x8, sx)
            elif getattr(x, "_tdl_fp8_only", False):
                # the producing BN wrote only the e4m3 copy (models.enable_fp8): the bf16 weight
                # gradient reads its dequantised values, never the unwritten bf16 bytes
                from .fp8 import dequantize
                x = dequantize(x8, sx).to(x.dtype)
        else:
            if getattr(x, "_tdl_fp8_only", False):
                raise RuntimeError("conv input has only an e4m3 copy (BatchNorm.fp8_only) but this "
                                   "conv does not run on fp8 operands")
            y = conv_fwd(x, w, geom, bias=b, relu=relu, stats=stats, residual=residual)
        ctx.has_res = residual is not None
        ctx.res_link = res_link
        ctx.geom = geom
        ctx.relu = relu
        ctx.layer = layer
        ctx.join = join
        ctx.x_shape = tuple(x.shape)
        # the ReLU-mask token of the BN that produced x (ops/gradjoin.py): a single-consumer conv
        # applies the mask in its dgrad and may fuse that BN's backward statistics
        ctx.bn_tok = getattr(x_in, "_tdl_mask_token", None) if join is None else None
        ctx.save_for_backward(None if getattr(ctx, "x8", None) is not None else x, weight, bias,
                              y if relu else None)
        if stats is None:
            stats = torch.empty(0, device=x.device)
        ctx.mark_non_differentiable(stats)
        # the stats output never receives a gradient: without this autograd zero-fills one
        # (a fill launch per conv per step)
        ctx.set_materialize_grads(False)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        x, weight, bias, y = ctx.saved_tensors
        geom = ctx.geom
        if dy is None:
            return (None,) * 10
        dy = dy.contiguous()
        if ctx.relu:
            dy = relu_bwd(dy, y)
        # the residual's gradient is the (masked) output gradient itself; it stays referenced by
        # the side-stream weight gradient's keep-alive list, so autograd never sums into it in
        # place while that kernel reads it
        dres = dy if ctx.has_res and ctx.needs_input_grad[8] else None
        if dres is not None and ctx.res_link is not None and ctx.res_link.offer(dres):
            dres = None  # the residual's BN adds it to its dx (ops/bn.py ResidualLink)
        ctx.res_link = None
        dx = None
        side = streams.side(dy.device) if (weight.requires_grad or
                                            (bias is not None and bias.requires_grad)) else None
        if side is not None and streams.EARLY_WAIT:  # dy is ready: wgrad may overlap this dgrad
            side.wait_stream(streams.current(dy.device))
        if ctx.needs_input_grad[0]:
            w = ctx.layer.compute_weight(dy.dtype) if ctx.layer is not None else \
                compute_weight(weight, dy.dtype)
            fp8_dg = fp8_dgrad_eligible(ctx.layer, dy, geom, tuple(w.shape))
            wf = None
            if fp8_dg:
                # fp8 dgrad: e5m2 dy (the BN backward's side output) × e4m3 W^T
                dy8, sdy = dy._tdl_fp8
                w8t, sw8 = ctx.layer.fp8_weight_t(w)
                # 1×1 stride 1: the transposed weight is the flipped filter — the dgrad runs as
                # the forward fp8 conv of dy (no extra weight pass)
                one = w8t.shape[0] == 1 and w8t.shape[1] == 1
                wf8 = (fp8_flip_weight(w8t) if geom.stride == (1, 1) and
                       (FP8_DGRAD_AS_FWD >= 2 or (FP8_DGRAD_AS_FWD == 1 and one)) else None)

                def dgrad(out=None, accumulate=False, mask=None):
                    return conv_dgrad_fp8(dy8, sdy, w8t, sw8, ctx.x_shape, geom, out=out,
                                          accumulate=accumulate, mask=mask, w_flip=wf8)

                def dgrad_bnstat(bn_x, mask=None, out=None):
                    return conv_dgrad_fp8(dy8, sdy, w8t, sw8, ctx.x_shape, geom, out=out,
                                          accumulate=out is not None, mask=mask, bn_x=bn_x,
                                          w_flip=wf8)
            else:
                # the flipped filter (strided: per-class sub-filters) lets the forward kernels
                # compute dx
                wf = None
                if ctx.layer is not None and dgrad_as_fwd_ok(dy, ctx.x_shape, geom):
                    wf = (ctx.layer.flip_weight(w) if geom.stride == (1, 1)
                          else ctx.layer.flip_weight_classes(w, geom))

                def dgrad(out=None, accumulate=False, mask=None):
                    return conv_dgrad(dy, w, ctx.x_shape, geom, out=out, accumulate=accumulate,
                                      mask=mask, w_flip=wf)

                def dgrad_bnstat(bn_x, mask=None, out=None):
                    return conv_dgrad_bnstat(dy, w, ctx.x_shape, geom, bn_x, out=out,
                                             accumulate=out is not None, mask=mask, w_flip=wf)
            join = ctx.join
            masks_ok = fused_gpu(dy) and ctx.x_shape[-1] % 64 == 0  # 64-channel mask slabs
            # (the kernel decides; strided: parity classes; fp8: no join)
            stats_ok = masks_ok and (not fp8_dg or FP8_DGRAD_STATS)
            if join is None:
                tok = ctx.bn_tok
                # a statistics-only token (BN without ReLU) needs no 64-channel mask slabs
                if tok is not None and tok.relu_y:
                    tok = None  # a ReLU without bit mask: only the depthwise dgrad applies it
                if tok is not None and (masks_ok or (fused_gpu(dy) and tok.mask is None)):
                    # sole consumer of a masked BN output: apply the mask here, and fuse the BN's
                    # backward statistics when the kernel can (ops/gradjoin.py)
                    if (stats_ok or tok.mask is None) and tok.x is not None \
                            and gradjoin.STATS_SINGLE:
                        dx, red = dgrad_bnstat(tok.x, mask=tok.mask)
                    else:
                        dx, red = dgrad(mask=tok.mask), None
                    tok.mark(dx, red)
                    ctx.bn_tok = None
                else:
                    dx = dgrad()
            else:  # residual-gradient join: first consumer writes, later ones accumulate
                # pre-masked join (ops/gradjoin.py)
                mask = join.mask if masks_ok else None
                if join.buf is None:
                    join.buf = dgrad(mask=mask)
                    join.note(mask is not None)
                elif (join.last and mask is not None and stats_ok and geom.stride == (1, 1)
                      and join.stats_x_for(fp8_dg and FP8_DGRAD_STATS) is not None):
                    # the final contribution writes every pixel through the mask: its epilogue
                    # sees the finished gradient and can fuse the BN statistics
                    _, join.red = dgrad_bnstat(join.stats_x_for(fp8_dg and FP8_DGRAD_STATS),
                                               mask=mask, out=join.buf)
                    join.note(True)
                else:
                    dgrad(out=join.buf, accumulate=True, mask=mask)
                    join.note(mask is not None, dgrad_covers_input(geom, w.shape[1], w.shape[2]))
                dx = join.take()
        if side is None:
            _conv_param_grads(ctx, dy, x, weight, bias)
        else:  # weight / bias gradients on the side stream, concurrent with the dgrad chain
            if not streams.EARLY_WAIT:
                side.wait_stream(streams.current(dy.device))
            with streams.on(side):
                _conv_param_grads(ctx, dy, x, weight, bias)
            # until the next join (no record_stream)
            streams.keep_alive(dy.device, *[t for t in (dy, x) if t is not None],
                               *getattr(ctx, "fp8_keep", ()))
            streams.join_at_backward_end(dy.device)  # backward() returns joined
        return dx, None, None, None, None, None, None, None, dres, None


def _conv_param_grads(ctx, dy, x, weight, bias):
    """dW (+ bias gradient) of one conv backward, delivered to the parameters."""
    geom = ctx.geom
    want_bias = bias is not None and bias.requires_grad
    bias_buf, bias_direct = None, False
    if want_bias:
        nb = dy.shape[-1]  # physical output channels (> bias.numel() when channel-padded)
        bt, bfresh = grad_target(bias)
        if bt is not None and nb != bias.numel():
            bt = flat_view(bias, nb, "grad")  # the zero slack after the bias takes the pad
        bias_direct = bt is not None and bfresh
        bias_buf = bt if bias_direct else torch.empty(nb, device=dy.device,
                                                      dtype=torch.float32)
    x8 = getattr(ctx, "x8", None)
    if x8 is not None and weight.requires_grad:
        # fp8 weight gradient: e5m2 dy (the BN backward's side output, else quantised here) ×
        # the forward's e4m3 input
        from .fp8 import quantize_e5m2
        ctx.x8 = None
        d8 = getattr(dy, "_tdl_fp8", None)
        dy8, sdy = d8 if d8 is not None else quantize_e5m2(dy)
        target, fresh = grad_target(weight)
        out = target if target is not None else torch.empty(tuple(weight.shape), device=dy.device,
                                                            dtype=torch.float32)
        (sh, sw), (dh, dw) = geom.stride, geom.dilation
        ext().conv_wgrad_fp8(dy8, x8[0], out, sdy, x8[1], sh, sw, geom.padding[0],
                             geom.padding[2], dh, dw, target is not None and not fresh)
        ctx.fp8_keep = (dy8, x8[0])
        if target is not None:
            deliver_grad(weight, written=True)
        else:
            deliver_grad(weight, out)
        return
    if weight.requires_grad:
        target, fresh = grad_target(weight)
        if ctx.layer is not None and ctx.layer.grad_needs_unpad():
            dw = conv_wgrad(dy, x, ctx.layer.padded_weight_shape(), geom, bias_grad=bias_buf)
            deliver_grad(weight, ctx.layer.unpad_grad(dw))
        elif target is not None:
            conv_wgrad(dy, x, tuple(weight.shape), geom, out=target, accumulate=not fresh,
                       bias_grad=bias_buf)
            deliver_grad(weight, written=True)
        else:
            dw = conv_wgrad(dy, x, tuple(weight.shape), geom, bias_grad=bias_buf)
            deliver_grad(weight, dw)
    elif want_bias:
        bias_buf.copy_(dy.float().reshape(-1, dy.shape[-1]).sum(0))
    if want_bias:
        if bias_direct:
            deliver_grad(bias, written=True)
        else:
            deliver_grad(bias, bias_buf[: bias.numel()])


def conv2d(x, weight, bias=None, geom: ConvGeom = ConvGeom(), relu=False, want_stats=False,
           layer=None, join=None, residual=None, res_link=None):
    """Differentiable NHWC conv. Returns (y, stats) where stats is fp32 [2, K] (sum, sumsq of y)
    when ``want_stats`` else an empty tensor.  ``join`` (ops.gradjoin.GradJoin) makes dx share one
    buffer with the other consumers of ``x``.  ``residual``: y = act(conv + bias + residual)."""
    if export_impl() is not None:  # serving trace: inference forward, no statistics
        sv = layer.__dict__.get("_serve") if layer is not None else None  # frozen (serving.py)
        if sv is not None:
            w, b = sv
        else:
            w = (layer.compute_weight(x.dtype) if layer is not None
                 else compute_weight(weight, x.dtype))
            b = None if bias is None else (layer.compute_bias() if layer is not None
                                           else bias.detach())
        return conv_fwd(x, w, geom, bias=b, relu=relu, residual=residual), None
    return _Conv2dFn.apply(x, weight, bias, geom, relu, want_stats, layer, join, residual,
                           res_link)
