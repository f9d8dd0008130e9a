"""Training-mode BatchNorm + ReLU folded into the dense convolution that consumes it.

In a ResNet bottleneck the outputs of the first two conv + BN + ReLU layers each feed exactly one
conv (conv1 → BN → ReLU → conv2 3×3 → BN → ReLU → conv3 1×1; the reference's slim arg scope puts
BN + ReLU after every conv, /root/reference/core/resnet.py:130-144 with :373-386).  Unfolded, the
BN's apply pass reads z and writes u = relu(a⊙z + b) (a = γ·invstd, b = β − μ·a) plus a 1-bit ReLU
mask, and the consumer conv reads u back.  Folded (SURVEY §7.4 "BN-apply + ReLU in the next conv's
prologue"), the consumer reads z and the BN's coefficients (``ConvArgs::aff``):

  forward   the conv_pc producer waves stage the A tile through registers and write
            u = relu(a·z + b), rounded to bf16 exactly as the apply pass stores it, into the LDS
            ring (conv_gemm's register staging for shapes the producer kernel does not take);
            padding taps and rows past M stay 0 — the consumers' K loop is unchanged
  dgrad     g_u = convᵀ(dy)·[a·z + b > 0]: the mask comes from z, which the fused BN-backward
            statistics epilogue (Σg, Σg·z) loads anyway, so no mask tensor exists at all
  BN bwd    dz = BN-backward(g_u) — the usual apply pass, its reduce already fused
  wgrad     dW = dyᵀ·relu(a·z + b): conv_gemm transforms the staged x rows

so u and its mask are never written or read (ResNet-50: 32 of 53 BN apply passes per step).  Exact
w.r.t. the unfolded step: same fma, same rounding, same mask.  Anything the kernels do not take
(CPU, fp32, fp8 layers, channel-padded or row-packed convs, a bias) materialises the BN the
ordinary way (:meth:`DeferredBNAct.materialize`).

Off by default (experimental: ``TDL_EXPERIMENTAL=bnconv`` turns it on): measured on MI355X it loses.  The transform
runs once per A element per filter tap and per output-column tile (9× for a 3×3 conv, Cout/128×
for a 1×1), and the producer waves' VALU does not overlap the consumers' MFMA issue on the same
SIMD — every transformed 8-channel chunk costs its ≈24 instructions of SIMD time.  ResNet-50 b1024
standalone per step (bench/bnconv_ab.py, profiles/r05_bnconv_fold_ab.txt): forward 11.74 →
14.10 ms *including* the 32 apply passes the fold removes, input gradients 11.21 → 12.74, weight
gradients 9.93 → 12.78 (the register-staged kernel instead of the halo / LDS-DMA ones); whole step
82.3 → 91.3 ms (serial streams), 13,196 → 11,676 img/s.
Numerics: tests/test_bnconv.py (CPU plumbing; on the GPU the three kernels and a ResNet-50 step).
"""
from __future__ import annotations

import os

import torch

from .common import on_gpu, fused_gpu, ext, compute_weight, grad_target, deliver_grad, export_impl
from . import workspace
from . import streams
from .bn import (bn_stats, bn_finalize, bn_apply, bn_bwd_reduce, bn_bwd_apply, bn_red_xhat,
                 _phys_params, _grad_target_phys)
from .conv import ConvGeom, conv_fwd, conv_dgrad, conv_wgrad

ENABLED = os.environ.get("TDL_EXP_BNCONV", "0") == "1"  # experimental (TDL_EXPERIMENTAL=bnconv)


class DeferredBNAct:
    """A training BN + ReLU whose apply is deferred to its single consumer: ``z`` the BN input,
    ``stats`` its (Σz, Σz²) if the producer accumulated them, ``bn`` the models.layers.BatchNorm.
    :meth:`materialize` applies it the ordinary way."""

    __slots__ = ("z", "stats", "bn")

    def __init__(self, z, stats, bn):
        self.z, self.stats, self.bn = z, stats, bn

    @property
    def shape(self):
        return self.z.shape

    def materialize(self):
        return self.bn(self.z, stats=self.stats, relu=True)


def foldable(z, layer) -> bool:
    """Can the dense conv ``layer`` (models.layers.Conv2d) consume BN + ReLU of ``z`` folded?"""
    from ..models.layers import Conv2d
    return (ENABLED and fused_gpu(z) and z.dtype == torch.bfloat16 and export_impl() is None
            and type(layer) is Conv2d and layer.bias is None and not layer.grad_needs_unpad()
            and not getattr(layer, "fp8", False) and z.shape[-1] % 8 == 0
            and layer.cout % 8 == 0 and torch.is_grad_enabled())


def _args(geom: ConvGeom):
    return (geom.stride[0], geom.stride[1], geom.padding[0], geom.padding[2], geom.dilation[0],
            geom.dilation[1])


class _BNActConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, stats_z, gamma, beta, weight, bn, layer, geom, want_stats):
        C = z.shape[-1]
        count = z.numel() // C
        if stats_z is None or stats_z.numel() == 0:
            stats_z = bn_stats(z)
        gp, bp = _phys_params(bn, gamma, beta)
        coef = bn_finalize(stats_z, count, gp, bp, bn.running_mean, bn.running_var, bn.decay,
                           bn.eps, True)
        w = layer.compute_weight(z.dtype)
        K = w.shape[0]
        stats = workspace.zeros((2, K), z.device) if want_stats else None
        if on_gpu(z):
            N, H, W, _ = z.shape
            Ho, Wo = geom.out_hw(H, W, w.shape[1], w.shape[2])
            y = torch.empty((N, Ho, Wo, K), device=z.device, dtype=z.dtype)
            ext().conv_fwd(z, w, y, None, stats, *_args(geom), False, None, coef)
        else:  # the plumbing on the CPU oracle: the same math with u materialised
            y = conv_fwd(bn_apply(z, coef, relu=True), w, geom, stats=stats)
        ctx.bn, ctx.layer, ctx.geom, ctx.count = bn, layer, geom, count
        ctx.save_for_backward(z, weight, gamma, beta, coef)
        if stats is None:
            stats = torch.empty(0, device=z.device)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        z, weight, gamma, beta, coef = ctx.saved_tensors
        if dy is None:
            return (None,) * 9
        dy = dy.contiguous()
        bn, layer, geom = ctx.bn, ctx.layer, ctx.geom
        C = z.shape[-1]
        gpu = on_gpu(dy)
        side = streams.side(dy.device) if (gpu and weight.requires_grad) else None
        if side is not None and streams.EARLY_WAIT:  # dy is ready: the wgrad overlaps the dgrad
            side.wait_stream(streams.current(dy.device))
        w = layer.compute_weight(dy.dtype)
        # input gradient through the conv, masked by the folded ReLU, with the BN-backward sums
        if gpu:
            gu = torch.empty_like(z)
            red = workspace.zeros((2, C), dy.device)
            fused = bool(ext().conv_dgrad(dy, w, gu, *_args(geom), False, None, None, z, red,
                                          coef))
        else:
            gu, fused = conv_dgrad(dy, w, tuple(z.shape), geom), False
        relu = 0 if fused else 2  # unfused: unmasked g_u, the BN masks by a·z + b > 0 itself
        if not fused:
            red = bn_bwd_reduce(gu, None, z, coef, relu)
        want_g = gamma is not None and gamma.requires_grad
        want_b = beta.requires_grad
        gt, gfresh = _grad_target_phys(gamma, C) if want_g else (None, False)
        bt, bfresh = _grad_target_phys(beta, C) if want_b else (None, False)
        direct_g = gpu and gt is not None and gfresh
        direct_b = gpu and bt is not None and bfresh
        gp, _ = _phys_params(bn, gamma, beta)
        dz, _ = bn_bwd_apply(gu, None, z, coef, red, gp, ctx.count, relu, False,
                             gt if direct_g else None, bt if direct_b else None, red_raw=fused)
        if fused and want_g and not direct_g:
            red = bn_red_xhat(red, coef)
        c = beta.numel()
        if want_g:
            deliver_grad(gamma, None if direct_g else red[1][:c], written=direct_g)
        if want_b:
            deliver_grad(beta, None if direct_b else red[0][:c], written=direct_b)
        # weight gradient on the folded input (side stream when enabled, as ops/conv.py does)
        if weight.requires_grad:
            if side is None:
                _wgrad(dy, z, coef, weight, geom)
            else:
                if not streams.EARLY_WAIT:
                    side.wait_stream(streams.current(dy.device))
                with streams.on(side):
                    _wgrad(dy, z, coef, weight, geom)
                # dy, z and the coefficients are read there: alive until the next join
                streams.keep_alive(dy.device, dy, z, coef)
                streams.join_at_backward_end(dy.device)
        return dz, None, None, None, None, None, None, None, None


def _wgrad(dy, z, coef, weight, geom):
    target, fresh = grad_target(weight)
    if on_gpu(dy):
        if target is not None:
            ext().conv_wgrad(dy, z, target, None, *_args(geom), not fresh, coef)
            deliver_grad(weight, written=True)
        else:
            dw = torch.empty(tuple(weight.shape), device=dy.device, dtype=torch.float32)
            ext().conv_wgrad(dy, z, dw, None, *_args(geom), False, coef)
            deliver_grad(weight, dw)
        return
    u = bn_apply(z, coef, relu=True)
    if target is not None:
        conv_wgrad(dy, u, tuple(weight.shape), geom, out=target, accumulate=not fresh)
        deliver_grad(weight, written=True)
    else:
        deliver_grad(weight, conv_wgrad(dy, u, tuple(weight.shape), geom))


def bn_act_conv(src: DeferredBNAct, layer, want_stats=False, force=False):
    """``layer(relu(BN(z)))`` for the deferred training BN ``src`` feeding the dense conv
    ``layer`` — folded when :func:`foldable` (or ``force``: the CPU plumbing tests), else the BN is
    applied first.  Returns ``(y, stats)`` like ``layer(x, want_stats=True)`` (stats None unless
    ``want_stats``)."""
    z, bn = src.z, src.bn
    if not (force or foldable(z, layer)):
        x = src.materialize()
        if want_stats:
            return layer(x, want_stats=True)
        return layer(x), None
    geom = layer.geom(z.shape[1], z.shape[2])
    y, st = _BNActConvFn.apply(z, src.stats, bn.gamma, bn.beta, layer.weight, bn, layer, geom,
                               bool(want_stats))
    return y, (st if want_stats else None)
