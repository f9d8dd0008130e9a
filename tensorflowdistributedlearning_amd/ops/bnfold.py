"""Training-mode BatchNorm folded into the 1×1 conv that consumes it (no activation between).

Xception's separable convs run depthwise → BN → pointwise 1×1 (core/xception.py:38-128 with
``activation_fn_in_separable_conv=False``: the BN after the depthwise has no ReLU).  The BN
output u = a⊙z + b (per channel: a = γ·invstd, b = β − μ·a from the batch statistics of z) has
the pointwise conv as its only consumer, so instead of materialising u (one read + one write of
the depthwise output per separable conv — an elementwise pass at HBM speed) the conv runs on z:

  forward   y = W·u = (W·diag a)·z + W·b          scaled weight copy (K×C) + bias vector, per step
  dgrad     du = Wᵀ·dy  (the unscaled W), with the BN-backward sums (Σdu, Σdu·z) in the dgrad
            epilogue, then dz = BN-backward(du) in one apply pass — what the unfolded path does
  wgrad     dW = dyᵀ·u = (dyᵀ·z)·diag a + (Σ_p dy) ⊗ b    the wgrad kernel reads z; the second
            term vanishes when y feeds a training-mode BN (Xception's pointwise BN): that BN's input
            gradient sums to zero per channel (Σ_p dy = γ·invstd·(Σg − N·ḡ − Σx̂·mean(g·x̂)) = 0,
            Σ_p x̂ = 0), so only a column scale remains — the column-sum pass over dy it would
            need cost more than the BN apply pass the fold removes (7 ms per Xception-41 b128
            step, profiles/r04_xception41_b128_fold_step_breakdown.txt)

Exact up to rounding (u is never rounded to bf16; the bias W·b goes through the conv's fp32 bias
epilogue).  The moving statistics update exactly as in ``batch_norm_act`` (bn_finalize).
Numerics: tests/test_bnfold.py (CPU oracle), tests/test_train_gpu.py (GPU, vs the unfolded step).
"""
from __future__ import annotations

import os

import torch

from .common import on_gpu, fused_gpu, grad_target, deliver_grad, ext
from . import streams
from . import workspace
from .bn import (bn_stats, bn_finalize, bn_bwd_reduce, bn_bwd_apply, bn_red_xhat, _phys_params,
                 _grad_target_phys)
from .conv import conv_fwd, conv_dgrad, conv_dgrad_bnstat, conv_wgrad

ENABLED = os.environ.get("TDL_BN_CONV_FOLD", "1") == "1"


def _scaled_weight(layer, dtype, coef):
    """(W·diag a in the compute dtype, fp32 W·b [+ the conv's own bias]) for this step — one
    HIP launch on the GPU (csrc/kernels/bnfold.hip)."""
    w = layer.compute_weight(dtype)
    K, C = w.shape[0], w.shape[-1]
    if on_gpu(w):
        wf = torch.empty_like(w)
        bias = torch.empty(K, device=w.device, dtype=torch.float32)
        bi = layer.compute_bias().float().contiguous() if layer.bias is not None else None
        ext().bn_fold_weight(w, coef, wf, bi, bias)
        return wf, bias
    w2 = w.float().reshape(K, C)
    wf = (w2 * coef[0][:C].view(1, C)).to(dtype).reshape(w.shape)
    bias = torch.mv(w2, coef[1][:C].contiguous())
    if layer.bias is not None:
        bias = bias + layer.compute_bias().float()
    return wf, bias.contiguous()


class _BNConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, stats_z, gamma, beta, weight, bn, layer, want_stats, dy_sums_zero):
        C = z.shape[-1]
        count = z.numel() // C
        if stats_z is None or stats_z.numel() == 0:
            stats_z = bn_stats(z)
        gp, bp = _phys_params(bn, gamma, beta)
        coef = bn_finalize(stats_z, count, gp, bp, bn.running_mean, bn.running_var, bn.decay,
                           bn.eps, True)
        wf, bias = _scaled_weight(layer, z.dtype, coef)
        geom = layer.geom(z.shape[1], z.shape[2])
        K = wf.shape[0]
        stats = workspace.zeros((2, K), z.device) if want_stats else None
        y = conv_fwd(z, wf, geom, bias=bias, stats=stats)
        ctx.bn, ctx.layer, ctx.geom, ctx.count = bn, layer, geom, count
        ctx.dy_sums_zero = dy_sums_zero
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
        layer, geom, bn = ctx.layer, ctx.geom, ctx.bn
        C = z.shape[-1]
        side = streams.side(dy.device) if weight.requires_grad else None
        if side is not None and streams.EARLY_WAIT:
            side.wait_stream(streams.current(dy.device))
        dz = None
        if ctx.needs_input_grad[0]:
            w = layer.compute_weight(dy.dtype)  # the unscaled W: du = Wᵀ·dy
            red = None
            if fused_gpu(dy) or not on_gpu(dy):
                du, red = conv_dgrad_bnstat(dy, w, tuple(z.shape), geom, z)
            else:
                du = conv_dgrad(dy, w, tuple(z.shape), geom)
            red_raw = red is not None
            if red is None:
                red = bn_bwd_reduce(du, None, z, coef, 0)
            want_g = gamma is not None and gamma.requires_grad
            want_b = beta.requires_grad
            gt, gfresh = _grad_target_phys(gamma, C) if want_g else (None, False)
            bt, bfresh = _grad_target_phys(beta, C) if want_b else (None, False)
            direct_g = on_gpu(dy) and gt is not None and gfresh
            direct_b = on_gpu(dy) and bt is not None and bfresh
            gp, _ = _phys_params(bn, gamma, beta)
            dz, _ = bn_bwd_apply(du, None, z, coef, red, gp, ctx.count, 0, False,
                                 gt if direct_g else None, bt if direct_b else None,
                                 red_raw=red_raw)
            if red_raw and want_g and not direct_g:
                red = bn_red_xhat(red, coef)
            c = beta.numel()
            if want_g:
                deliver_grad(gamma, None if direct_g else red[1][:c], written=direct_g)
            if want_b:
                deliver_grad(beta, None if direct_b else red[0][:c], written=direct_b)
        if weight.requires_grad:
            if side is None:
                _fold_wgrad(layer, weight, dy, z, geom, coef, ctx.dy_sums_zero)
            else:  # on the side stream, concurrent with the dgrad chain (ops/conv.py)
                if not streams.EARLY_WAIT:
                    side.wait_stream(streams.current(dy.device))
                with streams.on(side):
                    _fold_wgrad(layer, weight, dy, z, geom, coef, ctx.dy_sums_zero)
                streams.keep_alive(dy.device, dy, z, coef)
                streams.join_at_backward_end(dy.device)
        return dz, None, None, None, None, None, None, None, None


def _fold_wgrad(layer, weight, dy, z, geom, coef, dy_sums_zero):
    """dW = (dyᵀ·z)·diag a [+ (Σ dy) ⊗ b unless ``dy_sums_zero``], delivered to the parameter
    (before its grad hook, so a data-parallel bucket never all-reduces the unscaled product)."""
    K = dy.shape[-1]
    s = None
    if not dy_sums_zero:
        s = (workspace.zeros((K,), dy.device) if on_gpu(dy)
             else torch.zeros(K, dtype=torch.float32))
    pshape = layer.padded_weight_shape() if layer.grad_needs_unpad() else tuple(weight.shape)
    target, fresh = grad_target(weight)
    direct = target is not None and fresh and not layer.grad_needs_unpad()
    dw = conv_wgrad(dy, z, pshape, geom, out=target if direct else None, bias_grad=s)
    Cp = pshape[-1]
    d2 = dw.view(pshape[0], Cp)
    if on_gpu(d2):
        ext().scale_cols(d2, coef[0])
    else:
        d2.mul_(coef[0][:Cp].view(1, Cp))
    if s is not None:
        d2.addr_(s, coef[1][:Cp])
    if direct:
        deliver_grad(weight, written=True)
    else:
        deliver_grad(weight, layer.unpad_grad(dw) if layer.grad_needs_unpad() else dw)


def bn_conv1x1(z, stats, bn, layer, want_stats=False, dy_sums_zero=False):
    """``layer(BN(z))`` for a training-mode BN without activation whose only consumer is the 1×1
    conv ``layer`` (models.layers.Conv2d), without materialising BN(z).  ``stats``: (Σz, Σz²) if
    the producer accumulated them (else a reduce pass).  ``dy_sums_zero``: the conv's output
    feeds a training-mode BN (its gradient sums to zero per channel; see the module docstring).
    Returns ``(y, stats_of_y)`` (stats only with ``want_stats``)."""
    if layer.k != (1, 1) or layer.stride != (1, 1) or not bn.training:
        raise ValueError("bn_conv1x1: a training BN feeding a 1×1 stride-1 conv")
    y, st = _BNConvFn.apply(z, stats, bn.gamma, bn.beta, layer.weight, bn, layer,
                            bool(want_stats), bool(dy_sums_zero))
    return y, (st if want_stats else None)
