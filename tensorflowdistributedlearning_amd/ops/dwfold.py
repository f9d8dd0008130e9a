"""Training-mode BatchNorm + ReLU folded into the depthwise conv that consumes it.

Inside an Xception module the second and third separable convs read ReLU(BN(z)) of the previous
pointwise conv's output z (core/xception.py:38-128, the pre-activation ReLU of units 2 and 3 with
``activation_fn_in_separable_conv=False``) and nothing else reads it.  Unfolded, the BN's apply
pass writes u = relu(a⊙z + b) (a = γ·invstd, b = β − μ·a) and the depthwise conv reads u back;
its backward reads u again for the ReLU mask.  Here the depthwise kernels take (a, b) and read z
(csrc/kernels/dwconv.hip, ``DwArgs::aff``):

  forward   the LDS tile kernel transforms its staged input tile in place, u = relu(a·z + b)
            rounded to bf16 exactly as the apply pass stores it (out-of-image halo stays 0)
  dgrad     g_u = DWᵀ(dy)·[a·z + b > 0], with the BN-backward sums (Σg_u, Σg_u·z) in the same
            epilogue (z is read once for both), then dz = BN-backward(g_u) in one apply pass
  wgrad     dW = Σ dy ⊗ relu(a·z + b), the transform applied to the sliding window's x loads

so u is never written (one read + one write of the activation per fold) and the backward's mask
read is gone.  Exact w.r.t. the unfolded step (same fma, same bf16 rounding of u).  Stride-1 3×3
only (``ext().dwconv_aff_ok``); anything else, and the CPU, falls back to the unfolded ops.
Numerics: tests/test_dwfold.py (CPU plumbing; GPU against the unfolded step).
"""
from __future__ import annotations

import os

import torch

from .common import on_gpu, ext, compute_weight, grad_target, deliver_grad
from . import workspace
from .bn import (bn_stats, bn_finalize, bn_bwd_reduce, bn_bwd_apply, bn_red_xhat, _phys_params,
                 _grad_target_phys)
from .bnconv import DeferredBNAct  # noqa: F401  (shared with the dense-conv fold)

ENABLED = os.environ.get("TDL_BN_DW_FOLD", "1") == "1"


_FOLDABLE = {}  # (shape, padding) -> the kernels' answer (asked once per geometry)


def foldable(z, layer):
    """Can ``layer`` (models.layers.DepthwiseConv2d) consume BN + ReLU of ``z`` folded?"""
    if not (ENABLED and on_gpu(z) and z.dtype == torch.bfloat16 and layer.k == 3
            and layer.stride == (1, 1) and layer.dilation == (1, 1) and not layer.relu
            and layer.bias is None and z.shape[-1] % 8 == 0):
        return False
    from ..models.layers import resolve_padding
    pad = resolve_padding(layer.padding, z.shape[1], z.shape[2], 3, 3, layer.stride,
                          layer.dilation)
    if pad[0] != pad[1] or pad[2] != pad[3]:
        return False
    key = (tuple(z.shape), pad)
    ok = _FOLDABLE.get(key)
    if ok is None:
        w = torch.empty((3, 3, z.shape[-1]), dtype=torch.bfloat16, device="meta")
        ok = _FOLDABLE[key] = bool(ext().dwconv_aff_ok(z, w, 1, 1, pad[0], pad[2], 1, 1))
    return ok


class _BNActDwFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, stats_z, gamma, beta, weight, bn, pad, want_stats):
        C = z.shape[-1]
        count = z.numel() // C
        if stats_z is None or stats_z.numel() == 0:
            stats_z = bn_stats(z)
        gp, bp = _phys_params(bn, gamma, beta)
        coef = bn_finalize(stats_z, count, gp, bp, bn.running_mean, bn.running_var, bn.decay,
                           bn.eps, True)
        w = compute_weight(weight, z.dtype)
        y = torch.empty_like(z)
        stats = workspace.zeros((2, C), z.device) if want_stats else None
        fused = ext().dwconv_fwd(z, w, None, y, 1, 1, pad[0], pad[1], 1, 1, False, False, stats,
                                 aff=coef)
        if want_stats and not fused:
            bn_stats(y, stats)
        ctx.bn, ctx.pad, ctx.count = bn, pad, count
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
            return (None,) * 8
        dy = dy.contiguous()
        bn, pad = ctx.bn, ctx.pad
        C = z.shape[-1]
        w = compute_weight(weight, dy.dtype)
        dz = None
        if ctx.needs_input_grad[0]:
            gu = torch.empty_like(z)
            red = workspace.zeros((2, C), dy.device)
            fused = ext().dwconv_dgrad(dy, w, gu, 1, 1, pad[0], pad[1], 1, 1, None, z, red,
                                       aff=coef)
            red_raw = bool(fused)
            if not fused:  # (the mask is applied either way)
                red = bn_bwd_reduce(gu, None, z, coef, 0)
            want_g = gamma is not None and gamma.requires_grad
            want_b = beta.requires_grad
            gt, gfresh = _grad_target_phys(gamma, C) if want_g else (None, False)
            bt, bfresh = _grad_target_phys(beta, C) if want_b else (None, False)
            direct_g = gt is not None and gfresh
            direct_b = bt is not None and bfresh
            gp, _ = _phys_params(bn, gamma, beta)
            dz, _ = bn_bwd_apply(gu, None, z, coef, red, gp, ctx.count, 0, False,
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
            wt, wfresh = grad_target(weight)
            direct = wt is not None
            dw = wt if direct else workspace.zeros(tuple(weight.shape), dy.device)
            ext().dwconv_wgrad(dy, z, dw, None, 1, 1, pad[0], pad[1], 1, 1, False,
                               not (direct and wfresh), aff=coef)
            if direct:
                deliver_grad(weight, written=True)
            else:
                deliver_grad(weight, dw)
        return dz, None, None, None, None, None, None, None


def bn_act_dw(src: DeferredBNAct, layer, want_stats=False):
    """``layer(relu(BN(z)))`` for the deferred training BN ``src`` feeding the depthwise conv
    ``layer`` — folded when :func:`foldable`, else applied first.  Returns ``(y, stats)`` like
    ``layer(..., want_stats=True)`` (stats None unless ``want_stats``)."""
    z, bn = src.z, src.bn
    if not foldable(z, layer):
        x = src.materialize()
        if want_stats:
            return layer(x, want_stats=True)
        return layer(x), None
    from ..models.layers import resolve_padding
    p = resolve_padding(layer.padding, z.shape[1], z.shape[2], 3, 3, layer.stride, layer.dilation)
    y, st = _BNActDwFn.apply(z, src.stats, bn.gamma, bn.beta, layer.weight, bn, (p[0], p[2]),
                             bool(want_stats))
    return y, (st if want_stats else None)
