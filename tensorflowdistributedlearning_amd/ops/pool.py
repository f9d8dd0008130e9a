"""Pooling ops, NHWC.

* ``max_pool2d`` — k×k / stride s with explicit (top, bottom, left, right) padding (TF 'SAME' or
  PyTorch-style symmetric).  The forward stores the in-window argmax (uint8) so the backward is a
  deterministic gather (every input pixel sums the ≤⌈k/s⌉² windows that picked it), not a scatter.
  Reference: ``slim.max_pool2d(3, stride=2, padding='SAME')`` (core/resnet.py:241) and
  ``resnet_utils.subsample`` (1×1 max-pool stride s, core/resnet.py:73,81,128,140, K10).
* ``global_avg_pool`` — mean over H, W → [N, C].  Reference: ``tf.reduce_mean(net, [1,2])``
  (core/resnet.py:247,464, K12).

GPU kernels: ``csrc/kernels/pool.hip``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .common import on_gpu, ext, export_impl
from . import gradjoin
from . import workspace

import os

POOL_STATS = os.environ.get("TDL_POOL_BNSTAT", "1") == "1"  # 0: the stem BN reduces itself


def _out(size, k, s, pb, pa):
    return (size + pb + pa - k) // s + 1


def ref_max_pool(x, k, s, pad):
    pt, pb, pl, pr = pad
    xt = x.permute(0, 3, 1, 2).float()
    xt = F.pad(xt, (pl, pr, pt, pb), value=float("-inf"))
    y = F.max_pool2d(xt, k, s)
    return y.permute(0, 2, 3, 1).contiguous()


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        N, H, W, C = x.shape
        Ho = _out(H, k, s, pad[0], pad[1])
        Wo = _out(W, k, s, pad[2], pad[3])
        ctx.k, ctx.s, ctx.pad, ctx.x_shape = k, s, pad, tuple(x.shape)
        # ReLU-mask token of the producing BN (ops/gradjoin.py): the backward applies the mask
        # and fuses that BN's backward sums (the ResNet stem: BN+ReLU → max-pool)
        ctx.bn_tok = getattr(x, "_tdl_mask_token", None)
        if on_gpu(x):
            y = torch.empty((N, Ho, Wo, C), device=x.device, dtype=x.dtype)
            idx = torch.empty((N, Ho, Wo, C), device=x.device, dtype=torch.uint8)
            ext().maxpool_fwd(x, y, idx, k, s, pad[0], pad[2])
            ctx.save_for_backward(idx)
            return y
        xr = x.detach().float().requires_grad_(True)
        with torch.enable_grad():
            yr = ref_max_pool(xr, k, s, pad)
        ctx.save_for_backward(xr, yr)
        return yr.detach().to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        if on_gpu(dy):
            (idx,) = ctx.saved_tensors
            dx = torch.empty(ctx.x_shape, device=dy.device, dtype=dy.dtype)
            tok, ctx.bn_tok = ctx.bn_tok, None
            if (tok is not None and tok.x is not None and tok.mask is not None
                    and gradjoin.STATS_SINGLE and POOL_STATS):
                red = workspace.zeros((2, ctx.x_shape[-1]), dy.device)
                if ext().maxpool_bwd_stats(dy, idx, dx, ctx.k, ctx.s, ctx.pad[0], ctx.pad[2],
                                           tok.x, tok.mask, red):
                    tok.mark(dx, red)
                    return dx, None, None, None
            ext().maxpool_bwd(dy, idx, dx, ctx.k, ctx.s, ctx.pad[0], ctx.pad[2])
            return dx, None, None, None
        xr, yr = ctx.saved_tensors
        (g,) = torch.autograd.grad(yr, xr, dy.float())
        return g.to(dy.dtype), None, None, None


def max_pool2d(x, k, s, pad):
    ex = export_impl()
    if ex is not None:
        return ex.max_pool2d(x, k, s, tuple(pad))
    return _MaxPoolFn.apply(x, k, s, tuple(pad))


# the ResNet stem's BN + ReLU folded into its max-pool (bn_relu_max_pool); 0: apply pass + pool
STEM_FUSE = os.environ.get("TDL_STEM_POOL_FUSE", "1") == "1"
# its backward as BN sums per pool output + one gather-and-apply pass (0: gather pass writing g,
# then the BN backward apply)
FUSED_BWD = os.environ.get("TDL_STEM_POOL_FUSED_BWD", "1") == "1"


class _BNReluMaxPoolFn(torch.autograd.Function):
    """max_pool(relu(BN(z))) of a training BN in one pass over z (pool.hip bn_maxpool_fwd_kernel):
    the BN output — the largest activation of the network, 112×112×64 per ResNet image — is never
    written or read back.  The index bytes carry the ReLU bit of each window maximum, so the
    backward gather routes gradient only to positions the BN's ReLU passed, and accumulates the
    BN-backward sums (Σg, Σg·z) on the way (outside deterministic mode); the BN backward apply then
    produces dz.  Reference: the stem's conv + batch_norm(relu) + max_pool2d(3, 2, 'SAME')
    (/root/reference/core/resnet.py:238-241)."""

    @staticmethod
    def forward(ctx, z, stats, gamma, beta, bn, k, s, pad):
        from .bn import bn_stats, bn_finalize, _phys_params
        N, H, W, C = z.shape
        count = z.numel() // C
        if stats is None or stats.numel() == 0:
            stats = bn_stats(z)
        gp, bp = _phys_params(bn, gamma, beta)
        coef = bn_finalize(stats, count, gp, bp, bn.running_mean, bn.running_var, bn.decay,
                           bn.eps, True)
        Ho, Wo = _out(H, k, s, pad[0], pad[1]), _out(W, k, s, pad[2], pad[3])
        y = torch.empty((N, Ho, Wo, C), device=z.device, dtype=z.dtype)
        idx = torch.empty((N, Ho, Wo, C), device=z.device, dtype=torch.uint8)
        # z at each window's argmax: the two-pass fused backward (BN sums per pool output) reads
        # it; deterministic mode keeps the gather + reduce + apply backward
        zarg = (torch.empty_like(y) if FUSED_BWD and not ext().deterministic() else None)
        if not ext().bn_maxpool_fwd(z, coef, y, idx, k, s, pad[0], pad[2], zarg=zarg):
            raise RuntimeError("bn_relu_max_pool: channel count not a multiple of 8")
        ctx.k, ctx.s, ctx.pad, ctx.bn, ctx.count = k, s, pad, bn, count
        ctx.save_for_backward(z, idx, coef, gamma, beta, zarg)
        return y

    @staticmethod
    def backward(ctx, dy):
        from .bn import (bn_bwd_reduce, bn_bwd_apply, bn_red_xhat, _phys_params,
                         _grad_target_phys)
        from .common import deliver_grad
        z, idx, coef, gamma, beta, zarg = ctx.saved_tensors
        dy = dy.contiguous()
        C, c = z.shape[-1], beta.numel()
        red = workspace.zeros((2, C), dy.device)
        want_g = gamma is not None and gamma.requires_grad
        want_b = beta.requires_grad
        gt, gfresh = _grad_target_phys(gamma, C) if want_g else (None, False)
        bt, bfresh = _grad_target_phys(beta, C) if want_b else (None, False)
        direct_g, direct_b = gt is not None and gfresh, bt is not None and bfresh
        gp, _ = _phys_params(ctx.bn, gamma, beta)
        if zarg is not None:
            # two passes: (Σg, Σg·z) per pool output from zarg, then the gather + BN backward
            # apply per input pixel — g is never written
            dz = torch.empty_like(z)
            dg = gt if direct_g else (torch.empty(C, device=z.device) if want_g else None)
            db = bt if direct_b else (torch.empty(C, device=z.device) if want_b else None)
            if ext().maxpool_bn_bwd(dy, idx, zarg, z, coef, red,
                                    gp.detach().float().contiguous() if gp is not None else None,
                                    dz, dg, db, float(ctx.count), ctx.k, ctx.s, ctx.pad[0],
                                    ctx.pad[2]):
                if want_g:
                    deliver_grad(gamma, None if direct_g else dg[:c], written=direct_g)
                if want_b:
                    deliver_grad(beta, None if direct_b else db[:c], written=direct_b)
                return dz, None, None, None, None, None, None, None
            red.zero_()
        g = torch.empty_like(z)
        fused = ext().maxpool_bwd_rb(dy, idx, g, ctx.k, ctx.s, ctx.pad[0], ctx.pad[2], z, red)
        if not fused:
            red = bn_bwd_reduce(g, None, z, coef, 0)  # (Σg, Σg·ẑ), deterministic mode
        dz, _ = bn_bwd_apply(g, None, z, coef, red, gp, ctx.count, 0, False,
                             gt if direct_g else None, bt if direct_b else None, red_raw=fused)
        if fused and want_g and not direct_g:
            red = bn_red_xhat(red, coef)
        if want_g:
            deliver_grad(gamma, None if direct_g else red[1][:c], written=direct_g)
        if want_b:
            deliver_grad(beta, None if direct_b else red[0][:c], written=direct_b)
        return dz, None, None, None, None, None, None, None


def bn_relu_max_pool_ok(z, bn):
    """Can max_pool(relu(BN(z))) of this training BN run as one fused pass?"""
    from .common import fused_gpu
    return (STEM_FUSE and fused_gpu(z) and z.dtype == torch.bfloat16 and z.shape[-1] % 8 == 0
            and export_impl() is None and torch.is_grad_enabled()
            and not getattr(bn, "emit_fp8", False))


def bn_relu_max_pool(z, stats, bn, k, s, pad):
    """max_pool2d(relu(BN(z)), k, s, pad) for a training-mode ``bn`` (models.layers.BatchNorm)
    with the producer's BN sums ``stats`` — see :class:`_BNReluMaxPoolFn`."""
    return _BNReluMaxPoolFn.apply(z, stats, bn.gamma, bn.beta, bn, k, s, tuple(pad))


class _GAPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, keepdims, join=None):
        N, H, W, C = x.shape
        ctx.x_shape = tuple(x.shape)
        ctx.keepdims = keepdims
        ctx.join = join
        if on_gpu(x):
            y = torch.empty((N, C), device=x.device, dtype=x.dtype)
            ext().avgpool_fwd(x, y)
        else:
            y = x.float().mean(dim=(1, 2)).to(x.dtype)
        return y.view(N, 1, 1, C) if keepdims else y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.x_shape
        dy = dy.reshape(N, C).contiguous()
        join, ctx.join = ctx.join, None
        if on_gpu(dy):
            # residual-gradient join (ops/gradjoin.py): add the earlier contributions in place
            dadd = join.buf if join is not None else None
            dx = dadd if dadd is not None else torch.empty(ctx.x_shape, device=dy.device,
                                                           dtype=dy.dtype)
            ext().avgpool_bwd(dy, dx, dadd)
        else:
            dx = (dy.float() / (H * W)).view(N, 1, 1, C).expand(N, H, W, C).to(dy.dtype)
            if join is not None and join.buf is not None:
                join.buf += dx
                dx = join.buf
            else:
                dx = dx.contiguous()
        if join is not None:
            join.buf = dx
            join.note(False)
            dx = join.take()
        return dx, None, None


def global_avg_pool(x, keepdims=False, join=None):
    """Mean over H, W.  ``join``: gradient join of x (ops/gradjoin.py; the backward adds the
    join buffer's earlier contributions, C % 8 == 0 on the GPU)."""
    ex = export_impl()
    if ex is not None:
        return ex.avg_pool(x, keepdims)
    return _GAPFn.apply(x, keepdims, join)
