"""Depthwise k×k convolution (depth_multiplier 1), NHWC, weights [R, S, C], dilation/stride/
explicit padding, optional fused bias + ReLU.

GPU kernels (``csrc/kernels/dwconv.hip``): memory-bound, so no MFMA — each thread owns 8 channels
(one 16-B bf16 vector) of one output pixel; the wgrad is a per-(r, s, c-vector) reduction over
N·Ho·Wo with a per-block partial + fp32 atomic, bias-grad fused.

Reference parity: ``slim.separable_conv2d(num_outputs=None)`` (core/layers.py:34-42,
core/xception.py:90-110) and the fixed Laplacian of preprocessing.py:11-30.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .common import on_gpu, ext, compute_weight, grad_target, deliver_grad, export_impl
from .bn import bn_stats
from . import gradjoin
from . import workspace
from .conv import ConvGeom


def ref_dw_fwd(x, w, geom: ConvGeom, bias=None):
    C = x.shape[-1]
    pt, pb, pl, pr = geom.padding
    xt = F.pad(x.permute(0, 3, 1, 2).float(), (pl, pr, pt, pb))
    wt = w.float().permute(2, 0, 1).unsqueeze(1)  # [C,1,R,S]
    y = F.conv2d(xt, wt, None if bias is None else bias.float(), stride=geom.stride,
                 dilation=geom.dilation, groups=C)
    return y.permute(0, 2, 3, 1).contiguous()


# TDL_DW_STATS (default 1): the depthwise tile kernels fuse the neighbouring BNs' statistics
# (forward Σy, Σy²; dgrad Σg, Σg·x_bn with the ReLU mask applied as x > 0) instead of the BNs'
# reduce passes.  Round 3 (8-channel lanes) it lost: 2578 / 2577 img/s on vs 2595 / 2604 off;
# round 4 (LDS-DMA staging, 4-channel lanes) it wins narrowly: Xception-41 299² b128 2763 / 2765
# on vs 2761 / 2755 off (same box, alternating runs)
DW_STATS = os.environ.get("TDL_DW_STATS", "1") == "1"


def _fusable_relu_in(x, R, S):
    """The bf16 kernels fold an input ReLU into their loads for 3×3 filters on 8-channel vectors
    (the fp32 path applies it as a separate pass)."""
    return x.shape[-1] % 8 == 0 and R * S == 9 and x.dtype != torch.float32


def joinable(x, relu_in, R=3, S=3):
    """Can the depthwise backward take part in a residual-gradient join on ``x`` (ops/gradjoin.py:
    its dgrad adds the join buffer's earlier contribution in its epilogue)?  Not when an input
    ReLU it cannot fuse turns ``x`` into a separate tensor first."""
    return not relu_in or not on_gpu(x) or _fusable_relu_in(x, R, S)


class _DwConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, geom, relu, relu_in, want_stats, join=None):
        w = compute_weight(weight, x.dtype)
        N, H, W, C = x.shape
        R, S, _ = w.shape
        Ho, Wo = geom.out_hw(H, W, R, S)
        stats = workspace.zeros((2, C), x.device) if want_stats else None
        if on_gpu(x):
            y = torch.empty((N, Ho, Wo, C), device=x.device, dtype=x.dtype)
            fused = ext().dwconv_fwd(x, w, None if bias is None else bias.detach(), y,
                                     geom.stride[0], geom.stride[1], geom.padding[0],
                                     geom.padding[2], geom.dilation[0], geom.dilation[1],
                                     bool(relu), bool(relu_in), stats if DW_STATS else None)
            if want_stats and not fused:  # strided / dilated row kernels: a reduce pass
                bn_stats(y, stats)
        else:
            y = ref_dw_fwd(torch.relu(x) if relu_in else x, w, geom,
                           None if bias is None else bias.detach())
            if relu:
                y = torch.relu(y)
            y = y.to(x.dtype)
            if want_stats:
                bn_stats(y, stats)
        ctx.geom, ctx.relu, ctx.relu_in = geom, relu, relu_in
        ctx.join = join
        # the mask token of the BN that produced x (ops/gradjoin.py): this dgrad may mask by
        # x > 0 and fuse that BN's backward statistics
        ctx.bn_tok = getattr(x, "_tdl_mask_token", None)
        ctx.save_for_backward(x, weight, bias, y if relu else None)
        if stats is None:
            stats = torch.empty(0, device=x.device)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        x, weight, bias, y = ctx.saved_tensors
        geom = ctx.geom
        if dy is None:
            return (None,) * 8
        dy = dy.contiguous()
        if on_gpu(dy):
            if ctx.relu:
                g = torch.empty_like(dy)
                ext().relu_bwd(dy, y, g)
            else:
                g = dy
            w = compute_weight(weight, dy.dtype)
            dx = None
            if ctx.needs_input_grad[0]:
                join, ctx.join = ctx.join, None
                # residual-gradient join: the other consumer of x already wrote its gradient —
                # accumulate onto it in place (the kernel adds it in its epilogue)
                dadd = join.buf if join is not None else None
                dx = dadd if dadd is not None else torch.empty_like(x)
                R, S = weight.shape[0], weight.shape[1]
                tok, ctx.bn_tok = ctx.bn_tok, None
                # x is a BN output: its ReLU mask is x > 0 (the stored y), so this dgrad can apply
                # it through the relu_in mask path, and the tile kernel can accumulate that BN's
                # backward sums (Σg, Σg·x_bn) in its epilogue (ops/gradjoin.py)
                use_tok = (DW_STATS and tok is not None and tok.x is not None and join is None
                           and gradjoin.STATS_SINGLE and _fusable_relu_in(x, R, S))
                masked = ctx.relu_in or (use_tok and (tok.relu_y or tok.mask is not None))
                red = workspace.zeros((2, x.shape[-1]), dy.device) if use_tok else None
                fused = ext().dwconv_dgrad(g, w, dx, geom.stride[0], geom.stride[1],
                                           geom.padding[0], geom.padding[2], geom.dilation[0],
                                           geom.dilation[1], x if masked else None,
                                           tok.x if use_tok else None, red, dadd=dadd)
                if use_tok:
                    tok.mark(dx, red if fused else None)
                if join is not None:
                    if join.buf is None:
                        join.buf = dx
                    join.note(False)
                    dx = join.take()
            # straight into the flat gradient buffer (overwrite on the step's first contribution)
            # when the parameters are flat-backed; otherwise pre-zeroed slices of the per-step
            # arena (one fill per step) that deliver_grad copies out
            want_b = bias is not None and bias.requires_grad
            wt, wfresh = grad_target(weight) if weight.requires_grad else (None, False)
            bt, bfresh = grad_target(bias) if want_b else (None, wfresh)
            direct = (wt is not None and (not want_b or (bt is not None and bfresh == wfresh))
                      and (bias is None or want_b))
            if direct:
                dw, db = wt, (bt if want_b else None)
            else:
                dw = workspace.zeros(tuple(weight.shape), dy.device)
                db = workspace.zeros((x.shape[-1],), dy.device) if bias is not None else None
            ext().dwconv_wgrad(g, x, dw, db, geom.stride[0], geom.stride[1], geom.padding[0],
                               geom.padding[2], geom.dilation[0], geom.dilation[1],
                               bool(ctx.relu_in), not (direct and wfresh))
            if direct:
                deliver_grad(weight, written=True)
                if want_b:
                    deliver_grad(bias, written=True)
                return dx, None, None, None, None, None, None, None
        else:
            xr = x.detach().float().requires_grad_(True)
            wr = weight.detach().float().requires_grad_(True)
            br = bias.detach().float().requires_grad_(True) if bias is not None else None
            with torch.enable_grad():
                yr = ref_dw_fwd(torch.relu(xr) if ctx.relu_in else xr, wr, geom, br)
                if ctx.relu:
                    yr = torch.relu(yr)
                grads = torch.autograd.grad(yr, [xr, wr] + ([br] if br is not None else []),
                                            dy.float())
            dx = grads[0].to(x.dtype)
            dw = grads[1]
            db = grads[2] if br is not None else None
            join, ctx.join = ctx.join, None
            if join is not None:
                if join.buf is None:
                    join.buf = dx
                else:
                    join.buf += dx
                join.note(False)
                dx = join.take()
        if weight.requires_grad:
            deliver_grad(weight, dw)
        if bias is not None and bias.requires_grad:
            deliver_grad(bias, db)
        return dx, None, None, None, None, None, None, None


def depthwise_conv2d(x, weight, bias=None, geom: ConvGeom = ConvGeom(), relu=False,
                     relu_in=False, want_stats=False, join=None):
    """``relu_in``: convolve max(x, 0) without materialising it (Xception's pre-activation ReLU
    in front of each separable conv, core/xception.py:90-110); the backward masks dx by x > 0.
    ``want_stats``: also return fp32 [2, C] = (Σy, Σy²) of the stored output for the BN that
    normalises it (fused into the stride-1 tile kernel's epilogue) — returns ``(y, stats)``."""
    ex = export_impl()
    if ex is not None and not want_stats:
        w = compute_weight(weight, x.dtype)
        return ex.dwconv2d(x, w, None if bias is None else bias.detach().float(), geom, relu,
                           relu_in)
    if relu_in and on_gpu(x) and not _fusable_relu_in(x, weight.shape[0], weight.shape[1]):
        if join is not None:
            raise ValueError("depthwise_conv2d: a join on x needs the fused input ReLU "
                             "(see joinable())")
        from .elementwise import relu as relu_op
        x, relu_in = relu_op(x), False
    y, stats = _DwConvFn.apply(x, weight, bias, geom, relu, relu_in, bool(want_stats), join)
    return (y, stats) if want_stats else y


def laplace(x):
    """2-D Laplacian of a single-channel NHWC image batch, SAME zero padding
    (preprocessing.py:11-30; kernel [[.5,1,.5],[1,-6,1],[.5,1,.5]])."""
    k = torch.tensor([[0.5, 1.0, 0.5], [1.0, -6.0, 1.0], [0.5, 1.0, 0.5]], dtype=torch.float32,
                     device=x.device).view(3, 3, 1).expand(3, 3, x.shape[-1]).contiguous()
    geom = ConvGeom((1, 1), (1, 1, 1, 1), (1, 1))
    if on_gpu(x):
        with torch.no_grad():
            return depthwise_conv2d(x, k.to(x.dtype), None, geom, False)
    return ref_dw_fwd(x, k, geom).to(x.dtype)
