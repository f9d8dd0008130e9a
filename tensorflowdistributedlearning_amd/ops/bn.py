"""Batch normalisation (training: batch statistics + moving averages; eval: moving statistics)
fused with the optional residual add and ReLU, NHWC.

GPU kernels (``csrc/kernels/bn.hip``):
  * ``bn_stats``       per-channel Σx, Σx² (only when the producing conv did not already
                       accumulate them in its epilogue — see ``conv2d(want_stats=True)``);
  * ``bn_finalize``    mean / invstd / scale / shift + moving-average update in one tiny launch;
  * ``bn_apply``       y = act(x·scale + shift [+ residual]) — one vectorised pass;
  * ``bn_bwd_reduce``  Σg, Σg·x̂ with g = dy·[y>0] — skipped when the consumer conv's dgrad
                       epilogue already accumulated (Σg, Σg·x) (ops/gradjoin.py, fused statistics);
  * ``bn_bwd_apply``   dx = γ·invstd·(g − Σg/M − x̂·Σg·x̂/M), plus g for the residual branch.

Reference parity: ``slim.batch_norm`` under ``resnet_arg_scope`` (core/resnet.py:357-395,71,126,242)
with ``UPDATE_OPS`` moving averages (model.py:465-467) — TF FusedBatchNorm/FusedBatchNormGrad
(SURVEY N4, N5, K6, K8, K19).  Moving average: ``m ← decay·m + (1−decay)·batch`` (TF convention,
``decay`` = BATCH_NORM_DECAY); the moving variance uses the unbiased batch variance.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .common import on_gpu, fused_gpu, ext, deliver_grad, grad_target, flat_view, export_impl
from . import workspace
from . import gradjoin


# ----------------------------------------------------------------------------------------------
# raw ops
# ----------------------------------------------------------------------------------------------

def bn_stats(x, stats=None):
    C = x.shape[-1]
    if stats is None:
        stats = workspace.zeros((2, C), x.device)
    if on_gpu(x):
        ext().bn_stats(x, stats)
        return stats
    xf = x.float().reshape(-1, C)
    stats[0] += xf.sum(0)
    stats[1] += (xf * xf).sum(0)
    return stats


def bn_finalize(stats, count, gamma, beta, running_mean, running_var, decay, eps, training):
    """Returns fp32 [4, C] = (scale, shift, mean, invstd); updates moving stats in training.
    ``gamma``/``beta`` may be channel-padded (C physical channels) while the moving statistics
    cover the first ``running_mean.numel()`` (logical) channels only."""
    C = beta.shape[0]
    cr = running_mean.numel()
    if on_gpu(beta):
        coef = torch.empty((4, C), device=beta.device, dtype=torch.float32)
        ext().bn_finalize(stats if training else None, coef, gamma, beta, running_mean, running_var,
                          float(count), float(decay), float(eps), bool(training))
        return coef
    g = gamma.detach().float() if gamma is not None else torch.ones_like(beta)
    if training:
        mean = stats[0] / count
        var = (stats[1] / count - mean * mean).clamp_min(0.0)
        with torch.no_grad():
            unbiased = var * (count / max(count - 1, 1))
            running_mean.mul_(decay).add_((1 - decay) * mean[:cr])
            running_var.mul_(decay).add_((1 - decay) * unbiased[:cr])
    else:
        mean = torch.nn.functional.pad(running_mean.float(), (0, C - cr))
        var = torch.nn.functional.pad(running_var.float(), (0, C - cr), value=1.0)
    invstd = torch.rsqrt(var + eps)
    scale = g * invstd
    shift = beta.detach().float() - mean * scale
    return torch.stack([scale, shift, mean, invstd])


def bn_apply(x, coef, residual=None, relu=True, fp8=None, mask=None, out=None, store_y=True):
    """``out``: write y there instead (e.g. a channel slice ``buf[..., c0:c0+C]`` of a wider
    NHWC concat buffer — the kernel takes its pixel stride; no fp8 side output then).
    ``fp8`` = (amax_ring fp32[3], phase, scale fp32[1], emit): also write an e4m3 copy of y
    scaled by the previous call's |y|max (delayed scaling) — returned as ``y._tdl_fp8`` =
    (y8, scale) for an fp8 consumer conv (ops/conv.py) when ``emit``.  ``mask`` (uint8
    [numel/8], GPU): also write the ReLU mask y > 0 as one bit per element (relu mode 3).
    ``store_y=False`` (with an emitted e4m3 copy): y is NOT written — an fp8-only output whose
    every consumer reads ``y._tdl_fp8`` (models.enable_fp8 marks such BNs ``fp8_only``); the
    returned y is then an unwritten buffer carrying the shape and the attributes."""
    if out is not None and fp8 is not None:
        raise ValueError("bn_apply: no fp8 side output into a strided destination")
    if on_gpu(x):
        y = torch.empty_like(x) if out is None else out
        if fp8 is None:
            ext().bn_apply(x, coef, residual, y, bool(relu), mask=mask)
            return y
        ring, phase, scale, emit = fp8
        y8 = torch.empty(x.shape, device=x.device, dtype=torch.float8_e4m3fn) if emit else None
        ext().bn_apply(x, coef, residual, y, bool(relu), y8.view(torch.uint8) if emit else None,
                       ring, int(phase), scale, mask, store_y=bool(store_y or not emit))
        if emit:
            y._tdl_fp8 = (y8, scale)
        return y
    C = x.shape[-1]
    y = x.float() * coef[0].view(*([1] * (x.dim() - 1)), C) + coef[1]
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    if out is not None:
        out.copy_(y)
        return out
    return y.to(x.dtype)


def unpack_relu_mask(mask, C):
    """[M, C] bool from the 1-bit-per-element mask of relu mode 3 (bit j of byte i = element
    8·i + j)."""
    bits = torch.arange(8, device=mask.device, dtype=torch.uint8)
    return ((mask.view(-1, 1) >> bits) & 1).bool().reshape(-1, C)


def _relu_mask(relu, y, x, coef, C):
    """ReLU mask of the BN output: from y (relu=True / 1), or — without residual — recomputed as
    x·scale + shift > 0 (relu=2) so the backward never reads y, or unpacked from the bit mask the
    forward wrote (relu=3, ``y`` is then that uint8 mask)."""
    if relu == 2:
        return (x.float().reshape(-1, C) * coef[0] + coef[1]) > 0
    if relu == 3:
        return unpack_relu_mask(y, C)
    return y.float().reshape(-1, C) > 0


def bn_bwd_reduce(dy, y, x, coef, relu):
    """fp32 [2, C]: (Σg, Σg·x̂), g = dy·mask if relu else dy (relu: 0/False, 1/True = mask from y,
    2 = mask from x·scale+shift)."""
    C = x.shape[-1]
    if on_gpu(dy):
        red = workspace.zeros((2, C), dy.device)
        ext().bn_bwd_reduce(dy, y, x, coef, red, int(relu))
        return red
    g = dy.float().reshape(-1, C)
    if relu:
        g = g * _relu_mask(relu, y, x, coef, C)
    xhat = (x.float().reshape(-1, C) - coef[2]) * coef[3]
    return torch.stack([g.sum(0), (g * xhat).sum(0)])


PAIR_STATS = os.environ.get("TDL_BNSTAT_PAIR", "1") == "1"


def bn_bwd_reduce2(dy, x, coef, x2):
    """Backward sums of two BNs fed the same gradient ``dy`` (no mask): ((Σdy, Σdy·x̂) of ``x``,
    (Σdy, Σdy·x2) raw) — the residual BN of a downsampling bottleneck and its shortcut BN, in
    one pass that reads dy once.  None when the kernel does not take the shape."""
    C = x.shape[-1]
    if on_gpu(dy):
        red = workspace.zeros((2, C), dy.device)
        red2 = workspace.zeros((2, C), dy.device)
        if not ext().bn_bwd_reduce2(dy, x, x2, coef, red, red2):
            return None
        return red, red2
    g = dy.float().reshape(-1, C)
    xhat = (x.float().reshape(-1, C) - coef[2]) * coef[3]
    return (torch.stack([g.sum(0), (g * xhat).sum(0)]),
            torch.stack([g.sum(0), (g * x2.float().reshape(-1, C)).sum(0)]))


def bn_red_xhat(red, coef):
    """(Σg, Σg·x̂) from the raw (Σg, Σg·x) a fused dgrad epilogue accumulated:
    Σg·x̂ = invstd·(Σg·x − mean·Σg)."""
    return torch.stack([red[0], coef[3] * (red[1] - coef[2] * red[0])])


def bn_bwd_apply(dy, y, x, coef, red, gamma, count, relu, want_dres, dgamma=None, dbeta=None,
                 fp8=None, red_raw=False, dadd=None, fp8_only=False):
    """dx (same dtype as x) and optionally the masked gradient g for the residual branch.
    On the GPU, ``dgamma``/``dbeta`` (fp32 [C]) receive Σg·x̂ / Σg from the same launch.
    ``red_raw``: ``red`` holds (Σg, Σg·x) from a fused dgrad epilogue (:func:`bn_red_xhat`).
    ``fp8`` = (amax_ring, phase, scale, emit): also write an e5m2 copy of dx with delayed scaling
    (16× headroom over the previous call's |dx|max: fp8_policy) — attached as ``dx._tdl_fp8`` = (dx8, scale)
    for the fp8 dgrad of the producing conv.  ``dadd`` (shaped like x): another gradient of x
    added to dx in the same pass.  ``fp8_only`` (with an emitting ``fp8``): write only the e5m2
    copy — the returned bf16 dx is an unwritten placeholder carrying it (every reader of this
    gradient is the producing conv's fp8 dgrad / weight gradient)."""
    C = x.shape[-1]
    if on_gpu(dy):
        dx = torch.empty_like(x)
        dres = torch.empty_like(dy) if want_dres else None
        if fp8 is None:
            ext().bn_bwd_apply(dy, y, x, coef, red, gamma, dx, dres, dgamma, dbeta, float(count),
                               int(relu), red_raw=bool(red_raw), dadd=dadd)
            return dx, dres
        ring, phase, scale, emit = fp8
        dx8 = torch.empty(x.shape, device=x.device, dtype=torch.float8_e5m2) if emit else None
        ext().bn_bwd_apply(dy, y, x, coef, red, gamma, dx, dres, dgamma, dbeta, float(count),
                           int(relu), dx8.view(torch.uint8) if emit else None, ring, int(phase),
                           scale, red_raw=bool(red_raw), dadd=dadd,
                           store_dx=not (fp8_only and emit and C % 8 == 0))
        if emit:
            dx._tdl_fp8 = (dx8, scale)
        return dx, dres
    if red_raw:
        red = bn_red_xhat(red, coef)
    g = dy.float().reshape(-1, C)
    if relu:
        g = g * _relu_mask(relu, y, x, coef, C)
    xhat = (x.float().reshape(-1, C) - coef[2]) * coef[3]
    gam = gamma.detach().float() if gamma is not None else torch.ones(C)
    k = gam * coef[3]
    dx = k * (g - red[0] / count - xhat * red[1] / count)
    if dadd is not None:
        dx = dx + dadd.float().reshape(-1, C)
    dres = g.reshape(dy.shape).to(dy.dtype) if want_dres else None
    return dx.reshape(x.shape).to(x.dtype), dres


# ----------------------------------------------------------------------------------------------
# autograd
# ----------------------------------------------------------------------------------------------

class ResidualLink:
    """Hands the residual-path gradient of a tensor x to the BN that normalises x, so the BN
    backward adds it to its dx in the same pass (``bn_bwd_apply(dadd=…)``) instead of autograd
    summing the two gradients (a DeepLab unit input feeds its pre-activation BN and, as the
    identity shortcut, conv3's residual epilogue).  Order independent: whichever backward runs
    second sees the other's state — a residual gradient arriving after the BN backward already
    ran is returned to autograd as usual."""
    __slots__ = ("g", "bn_done")

    def __init__(self):
        self.g = None
        self.bn_done = False

    def offer(self, g):
        """Residual side: True if the BN will add ``g`` (return None to autograd then)."""
        if self.bn_done:
            return False
        self.g = g
        return True

    def take(self):
        """BN side: the residual gradient if it arrived first, else None (and mark done)."""
        g, self.g = self.g, None
        self.bn_done = True
        return g


class _BatchNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, stats, gamma, beta, residual, bn, relu, training, res_join, need_grad,
                link=None):
        C = x.shape[-1]
        count = x.numel() // C
        if training:
            if stats is None or stats.numel() == 0:
                stats = bn_stats(x)
        gp, bp = _phys_params(bn, gamma, beta)
        coef = bn_finalize(stats, count, gp, bp, bn.running_mean, bn.running_var,
                           bn.decay, bn.eps, training)
        fp8 = bn.fp8_state(x) if getattr(bn, "emit_fp8", False) else None
        # ReLU mask for the backward: without a residual it is recomputed from x (relu mode 2,
        # nothing saved); with one, the forward writes it as 1 bit per element (mode 3: the two
        # backward kernels read 1/16 of y's bytes instead of y itself)
        mask = None
        if relu and need_grad and fused_gpu(x) and C % 8 == 0 and C <= 2048 and (
                residual is not None or (C % 64 == 0 and gradjoin.STATS_ENABLED
                                         and gradjoin.MASK_ENABLED)):
            # without a residual only for the fused-statistics path: the consuming conv's dgrad
            # applies the mask and accumulates this BN's backward sums (ops/gradjoin.py)
            mask = torch.empty(x.numel() // 8, device=x.device, dtype=torch.uint8)
        # fp8-only output (models.enable_fp8): every consumer is an fp8 conv that reads the e4m3
        # copy and keeps it for its weight gradient — the bf16 y is not written
        # (no residual: the backward never saves y — relu mode 3 reads the bit mask, mode 2
        # recomputes from x; a ReLU without the mask would leave y > 0 to a depthwise consumer)
        fp8_only = (fp8 is not None and getattr(bn, "fp8_only", False) and residual is None
                    and (mask is not None or not relu))
        y = bn_apply(x, coef, residual, relu, fp8, mask, store_y=not fp8_only)
        if fp8_only:  # the bf16 bytes of y are unwritten: consumers must read y._tdl_fp8
            y._tdl_fp8_only = True
        ctx.mask_token = None
        if mask is not None:  # the consumers' dgrads may apply it for us (ops/gradjoin.py)
            ctx.mask_token = y._tdl_mask_token = gradjoin.MaskToken(mask, x)
        elif (not relu and residual is None and need_grad and fused_gpu(x) and PAIR_STATS
              and gradjoin.STATS_ENABLED):
            # no ReLU: a statistics-only token — the residual BN this output feeds (a shortcut
            # BN) computes both BNs' backward sums in one pass over the shared gradient, or the
            # consuming conv's dgrad fuses them
            ctx.mask_token = y._tdl_mask_token = gradjoin.MaskToken(None, x)
        elif relu and residual is None and need_grad and fused_gpu(x) and C % 8 == 0 \
                and gradjoin.STATS_ENABLED:
            # ReLU without a bit mask: a consuming depthwise dgrad masks by y > 0 itself
            ctx.mask_token = y._tdl_mask_token = gradjoin.MaskToken(None, x, relu_y=True)
        ctx.res_tok = None
        if residual is not None:
            rt = getattr(residual, "_tdl_mask_token", None)
            if rt is not None and rt.mask is None and not rt.relu_y and rt.x is not None:
                ctx.res_tok = rt
        ctx.count = count
        ctx.bn = bn
        ctx.training = training
        ctx.link = link
        ctx.has_res = residual is not None
        ctx.res_join = res_join if residual is not None else None
        ctx.relu = 0 if not relu else (3 if mask is not None else (2 if residual is None else 1))
        ctx.save_for_backward(x, mask if ctx.relu == 3 else (y if ctx.relu == 1 else None), coef,
                              gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, coef, gamma, beta = ctx.saved_tensors
        dy = dy.contiguous()
        relu = ctx.relu
        C = x.shape[-1]  # physical channels (≥ beta.numel() when channel-padded)
        c = beta.numel()
        premasked = ctx.mask_token is not None and ctx.mask_token.is_premasked(dy)
        if not ctx.training and not on_gpu(dy):
            # eval-mode backward (frozen BN): treat statistics as constants.  On the GPU this is
            # the training path's kernels with 1/count = 0 (no batch-statistics terms)
            g = dy.float().reshape(-1, C)
            if relu and not premasked:
                g = g * _relu_mask(relu, y, x, coef, C)
            dx = (g * coef[0]).reshape(x.shape).to(x.dtype)
            xhat = (x.float().reshape(-1, C) - coef[2]) * coef[3]
            if gamma is not None and gamma.requires_grad:
                deliver_grad(gamma, (g * xhat).sum(0)[:c])
            if beta.requires_grad:
                deliver_grad(beta, g.sum(0)[:c])
            dres = None
            if ctx.has_res:
                dres = dy if premasked else g.reshape(dy.shape).to(dy.dtype)
            if ctx.link is not None:
                extra = ctx.link.take()
                if extra is not None:
                    dx = (dx.float() + extra.float()).to(x.dtype)
            return dx, None, None, None, _join_res(ctx, dres), None, None, None, None, None, None
        # pre-masked: the block output's consumers already applied this ReLU's mask to dy
        # (ops/gradjoin.py) — no mask reads, and dy itself is the residual gradient
        if premasked:
            relu, y = 0, None
        # (Σg, Σg·x) fused into the last writer's dgrad epilogue, else a reduce pass
        red = ctx.mask_token.red if premasked else None
        red_raw = red is not None
        rt, ctx.res_tok = ctx.res_tok, None
        if red is None and premasked and rt is not None and rt.x is not None \
                and tuple(rt.x.shape) == tuple(x.shape):
            # the shortcut BN gets this same gradient (dres = dy): both sums in one pass
            pair = bn_bwd_reduce2(dy, x, coef, rt.x)
            if pair is not None:
                red = pair[0]
                rt.mark(dy, pair[1])
        if red is None:
            red = bn_bwd_reduce(dy, y, x, coef, relu)
        want_g = gamma is not None and gamma.requires_grad
        want_b = beta.requires_grad
        gt, gfresh = _grad_target_phys(gamma, C) if want_g else (None, False)
        bt, bfresh = _grad_target_phys(beta, C) if want_b else (None, False)
        direct_g = on_gpu(dy) and gt is not None and gfresh
        direct_b = on_gpu(dy) and bt is not None and bfresh
        gp, _ = _phys_params(ctx.bn, gamma, beta)
        count = ctx.count if ctx.training else float("inf")  # frozen BN: dx = γ·invstd·g
        fp8 = ctx.bn.fp8_bwd_state(x) if getattr(ctx.bn, "emit_fp8_bwd", False) else None
        extra = ctx.link.take() if ctx.link is not None else None
        fuse_add = extra is not None and tuple(extra.shape) == tuple(x.shape) and (
            not on_gpu(dy) or C % 8 == 0)
        dx, dres = bn_bwd_apply(dy, y, x, coef, red, gp, count, relu,
                                ctx.has_res and not premasked and relu != 0,
                                gt if direct_g else None, bt if direct_b else None, fp8=fp8,
                                red_raw=red_raw, dadd=extra.contiguous() if fuse_add else None,
                                fp8_only=getattr(ctx.bn, "fp8_bwd_only", False) and extra is None)
        if extra is not None and not fuse_add:
            dx = dx + extra
        if ctx.has_res and (premasked or relu == 0):
            dres = dy  # no mask to apply: the residual gradient is the incoming one, no copy
        if red_raw and want_g and not direct_g:
            red = bn_red_xhat(red, coef)
        if want_g:
            deliver_grad(gamma, None if direct_g else red[1][:c], written=direct_g)
        if want_b:
            deliver_grad(beta, None if direct_b else red[0][:c], written=direct_b)
        if ctx.mask_token is not None:
            ctx.mask_token.release()
        return dx, None, None, None, _join_res(ctx, dres), None, None, None, None, None, None


def _phys_params(bn, gamma, beta):
    """γ/β padded to the physical channel count of a channel-padded BN (models.layers.BatchNorm
    ``c_phys``); the parameters themselves otherwise."""
    if getattr(bn, "c_phys", None) not in (None, beta.numel()):
        return bn.phys_params()
    return gamma, beta


def _grad_target_phys(p, C):
    """grad_target for a gradient of C ≥ p.numel() channels: the flat gradient buffer's slack
    after p takes the padding channels (their gradient is exactly zero)."""
    t, fresh = grad_target(p)
    if t is not None and C != p.numel():
        t = flat_view(p, C, "grad")
    return t, fresh


def _join_res(ctx, dres):
    """Residual gradient into the block input's shared buffer (ops/gradjoin.py)."""
    join = ctx.res_join
    if join is None or dres is None:
        return dres
    if join.buf is None:
        join.buf = dres
    else:  # another consumer ran first (not the usual order): plain add
        join.buf.add_(dres)
    join.note(False)  # not masked (a later full-coverage masking dgrad re-masks everything)
    return join.take()


def eval_coef(bn, device):
    """fp32 [4, C_phys] (scale, shift, mean, invstd) of an eval-mode BN — bn_finalize's layout
    in plain tensor ops (traceable): y = x·scale + shift, zero on padding channels."""
    gamma, beta = bn.phys_params()
    C, c = beta.shape[0], bn.c
    mean = bn.running_mean.float().to(device)
    inv = torch.rsqrt(bn.running_var.float().to(device) + bn.eps)
    scale = inv * gamma[:c].float().to(device) if gamma is not None else inv
    shift = beta[:c].float().to(device) - mean * scale
    pad = (0, C - c)
    return torch.stack([F.pad(scale, pad), F.pad(shift, pad), F.pad(mean, pad), F.pad(inv, pad)])


def batch_norm_act(x, bn, stats=None, residual=None, relu=True, training=True, res_join=None,
                   link=None):
    """act(BN(x) [+ residual]).  ``bn`` is a :class:`models.layers.BatchNorm` (holds γ, β and the
    moving statistics).  ``stats`` may carry Σx, Σx² already accumulated by the producer conv.
    ``res_join`` shares the residual's gradient buffer with its other consumers; ``link``
    (:class:`ResidualLink`) adds x's residual-path gradient to dx in the backward pass."""
    ex = export_impl()
    if ex is not None:  # serving trace: eval-mode BN as one affine (+residual, ReLU) pass
        if training:
            raise RuntimeError("batch_norm_act: export needs the network in eval mode")
        coef = bn.__dict__.get("_serve")  # frozen by engine/serving.py
        return ex.bn_act(x, coef if coef is not None else eval_coef(bn, x.device), residual,
                         relu)
    # (grad mode is off inside Function.forward: decide here whether a backward will follow)
    need_grad = torch.is_grad_enabled() and (
        x.requires_grad or (residual is not None and residual.requires_grad))
    return _BatchNormActFn.apply(x, stats, bn.gamma, bn.beta, residual, bn, relu, training,
                                 res_join, need_grad, link)


# ----------------------------------------------------------------------------------------------
# BN(+ReLU) written straight into a channel slice of a concat buffer (concat-free ASPP / decoder)
# ----------------------------------------------------------------------------------------------

class _BatchNormActIntoFn(torch.autograd.Function):
    """``buf[..., c0:c0+C] = act(BN(x))`` in place, returning ``buf``: the DeepLab ASPP branches
    and the decoder's low-level features land in the consumer conv's input without a
    ``torch.cat`` pass (core/resnet.py:438-448,476-486 concatenate them).  The backward reads its
    branch's gradient as a strided slice of the concat gradient — no split copy — and passes that
    gradient on to the other writers.  The ReLU mask is recomputed from x (relu mode 2)."""

    @staticmethod
    def forward(ctx, buf, x, stats, gamma, beta, bn, c0, relu, training):
        C = x.shape[-1]
        count = x.numel() // C
        if training and (stats is None or stats.numel() == 0):
            stats = bn_stats(x)
        gp, bp = _phys_params(bn, gamma, beta)
        coef = bn_finalize(stats, count, gp, bp, bn.running_mean, bn.running_var,
                           bn.decay, bn.eps, training)
        bn_apply(x, coef, None, relu, out=buf[..., c0:c0 + C])
        ctx.mark_dirty(buf)
        ctx.count, ctx.bn, ctx.training, ctx.c0 = count, bn, training, c0
        ctx.relu = 2 if relu else 0
        ctx.save_for_backward(x, coef, gamma, beta)
        return buf

    @staticmethod
    def backward(ctx, gbuf):
        x, coef, gamma, beta = ctx.saved_tensors
        if gbuf.stride(-1) != 1 or not gbuf.is_contiguous():
            gbuf = gbuf.contiguous()
        C = x.shape[-1]
        dy = gbuf[..., ctx.c0:ctx.c0 + C]  # strided view: the kernels take the pixel stride
        if not on_gpu(dy):
            dy = dy.contiguous()
        red = bn_bwd_reduce(dy, None, x, coef, ctx.relu)
        want_g = gamma is not None and gamma.requires_grad
        want_b = beta.requires_grad
        gt, gfresh = _grad_target_phys(gamma, C) if want_g else (None, False)
        bt, bfresh = _grad_target_phys(beta, C) if want_b else (None, False)
        direct_g = on_gpu(dy) and gt is not None and gfresh
        direct_b = on_gpu(dy) and bt is not None and bfresh
        gp, _ = _phys_params(ctx.bn, gamma, beta)
        count = ctx.count if ctx.training else float("inf")
        dx, _ = bn_bwd_apply(dy, None, x, coef, red, gp, count, ctx.relu, False,
                             gt if direct_g else None, bt if direct_b else None)
        c = beta.numel()
        if want_g:
            deliver_grad(gamma, None if direct_g else red[1][:c], written=direct_g)
        if want_b:
            deliver_grad(beta, None if direct_b else red[0][:c], written=direct_b)
        return gbuf, dx, None, None, None, None, None, None, None


def batch_norm_act_into(buf, c0, x, bn, stats=None, relu=True, training=True):
    """``buf[..., c0:c0+C] = act(BN(x))`` (in place; returns ``buf`` for the autograd chain).
    ``x`` must not be channel-padded (its channels are the slice's channels)."""
    C = x.shape[-1]
    if C != bn.beta.numel() or buf.shape[:-1] != x.shape[:-1] or c0 + C > buf.shape[-1]:
        raise ValueError(f"batch_norm_act_into: x {tuple(x.shape)} into buf {tuple(buf.shape)} "
                         f"at channel {c0} (BN of {bn.beta.numel()} channels)")
    return _BatchNormActIntoFn.apply(buf, x, stats, bn.gamma, bn.beta, bn, c0, relu, training)
