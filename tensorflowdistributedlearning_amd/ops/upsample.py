"""The reference's ``_upsample``: 1-px SYMMETRIC pad → TF1 legacy ``resize_bilinear``
(align_corners=False, src = dst·in/out, no half-pixel) to (out+4) → crop [2:-2]
(core/layers.py:82-109).

The whole chain is one linear map per spatial axis, so the op is expressed as
``y[n, i, j, c] = Σ_a Σ_b Ah[i, a] · Aw[j, b] · x[n, a, b, c]`` where each row of Ah/Aw has at most
two non-zeros (the two bilinear taps, after folding the symmetric pad back onto the edge pixels).
GPU: ``csrc/kernels/upsample.hip`` evaluates the 4 taps per output vector (fwd) and the transposed
map as a gather over the taps' inverse index lists (bwd, deterministic); the tap tables are built
once per shape on the host.  D12 (swapped height/width names) is fixed: out_shape is (H, W).
"""
from __future__ import annotations

import functools

import torch

from .common import on_gpu, ext, export_impl


@functools.lru_cache(maxsize=256)
def _taps(in_size, out_size):
    """Row-wise taps (i0, i1, w0, w1) of the 1-D map out_size <- in_size (as python lists)."""
    padded = in_size + 2
    new = out_size + 4
    scale = padded / new
    i0s, i1s, w0s, w1s = [], [], [], []
    for o in range(out_size):
        d = o + 2
        src = d * scale
        y0 = int(src)  # floor, src >= 0
        y1 = min(y0 + 1, padded - 1)
        f = src - y0

        def unpad(j):  # symmetric pad by 1: padded[0] = x[0], padded[n+1] = x[n-1]
            return min(max(j - 1, 0), in_size - 1)

        i0s.append(unpad(y0))
        i1s.append(unpad(y1))
        w0s.append(1.0 - f)
        w1s.append(f)
    return i0s, i1s, w0s, w1s


def interp_matrix(in_size, out_size, device=None):
    i0, i1, w0, w1 = _taps(in_size, out_size)
    A = torch.zeros(out_size, in_size, dtype=torch.float32)
    for o in range(out_size):
        A[o, i0[o]] += w0[o]
        A[o, i1[o]] += w1[o]
    return A.to(device) if device is not None else A


@functools.lru_cache(maxsize=256)
def _tap_tensor_cpu(in_size, out_size):
    """Kernel tap tables: idx int32 [i0(O) | i1(O) | lo(I) | hi(I)], wt fp32 [w0(O) | w1(O)].
    lo/hi = inclusive range of outputs whose taps touch input i (empty: lo > hi)."""
    i0, i1, w0, w1 = _taps(in_size, out_size)
    lo = [out_size] * in_size
    hi = [-1] * in_size
    for o in range(out_size):
        for a in (i0[o], i1[o]):
            lo[a] = min(lo[a], o)
            hi[a] = max(hi[a], o)
    idx = torch.tensor(i0 + i1 + lo + hi, dtype=torch.int32)
    wt = torch.tensor(w0 + w1, dtype=torch.float32)
    return idx, wt


_DEV_CACHE = {}


def _tap_tensor(in_size, out_size, device):
    key = (in_size, out_size, str(device))
    t = _DEV_CACHE.get(key)
    if t is None:
        idx, wt = _tap_tensor_cpu(in_size, out_size)
        t = (idx.to(device), wt.to(device))
        _DEV_CACHE[key] = t
    return t


class _UpsampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_h, out_w):
        N, H, W, C = x.shape
        ctx.x_shape = tuple(x.shape)
        ctx.out = (out_h, out_w)
        if on_gpu(x):
            ih, wh = _tap_tensor(H, out_h, x.device)
            iw, ww = _tap_tensor(W, out_w, x.device)
            y = torch.empty((N, out_h, out_w, C), device=x.device, dtype=x.dtype)
            ext().upsample_fwd(x, y, ih, wh, iw, ww)
            return y
        Ah = interp_matrix(H, out_h)
        Aw = interp_matrix(W, out_w)
        y = torch.einsum("ia,jb,nabc->nijc", Ah, Aw, x.float())
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.x_shape
        out_h, out_w = ctx.out
        dy = dy.contiguous()
        if on_gpu(dy):
            ih, wh = _tap_tensor(H, out_h, dy.device)
            iw, ww = _tap_tensor(W, out_w, dy.device)
            dx = torch.empty(ctx.x_shape, device=dy.device, dtype=dy.dtype)
            ext().upsample_bwd(dy, dx, ih, wh, iw, ww)
            return dx, None, None
        Ah = interp_matrix(H, out_h)
        Aw = interp_matrix(W, out_w)
        dx = torch.einsum("ia,jb,nijc->nabc", Ah, Aw, dy.float())
        return dx.to(dy.dtype), None, None


def upsample(x, out_shape):
    """Reference ``_upsample(inputs, out_shape)``; ``out_shape`` = (H, W)."""
    ex = export_impl()
    if ex is not None:
        return ex.upsample(x, int(out_shape[0]), int(out_shape[1]))
    return _UpsampleFn.apply(x, int(out_shape[0]), int(out_shape[1]))


class _UpsampleIntoFn(torch.autograd.Function):
    """``buf[..., c0:c0+C] = upsample(x)`` in place (the kernel takes the destination's pixel
    stride), returning ``buf`` — the concat-free ASPP pooling branch and decoder input."""

    @staticmethod
    def forward(ctx, buf, x, c0):
        N, H, W, C = x.shape
        out_h, out_w = buf.shape[1], buf.shape[2]
        ctx.x_shape, ctx.c0 = tuple(x.shape), c0
        dst = buf[..., c0:c0 + C]
        if on_gpu(x):
            ih, wh = _tap_tensor(H, out_h, x.device)
            iw, ww = _tap_tensor(W, out_w, x.device)
            ext().upsample_fwd(x.contiguous(), dst, ih, wh, iw, ww)
        else:
            dst.copy_(torch.einsum("ia,jb,nabc->nijc", interp_matrix(H, out_h),
                                   interp_matrix(W, out_w), x.float()).to(buf.dtype))
        ctx.mark_dirty(buf)
        ctx.out = (out_h, out_w)
        return buf

    @staticmethod
    def backward(ctx, gbuf):
        N, H, W, C = ctx.x_shape
        out_h, out_w = ctx.out
        if not gbuf.is_contiguous():
            gbuf = gbuf.contiguous()
        dy = gbuf[..., ctx.c0:ctx.c0 + C]
        if on_gpu(dy):
            ih, wh = _tap_tensor(H, out_h, dy.device)
            iw, ww = _tap_tensor(W, out_w, dy.device)
            dx = torch.empty(ctx.x_shape, device=dy.device, dtype=dy.dtype)
            ext().upsample_bwd(dy, dx, ih, wh, iw, ww)
        else:
            dx = torch.einsum("ia,jb,nijc->nabc", interp_matrix(H, out_h),
                              interp_matrix(W, out_w), dy.float()).to(dy.dtype)
        return gbuf, dx, None


def upsample_into(buf, c0, x):
    """``buf[..., c0:c0+C] = upsample(x, buf.shape[1:3])`` in place; returns ``buf``."""
    if buf.shape[0] != x.shape[0] or c0 + x.shape[-1] > buf.shape[-1]:
        raise ValueError(f"upsample_into: x {tuple(x.shape)} into buf {tuple(buf.shape)} at {c0}")
    return _UpsampleIntoFn.apply(buf, x, int(c0))
