"""Shared helpers for ops: device dispatch, gradient delivery into flat buffers.

Parameters of our models live in flat buffers (see :mod:`models.params`):
``p.data`` is a view of the fp32 master buffer, ``p.grad`` a view of the fp32 gradient buffer and
``p._lowp`` a view of the bf16 compute copy.  Our autograd Functions never hand weight gradients back
to autograd; they write them straight into ``p.grad`` (the HIP wgrad kernels write there directly)
and then call ``p._grad_hook(p)`` so the data-parallel bucketer can launch the all-reduce of a
bucket as soon as its last gradient lands (SURVEY.md §5.8 "GradBucketer").  This replaces the
reference's MirroredStrategy gradient aggregation (model.py:114-116, Test.ipynb:200).
"""
from __future__ import annotations

import torch

from .. import _native


def on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def fused_gpu(t: torch.Tensor) -> bool:
    """A GPU tensor on the bf16 fast path: the fused epilogue features (ReLU bit masks, BN-backward
    statistics in the consumer's dgrad, fp8 side outputs) apply.  fp32 GPU tensors — the
    reference-precision path (``--dtype fp32``) — run the plain fp32 kernels
    (``csrc/kernels/f32.hip``), which take none of those fusions."""
    return t.is_cuda and t.dtype != torch.float32


def ext():
    return _native.ext()


# the serving-export lowering while a model is traced (engine/serving.py export_mode), else None
_EXPORT = [None]


def export_impl():
    """The active export lowering: the ops layer hands each primitive to it instead of launching
    a kernel (the tracer's tensors are fakes)."""
    return _EXPORT[0]


def compute_weight(p: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """The tensor the kernels read for parameter ``p`` (bf16 shadow on GPU, else fp32 master)."""
    lp = getattr(p, "_lowp", None)
    if lp is not None and lp.dtype == dtype:
        return lp
    if p.dtype == dtype:
        return p.detach()
    return p.detach().to(dtype)


def grad_target(p: torch.Tensor):
    """Return (tensor, overwrite) where a kernel may write p's gradient directly.

    ``overwrite`` is True when this is the first contribution of the step (the kernel may store
    instead of accumulate)."""
    g = p.grad
    if g is None:
        return None, True
    return g, bool(getattr(p, "_grad_fresh", True))


def deliver_grad(p: torch.Tensor, g: torch.Tensor | None = None, written: bool = False):
    """Deliver gradient ``g`` of parameter ``p``.

    If ``written`` the kernel already stored the gradient into ``p.grad``.  Otherwise ``g`` is
    copied (first contribution) or accumulated into ``p.grad``."""
    if not written:
        g = g.to(torch.float32).reshape(p.shape)
        if p.grad is None:
            p.grad = g.clone()
        elif getattr(p, "_grad_fresh", True):
            p.grad.copy_(g)
        else:
            p.grad.add_(g)
    p._grad_fresh = False
    hook = getattr(p, "_grad_hook", None)
    if hook is not None:
        hook(p)


def flat_view(p: torch.Tensor, n: int, which: str = "master"):
    """``n`` ≥ p.numel() fp32 elements of p's flat buffer starting at p (``which``: "master" data or
    "grad"), or None when p is not flat-backed or its 64-aligned slot is shorter than ``n``.

    The slack between p.numel() and the aligned slot belongs to p and stays zero (models/params.py:
    zero-initialised, zero gradient, so the optimizer never moves it), which is what lets
    channel-padded layers read γ/β/bias as one padded vector and write their padded gradients
    straight into the flat gradient buffer."""
    buf = getattr(p, "_flat_master" if which == "master" else "_flat_grad", None)
    if buf is None:
        return None
    o = p._flat_offset
    if n > (p.numel() + 63) // 64 * 64 or o + n > buf.numel():
        return None
    return buf[o:o + n]


def reset_grad_state(params):
    for p in params:
        p._grad_fresh = True


def param_requires_grad(p) -> bool:
    return p is not None and p.requires_grad and torch.is_grad_enabled()
