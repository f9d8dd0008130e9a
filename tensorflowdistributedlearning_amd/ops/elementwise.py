"""Small fused elementwise ops (vectorised 16-B bf16 HIP kernels in ``csrc/kernels/elementwise.hip``).

* ``relu`` / ``add_relu`` — the reference's ``tf.nn.relu(shortcut + residual)``
  (core/resnet.py:87,148) and Xception's pre-activation ReLUs (core/xception.py:190).
* ``add`` — Xception ``sum`` skip connections (core/xception.py:216-219).
* ``sigmoid_threshold`` — ``sigmoid`` + ``> threshold`` (model.py:371-372, K15).
"""
from __future__ import annotations

import torch

from .common import on_gpu, ext, export_impl


class _AddReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, relu):
        if on_gpu(a):
            y = torch.empty_like(a)
            ext().add_act(a, b, y, bool(relu))
        else:
            y = a.float() + (b.float() if b is not None else 0.0)
            if relu:
                y = torch.relu(y)
            y = y.to(a.dtype)
        ctx.relu = relu
        ctx.has_b = b is not None
        ctx.save_for_backward(y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        if ctx.relu:
            (y,) = ctx.saved_tensors
            if on_gpu(dy):
                g = torch.empty_like(dy)
                ext().relu_bwd(dy, y, g)
            else:
                g = (dy.float() * (y.float() > 0)).to(dy.dtype)
        else:
            g = dy
        return g, (g if ctx.has_b else None), None


def _add_act(a, b, act):
    ex = export_impl()
    if ex is not None:
        return ex.add_act(a, b, act)
    return _AddReluFn.apply(a, b, act)


def add_relu(a, b):
    return _add_act(a, b, True)


def relu(a):
    return _add_act(a, None, True)


def add(a, b):
    return _add_act(a, b, False)


def sigmoid_threshold(logits, threshold=0.5):
    """(probabilities fp32, prediction {0,1} fp32)."""
    ex = export_impl()
    if ex is not None:
        return ex.sigmoid_threshold(logits, threshold)
    if on_gpu(logits):
        prob = torch.empty(logits.shape, device=logits.device, dtype=torch.float32)
        pred = torch.empty_like(prob)
        ext().sigmoid_threshold(logits.contiguous(), prob, pred, float(threshold))
        return prob, pred
    prob = torch.sigmoid(logits.float())
    return prob, (prob > threshold).float()
