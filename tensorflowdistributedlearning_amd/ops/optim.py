"""Fused optimizer updates over the flat parameter buffers.

Every parameter of a model lives in one flat fp32 master buffer (64-element aligned), its gradient
in one flat fp32 buffer and its bf16 compute copy in one flat bf16 buffer (models/params.py).  The
update is therefore ONE kernel launch over the whole model: it reads a per-64-element-group
weight-decay flag, applies the data-parallel 1/world gradient scale, and writes both the new fp32
master and the bf16 copy the conv kernels read (``csrc/kernels/optim.hip``).  Scalars are passed
by value (no host→device copy, no sync).

Reference parity: ``tf.contrib.optimizer_v2.AdamOptimizer`` + ``exponential_decay`` (model.py:457-467,
SURVEY N13/K18) — TF Adam formulation (bias correction folded into lr_t, ε added to √v after
correction); plus the north-star SGD + momentum (TF/PyTorch convention
v = μv + g, p -= lr·v).
"""
from __future__ import annotations

import math

import torch

from .common import on_gpu, ext


def exponential_decay(lr, step, decay_steps=10000, decay_rate=0.5, staircase=False):
    """tf.train.exponential_decay (model.py:457-459)."""
    p = step / decay_steps
    if staircase:
        p = math.floor(p)
    return lr * decay_rate ** p


def _flags(decay_flags, n):
    return decay_flags.repeat_interleave(64)[:n].float()


def sgd_momentum_(master, grad, mom, lowp, decay_flags, lr, momentum, weight_decay,
                  grad_scale=1.0, nesterov=False, lr_scale=None):
    """g' = g·grad_scale + wd·p·flag;  v = μv + g';  p -= lr·(g' + μv if nesterov else v).
    ``lr_scale``: optional fp32 [1] device tensor multiplying ``lr`` (read by the kernel)."""
    if on_gpu(master):
        ext().sgd_momentum(master, grad, mom, lowp, decay_flags, float(lr), float(momentum),
                           float(weight_decay), float(grad_scale), bool(nesterov), lr_scale)
        return
    if lr_scale is not None:
        lr = lr * float(lr_scale)
    g = grad * grad_scale + weight_decay * _flags(decay_flags, master.numel()) * master
    mom.mul_(momentum).add_(g)
    upd = g + momentum * mom if nesterov else mom
    master.sub_(lr * upd)
    if lowp is not None:
        lowp.copy_(master.to(lowp.dtype))


def adam_(master, grad, m, v, lowp, decay_flags, lr_t, beta1, beta2, eps, weight_decay=0.0,
          grad_scale=1.0, lr_scale=None):
    """TF Adam: m = β1 m + (1-β1) g; v = β2 v + (1-β2) g²; p -= lr_t·m/(√v + ε), with
    lr_t = lr·√(1-β2^t)/(1-β1^t) computed on the host (times the optional device ``lr_scale``)."""
    if on_gpu(master):
        ext().adam(master, grad, m, v, lowp, decay_flags, float(lr_t), float(beta1), float(beta2),
                   float(eps), float(weight_decay), float(grad_scale), lr_scale)
        return
    if lr_scale is not None:
        lr_t = lr_t * float(lr_scale)
    g = grad * grad_scale + weight_decay * _flags(decay_flags, master.numel()) * master
    m.mul_(beta1).add_((1 - beta1) * g)
    v.mul_(beta2).add_((1 - beta2) * g * g)
    master.sub_(lr_t * m / (v.sqrt() + eps))
    if lowp is not None:
        lowp.copy_(master.to(lowp.dtype))
