"""Optimizers over :class:`models.params.FlatParams` — one fused kernel per step.

``FusedSGD``  : momentum SGD (north-star ResNet/Xception configs).
``FusedAdam`` : TF AdamOptimizer semantics (reference model.py:462) with the reference's
                ``exponential_decay(lr, step, 10000, 0.5)`` schedule available via
                :func:`ops.optim.exponential_decay`.
Both apply the data-parallel 1/world gradient averaging inside the update kernel.
"""
from __future__ import annotations

import math

import torch

from ..ops import optim as _ops
from ..models import params as _params


class _FlatOptimizer:
    def __init__(self, flat, lr=0.1, weight_decay=0.0, lr_schedule=None):
        self.flat = flat
        self.base_lr = lr
        self.weight_decay = weight_decay
        self.lr_schedule = lr_schedule
        self.step_count = 0

    def lr_at(self, step):
        return self.lr_schedule(step) if self.lr_schedule is not None else self.base_lr

    @property
    def lr(self):
        return self.lr_at(self.step_count)

    def step(self, grad_scale=1.0):
        self._update(self.lr_at(self.step_count), grad_scale)
        self.step_count += 1
        _params.bump_version()

    def state_tensors(self):
        return {}

    def load_state_tensors(self, d):
        for k, v in self.state_tensors().items():
            if k in d:
                v.copy_(d[k].to(v.device, v.dtype).reshape(v.shape))


class FusedSGD(_FlatOptimizer):
    def __init__(self, flat, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=False,
                 lr_schedule=None):
        super().__init__(flat, lr, weight_decay, lr_schedule)
        self.momentum = momentum
        self.nesterov = nesterov
        self.mom = torch.zeros_like(flat.master)

    def _update(self, lr, grad_scale):
        f = self.flat
        _ops.sgd_momentum_(f.master, f.grad, self.mom, f.lowp, f.decay_flags, lr, self.momentum,
                           self.weight_decay, grad_scale, self.nesterov)

    def state_tensors(self):
        return {"Momentum": self.mom}


class FusedAdam(_FlatOptimizer):
    def __init__(self, flat, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
                 lr_schedule=None):
        super().__init__(flat, lr, weight_decay, lr_schedule)
        self.beta1, self.beta2, self.eps = beta1, beta2, eps
        self.m = torch.zeros_like(flat.master)
        self.v = torch.zeros_like(flat.master)

    def _update(self, lr, grad_scale):
        t = self.step_count + 1
        lr_t = lr * math.sqrt(1 - self.beta2 ** t) / (1 - self.beta1 ** t)
        f = self.flat
        _ops.adam_(f.master, f.grad, self.m, self.v, f.lowp, f.decay_flags, lr_t, self.beta1,
                   self.beta2, self.eps, self.weight_decay, grad_scale)

    def state_tensors(self):
        return {"Adam": self.m, "Adam_1": self.v}


def build_optimizer(kind, flat, **kw):
    kind = kind.lower()
    if kind in ("sgd", "momentum", "sgd_momentum"):
        return FusedSGD(flat, **kw)
    if kind == "adam":
        return FusedAdam(flat, **kw)
    raise ValueError(f"unknown optimizer {kind}")
