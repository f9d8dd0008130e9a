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
        self.lr_dev = None  # graph mode: fp32 [1] device lr the kernel reads (set_device_lr)

    def set_device_lr(self, enabled=True):
        """HIP-graph mode: the update kernel reads the learning rate from a device scalar that
        :meth:`prepare_replay` refreshes before every replay (a captured launch keeps its host
        arguments frozen, and the schedule / Adam bias correction change every step)."""
        self.lr_dev = (torch.zeros(1, device=self.flat.master.device, dtype=torch.float32)
                       if enabled else None)

    def prepare_replay(self):
        """Write this step's effective lr into the device scalar (stream-ordered fill)."""
        self.lr_dev.fill_(self._effective_lr(self.step_count))

    def _effective_lr(self, step):
        return self.lr_at(step)

    def lr_at(self, step):
        return self.lr_schedule(step) if self.lr_schedule is not None else self.base_lr

    @property
    def lr(self):
        return self.lr_at(self.step_count)

    def step(self, grad_scale=1.0):
        self._update(self._effective_lr(self.step_count), grad_scale)
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
        if self.lr_dev is not None:
            lr = 1.0
        _ops.sgd_momentum_(f.master, f.grad, self.mom, f.lowp, f.decay_flags, lr, self.momentum,
                           self.weight_decay, grad_scale, self.nesterov, self.lr_dev)

    def state_tensors(self):
        return {"Momentum": self.mom}


class FusedAdam(_FlatOptimizer):
    def __init__(self, flat, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
                 lr_schedule=None):
        super().__init__(flat, lr, weight_decay, lr_schedule)
        self.beta1, self.beta2, self.eps = beta1, beta2, eps
        self.m = torch.zeros_like(flat.master)
        self.v = torch.zeros_like(flat.master)

    def _effective_lr(self, step):
        t = step + 1  # TF: bias correction folded into the step size
        return self.lr_at(step) * math.sqrt(1 - self.beta2 ** t) / (1 - self.beta1 ** t)

    def _update(self, lr_t, grad_scale):
        f = self.flat
        if self.lr_dev is not None:
            lr_t = 1.0
        _ops.adam_(f.master, f.grad, self.m, self.v, f.lowp, f.decay_flags, lr_t, self.beta1,
                   self.beta2, self.eps, self.weight_decay, grad_scale, self.lr_dev)

    def state_tensors(self):
        return {"Adam": self.m, "Adam_1": self.v}


def build_optimizer(kind, flat, **kw):
    kind = kind.lower()
    if kind in ("sgd", "momentum", "sgd_momentum"):
        return FusedSGD(flat, **kw)
    if kind == "adam":
        return FusedAdam(flat, **kw)
    raise ValueError(f"unknown optimizer {kind}")
