"""Learning-rate schedules (host callables ``step -> lr``; the fused optimizers read them once per
step, or write them into their device scalar before a HIP-graph replay).

* ``exponential`` — ``tf.train.exponential_decay(lr, step, decay_steps, decay_rate)``, the
  reference's schedule (/root/reference/model.py:457-459: 10000 steps, rate 0.5, continuous).
* ``cosine`` — linear warm-up then half-cosine to ``final_fraction·lr`` at ``total_steps``
  (the usual ImageNet ResNet recipe for the north-star workloads).
* ``step`` — multiply by ``decay_rate`` every ``decay_steps`` (staircase), with warm-up.
* ``constant`` — ``lr`` (after warm-up).
"""
from __future__ import annotations

import functools
import math

from ..ops.optim import exponential_decay

SCHEDULES = ("exponential", "cosine", "step", "constant")


def _warm(lr, step, warmup):
    return lr * (step + 1) / warmup if warmup and step < warmup else None


def cosine(lr, step, total_steps, warmup_steps=0, final_fraction=0.0):
    w = _warm(lr, step, warmup_steps)
    if w is not None:
        return w
    span = max(1, total_steps - warmup_steps)
    t = min(1.0, max(0.0, (step - warmup_steps) / span))
    return lr * (final_fraction + (1 - final_fraction) * 0.5 * (1 + math.cos(math.pi * t)))


def staircase(lr, step, decay_steps, decay_rate, warmup_steps=0):
    w = _warm(lr, step, warmup_steps)
    if w is not None:
        return w
    return lr * decay_rate ** (step // max(1, decay_steps))


def constant(lr, step, warmup_steps=0):
    w = _warm(lr, step, warmup_steps)
    return lr if w is None else w


def make(kind, lr, total_steps=None, decay_steps=10000, decay_rate=0.5, warmup_steps=0):
    """The schedule ``kind`` as a ``step -> lr`` callable."""
    if kind == "exponential":
        return functools.partial(exponential_decay, lr, decay_steps=decay_steps,
                                 decay_rate=decay_rate, staircase=False)
    if kind == "cosine":
        if not total_steps:
            raise ValueError("the cosine schedule needs total_steps")
        return functools.partial(cosine, lr, total_steps=total_steps, warmup_steps=warmup_steps)
    if kind == "step":
        return functools.partial(staircase, lr, decay_steps=decay_steps, decay_rate=decay_rate,
                                 warmup_steps=warmup_steps)
    if kind == "constant":
        return functools.partial(constant, lr, warmup_steps=warmup_steps)
    raise ValueError(f"unknown lr schedule {kind!r}; have {SCHEDULES}")
