"""Per-step pre-zeroed scratch for atomically accumulated reductions.

BN statistics (Σx, Σx² from the conv epilogue) and BN-backward sums (Σg, Σg·x̂) are accumulated
with fp32 atomics and therefore need zeroed destinations.  Allocating each with ``torch.zeros``
costs one fill launch per BN layer per pass (≈800 launches per ResNet-50 step); instead every
such buffer is a slice of one arena that is zeroed by a single fill at the start of each training
step (``reset()``, called by the Trainer).  The first step discovers the required size.
"""
from __future__ import annotations

import torch

_ALIGN = 64


class ZeroArena:
    def __init__(self):
        self.buf = None
        self.off = 0
        self.need = 0

    def take(self, shape, device):
        n = 1
        for s in shape:
            n *= int(s)
        na = (n + _ALIGN - 1) // _ALIGN * _ALIGN
        if (self.buf is None or self.buf.device != torch.device(device)
                or self.off + na > self.buf.numel()):
            self.off += na
            self.need = max(self.need, self.off)
            return torch.zeros(shape, dtype=torch.float32, device=device)
        v = self.buf[self.off:self.off + n].view(shape)
        self.off += na
        return v

    def reset(self, device):
        device = torch.device(device)
        used = max(self.need, self.off)
        if self.buf is None or self.buf.device != device or used > self.buf.numel():
            if used > 0:
                self.buf = torch.zeros(int(used * 1.25) + _ALIGN, dtype=torch.float32,
                                       device=device)
        elif self.off > 0:
            self.buf[: self.off].zero_()
        self.off = 0
        self.need = 0


_ARENA = ZeroArena()


class use_arena:
    """Route ``zeros`` / ``reset`` to ``arena`` inside the block.  A HIP-graph capture gives its
    step a private arena (engine/trainer.py ``capture``): the graph bakes the arena's addresses
    in, so eager steps of other trainers in the process must not grow or reallocate it."""

    def __init__(self, arena):
        self.arena = arena

    def __enter__(self):
        global _ARENA
        self.prev, _ARENA = _ARENA, self.arena
        return self.arena

    def __exit__(self, *exc):
        global _ARENA
        _ARENA = self.prev
        return False


def zeros(shape, device):
    """A zero-filled fp32 tensor valid until the next ``reset`` (i.e. within one step)."""
    if torch.device(device).type != "cuda":
        return torch.zeros(shape, dtype=torch.float32, device=device)
    return _ARENA.take(shape, device)


def reset(device):
    if torch.device(device).type == "cuda":
        _ARENA.reset(device)
