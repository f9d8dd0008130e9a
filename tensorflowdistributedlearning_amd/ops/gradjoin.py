"""Residual-gradient join: one gradient buffer shared by all consumers of a tensor.

In a residual block the block input ``x`` feeds two branches (conv1 and the shortcut — identity
into the final BN+add, or a 1×1 downsample conv), so autograd receives two gradients for ``x`` and
sums them with a separate elementwise ``add`` kernel (a full read-read-write pass over the block
input every block; 1.3 ms of a ResNet-50 b256 step).  With a :class:`GradJoin` the consumers'
backward kernels write into ONE buffer instead: the first consumer produces it (the BN backward
writes its residual gradient there, or a dgrad overwrites it), the later ones accumulate in their
epilogue (``conv_dgrad(accumulate=True)``: dx += …), and only the last consumer hands the buffer to
autograd — the others return ``None`` (zero) for ``x``.

Order independence: whichever consumer's backward runs first creates the buffer; correctness
only needs every consumer to run, which holds inside a block (all branches reach the loss).
"""
from __future__ import annotations

ENABLED = True


class GradJoin:
    __slots__ = ("n", "count", "buf")

    def __init__(self, n):
        self.n = n
        self.count = 0
        self.buf = None

    def take(self):
        """Register one consumer's contribution; returns the buffer for the last one, else None."""
        self.count += 1
        return self.buf if self.count == self.n else None


def make(n, x):
    """A join for ``n`` consumers of ``x`` when enabled and ``x`` needs a gradient."""
    if ENABLED and x.requires_grad:
        return GradJoin(n)
    return None
