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

Pre-masked joins: when ``x`` is the output of a residual BN + ReLU (the previous block's
``relu(bn3(y) + shortcut)``), that BN's backward needs g = dx·[x > 0].  The forward attached a
:class:`MaskToken` (the 1-bit ReLU mask) to ``x``; the join's dgrad consumers apply the mask in
their epilogue (dx = ([dx +] dgrad)·[bit], exact: masking is linear in the contributions), and if
the finished buffer is masked everywhere the token records it — the BN backward then reads no
mask and returns the incoming gradient itself as the residual gradient instead of writing a copy
(ResNet-50 b256: one full activation write and the mask reads of 16 residual BN backwards).
Anything that breaks the protocol (an unmasked contribution last, autograd summing another
gradient into the buffer) leaves the token unset, and the BN applies the mask itself as before.

Fused BN-backward statistics: the token also carries the BN's input x.  A stride-1 dgrad that
writes the final gradient (the only consumer, or the join's last contribution) accumulates
(Σg, Σg·x) of what it stores in its epilogue (``conv_dgrad_bnstat``); the token records them with
the pre-masked stamp and the BN backward skips its reduce pass (a read of dy and x).  Non-residual
ReLU BNs (bottleneck conv1 / conv2 outputs) write the 1-bit mask too so their single consumer
conv can take the same path.
"""
from __future__ import annotations

import os

ENABLED = True


MASK_ENABLED = os.environ.get("TDL_PREMASK", "1") == "1"  # 0: the BN applies its mask
# TDL_BNSTAT_FUSE: 0 — the BN backward always runs its own reduce pass; 1 — statistics fused into
# the last writer's dgrad epilogue, residual joins included; 2 (default) — only for
# single-consumer convs; 3 — only for residual joins.  ResNet-50 b1024 same-box A/B
# (profiles/r02_bnstat_fuse_ab.txt): 0 11993 / 11999, 1 11994 / 11984, 2 12029 / 12012,
# 3 11882 / 11840 img/s — the join variant's smaller tiles (the 256×128 ones spill with both the
# previous-dx and the x loads) lose next to the side-stream weight gradients.  Round 5, with the
# joins' statistics on the dgrad-as-forward 8-wave tiles (route row dgrad.asfwd.glds.join): 1
# 12,990 / 12,992 vs 2 13,179 / 13,170 img/s (dev/scripts/gpu_r05_statsjoin.sh) — still slower.
# Round 6, the joins on the 256×128 tiles (route row dgrad.asfwd.glds.join.wide): a tie — serial
# 77.19 vs 77.23 ms (12 fused joins +2.2 ms, 8 reduce passes −2.1 ms), bench 14,027 / 13,989 /
# 14,028 vs 14,020 / 14,024 / 14,026 img/s (profiles/r06_join_stats.txt)
_FUSE = os.environ.get("TDL_BNSTAT_FUSE", "2")
STATS_ENABLED = _FUSE != "0"
STATS_SINGLE = _FUSE in ("1", "2")
STATS_JOIN = _FUSE in ("1", "3")
# the fp8 dgrads (e5m2 × e4m3) fuse the join's statistics unless TDL_FP8_JOIN_STATS=0 (A/B)
FP8_JOIN_STATS = STATS_ENABLED and os.environ.get("TDL_FP8_JOIN_STATS", "1") == "1"


class MaskToken:
    """The ReLU bit mask of a BN output, the BN's input ``x`` (for fused statistics), and (after
    backward) which gradient buffer the consumers handed back already masked:
    ``(data_ptr, version)`` of that tensor, plus its (Σg, Σg·x) when the last writer fused them."""
    __slots__ = ("mask", "premasked", "x", "red", "relu_y")

    def __init__(self, mask, x=None, relu_y=False):
        self.mask = mask
        self.premasked = None
        self.x = x if STATS_ENABLED else None
        self.red = None
        # relu_y: the BN output is ReLU'd but no bit mask was written (channel counts that do
        # not fill the 64-channel mask slabs): a consumer may apply the mask as "its input > 0"
        # (the depthwise dgrad's relu_in path); the conv dgrads, which only take bit masks,
        # leave such tokens alone
        self.relu_y = relu_y

    def is_premasked(self, g):
        return self.premasked is not None and self.premasked == (g.data_ptr(), g._version)

    def mark(self, g, red=None):
        """``g`` is the finished, masked gradient; ``red`` its fused (Σg, Σg·x) or None."""
        self.premasked = (g.data_ptr(), g._version)
        self.red = red

    def stats_for(self, g):
        """The fused (Σg, Σg·x) of ``g`` if its last writer produced them, else None."""
        return self.red if self.is_premasked(g) else None

    def release(self):
        """Drop the tensors once the BN backward has used them (the token is reachable from
        autograd nodes that live until the whole backward ends: it must not pin x)."""
        self.x = None
        self.red = None
        self.mask = None
        # a second backward over the same graph (retain_graph) must not see this backward's
        # stamp: a fresh unmasked gradient can reuse the address at version 0
        self.premasked = None


class GradJoin:
    __slots__ = ("n", "count", "buf", "mask_token", "unmasked", "red")

    def __init__(self, n, mask_token=None):
        self.n = n
        self.count = 0
        self.buf = None
        self.mask_token = mask_token
        self.unmasked = False  # some element of buf holds a contribution not yet masked
        self.red = None        # (Σg, Σg·x) fused by the last contribution (conv_dgrad_bnstat)

    @property
    def last(self):
        """The next contribution is the last one."""
        return self.count + 1 == self.n

    @property
    def stats_x(self):
        """The BN input to fuse statistics against (None: not applicable)."""
        return self.stats_x_for(False)

    def stats_x_for(self, fp8):
        """:attr:`stats_x` for a last contribution that is an fp8 dgrad (``fp8``): fused there by
        default (FP8_JOIN_STATS), the bf16 joins per STATS_JOIN."""
        t = self.mask_token
        return t.x if t is not None and (STATS_JOIN or (fp8 and FP8_JOIN_STATS)) else None

    @property
    def mask(self):
        """The ReLU bit mask the dgrad consumers apply in their epilogue (None: no masking)."""
        return self.mask_token.mask if self.mask_token is not None else None

    def note(self, masked, full=True):
        """Record a contribution: ``masked`` — written through the mask epilogue; ``full`` — it
        rewrote every element (a strided dgrad leaves some pixels untouched)."""
        if not masked:
            self.unmasked = True
        elif full:
            self.unmasked = False

    def take(self):
        """Register one consumer's contribution; returns the buffer for the last one, else None."""
        self.count += 1
        if self.count > self.n:
            raise RuntimeError(
                "fused residual-gradient join reached more than once per forward (a second "
                "backward over a retained graph?): run the forward again for every backward")
        if self.count != self.n:
            return None
        if self.mask_token is not None and not self.unmasked and self.buf is not None:
            self.mask_token.mark(self.buf, self.red)
        buf, self.buf = self.buf, None  # autograd owns it now: the join (kept by the graph
        return buf                       # nodes until backward ends) must not pin it


def make(n, x):
    """A join for ``n`` consumers of ``x`` when enabled and ``x`` needs a gradient (pre-masked
    when ``x`` carries the ReLU mask token of a residual BN)."""
    if ENABLED and x.requires_grad:
        tok = getattr(x, "_tdl_mask_token", None) if MASK_ENABLED else None
        return GradJoin(n, tok)
    return None
