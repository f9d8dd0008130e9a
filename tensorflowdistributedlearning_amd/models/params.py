"""Flat parameter storage: fp32 master + fp32 gradient + bf16 compute copy in three flat buffers.

Why flat: on MI355X the optimizer update, the data-parallel all-reduce and the checkpoint D2H copy
all become a handful of large contiguous operations instead of hundreds of small ones (one fused
optimizer launch for the whole model, bucketed RCCL all-reduces that are plain slices of one
buffer, one async D2H copy).  Offsets are 64-element aligned (256 B) so every parameter starts on
a 16-B vector boundary and owns whole weight-decay groups.

Layout is *registration order* (= forward order); the data-parallel bucketer walks it backwards so
buckets fill in the order backward produces gradients.

Replaces the reference's per-variable mirrored variables + Adam slots (model.py:115-116,462;
SURVEY N13/N15).
"""
from __future__ import annotations

import torch

ALIGN = 64

# bumped after every optimizer step; layers that keep derived copies (e.g. channel-padded stem
# weights) refresh lazily when it changes
_VERSION = [0]


def version() -> int:
    return _VERSION[0]


def bump_version():
    _VERSION[0] += 1


def _align(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


class FlatParams:
    """Owns the flat buffers of ``module``'s trainable parameters.

    After construction every trainable parameter ``p`` satisfies
    ``p.data`` = view of ``self.master``, ``p.grad`` = view of ``self.grad``,
    ``p._lowp`` = view of ``self.lowp`` (bf16; only if ``lowp_dtype``).
    """

    def __init__(self, module: torch.nn.Module, device, lowp_dtype=torch.bfloat16,
                 no_decay=None, with_grad=True):
        """``with_grad=False`` (inference: ``Model.predict``): no gradient buffer — parameters get
        their fp32 master views and bf16 compute views only."""
        self.device = torch.device(device)
        self.params = []
        self.names = []
        seen = set()
        for name, p in module.named_parameters():
            if not p.requires_grad or id(p) in seen:
                continue
            seen.add(id(p))
            self.params.append(p)
            self.names.append(name)
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _align(p.numel())
        self.total = max(off, ALIGN)
        self.master = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.grad = (torch.zeros(self.total, dtype=torch.float32, device=self.device)
                     if with_grad else None)
        self.lowp = (torch.zeros(self.total, dtype=lowp_dtype, device=self.device)
                     if lowp_dtype is not None else None)
        flags = torch.ones(self.total // ALIGN, dtype=torch.uint8)
        if no_decay is None:
            # exempt from weight decay: parameters a module lists in ``no_decay_params`` (BN γ/β,
            # biases — a class attribute, so it survives copy.deepcopy, which drops attributes
            # set on a Parameter) or flagged ``_no_decay`` directly
            exempt = {id(getattr(m, a)) for m in module.modules()
                      for a in getattr(m, "no_decay_params", ())
                      if isinstance(getattr(m, a, None), torch.nn.Parameter)}
            no_decay = lambda name, p: id(p) in exempt or getattr(p, "_no_decay", False)  # noqa: E731
        for name, p, o in zip(self.names, self.params, self.offsets):
            n = p.numel()
            with torch.no_grad():
                self.master[o:o + n].copy_(p.detach().reshape(-1).to(self.device, torch.float32))
            if no_decay(name, p):
                flags[o // ALIGN:(o + _align(n)) // ALIGN] = 0
        self.decay_flags = flags.to(self.device)
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            p.data = self.master[o:o + n].view(p.shape)
            p.grad = self.grad[o:o + n].view(p.shape) if self.grad is not None else None
            p._lowp = self.lowp[o:o + n].view(p.shape) if self.lowp is not None else None
            p._flat_offset = o
            p._flat_lowp = self.lowp
            p._flat_master = self.master
            p._flat_grad = self.grad
            p._grad_fresh = True
        self.sync_lowp()

    # ------------------------------------------------------------------------------------------
    def sync_lowp(self):
        """Refresh the bf16 compute copy from the fp32 master (after init / checkpoint load)."""
        if self.lowp is not None:
            with torch.no_grad():
                self.lowp.copy_(self.master.to(self.lowp.dtype))
        bump_version()

    def begin_step(self):
        for p in self.params:
            p._grad_fresh = True

    def finish_grads(self):
        """Zero the gradient slices of parameters that received no gradient this step.
        Returns the list of such parameters."""
        missing = [p for p in self.params if getattr(p, "_grad_fresh", True)]
        for p in missing:
            p.grad.zero_()
            p._grad_fresh = False
        return missing

    def num_params(self):
        return sum(p.numel() for p in self.params)

    def slice_of(self, p):
        o = p._flat_offset
        return o, o + p.numel()
