"""fp8 (OCP e4m3fn) per-tensor quantisation for the fp8 forward convolution.

``quantize_e4m3(x)`` → ``(x8, scale)`` with ``scale = amax(|x|) / 448`` kept on the device (a [1]
fp32 tensor: no host synchronisation) and ``x8 = sat(x / scale)`` in ``torch.float8_e4m3fn``.
GPU: ``csrc/kernels/fp8.hip`` (amax reduction + vectorised ``v_cvt_pk_fp8_f32`` quantiser).
CPU: the same math in PyTorch (the reference for the tests).
"""
from __future__ import annotations

import torch

from .common import on_gpu, ext

E4M3 = torch.float8_e4m3fn
E4M3_MAX = 448.0
E5M2 = torch.float8_e5m2
E5M2_MAX = 57344.0


AMAX_SLOT = 1024  # fp32 partial maxima per amax slot (csrc/kernels/kernels.h AMAX_SLOT)


def _new_ring(device):
    return torch.zeros(3, AMAX_SLOT, device=device, dtype=torch.float32)


# ---- device-side rotation of the delayed-scaling state (graph-capturable) --------------------
# Every delayed-scaling ring keeps fixed slot roles: slot 0 = the previous call's |x|max (scale
# source), slot 1 = accumulates this call's.  The data moves instead of the roles: ONE launch per
# training step rolls every ring of the model (slot 0 ← slot 1, slot 1 ← 0; fp8_roll), issued by
# the Trainer after the optimizer — so no kernel argument changes from step to step and the whole
# fp8 step can be captured as a HIP graph.  A scaler called twice with no roll in between (direct
# use outside a Trainer) rolls its own ring first, which keeps the per-call delayed semantics.
_STATE = {"rings_made": 0}


def _rolls(owner):
    """Step rolls seen by ``owner``'s ring so far: the count of the RingRoller that rolls it
    (per model, so one Trainer's roll never suppresses another model's self-roll), or 0 for a
    scaler no roller has claimed (used outside a Trainer: every second call self-rolls)."""
    roller = getattr(owner, "_roller", None)
    return roller.rolls if roller is not None else 0


def _self_roll(table):
    ext().fp8_roll(table)


class RingRoller:
    """The end-of-step roll of every delayed-scaling ring of ``model`` (its DelayedScalers and
    the FlatFp8Weights of its flat parameter buffer): one launch over a device pointer table,
    rebuilt only when scalers were created since (they appear lazily in the first forwards)."""

    def __init__(self, model):
        self.model = model
        self.table = None
        self.keep = []
        self.built_at = -1
        self.rolls = 0  # device rolls of this model's rings (eager launches + graph replays)

    def _scan(self):
        rings = []
        seen = set()
        for m in self.model.modules():
            for k in ("_fp8_w", "_fp8_x", "_fp8", "_fp8_bwd"):
                sc = m.__dict__.get(k)
                if isinstance(sc, DelayedScaler) and sc.ring is not None:
                    rings.append((sc.ring, 0))
                    self._claim(sc)
            for prm in m.parameters(recurse=False):
                flat = getattr(prm, "_flat_lowp", None)
                fw = getattr(flat, "_tdl_fp8w", None) if flat is not None else None
                if fw is not None and id(fw) not in seen and getattr(fw, "rings", None) is not None:
                    seen.add(id(fw))
                    self._claim(fw)
                    for seg in range(fw.rings.shape[0]):
                        rings.append((fw.rings, seg * 3 * AMAX_SLOT * 4))
        return rings

    def _claim(self, owner):
        # called right before this roller's next roll: from the owner's point of view a roll
        # has happened since its last call, so its next call must not self-roll
        if getattr(owner, "_roller", None) is not self:
            owner._roller = self
            owner.last_roll = None

    def note_replay(self):
        """A captured step that contains this roller's launch was replayed: the rings rolled
        on the device without a host-side roll() call (engine/trainer.Trainer.replay)."""
        if self.table is not None:
            self.rolls += 1

    def roll(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            return
        if self.built_at != _STATE["rings_made"]:
            rings = self._scan()
            self.keep = [t for t, _ in rings]
            self.table = (torch.tensor([t.data_ptr() + o for t, o in rings], dtype=torch.int64)
                          .to(device) if rings else None)
            self.built_at = _STATE["rings_made"]
        if self.table is not None:
            ext().fp8_roll(self.table)
            self.rolls += 1


def quantize_e4m3(x):
    """Just-in-time scaling: scale from this tensor's own amax (amax pass + quantise pass)."""
    if on_gpu(x):
        ring = _new_ring(x.device)
        scale = torch.empty(1, device=x.device, dtype=torch.float32)
        y8 = torch.empty(x.shape, device=x.device, dtype=E4M3)
        xc = x.contiguous()
        ext().fp8_amax(xc, ring, 0)
        ext().fp8_quantize(xc, ring, 0, False, scale, y8.view(torch.uint8))
        return y8, scale
    xf = x.float()
    amax = xf.abs().max().clamp_min(1e-12)
    scale = (amax / E4M3_MAX).reshape(1)
    y8 = (xf / scale).clamp(-E4M3_MAX, E4M3_MAX).to(E4M3)
    return y8, scale


def quantize_e5m2(x):
    """Just-in-time e5m2 (OCP bf8) quantisation — output gradients of the fp8 dgrad."""
    if on_gpu(x):
        ring = _new_ring(x.device)
        scale = torch.empty(1, device=x.device, dtype=torch.float32)
        y8 = torch.empty(x.shape, device=x.device, dtype=E5M2)
        xc = x.contiguous()
        ext().fp8_amax(xc, ring, 0)
        ext().fp8_quantize_e5m2(xc, ring, 0, False, scale, y8.view(torch.uint8))
        return y8, scale
    xf = x.float()
    amax = xf.abs().max().clamp_min(1e-30)
    scale = (amax / E5M2_MAX).reshape(1)
    y8 = (xf / scale).clamp(-E5M2_MAX, E5M2_MAX).to(E5M2)
    return y8, scale


def transpose_weight(w8):
    """[K, R, S, C] fp8 → [R, S, C, K] (the fp8 dgrad's B operand layout)."""
    K = w8.shape[0]
    t = w8.view(torch.uint8).reshape(K, -1).t().contiguous()
    return t.view(w8.dtype).reshape(*w8.shape[1:], K)


class DelayedScaler:
    """Per-tensor delayed scaling (the fp8 training recipe): call t quantises with the |x|max
    measured by call t−1 while measuring its own — one pass over x, no host sync, no memset.
    The ring's slot 0 holds the previous |x|max, slot 1 accumulates this call's; the end-of-step
    :func:`roll_all` moves slot 1 into slot 0 on the device (a self-roll covers back-to-back
    calls without a Trainer step in between), so the kernel arguments never change and the step
    is graph-capturable.  The very first call primes the ring with an amax pass, so it is exact.
    Values beyond the previous amax saturate at ±448.  ``bn_args`` hands the same state to the BN
    apply kernel's fused e4m3 side output (ops/bn.py), whose first call only measures.  The
    scale a call produces lives in one preallocated slot: its consumers (the conv of the same
    step) are stream-ordered before the next call rewrites it."""

    def __init__(self):
        self.ring = None
        self.scale = None
        self.calls = 0
        self.last_roll = None
        self._roller = None

    def _ensure(self, device):
        if self.ring is None or self.ring.device != device:
            self.ring = _new_ring(device)
            self.scale = torch.zeros(1, device=device, dtype=torch.float32)
            self.self_table = torch.tensor([self.ring.data_ptr()], dtype=torch.int64).to(device)
            _STATE["rings_made"] += 1
            self.calls = 0
            self.last_roll = None

    def _begin(self, device):
        rolls = _rolls(self)
        if self.calls > 0 and self.last_roll == rolls:
            _self_roll(self.self_table)  # second call since the last step roll
        self.last_roll = rolls

    def quantize(self, x):
        if not on_gpu(x):
            return quantize_e4m3(x)
        self._ensure(x.device)
        self._begin(x.device)
        xc = x.contiguous()
        if self.calls == 0:
            ext().fp8_amax(xc, self.ring, 0)
        y8 = torch.empty(x.shape, device=x.device, dtype=E4M3)
        ext().fp8_quantize(xc, self.ring, 0, True, self.scale, y8.view(torch.uint8))
        self.calls += 1
        return y8, self.scale

    def bn_args(self, x):
        self._ensure(x.device)
        self._begin(x.device)
        out = (self.ring, 0, self.scale, self.calls > 0)
        self.calls += 1
        return out


class FlatFp8Weights:
    """e4m3 copies of every fp8 conv weight that lives in one flat bf16 buffer
    (models/params.FlatParams), refreshed by ONE launch per optimizer step
    (``fp8_multi_quantize``: delayed scaling per weight tensor) instead of one amax+quantise pair
    per layer.  Layers join on their first call (served by their own scaler for that call) and the
    work list is rebuilt at the next parameter version."""

    CHUNK = 16384  # elements per workgroup

    def __init__(self, flat_lowp):
        self.flat = flat_lowp
        self.w8 = torch.empty(flat_lowp.numel(), device=flat_lowp.device, dtype=E4M3)
        # transposed copies [R][S][C][K] for the fp8 dgrad, refreshed by one transpose launch
        self.w8t = torch.zeros(flat_lowp.numel(), device=flat_lowp.device, dtype=E4M3)
        self.tviews = {}
        self.views = {}     # id(param) -> (w8 view, scale view), valid for the buffers' lifetime
        self.pending = {}   # id(param) -> (offset, numel, shape)
        self.spans = []     # segment -> (offset, numel, shape)
        self.version = None
        self.last_roll = None
        self.rings = None
        self._roller = None

    def _rebuild(self):
        keys = list(self.views) + list(self.pending)
        self.spans = [s for s in self.spans] + list(self.pending.values())
        self.pending = {}
        rows = []
        total = self.flat.numel()
        for seg, (off, n, _) in enumerate(self.spans):
            if n % 16 or off % 16 or off + n > total:
                raise ValueError(f"fp8 weight span ({off}, {n}) not 16-aligned inside the buffer")
            for c in range(0, n, self.CHUNK):
                rows.append((seg, off + c, min(self.CHUNK, n - c), int(c == 0)))
        dev = self.flat.device
        self.chunks = torch.tensor(rows, dtype=torch.int64).to(dev)
        self.rings = torch.zeros(len(self.spans), 3, AMAX_SLOT, device=dev)
        _STATE["rings_made"] += 1  # rolled with the model's other rings (RingRoller)
        self.self_table = torch.tensor([self.rings.data_ptr() + seg * 3 * AMAX_SLOT * 4
                                        for seg in range(len(self.spans))],
                                       dtype=torch.int64).to(dev)
        self.scales = torch.zeros(len(self.spans), device=dev)
        self.views = {k: (self.w8[off:off + n].view(shape), self.scales[seg:seg + 1])
                      for seg, (k, (off, n, shape)) in enumerate(zip(keys, self.spans))}
        trows = []
        self.tviews = {}
        for seg, (k, (off, n, shape)) in enumerate(zip(keys, self.spans)):
            K = shape[0]
            cols = n // K
            if len(shape) == 4 and K % 16 == 0 and cols % 16 == 0:
                tiles = ((K + 63) // 64) * ((cols + 63) // 64)
                trows += [(off, K, cols, t) for t in range(tiles)]
                self.tviews[k] = (self.w8t[off:off + n].view(*shape[1:], K),
                                  self.scales[seg:seg + 1])
        self.tiles = torch.tensor(trows if trows else [(0, 16, 16, 0)],
                                  dtype=torch.int64).to(dev)
        self.ntiles = len(trows)
        self.last_roll = None
        ext().fp8_multi_quantize(self.flat, self.w8.view(torch.uint8), self.chunks, self.rings,
                                 self.scales, 0, True)  # prime: exact first scales

    def get(self, p, version):
        """(w8, scale) for parameter ``p`` at parameter version ``version``, or None the first
        time ``p`` is seen (caller quantises it itself)."""
        k = id(p)
        if k not in self.views and k not in self.pending:
            self.pending[k] = (p._flat_offset, p.numel(), tuple(p.shape))
            return None
        self._refresh(version)
        return self.views.get(k)  # None: joined during this version

    def _refresh(self, version):
        if self.version != version:
            if self.pending:
                self._rebuild()
            rolls = _rolls(self)
            if self.last_roll == rolls:
                _self_roll(self.self_table)  # refreshed twice with no step roll in between
            self.last_roll = rolls
            ext().fp8_multi_quantize(self.flat, self.w8.view(torch.uint8), self.chunks, self.rings,
                                     self.scales, 0, False)
            if self.ntiles:
                ext().fp8_multi_transpose(self.w8.view(torch.uint8), self.w8t.view(torch.uint8),
                                          self.tiles)
            self.version = version

    def get_t(self, p, version):
        """(W^T [R, S, C, K] e4m3, scale) of parameter ``p`` for the fp8 dgrad, or None if ``p``
        has no flat copy yet (it joins at its first forward)."""
        if id(p) not in self.tviews:
            return None
        self._refresh(version)
        return self.tviews.get(id(p))


def flat_weights_for(p):
    """The :class:`FlatFp8Weights` of ``p``'s flat buffer (None if ``p`` is not flat-backed);
    kept on the buffer tensor itself, so it lives and dies with the FlatParams."""
    flat = getattr(p, "_flat_lowp", None)
    if flat is None or not on_gpu(flat):
        return None
    fw = getattr(flat, "_tdl_fp8w", None)
    if fw is None:
        fw = flat._tdl_fp8w = FlatFp8Weights(flat)
    return fw


def dequantize_e5m2(y8, scale):
    if on_gpu(y8):
        out = torch.empty(y8.shape, device=y8.device, dtype=torch.float32)
        ext().fp8_dequantize_e5m2(y8.contiguous().view(torch.uint8), scale, out)
        return out
    return y8.float() * scale


def dequantize(y8, scale):
    if on_gpu(y8):
        out = torch.empty(y8.shape, device=y8.device, dtype=torch.float32)
        ext().fp8_dequantize(y8.contiguous(), scale, out)
        return out
    return y8.float() * scale
