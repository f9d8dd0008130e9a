"""NHWC layer modules built on our fused ops.

All activations are NHWC (bf16 on the GPU, fp32 on the CPU oracle path); conv weights are KRSC
([Cout, R, S, Cin]) so both implicit-GEMM operands of the forward conv are K-contiguous.
These are the L2 "layer primitives" of the reference (core/layers.py + tf.contrib.slim conv2d /
batch_norm / max_pool2d / separable_conv2d under resnet_arg_scope, core/resnet.py:357-395).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

import os

from ..ops.conv import ConvGeom, conv2d, conv_fwd, same_padding, symmetric_padding, row_pack
from ..ops.bn import batch_norm_act, batch_norm_act_into
from ..ops.pool import max_pool2d, global_avg_pool
from ..ops.dwconv import depthwise_conv2d
from ..ops import bnconv
from ..ops.bnconv import DeferredBNAct, bn_act_conv
from ..ops.common import compute_weight, flat_view
from ..ops.fp8 import DelayedScaler, flat_weights_for, transpose_weight
from . import params as _params


def _round_up(c, multiple):
    return c if not multiple else (c + multiple - 1) // multiple * multiple


# ----------------------------------------------------------------------------------------------
# initialisers
# ----------------------------------------------------------------------------------------------

def trunc_normal_(t, std, a=-2.0, b=2.0):
    with torch.no_grad():
        t.normal_(0, 1)
        while True:
            bad = (t < a) | (t > b)
            if not bad.any():
                break
            t[bad] = torch.randn(int(bad.sum()))
        t.mul_(std)
    return t


def variance_scaling_(t, fan_in, factor=2.0):
    """tf.contrib.layers.variance_scaling_initializer() default (FAN_IN, truncated normal,
    stddev = sqrt(1.3·factor/fan_in)) — resnet_arg_scope's initializer (core/resnet.py:383)."""
    return trunc_normal_(t, math.sqrt(1.3 * factor / fan_in))


def kaiming_normal_fan_out_(t, fan_out):
    with torch.no_grad():
        return t.normal_(0, math.sqrt(2.0 / fan_out))


# ----------------------------------------------------------------------------------------------
# padding modes
# ----------------------------------------------------------------------------------------------

def resolve_padding(mode, H, W, R, S, stride, dilation):
    """mode: 'SAME' (TF, possibly asymmetric), 'VALID', 'sym' (PyTorch-style (k-1)/2 both sides),
    int, or explicit 4-tuple (top, bottom, left, right)."""
    if isinstance(mode, tuple) and len(mode) == 4:
        return mode
    if isinstance(mode, int):
        return (mode, mode, mode, mode)
    if mode == "VALID":
        return (0, 0, 0, 0)
    if mode == "SAME":
        t, b = same_padding(H, R, stride[0], dilation[0])
        l, r = same_padding(W, S, stride[1], dilation[1])
        return (t, b, l, r)
    if mode == "sym":
        t, b = symmetric_padding(R, dilation[0])
        l, r = symmetric_padding(S, dilation[1])
        return (t, b, l, r)
    raise ValueError(f"unknown padding {mode}")


# ----------------------------------------------------------------------------------------------
# layers
# ----------------------------------------------------------------------------------------------

class FlatFlips:
    """The flipped filters (Conv2d.flip_weight) of every flat-backed conv of one flat bf16 weight
    buffer (models/params.FlatParams), refreshed by ONE launch per parameter version
    (``conv_flip_weights_multi``) instead of one per layer (46 per ResNet-50 step).  The flips sit
    at their weights' offsets in a parallel buffer, so a view never moves (HIP-graph replays
    refresh it in place).  A layer joins at its first call (flipped on its own for that version)
    and the work list is rebuilt at the next version.

    The work list is never rebuilt while a HIP graph is being captured: its host-to-device copy
    would read a pageable temporary freed after capture.  Layers still pending then flip on their
    own inside the graph (``get`` returns None), and every work-list tensor a launch ever read is
    kept alive, so a graph captured against an older list replays valid offsets."""

    def __init__(self, flat):
        self.flat = flat
        self.buf = torch.empty_like(flat)
        self.segs = {}      # id(param) -> (offset, (K, R, S, C))
        self.pending = {}
        self.rows = None
        self.retired = []   # earlier work lists (a captured graph may still read one)
        self.version = None

    @staticmethod
    def of(p, w):
        """The FlatFlips of ``p``'s flat buffer when ``w`` (the compute weight handed to the
        backward) is ``p``'s own slice of it, else None."""
        flat = getattr(p, "_flat_lowp", None)
        if flat is None or not flat.is_cuda or flat.dtype != torch.bfloat16 or w.dim() != 4:
            return None
        off = getattr(p, "_flat_offset", None)
        if off is None or w.data_ptr() != flat.data_ptr() + off * flat.element_size() \
                or not w.is_contiguous():
            return None
        fl = getattr(flat, "_tdl_flips", None)
        if fl is None:
            fl = flat._tdl_flips = FlatFlips(flat)
        return fl

    def get(self, p, version):
        capturing = torch.cuda.is_current_stream_capturing()
        if self.version != version:  # first call of a parameter version: flip every member
            if self.pending and not capturing:
                self._rebuild()
            if self.segs:
                from ..ops.common import ext
                ext().conv_flip_weights_multi(self.flat, self.buf, self.rows)
            self.version = version
        k = id(p)
        if k not in self.segs:
            self.pending[k] = (p._flat_offset, tuple(p.shape))
            return None  # flipped on its own (Conv2d.flip_weight) until the next rebuild
        off, (K, R, S, C) = self.segs[k]
        return self.buf[off:off + K * R * S * C].view(C, R, S, K)

    def _rebuild(self):
        self.segs.update(self.pending)
        self.pending = {}
        rows = []
        n = self.flat.numel()
        for off, (K, R, S, C) in self.segs.values():
            if off < 0 or off + K * R * S * C > n:
                raise ValueError(f"flip span ({off}, {K}x{R}x{S}x{C}) outside the flat buffer")
            for tap in range(R * S):
                for kb in range((K + 31) // 32):
                    for cb in range((C + 31) // 32):
                        rows.append((off, K, R, S, C, tap, kb, cb))
        if self.rows is not None:
            self.retired.append(self.rows)
        self.rows = torch.tensor(rows, dtype=torch.int64).to(self.flat.device)


class Conv2d(nn.Module):
    """NHWC conv, KRSC weight, optional bias and fused ReLU.

    ``pad_cin_to``: the bf16 compute copy of the weight is zero-padded along Cin to this multiple
    (the kernels need Cin % 8 == 0; used for the 3-channel RGB / 2-channel TGS stems whose input
    tensors are padded the same way).  ``pad_cout_to``: likewise along Cout, so the output tensor
    carries zero channels up to the multiple (the reference preset's 258-wide block2 bottleneck,
    defect D7, runs on the LDS-DMA kernels as 264 channels).  The fp32 parameter keeps its true
    shape; gradients are un-padded on delivery.
    """

    no_decay_params = ("bias",)  # (models/params.FlatParams)

    def __init__(self, cin, cout, k, stride=1, padding="sym", dilation=1, bias=False, relu=False,
                 init="he_tf", init_std=None, pad_cin_to=None, pad_cout_to=None):
        super().__init__()
        kh, kw = (k, k) if isinstance(k, int) else k
        self.cin, self.cout, self.k = cin, cout, (kh, kw)
        self.stride = (stride, stride) if isinstance(stride, int) else tuple(stride)
        self.dilation = (dilation, dilation) if isinstance(dilation, int) else tuple(dilation)
        self.padding = padding
        self.relu = relu
        self.weight = nn.Parameter(torch.empty(cout, kh, kw, cin))
        fan_in = cin * kh * kw
        if init == "he_tf":
            variance_scaling_(self.weight.data, fan_in)
        elif init == "kaiming_fan_out":
            kaiming_normal_fan_out_(self.weight.data, cout * kh * kw)
        elif init == "trunc_normal":
            trunc_normal_(self.weight.data, init_std)
        elif init == "zeros":
            self.weight.data.zero_()
        else:
            raise ValueError(init)
        if bias:
            self.bias = nn.Parameter(torch.zeros(cout))
            self.bias._no_decay = True
        else:
            self.bias = None
        self.pad_cin_to = pad_cin_to
        self._cin_store = _round_up(cin, pad_cin_to)
        self._cout_store = _round_up(cout, pad_cout_to)
        self._padded = None
        self._padded_version = -1
        self._geom_cache = {}

    # weight handling for the kernels -----------------------------------------------------------
    def grad_needs_unpad(self):
        return self._cin_store != self.cin or self._cout_store != self.cout

    def padded_weight_shape(self):
        return (self._cout_store, self.k[0], self.k[1], self._cin_store)

    def unpad_grad(self, dw):
        return dw[: self.cout, ..., : self.cin]

    def compute_weight(self, dtype):
        w = compute_weight(self.weight, dtype)
        if not self.grad_needs_unpad():
            return w
        # one persistent zero-padded copy, refreshed in place once per parameter version (the
        # padding never changes; a fixed address also keeps HIP-graph replays valid)
        if (self._padded is None or self._padded.dtype != dtype
                or self._padded.device != w.device):
            self._padded = torch.zeros(self.padded_weight_shape(), dtype=dtype, device=w.device)
            self._padded_version = -1
        v = _params.version()
        if self._padded_version != v:
            self._padded[: self.cout, ..., : self.cin].copy_(w)
            self._padded_version = v
        return self._padded

    def flip_weight(self, w):
        """[C, R, S, K] flipped transpose of the compute weight ``w`` (w_flip[c][r][s][k] =
        w[k][R−1−r][S−1−s][c]): the stride-1 input gradient then runs as the forward conv of dy
        (ops/conv.py, conv_glds.hip conv_dgrad_as_fwd).  One HIP launch per parameter version into
        a persistent buffer (fixed address: HIP-graph replays refresh it in place); flat-backed
        weights join their buffer's :class:`FlatFlips` — every flip of the model in one launch."""
        v = _params.version()
        fl = FlatFlips.of(self.weight, w)
        if fl is not None:
            wf = fl.get(self.weight, v)
            if wf is not None:
                return wf
        c = self.__dict__.get("_flip")
        shape = (w.shape[3], w.shape[1], w.shape[2], w.shape[0])
        if c is not None and c[0] == v and c[1].device == w.device and tuple(c[1].shape) == shape:
            return c[1]
        if c is not None and c[1].device == w.device and tuple(c[1].shape) == shape \
                and c[1].dtype == w.dtype:
            wf = c[1]
        else:
            wf = torch.empty(shape, dtype=w.dtype, device=w.device)
        from ..ops.common import ext
        ext().conv_flip_weight(w.contiguous(), wf)
        self.__dict__["_flip"] = (v, wf)
        return wf

    def flip_weight_classes(self, w, geom):
        """The per-parity-class flipped sub-filters of this strided conv (ops/conv.flip_classes),
        rebuilt once per parameter version into a persistent buffer (HIP-graph replays refresh
        it in place)."""
        from ..ops.conv import flip_classes
        v = _params.version()
        c = self.__dict__.get("_flipc")
        if c is not None and c[0] == v and c[1].device == w.device:
            return c[1]
        f = flip_classes(w, geom, out=c[1] if c is not None else None)  # (in place when it fits)
        self.__dict__["_flipc"] = (v, f)
        return f

    def compute_bias(self):
        """fp32 bias as the kernels read it, ``_cout_store`` long with zero padding channels (the
        flat master buffer's slack when flat-backed, else a padded copy)."""
        b = self.bias.detach()
        if self._cout_store == self.cout:
            return b
        v = flat_view(self.bias, self._cout_store)
        return v if v is not None else torch.nn.functional.pad(b, (0, self._cout_store - self.cout))

    def geom(self, H, W):
        g = self._geom_cache.get((H, W))
        if g is None:
            pad = resolve_padding(self.padding, H, W, self.k[0], self.k[1], self.stride,
                                  self.dilation)
            g = ConvGeom(self.stride, pad, self.dilation)
            self._geom_cache[(H, W)] = g
        return g

    fp8 = False  # set by models.enable_fp8: e4m3 forward GEMM (ops/fp8.py)
    fp8_dgrad = False  # … and the e5m2 × e4m3 input gradient
    fp8_wgrad = False  # … and the e5m2 × e4m3 weight gradient (the forward's e4m3 input saved)

    def fp8_weight(self, w_lowp):
        """e4m3 copy of the weight + its scale, re-quantised once per optimizer step (delayed
        scaling: one pass per step)."""
        v = _params.version()
        if not self.grad_needs_unpad():  # the weight is the flat bf16 buffer slice itself
            fw = flat_weights_for(self.weight)
            got = fw.get(self.weight, v) if fw is not None else None
            if got is not None:
                return got
        cache = self.__dict__.get("_fp8_cache")
        if cache is None or cache[0] != v or cache[1].device != w_lowp.device:
            sc = self.__dict__.get("_fp8_w")
            if sc is None:
                sc = self.__dict__["_fp8_w"] = DelayedScaler()
            w8, sw = sc.quantize(w_lowp)
            cache = (v, w8, sw)
            self.__dict__["_fp8_cache"] = cache
        return cache[1], cache[2]

    def fp8_weight_t(self, w_lowp):
        """Transposed e4m3 weight [R, S, C, K] + scale for the fp8 dgrad (same quantisation as
        :meth:`fp8_weight`, refreshed once per optimizer step)."""
        v = _params.version()
        if not self.grad_needs_unpad():
            fw = flat_weights_for(self.weight)
            got = fw.get_t(self.weight, v) if fw is not None else None
            if got is not None:
                return got
        cache = self.__dict__.get("_fp8_t_cache")
        if cache is None or cache[0] != v or cache[1].device != w_lowp.device:
            w8, sw = self.fp8_weight(w_lowp)
            cache = (v, transpose_weight(w8), sw)
            self.__dict__["_fp8_t_cache"] = cache
        return cache[1], cache[2]

    def fp8_input(self, x):
        """e4m3 copy of an input no BN pre-quantised (delayed scaling, per layer)."""
        sc = self.__dict__.get("_fp8_x")
        if sc is None:
            sc = self.__dict__["_fp8_x"] = DelayedScaler()
        return sc.quantize(x)

    def forward(self, x, want_stats=False, join=None, residual=None, relu=None, res_link=None):
        """``residual``: y = act(conv(x) + bias + residual) (the epilogue adds it); ``relu``
        overrides the layer's activation for this call; ``res_link`` (ops/bn.ResidualLink)
        hands the residual's gradient to the BN that normalises it."""
        g = self.geom(x.shape[1], x.shape[2])
        y, stats = conv2d(x, self.weight, self.bias, g, self.relu if relu is None else relu,
                          want_stats, self, join, residual, res_link)
        return (y, stats) if want_stats else y

    def _load_from_state_dict(self, *args, **kw):
        # derived copies (channel-padded / row-packed weights, folded BN) key on the parameter
        # version: a load outside the optimizer must refresh them too
        _params.bump_version()
        return super()._load_from_state_dict(*args, **kw)

    def forward_folded(self, x, w, bias, relu, residual=None):
        """Inference forward with a given compute weight and fp32 bias (ConvBN's folded BN):
        act(conv(x, w) + bias [+ residual]) in the conv epilogue, no autograd record."""
        return conv_fwd(x, w, self.geom(x.shape[1], x.shape[2]), bias=bias, relu=relu,
                        residual=residual)

    def extra_repr(self):
        return (f"{self.cin}->{self.cout}, k={self.k}, s={self.stride}, d={self.dilation}, "
                f"pad={self.padding}, bias={self.bias is not None}, relu={self.relu}")


class RowPackedConv2d(Conv2d):
    """k×k conv on a few-channel image (the 7×7 RGB stem) computed as a k×1 conv over the
    row-packed input (:func:`ops.conv.row_pack`: each output column's k taps × C channels become
    one contiguous channel vector, padded to a multiple of 8).  Same math as :class:`Conv2d` with
    the input padded to 8 channels, but the GEMM K is k·⌈k·C/8⌉·8 instead of k·k·8 (168 vs 392
    for 7×7×3: 2.3× fewer MFMA FLOPs in the stem's forward and weight gradient).  The parameter
    keeps its [Cout, k, k, C] shape (checkpoints, optimizer); the compute copy is re-laid to
    [Cout, k, 1, Cp] once per parameter version and the weight gradient folded back.  An input
    gradient (rare for an image) flows through the packing's transposed gather."""

    def __init__(self, cin, cout, k, stride=1, padding="sym", **kw):
        super().__init__(cin, cout, k, stride, padding, **kw)
        assert self.k[0] == self.k[1] and self.dilation == (1, 1)
        self._cp = _round_up(self.k[1] * cin, 8)
        self._packed = None
        self._packed_version = -1
        self._pgeom = {}

    def grad_needs_unpad(self):
        return True

    def padded_weight_shape(self):
        return (self._cout_store, self.k[0], 1, self._cp)

    def unpad_grad(self, dw):
        k = self.k[1]
        return dw[: self.cout, :, 0, : k * self.cin].reshape(self.cout, self.k[0], k, self.cin)

    def compute_weight(self, dtype):
        w = compute_weight(self.weight, dtype)
        if (self._packed is None or self._packed.dtype != dtype
                or self._packed.device != w.device):
            self._packed = torch.zeros(self.padded_weight_shape(), dtype=dtype, device=w.device)
            self._packed_version = -1
        v = _params.version()
        if self._packed_version != v:
            k = self.k[1]
            self._packed[: self.cout, :, 0, : k * self.cin].copy_(
                w.reshape(self.cout, self.k[0], k * self.cin))
            self._packed_version = v
        return self._packed

    def packed_geom(self, H, W):
        """(k×1 conv geometry over the packed rows, left padding, output width)."""
        pg = self._pgeom.get((H, W))
        if pg is None:
            pt, pb, pl, pr = resolve_padding(self.padding, H, W, self.k[0], self.k[1],
                                             self.stride, self.dilation)
            Wo = (W + pl + pr - self.k[1]) // self.stride[1] + 1
            pg = self._pgeom[(H, W)] = (ConvGeom((self.stride[0], 1), (pt, pb, 0, 0)), pl, Wo)
        return pg

    def forward(self, x, want_stats=False, join=None):
        g, pl, Wo = self.packed_geom(x.shape[1], x.shape[2])
        t = row_pack(x, self.cin, self.k[1], self.stride[1], pl, Wo, self._cp)
        y, stats = conv2d(t, self.weight, self.bias, g, self.relu, want_stats, self, join)
        return (y, stats) if want_stats else y

    def forward_folded(self, x, w, bias, relu, residual=None):
        g, pl, Wo = self.packed_geom(x.shape[1], x.shape[2])
        t = row_pack(x, self.cin, self.k[1], self.stride[1], pl, Wo, self._cp)
        return conv_fwd(t, w, g, bias=bias, relu=relu, residual=residual)


class BatchNorm(nn.Module):
    """BN over the channel (last) axis with TF-style moving averages
    (``m ← decay·m + (1−decay)·batch``).  ``scale=False`` drops γ (slim ``scale`` flag).

    ``c_phys`` > ``c``: the input carries zero padding channels up to ``c_phys`` (channel-padded
    convs, :class:`Conv2d` ``pad_cout_to``); γ/β are read zero-padded so those channels stay
    exactly zero, and the moving statistics keep their logical size ``c``."""

    no_decay_params = ("gamma", "beta")  # (models/params.FlatParams)

    def __init__(self, c, decay=0.997, eps=1e-5, scale=True, zero_init=False, c_phys=None):
        super().__init__()
        self.c, self.decay, self.eps = c, decay, eps
        self.c_phys = c_phys or c
        self.gamma = nn.Parameter(torch.zeros(c) if zero_init else torch.ones(c)) if scale else None
        if self.gamma is not None:
            self.gamma._no_decay = True
        self.beta = nn.Parameter(torch.zeros(c))
        self.beta._no_decay = True
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))

    def phys_params(self):
        """(γ, β) as the kernels read them: fp32 vectors of ``c_phys`` with zero padding (views of
        the flat master buffer's slack when flat-backed, else padded copies)."""
        g = None if self.gamma is None else self.gamma.detach()
        b = self.beta.detach()
        if self.c_phys == self.c:
            return g, b

        def pad(p, t):
            v = flat_view(p, self.c_phys)
            return v if v is not None else torch.nn.functional.pad(t, (0, self.c_phys - self.c))
        return (None if g is None else pad(self.gamma, g)), pad(self.beta, b)

    emit_fp8 = False  # set by models.enable_fp8: also emit an e4m3 copy for the fp8 consumer conv
    fp8_only = False  # … and write only that copy (every consumer is an fp8 conv with fp8 wgrad)

    def fp8_state(self, x):
        """(amax ring, phase, scale, emit) for the delayed-scaling e4m3 side output of bn_apply
        (ops/bn.py, ops/fp8.DelayedScaler), or None where it does not apply."""
        if not (x.is_cuda and self.c_phys % 16 == 0):
            return None
        sc = self.__dict__.get("_fp8")
        if sc is None:
            sc = self.__dict__["_fp8"] = DelayedScaler()
        return sc.bn_args(x)

    emit_fp8_bwd = False  # set by models.enable_fp8: e5m2 copy of dx for the fp8 dgrad
    fp8_bwd_only = False  # … and write only that copy (the conv's dgrad and wgrad are both fp8)

    def fp8_bwd_state(self, x):
        """(amax ring, phase, scale, emit) for the e5m2 side output of the backward apply (the
        producing conv's fp8 dgrad needs K % 128 == 0), or None where it does not apply."""
        if not (x.is_cuda and self.c_phys % 128 == 0):
            return None
        sc = self.__dict__.get("_fp8_bwd")
        if sc is None:
            sc = self.__dict__["_fp8_bwd"] = DelayedScaler()
        return sc.bn_args(x)

    def forward(self, x, stats=None, residual=None, relu=False, res_join=None, link=None):
        return batch_norm_act(x, self, stats=stats, residual=residual, relu=relu,
                              training=self.training, res_join=res_join, link=link)


def bn_fold_enabled():
    """Inference BN folding (ConvBN, eval mode, no autograd): on unless TDL_BN_FOLD=0."""
    return os.environ.get("TDL_BN_FOLD", "1") != "0"


def fold_bn_affine(bn, device):
    """(s, b') fp32 over ``bn.c_phys`` channels: eval-mode BN(y) = y·s + b' with
    s = γ/√(σ²+ε), b' = β − μ·s (zero on padding channels)."""
    gamma, beta = bn.phys_params()
    s = torch.zeros(bn.c_phys, dtype=torch.float32, device=device)
    sh = torch.zeros(bn.c_phys, dtype=torch.float32, device=device)
    inv = torch.rsqrt(bn.running_var.float().to(device) + bn.eps)
    if gamma is not None:
        inv = inv * gamma[: bn.c].float().to(device)
    s[: bn.c] = inv
    sh[: bn.c] = beta[: bn.c].float().to(device) - bn.running_mean.float().to(device) * inv
    return s, sh


class ConvBN(nn.Module):
    """conv → BN → [+residual] → [ReLU] with BN statistics accumulated in the conv epilogue.

    Inference (eval mode under ``torch.no_grad``): the BN's moving statistics are folded into
    the conv — W' = W·s, b' = β − μ·s with s = γ/√(σ²+ε) per output channel — so the layer is one
    conv whose epilogue adds b' (+ the residual) and applies the ReLU: no BN pass at all (the
    reference's eval graph runs slim.batch_norm(is_training=False) as separate ops,
    core/resnet.py:373-386).  The folded weights are cached per parameter version and dropped on
    every train()/eval() switch and state-dict load (the moving statistics change only in
    training).  ``TDL_BN_FOLD=0`` keeps the unfolded conv + BN-apply path."""

    def __init__(self, cin, cout, k, stride=1, padding="sym", dilation=1, relu=True,
                 bn_decay=0.997, bn_eps=1e-5, bn_scale=True, zero_init_gamma=False, init="he_tf",
                 init_std=None, pad_cin_to=None, pad_cout_to=None, conv_cls=None):
        super().__init__()
        self.conv = (conv_cls or Conv2d)(cin, cout, k, stride, padding, dilation=dilation,
                                         bias=False, relu=False, init=init, init_std=init_std,
                                         pad_cin_to=pad_cin_to, pad_cout_to=pad_cout_to)
        self.bn = BatchNorm(cout, bn_decay, bn_eps, bn_scale, zero_init_gamma,
                            c_phys=self.conv._cout_store)
        self.relu = relu

    # inference BN folding ------------------------------------------------------------------------
    def train(self, mode=True):
        self.__dict__.pop("_fold", None)
        return super().train(mode)

    def _load_from_state_dict(self, *args, **kw):
        self.__dict__.pop("_fold", None)
        _params.bump_version()
        return super()._load_from_state_dict(*args, **kw)

    def folded_params(self, dtype, device):
        """(W·s in the compute dtype, fp32 b') over the stored (padded) output channels."""
        key = (_params.version(), dtype, device)
        c = self.__dict__.get("_fold")
        if c is not None and c[0] == key:
            return c[1], c[2]
        bn, conv = self.bn, self.conv
        with torch.no_grad():
            s, sh = fold_bn_affine(bn, device)
            if conv.bias is not None:
                sh += conv.compute_bias().float().to(device) * s
            w = conv.compute_weight(dtype)
            wf = (w.float() * s.view(-1, 1, 1, 1)).to(dtype).contiguous()
        self.__dict__["_fold"] = (key, wf, sh.contiguous())
        return wf, self.__dict__["_fold"][2]

    def forward(self, x, residual=None, join=None, res_join=None, into=None, defer=False):
        """``join``: gradient join for x (ops/gradjoin.py); ``res_join``: for the residual.
        ``into`` = (buf, c0): write act(BN(conv(x))) into ``buf[..., c0:c0+C]`` (a concat
        buffer, ops/bn.batch_norm_act_into) and return ``buf``.
        ``x`` may be an ops.bnconv.DeferredBNAct (the previous layer's BN + ReLU, folded into
        this conv where the kernels take it); ``defer``: in training, return this layer's own
        BN + ReLU deferred the same way for a single consumer conv (ops/bnconv.py)."""
        if isinstance(x, DeferredBNAct):
            if join is not None or not self.training:
                x = x.materialize()
            else:
                y, stats = bn_act_conv(x, self.conv, want_stats=True)
                return self._bn_out(y, stats, residual, res_join, into, defer)
        if (not self.training and into is None and not torch.is_grad_enabled()
                and bn_fold_enabled()):
            wf, bf = self.folded_params(x.dtype, x.device)
            return self.conv.forward_folded(x, wf, bf, self.relu, residual)
        if self.training:
            y, stats = self.conv(x, want_stats=True, join=join)
        else:
            y, stats = self.conv(x, join=join), None
        return self._bn_out(y, stats, residual, res_join, into, defer)

    def _bn_out(self, y, stats, residual, res_join, into, defer):
        if (defer and self.relu and self.training and residual is None and into is None
                and bnconv.ENABLED and torch.is_grad_enabled()):
            return DeferredBNAct(y, stats, self.bn)
        if into is not None:
            if residual is not None:
                raise ValueError("ConvBN: no residual with into=")
            return batch_norm_act_into(into[0], into[1], y, self.bn, stats, self.relu,
                                       self.bn.training)
        return self.bn(y, stats=stats, residual=residual, relu=self.relu, res_join=res_join)


class BNAct(nn.Module):
    """standalone BN(+ReLU) — slim.batch_norm(activation_fn=relu) pre-activation / postnorm."""

    def __init__(self, c, decay=0.997, eps=1e-5, scale=True, relu=True, c_phys=None):
        super().__init__()
        self.bn = BatchNorm(c, decay, eps, scale, c_phys=c_phys)
        self.relu = relu

    def forward(self, x, stats=None, link=None):
        """``stats``: the input's BN sums (Σx, Σx²) if its producer already accumulated them;
        ``link``: ops/bn.ResidualLink of x's residual-path gradient."""
        return self.bn(x, stats=stats, relu=self.relu, link=link)


class MaxPool(nn.Module):
    def __init__(self, k, stride, padding="sym"):
        super().__init__()
        self.k, self.stride, self.padding = k, stride, padding

    def forward(self, x):
        pad = resolve_padding(self.padding, x.shape[1], x.shape[2], self.k, self.k,
                              (self.stride, self.stride), (1, 1))
        return max_pool2d(x, self.k, self.stride, pad)


class GlobalAvgPool(nn.Module):
    def __init__(self, keepdims=False):
        super().__init__()
        self.keepdims = keepdims

    def forward(self, x):
        return global_avg_pool(x, self.keepdims)


class Linear(nn.Module):
    """Fully connected layer = 1×1 conv on a [N, 1, 1, C] view (same MFMA GEMM kernels)."""

    def __init__(self, cin, cout, bias=True, init_std=None):
        super().__init__()
        self.conv = Conv2d(cin, cout, 1, bias=bias, padding=0, init="trunc_normal" if init_std
                           else "he_tf", init_std=init_std)
        if init_std is None:
            bound = 1.0 / math.sqrt(cin)
            with torch.no_grad():
                self.conv.weight.uniform_(-bound, bound)

    def forward(self, x):
        N, C = x.shape
        y = self.conv(x.reshape(N, 1, 1, C))
        return y.reshape(N, -1)


class DepthwiseConv2d(nn.Module):
    """Depthwise k×k (depth multiplier 1), weight [R, S, C], optional bias + ReLU."""

    no_decay_params = ("bias",)  # (models/params.FlatParams)

    def __init__(self, c, k=3, stride=1, padding="SAME", dilation=1, bias=True, relu=True,
                 init_std=0.33):
        super().__init__()
        self.c, self.k = c, k
        self.stride = (stride, stride)
        self.dilation = (dilation, dilation)
        self.padding = padding
        self.relu = relu
        self.weight = nn.Parameter(trunc_normal_(torch.empty(k, k, c), init_std))
        if bias:
            self.bias = nn.Parameter(torch.zeros(c))
            self.bias._no_decay = True
        else:
            self.bias = None

    def forward(self, x, relu_in=False, want_stats=False, join=None):
        """``want_stats``: returns ``(y, stats)`` with the BN sums (Σy, Σy²) of y.  ``join``:
        residual-gradient join for x (ops/gradjoin.py; see ops.dwconv.joinable)."""
        pad = resolve_padding(self.padding, x.shape[1], x.shape[2], self.k, self.k, self.stride,
                              self.dilation)
        w, b = self.__dict__.get("_serve") or (self.weight, self.bias)  # frozen: serving.py
        return depthwise_conv2d(x, w, b, ConvGeom(self.stride, pad, self.dilation), self.relu,
                                relu_in, want_stats, join)

    def forward_folded(self, x, w, bias, relu, relu_in=False):
        """Inference forward with a given weight (x's dtype) and fp32 bias: a BN folded into
        the depthwise conv (models/xception.SeparableConvBN), no autograd record."""
        pad = resolve_padding(self.padding, x.shape[1], x.shape[2], self.k, self.k, self.stride,
                              self.dilation)
        return depthwise_conv2d(x, w, bias, ConvGeom(self.stride, pad, self.dilation), relu,
                                relu_in)
