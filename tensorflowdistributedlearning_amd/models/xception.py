"""Xception-41 (DeepLab variant), NHWC — the *intended* network of core/xception.py:405-465.

The reference file is not importable (``resnet_utils`` missing, D8), builds only the last unit of
each block (scope dedented out of the loop, D9) and has no BN on its convs (D10); this is the
intended DeepLab Xception-41: BN after every conv, 8-unit middle flow, depthwise-separable convs
with explicit ``fixed_padding`` at stride 2 (core/xception.py:18-35,38-128), skip connections
'conv' / 'sum' / 'none' (:131-228), atrous output-stride control (:231-292) and optional
classification head (global pool + logits) for the north-star Xception 299×299 benchmark.

The depthwise 3×3 (+BN) runs on the HIP depthwise kernels; the pointwise 1×1 convs on the MFMA
GEMM kernels with BN statistics fused into their epilogue.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import params as _params
from .layers import (ConvBN, DepthwiseConv2d, BatchNorm, GlobalAvgPool, Linear, bn_fold_enabled,
                     fold_bn_affine)
from ..ops import bnfold, dwfold, gradjoin
from ..ops.dwconv import joinable


def _fixed_pad(k, rate):
    keff = k + (k - 1) * (rate - 1)
    beg = (keff - 1) // 2
    return (beg, keff - 1 - beg, beg, keff - 1 - beg)


class SeparableConvBN(nn.Module):
    """separable_conv2d_same (split form): [ReLU →] depthwise k×k (stride, rate) → BN [→ReLU] →
    pointwise 1×1 → BN [→ReLU].  ``relu_out`` rectifies the pointwise BN output even when the
    activation is not 'inside' (it then belongs to the next unit's pre-activation ReLU)."""

    def __init__(self, cin, cout, stride, rate, act_inside, bn_kw, relu_out=None):
        super().__init__()
        pad = "SAME" if stride == 1 else _fixed_pad(3, rate)
        self.depthwise = DepthwiseConv2d(cin, 3, stride, pad, rate, bias=False, relu=False,
                                         init_std=0.33)
        self.dw_bn = BatchNorm(cin, bn_kw["bn_decay"], bn_kw["bn_eps"])
        self.pointwise = ConvBN(cin, cout, 1, 1, 0,
                                relu=act_inside if relu_out is None else relu_out,
                                init="trunc_normal", init_std=0.06, **bn_kw)
        self.act_inside = act_inside

    def train(self, mode=True):
        self.__dict__.pop("_fold", None)
        return super().train(mode)

    def _load_from_state_dict(self, *args, **kw):
        self.__dict__.pop("_fold", None)
        return super()._load_from_state_dict(*args, **kw)

    def _dw_folded(self, dtype, device):
        """depthwise weight × s and b' of the depthwise BN (inference; see layers.ConvBN)."""
        key = (_params.version(), dtype, device)
        c = self.__dict__.get("_fold")
        if c is None or c[0] != key:
            with torch.no_grad():
                s, sh = fold_bn_affine(self.dw_bn, device)
                w = self.depthwise.weight.detach().to(device).float() * s.view(1, 1, -1)
                c = self.__dict__["_fold"] = (key, w.to(dtype).contiguous(), sh.contiguous())
        return c[1], c[2]

    def forward(self, x, relu_in=False, residual=None, join=None, res_join=None, defer=False):
        """``join``: gradient join of x (its depthwise dgrad accumulates onto the other
        consumer's contribution); ``res_join``: gradient join of the residual.  ``x`` may be a
        deferred BN + ReLU (ops/dwfold.DeferredBNAct) that the depthwise conv applies on its
        loads; ``defer``: return this conv's own BN + ReLU deferred the same way (training,
        no residual) for the next separable conv."""
        if isinstance(x, dwfold.DeferredBNAct):
            fold_in = (self.training and not self.act_inside and bnfold.ENABLED and not relu_in
                       and join is None)
            if not fold_in:
                x = x.materialize()
        else:
            fold_in = False
        if not self.training and not torch.is_grad_enabled() and bn_fold_enabled():
            # inference: the depthwise BN (+ReLU) folded into the depthwise conv's bias epilogue
            w, b = self._dw_folded(x.dtype, x.device)
            y = self.depthwise.forward_folded(x, w, b, self.act_inside, relu_in)
            return self.pointwise(y, residual=residual)
        # training: the depthwise kernel accumulates the BN statistics of its output in its
        # epilogue (no separate reduce pass over y)
        if self.training and not self.act_inside and bnfold.ENABLED:
            # no activation between the depthwise BN and the pointwise conv: the BN is folded
            # into the conv (scaled weights + bias, ops/bnfold.py) — its output never exists
            if fold_in:  # the previous pointwise BN + ReLU applied by the depthwise kernels
                z, stats = dwfold.bn_act_dw(x, self.depthwise, want_stats=True)
            else:
                z, stats = self.depthwise(x, relu_in=relu_in, want_stats=True, join=join)
            pw = self.pointwise
            y, st2 = bnfold.bn_conv1x1(z, stats, self.dw_bn, pw.conv, want_stats=True,
                                       dy_sums_zero=pw.bn.training)
            if defer and pw.relu and residual is None and res_join is None and dwfold.ENABLED:
                return dwfold.DeferredBNAct(y, st2, pw.bn)
            return pw.bn(y, stats=st2, residual=residual, relu=pw.relu, res_join=res_join)
        if self.training:
            y, stats = self.depthwise(x, relu_in=relu_in, want_stats=True, join=join)
        else:
            y, stats = self.depthwise(x, relu_in=relu_in, join=join), None
        y = self.dw_bn(y, stats=stats, relu=self.act_inside)
        return self.pointwise(y, residual=residual, res_join=res_join)


class XceptionModule(nn.Module):
    def __init__(self, cin, depth_list, skip, stride, rate, unit_rates, act_inside, bn_kw):
        super().__init__()
        self.skip = skip
        self.act_inside = act_inside
        convs = []
        c = cin
        for i in range(3):
            # pre-activation (act_inside False): the ReLU in front of separable convs 2 and 3
            # reads only the previous pointwise BN output, so it is fused into that BN's apply;
            # the one in front of conv 1 reads the unit input (also the skip path's operand), so
            # the depthwise kernel applies it on load instead.
            convs.append(SeparableConvBN(c, depth_list[i], stride if i == 2 else 1,
                                         rate * unit_rates[i], act_inside, bn_kw,
                                         relu_out=(not act_inside and i < 2) or act_inside))
            c = depth_list[i]
        self.convs = nn.ModuleList(convs)
        self.shortcut = (ConvBN(cin, depth_list[-1], 1, stride, 0, relu=False, **bn_kw)
                         if skip == "conv" else None)
        self.out_channels = depth_list[-1]

    # x feeds the first separable conv and the skip: their gradients meet in one buffer — the
    # skip's contribution (the residual BN's dres, or the 1×1 shortcut's dgrad) is written first
    # and the depthwise dgrad adds its own in its epilogue (ops/gradjoin.py) instead of autograd
    # summing two tensors (TDL_XC_JOIN=0: autograd add)
    grad_join = os.environ.get("TDL_XC_JOIN", "1") == "1"

    def forward(self, x):
        relu_in = not self.act_inside
        join = None
        if (self.grad_join and self.skip in ("sum", "conv") and torch.is_grad_enabled()
                and x.requires_grad and joinable(x, relu_in)):
            join = gradjoin.GradJoin(2)
        # units 2 and 3 read only the previous pointwise BN + ReLU: it is deferred into their
        # depthwise kernels (ops/dwfold.py; a geometry they cannot take applies it as usual)
        kw = {"defer": True} if (dwfold.ENABLED and self.training and torch.is_grad_enabled()) \
            else {}
        r = self.convs[0](x, relu_in=relu_in, join=join, **kw)
        r = self.convs[1](r, **kw)
        if self.skip == "sum":
            # identity skip: the add is folded into the last pointwise BN's apply (one pass,
            # one bf16 rounding of BN(y) + x instead of two)
            return self.convs[2](r, residual=x, res_join=join)
        r = self.convs[2](r)
        if self.skip == "conv":
            return self.shortcut(x, residual=r, join=join)  # BN(shortcut) + residual, no act
        return r


# Xception-41 (core/xception.py:405-465): (block scope, depth_list, skip, num_units, stride,
# unit_rate_list, activation inside the separable convs)
XCEPTION41_BLOCKS = [
    ("entry_flow/block1", [128, 128, 128], "conv", 1, 2, [1, 1, 1], False),
    ("entry_flow/block2", [256, 256, 256], "conv", 1, 2, [1, 1, 1], False),
    ("entry_flow/block3", [728, 728, 728], "conv", 1, 2, [1, 1, 1], False),
    ("middle_flow/block1", [728, 728, 728], "sum", 8, 1, [1, 1, 1], False),
    ("exit_flow/block1", [728, 1024, 1024], "conv", 1, 2, [1, 1, 1], False),
    ("exit_flow/block2", [1536, 1536, 2048], "none", 1, 1, None, True),
]


class Xception(nn.Module):
    """The generic Xception generator (core/xception.py:295-364): the root (3×3/s2 32 → 3×3 64,
    conv+BN+ReLU) then ``stack_blocks_dense`` over ``blocks`` — a list of (scope, depth_list,
    skip_connection_type, num_units, stride, unit_rate_list, activation_fn_in_separable_conv);
    the stride of a block is in its last unit — with atrous output-stride control, and an
    optional global-pool + logits head."""

    def __init__(self, blocks, num_classes=0, in_channels=3, output_stride=None, bn_decay=0.9997,
                 bn_eps=1e-3):
        super().__init__()
        bn_kw = dict(bn_decay=bn_decay, bn_eps=bn_eps)
        self.conv1_1 = ConvBN(in_channels, 32, 3, 2, _fixed_pad(3, 1), relu=True, pad_cin_to=8,
                              **bn_kw)
        self.conv1_2 = ConvBN(32, 64, 3, 1, "SAME", relu=True, **bn_kw)
        target = None if output_stride is None else output_stride // 2
        if output_stride is not None and output_stride % 2 != 0:
            raise ValueError("The output_stride needs to be a multiple of 2.")
        current, rate = 1, 1
        self.units = nn.ModuleList()
        self.unit_names = []
        cin = 64
        seen = {}
        for name, depths, skip, n, stride, urates, act in blocks:
            urates = list(urates) if urates else [1, 1, 1]
            if len(depths) != 3 or len(urates) != 3:
                raise ValueError("Expect three elements in depth_list and unit_rate_list.")
            if skip not in ("conv", "sum", "none"):
                raise ValueError("Unsupported skip connection type.")
            for u in range(n):
                s = stride if u == n - 1 else 1
                if target is not None and current > target:
                    raise ValueError("The target output_stride cannot be reached.")
                if target is not None and current == target:
                    m = XceptionModule(cin, depths, skip, 1, rate, urates, act, bn_kw)
                    rate *= s
                else:
                    m = XceptionModule(cin, depths, skip, s, 1, urates, act, bn_kw)
                    current *= s
                cin = m.out_channels
                self.units.append(m)
                seen[name] = seen.get(name, 0) + 1
                self.unit_names.append(f"{name}/unit_{seen[name]}")
        if target is not None and current != target:
            raise ValueError("The target output_stride cannot be reached.")
        self.num_features = cin
        self.gap = GlobalAvgPool() if num_classes else None
        self.fc = Linear(cin, num_classes) if num_classes else None

    def forward(self, x, return_end_points=False):
        if x.shape[-1] != self.conv1_1.conv._cin_store:
            if x.shape[-1] > self.conv1_1.conv._cin_store:  # never crop input channels
                raise ValueError(f"input has {x.shape[-1]} channels, the stem takes "
                                 f"{self.conv1_1.conv.cin}")
            x = nn.functional.pad(x, (0, self.conv1_1.conv._cin_store - x.shape[-1]))
        x = self.conv1_2(self.conv1_1(x))
        ep = {}
        for name, u in zip(self.unit_names, self.units):
            x = u(x)
            if return_end_points:
                ep[name] = x
        if self.fc is not None:
            x = self.fc(self.gap(x))
        return (x, ep) if return_end_points else x


class Xception41(Xception):
    def __init__(self, num_classes=1000, in_channels=3, output_stride=None, multi_grid=None,
                 bn_decay=0.9997, bn_eps=1e-3):
        blocks = [b if b[5] is not None else b[:5] + (list(multi_grid or [1, 1, 1]),) + b[6:]
                  for b in XCEPTION41_BLOCKS]
        super().__init__(blocks, num_classes, in_channels, output_stride, bn_decay, bn_eps)


def xception_41(num_classes=1000, **kw):
    return Xception41(num_classes=num_classes, **kw)
