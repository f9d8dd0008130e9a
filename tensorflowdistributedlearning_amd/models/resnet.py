"""Standard ImageNet ResNets (v1.5: stride on the 3×3 conv) in NHWC — the north-star workloads of
BASELINE.json (ResNet-18/50/152 at 224×224).  Not present in the reference, whose only ResNet is the
beta-variant DeepLab encoder (core/resnet.py:284-354, see :mod:`models.deeplab`); the reference's
optional classification head (core/resnet.py:246-256) is what ``num_classes`` reproduces.

Every conv is followed by BN whose batch statistics are accumulated in the conv's epilogue; the
bottleneck's last BN, the residual add and the ReLU are a single fused kernel pass; the first two
BN + ReLU of a block are folded into the next conv's operand staging (ops/bnconv.py).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops import gradjoin

from .layers import ConvBN, MaxPool, GlobalAvgPool, Linear, RowPackedConv2d, resolve_padding
from ..ops.pool import bn_relu_max_pool, bn_relu_max_pool_ok


_CFG = {
    18: ("basic", (2, 2, 2, 2)),
    34: ("basic", (3, 4, 6, 3)),
    50: ("bottleneck", (3, 4, 6, 3)),
    101: ("bottleneck", (3, 4, 23, 3)),
    152: ("bottleneck", (3, 8, 36, 3)),
}


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, width, stride, bn_kw):
        super().__init__()
        self.conv1 = ConvBN(cin, width, 3, stride, "sym", relu=True, init="kaiming_fan_out", **bn_kw)
        self.conv2 = ConvBN(width, width, 3, 1, "sym", relu=True, init="kaiming_fan_out", **bn_kw)
        self.downsample = None
        if stride != 1 or cin != width:
            self.downsample = ConvBN(cin, width, 1, stride, 0, relu=False,
                                     init="kaiming_fan_out", **bn_kw)

    def forward(self, x):
        # x feeds conv1 and the shortcut: one shared gradient buffer (ops/gradjoin.py)
        join = gradjoin.make(2, x) if self.training else None
        if self.downsample is None:
            sc, res_join = x, join
        else:
            sc, res_join = self.downsample(x, join=join), None
        # conv1's BN + ReLU is folded into conv2 (ops/bnconv.py; applied where it cannot be)
        out = self.conv1(x, join=join, defer=True)
        return self.conv2(out, residual=sc, res_join=res_join)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride, bn_kw):
        super().__init__()
        out = width * 4
        self.conv1 = ConvBN(cin, width, 1, 1, 0, relu=True, init="kaiming_fan_out", **bn_kw)
        self.conv2 = ConvBN(width, width, 3, stride, "sym", relu=True, init="kaiming_fan_out",
                            **bn_kw)
        self.conv3 = ConvBN(width, out, 1, 1, 0, relu=True, init="kaiming_fan_out", **bn_kw)
        self.downsample = None
        if stride != 1 or cin != out:
            self.downsample = ConvBN(cin, out, 1, stride, 0, relu=False, init="kaiming_fan_out",
                                     **bn_kw)

    def forward(self, x):
        # x feeds conv1 and the shortcut: one shared gradient buffer (ops/gradjoin.py)
        join = gradjoin.make(2, x) if self.training else None
        if self.downsample is None:
            sc, res_join = x, join
        else:
            sc, res_join = self.downsample(x, join=join), None
        # bn1 + ReLU folded into conv2, bn2 + ReLU into conv3 (ops/bnconv.py): their outputs are
        # never written (/root/reference/core/resnet.py:134-144 conv+BN+ReLU, single consumers)
        y = self.conv1(x, join=join, defer=True)
        y = self.conv2(y, defer=True)
        return self.conv3(y, residual=sc, res_join=res_join)


class ResNet(nn.Module):
    """ResNet-{18,34,50,101,152}. Input NHWC [N, H, W, 3 or 8] (channels 3..7 zero)."""

    def __init__(self, depth=50, num_classes=1000, bn_decay=0.9, bn_eps=1e-5, in_channels=3,
                 width=64):
        super().__init__()
        kind, layers = _CFG[depth]
        block = Bottleneck if kind == "bottleneck" else BasicBlock
        bn_kw = dict(bn_decay=bn_decay, bn_eps=bn_eps)
        self.depth = depth
        self.in_channels = in_channels
        # 7×7/s2 stem on the row-packed image (K = 7·24 instead of 7·7·8, RowPackedConv2d);
        # TDL_STEM_PACK=0: the plain conv on the 8-channel padded input
        packed = in_channels * 7 <= 64 and os.environ.get("TDL_STEM_PACK", "1") == "1"
        self.stem = ConvBN(in_channels, width, 7, 2, "sym", relu=True, init="kaiming_fan_out",
                           pad_cin_to=8, conv_cls=RowPackedConv2d if packed else None, **bn_kw)
        self.pool = MaxPool(3, 2, "sym")
        stages = []
        cin = width
        for i, n in enumerate(layers):
            w = width * (2 ** i)
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(block(cin, w, stride, bn_kw))
                cin = w * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.gap = GlobalAvgPool()
        self.num_features = cin
        self.fc = Linear(cin, num_classes) if num_classes else None

    @property
    def input_channels_padded(self):
        return self.stem.conv._cin_store

    def forward_features(self, x):
        if x.shape[-1] != self.stem.conv._cin_store:
            x = nn.functional.pad(x, (0, self.stem.conv._cin_store - x.shape[-1]))
        if (self.training and self.stem.bn.training and self.stem.relu
                and bn_relu_max_pool_ok(x, self.stem.bn)):
            # training BN: the stem BN + ReLU runs inside the max-pool (ops/pool.bn_relu_max_pool)
            z, stats = self.stem.conv(x, want_stats=True)
            pad = resolve_padding(self.pool.padding, z.shape[1], z.shape[2], self.pool.k,
                                  self.pool.k, (self.pool.stride, self.pool.stride), (1, 1))
            x = bn_relu_max_pool(z, stats, self.stem.bn, self.pool.k, self.pool.stride, pad)
        else:
            x = self.stem(x)
            x = self.pool(x)
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        return x

    def forward(self, x):
        x = self.forward_features(x)
        x = self.gap(x)
        if self.fc is not None:
            x = self.fc(x)
        return x


def resnet18(**kw):
    return ResNet(18, **kw)


def resnet34(**kw):
    return ResNet(34, **kw)


def resnet50(**kw):
    return ResNet(50, **kw)


def resnet101(**kw):
    return ResNet(101, **kw)


def resnet152(**kw):
    return ResNet(152, **kw)
