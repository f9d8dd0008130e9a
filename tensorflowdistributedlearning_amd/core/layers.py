"""core.layers — reference API (core/layers.py).

* ``split_separable_conv2d`` (layers.py:6-49): depthwise 3×3 (rate, σ=0.33, bias+ReLU) →
  pointwise 1×1 (σ=0.06, BN+ReLU); module cached per ``scope``.
* ``_fixed_padding`` (:52-79): pad (k−1)//2 before / rest after, CONSTANT or SYMMETRIC.
* ``_upsample`` (:82-109): symmetric pad 1 → TF1 legacy bilinear → crop (HIP kernel on GPU);
  ``out_shape`` is (H, W) (D12 fixed).
"""
from __future__ import annotations

import torch.nn.functional as F

from ..models.deeplab import SplitSeparableConv
from ..ops.upsample import upsample as _up
from ._scope import get_or_create, to_nhwc, from_nhwc, device_of


def split_separable_conv2d(inputs, filters, kernel_size=3, rate=1, weight_decay=0.00004,
                           depthwise_weights_initializer_stddev=0.33,
                           pointwise_weights_initializer_stddev=0.06, scope=None,
                           data_format="NHWC", batch_norm_decay=0.997, batch_norm_epsilon=1e-5,
                           batch_norm_scale=True):
    if kernel_size != 3:
        raise ValueError("only 3x3 depthwise kernels are provided")
    x = to_nhwc(inputs, data_format)
    m = get_or_create(("split_separable_conv2d", scope, x.shape[-1], filters, rate),
                      lambda: SplitSeparableConv(x.shape[-1], filters, rate,
                                                 dict(decay=batch_norm_decay,
                                                      eps=batch_norm_epsilon,
                                                      scale=batch_norm_scale)),
                      device_of(x))
    return from_nhwc(m(x), data_format)


def _fixed_padding(inputs, kernel_size, data_format="NCHW", mode="CONSTANT"):
    pad_total = kernel_size - 1
    b = pad_total // 2
    e = pad_total - b
    x = to_nhwc(inputs, data_format)
    t = x.permute(0, 3, 1, 2)
    if mode == "CONSTANT":
        t = F.pad(t, (b, e, b, e))
    elif mode == "SYMMETRIC":
        # symmetric (edge repeated): reflect of the edge-padded tensor
        if b == 0 and e == 0:
            pass
        else:
            idx_h = _sym_index(t.shape[2], b, e, t.device)
            idx_w = _sym_index(t.shape[3], b, e, t.device)
            t = t.index_select(2, idx_h).index_select(3, idx_w)
    elif mode == "REFLECT":
        t = F.pad(t, (b, e, b, e), mode="reflect")
    else:
        raise ValueError(mode)
    return from_nhwc(t.permute(0, 2, 3, 1).contiguous(), data_format)


def _sym_index(n, b, e, device):
    import torch
    idx = []
    for i in range(-b, n + e):
        j = i
        while j < 0 or j >= n:
            j = -j - 1 if j < 0 else 2 * n - 1 - j
        idx.append(j)
    return torch.tensor(idx, device=device)


def _upsample(inputs, out_shape, data_format="NCHW"):
    x = to_nhwc(inputs, data_format)
    return from_nhwc(_up(x, out_shape), data_format)
