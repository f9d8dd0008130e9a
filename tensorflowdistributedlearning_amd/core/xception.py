"""core.xception — reference API (core/xception.py:6-509), built as the *intended* DeepLab
Xception-41 (D8–D10 fixed: importable, 8-unit middle flow, BN after every conv); see
:mod:`models.xception`.
"""
from __future__ import annotations

import collections

import torch.nn.functional as F

from ..models.xception import Xception, Xception41, XceptionModule, SeparableConvBN, _fixed_pad
from ..models.deeplab import SplitSeparableConv  # noqa: F401  (split_separable_conv2d lives in core.layers)
from .layers import split_separable_conv2d  # noqa: F401
from ._scope import get_or_create, to_nhwc, from_nhwc, device_of

Block = collections.namedtuple("Block", ["scope", "unit_fn", "args"])


def fixed_padding(inputs, kernel_size, rate=1):
    """Zero-pad for a k×k (rate) conv with 'VALID' padding (xception.py:18-35), NHWC."""
    t, b, l, r = _fixed_pad(kernel_size, rate)
    return F.pad(inputs, (0, 0, l, r, t, b))


def separable_conv2d_same(in_channels, num_outputs, kernel_size=3, depth_multiplier=1, stride=1,
                          rate=1, activation_fn_in_separable_conv=False, bn_decay=0.9997,
                          bn_eps=1e-3):
    """Module: depthwise (explicit fixed padding at stride>1) + BN → pointwise + BN."""
    if kernel_size != 3 or depth_multiplier != 1:
        raise ValueError("3x3, depth_multiplier 1 only")
    return SeparableConvBN(in_channels, num_outputs, stride, rate, activation_fn_in_separable_conv,
                           dict(bn_decay=bn_decay, bn_eps=bn_eps))


def xception_module(in_channels, depth_list, skip_connection_type, stride, unit_rate_list=None,
                    rate=1, activation_fn_in_separable_conv=False, bn_decay=0.9997, bn_eps=1e-3):
    if len(depth_list) != 3:
        raise ValueError("Expect three elements in depth_list.")
    unit_rate_list = unit_rate_list or [1, 1, 1]
    if len(unit_rate_list) != 3:
        raise ValueError("Expect three elements in unit_rate_list.")
    if skip_connection_type not in ("conv", "sum", "none"):
        raise ValueError("Unsupported skip connection type.")
    return XceptionModule(in_channels, depth_list, skip_connection_type, stride, rate,
                          unit_rate_list, activation_fn_in_separable_conv,
                          dict(bn_decay=bn_decay, bn_eps=bn_eps))


def xception_block(scope, depth_list, skip_connection_type, activation_fn_in_separable_conv,
                   regularize_depthwise, num_units, stride, unit_rate_list=None):
    if unit_rate_list is None:
        unit_rate_list = [1, 1, 1]
    return Block(scope, xception_module, [{
        "depth_list": depth_list, "skip_connection_type": skip_connection_type,
        "activation_fn_in_separable_conv": activation_fn_in_separable_conv,
        "regularize_depthwise": regularize_depthwise, "stride": stride,
        "unit_rate_list": unit_rate_list}] * num_units)


def stack_blocks_dense(in_channels, blocks, output_stride=None):
    """Build the units of ``blocks`` (xception_block specs) with atrous output-stride control
    (core/xception.py:231-292): once the running stride reaches ``output_stride`` further strides
    become dilation.  Returns (nn.ModuleList of units, out_channels)."""
    import torch.nn as nn
    if output_stride is not None and output_stride <= 0:
        raise ValueError("output_stride must be positive")
    current, rate = 1, 1
    units = nn.ModuleList()
    cin = in_channels
    for block in blocks:
        for args in block.args:
            stride = args["stride"]
            if output_stride is not None and current > output_stride:
                raise ValueError("The target output_stride cannot be reached.")
            if output_stride is not None and current == output_stride:
                m = block.unit_fn(cin, args["depth_list"], args["skip_connection_type"], 1,
                                  args.get("unit_rate_list"), rate,
                                  args["activation_fn_in_separable_conv"])
                rate *= stride
            else:
                m = block.unit_fn(cin, args["depth_list"], args["skip_connection_type"], stride,
                                  args.get("unit_rate_list"), 1,
                                  args["activation_fn_in_separable_conv"])
                current *= stride
            units.append(m)
            cin = m.out_channels
    if output_stride is not None and current != output_stride:
        raise ValueError("The target output_stride cannot be reached.")
    return units, cin


def _block_specs(blocks):
    """xception_block specs (Block namedtuples, core/xception.py:367-402) → the model's
    (scope, depth_list, skip, num_units, stride, unit_rate_list, act) rows."""
    rows = []
    for b in blocks:
        # xception_block repeats one unit dict num_units times with the block stride in every
        # unit; the reference stack applies each unit's own stride (stack_blocks_dense, :270-290)
        for a in b.args:
            rows.append((b.scope, list(a["depth_list"]), a["skip_connection_type"], 1,
                         a["stride"], list(a.get("unit_rate_list") or [1, 1, 1]),
                         bool(a["activation_fn_in_separable_conv"])))
    return rows


def xception(inputs, blocks=None, num_classes=None, is_training=True, global_pool=True,
             keep_prob=0.5, output_stride=None, reuse=None, scope=None, data_format="NHWC"):
    """Generic Xception generator (core/xception.py:295-364): the root block, then
    ``stack_blocks_dense`` over ``blocks`` (a list of :func:`xception_block` specs; default: the
    Xception-41 blocks) with atrous output-stride control, and — with ``num_classes`` — global
    pooling + logits.  Builds (or reuses, per ``scope``) the module; returns (net, end_points)
    with one end point per unit ('<scope>/<block>/unit_<i>')."""
    scope = scope or "xception"
    if blocks is None:
        return xception_41(inputs, is_training=is_training, keep_prob=keep_prob,
                           output_stride=output_stride, scope=scope, num_classes=num_classes,
                           data_format=data_format)
    rows = _block_specs(blocks)
    x = to_nhwc(inputs, data_format)
    key = ("xception", scope, output_stride, num_classes, x.shape[-1],
           tuple((r[0], tuple(r[1]), r[2], r[4], tuple(r[5]), r[6]) for r in rows))
    m = get_or_create(key, lambda: Xception(rows, num_classes=num_classes or 0,
                                            in_channels=x.shape[-1],
                                            output_stride=output_stride), device_of(x))
    m.train(bool(is_training))
    y, ep = m(x, return_end_points=True)
    ep = {f"{scope}/{k}": v for k, v in ep.items()}
    return (from_nhwc(y, data_format) if y.dim() == 4 else y), ep


def xception_41(inputs, is_training=True, keep_prob=0.5, output_stride=None,
                regularize_depthwise=False, multi_grid=None, reuse=None, scope="xception_41",
                num_classes=None, data_format="NHWC"):
    """Builds (or reuses, per ``scope``) Xception-41 and applies it.  Returns (net, end_points)
    with ``net`` the exit-flow features (or logits when ``num_classes``)."""
    x = to_nhwc(inputs, data_format)
    m = get_or_create(("xception_41", scope, output_stride, tuple(multi_grid or []), num_classes),
                      lambda: Xception41(num_classes=num_classes or 0,
                                         in_channels=x.shape[-1],
                                         output_stride=output_stride, multi_grid=multi_grid),
                      device_of(x))
    m.train(bool(is_training))
    y = m(x)
    return from_nhwc(y, data_format) if y.dim() == 4 else y, {f"{scope}/output": y}
