"""core.resnet — reference API (core/resnet.py) on :mod:`models.deeplab`.

Reference functions and where they map:
  channel_dimension / _get_dimension (resnet.py:16-54)      → shape helpers
  resnet_arg_scope (:357-395)                               → layer defaults; a context manager
                                                              (``with resnet_arg_scope(...)``,
                                                              slim.arg_scope) the builders read
  bottleneck / basic_block (:57-152)                        → :class:`models.deeplab.BetaUnit`
  root_block_fn_for_beta_variant (:155-168)                 → beta stem (3 × conv+BN+ReLU)
  resnet_v2_beta_block (:260-281), resnet_v2 (:284-354),
  resnet_v2_beta (:171-257)                                 → block specs / encoder
  resnet_model (:398-496)                                   → :class:`models.deeplab.DeepLabResNet`
Tensors are NHWC (``data_format="NCHW"`` inputs are transposed at the boundary).
"""
from __future__ import annotations

import collections

import torch
import torch.nn as nn

from ..models.deeplab import DeepLabResNet, BetaUnit
from ..models.layers import ConvBN, Conv2d
from ..ops.pool import global_avg_pool
from ..ops.loss import softmax_eval
from ._scope import get_or_create, to_nhwc, from_nhwc, device_of

_DEFAULT_MULTI_GRID = [2, 2, 2]

Block = collections.namedtuple("Block", ["scope", "unit_fn", "args"])


def _get_dimension(shape, dim, min_rank=1):
    dims = list(shape)
    if len(dims) < min_rank:
        raise ValueError(f"rank of shape must be at least {min_rank} not: {len(dims)}")
    v = dims[dim]
    if v is None:
        raise ValueError(f"dimension {dim} of shape must be known but is None: {shape}")
    return int(v)


def channel_dimension(shape, data_format, min_rank=1):
    return _get_dimension(shape, 1 if data_format == "NCHW" else -1, min_rank=min_rank)


_ARG_DEFAULTS = {"weight_decay": 0.0001, "batch_norm_decay": 0.997, "batch_norm_epsilon": 1e-5,
                 "batch_norm_scale": True}
_ARG_STACK = []


class ResNetArgScope(dict):
    """What ``resnet_arg_scope`` returns (core/resnet.py:357-395): the layer defaults of every
    conv — L2 weight decay, He (variance-scaling) init, BN + ReLU post-activation, SAME max-pool.

    As in slim, it is applied with a ``with`` block (``with resnet_arg_scope(...):`` or
    ``with arg_scope(sc):``): builders called inside — :func:`bottleneck`, :func:`basic_block`,
    :func:`root_block_fn_for_beta_variant`, :func:`resnet_v2` — take their BN decay / epsilon /
    scale and weight decay from the innermost active scope unless given explicitly."""

    def __enter__(self):
        _ARG_STACK.append(self)
        return self

    def __exit__(self, *exc):
        _ARG_STACK.remove(self)
        return False


def arg_scope(sc):
    """slim.arg_scope(sc) for a :class:`ResNetArgScope` (it is its own context manager)."""
    return sc


def _arg(name, value):
    if value is not None:
        return value
    for sc in reversed(_ARG_STACK):
        if name in sc:
            return sc[name]
    return _ARG_DEFAULTS[name]


def resnet_arg_scope(weight_decay=0.0001, batch_norm_decay=0.997, batch_norm_epsilon=1e-5,
                     batch_norm_scale=True):
    """Defaults applied to every conv of the ResNet (L2 decay, He init, BN+ReLU, SAME pooling)."""
    return ResNetArgScope({
        "weight_decay": weight_decay, "batch_norm_decay": batch_norm_decay,
        "batch_norm_epsilon": batch_norm_epsilon, "batch_norm_scale": batch_norm_scale,
        "initializer": "variance_scaling(2.0, fan_in, truncated_normal)",
        "normalizer": "batch_norm", "activation": "relu", "max_pool_padding": "SAME"})


def _bn_kw(decay, eps, scale):
    return dict(decay=_arg("batch_norm_decay", decay), eps=_arg("batch_norm_epsilon", eps),
                scale=_arg("batch_norm_scale", scale))


def bottleneck(depth_in, depth, depth_bottleneck, stride, unit_rate=1, rate=1,
               batch_norm_decay=None, batch_norm_epsilon=None, batch_norm_scale=None):
    """Hybrid pre/post-activation bottleneck unit module (core/resnet.py:94-152)."""
    return BetaUnit(depth_in, depth, depth_bottleneck, stride, rate * unit_rate, "bottleneck",
                    _bn_kw(batch_norm_decay, batch_norm_epsilon, batch_norm_scale))


def basic_block(depth_in, depth, depth_bottleneck, stride, unit_rate=1, rate=1,
                batch_norm_decay=None, batch_norm_epsilon=None, batch_norm_scale=None):
    """basic_block unit module (core/resnet.py:57-91)."""
    return BetaUnit(depth_in, depth, depth_bottleneck, stride, rate * unit_rate, "basic_block",
                    _bn_kw(batch_norm_decay, batch_norm_epsilon, batch_norm_scale))


def root_block_fn_for_beta_variant(in_channels=2, batch_norm_decay=None, batch_norm_epsilon=None):
    """3×3/s2 64 → 3×3 64 → 3×3 128, each conv+BN+ReLU (core/resnet.py:155-168)."""
    kw = dict(bn_decay=_arg("batch_norm_decay", batch_norm_decay),
              bn_eps=_arg("batch_norm_epsilon", batch_norm_epsilon))
    return nn.Sequential(ConvBN(in_channels, 64, 3, 2, "SAME", relu=True, pad_cin_to=8, **kw),
                         ConvBN(64, 64, 3, 1, "SAME", relu=True, **kw),
                         ConvBN(64, 128, 3, 1, "SAME", relu=True, **kw))


def resnet_v2_beta_block(scope, base_depth, num_units, stride, block_fn=bottleneck):
    """Block spec: num_units-1 units of stride 1 + a final unit with ``stride``."""
    unit = {"depth": base_depth * 4, "depth_bottleneck": base_depth, "stride": 1, "unit_rate": 1}
    return Block(scope, block_fn, [dict(unit)] * (num_units - 1) + [dict(unit, stride=stride)])


class ResNetV2Beta(nn.Module):
    """``resnet_v2_beta`` as a module (core/resnet.py:171-257): the beta-stem encoder, then the
    optional ``global_pool`` (spatial mean, keepdims, 'pool5') and the ``num_classes`` head — a
    1×1 conv with bias and no normaliser ('logits') whose softmax is end_points['predictions']."""

    def __init__(self, encoder, num_classes=None, global_pool=False):
        super().__init__()
        self.encoder = encoder
        self.global_pool = global_pool
        self.logits = (Conv2d(encoder.encoder_channels, num_classes, 1, 1, 0, bias=True,
                              pad_cout_to=8) if num_classes else None)
        self.num_classes = num_classes

    def forward(self, x):
        net, ep = self.encoder.forward_encoder(x)
        scope = f"{self.encoder.model_name}/resnet_v2"
        if self.global_pool:
            net = global_avg_pool(net.contiguous(), keepdims=True)
            ep[f"{scope}/pool5"] = net
        if self.logits is not None:
            net = self.logits(net.contiguous())
            if net.shape[-1] != self.num_classes:
                net = net[..., :self.num_classes].contiguous()
            ep[f"{scope}/logits"] = net
            # the HIP softmax head (ops/loss.softmax_eval; fp32 rows on the CPU)
            ep["predictions"] = softmax_eval(net.reshape(-1, net.shape[-1]), probs=True)[2] \
                .reshape(net.shape)
        return net, ep


def resnet_v2(inputs=None, n_blocks=(3, 4, 6), block_type="bottleneck", num_classes=None,
              is_training=None, global_pool=False, output_stride=None, multi_grid=None,
              reuse=None, scope="resnet_v2_34", data_format="NHWC", **kw):
    """Block specs of the reference encoder (core/resnet.py:284-354); when ``inputs`` is given,
    builds (or reuses, per ``scope``) the ``resnet_v2_beta`` network and returns
    (net, end_points): ``net`` is the block4 features, their global mean (``global_pool``) or
    the logits of the 1×1 classification conv (``num_classes``; end_points['predictions'] holds
    the softmax), as at core/resnet.py:246-256."""
    if multi_grid is None:
        multi_grid = _DEFAULT_MULTI_GRID
    elif len(multi_grid) != 3:
        raise ValueError("Expect multi_grid to have length 3.")
    if inputs is None:
        fn = basic_block if block_type == "basic_block" else bottleneck
        return [resnet_v2_beta_block("block1", 128, n_blocks[0], 2, fn),
                resnet_v2_beta_block("block2", 258, n_blocks[1], 2, fn),
                resnet_v2_beta_block("block3", 512, n_blocks[2], 2, fn),
                Block("block4", fn, [{"depth": 1024, "depth_bottleneck": 256, "stride": 1,
                                      "unit_rate": r} for r in multi_grid])]
    x = to_nhwc(inputs, data_format)
    bn = _bn_kw(kw.pop("batch_norm_decay", None), kw.pop("batch_norm_epsilon", None),
                kw.pop("batch_norm_scale", None))
    wd = _arg("weight_decay", kw.pop("weight_decay", None))
    m = get_or_create(("resnet_v2", scope, tuple(n_blocks), block_type, output_stride,
                       tuple(multi_grid), num_classes, bool(global_pool),
                       x.shape[1], x.shape[2], x.shape[3]),
                      lambda: ResNetV2Beta(
                          DeepLabResNet(model_name=scope, in_channels=x.shape[3],
                                        output_stride=output_stride,
                                        input_shape=(x.shape[1], x.shape[2]),
                                        n_blocks=n_blocks, block_type=block_type,
                                        multi_grid=tuple(multi_grid), batch_norm_decay=bn["decay"],
                                        batch_norm_epsilon=bn["eps"], batch_norm_scale=bn["scale"],
                                        weight_decay=wd, **kw),
                          num_classes=num_classes, global_pool=global_pool),
                      device_of(x))
    m.train(bool(is_training) if is_training is not None else m.training)
    net, ep = m(x)
    return from_nhwc(net, data_format), ep


resnet_v2_beta = resnet_v2


def resnet_model(input, model_name, weight_decay, batch_norm_decay, batch_norm_epsilon,
                 batch_norm_scale, data_format, is_training, output_stride, base_depth, input_shape,
                 n_blocks, block_type):
    """The reference's DeepLab net (core/resnet.py:398-496): returns pre-activation logits
    [N, H, W, 1] (NHWC) / [N, 1, H, W] (NCHW).  Variables live in the module cached under
    ``model_name`` (the reference's root variable scope)."""
    if len(n_blocks) != 3:
        raise ValueError("Expect n_blocks to have length 3.")
    x = to_nhwc(input, data_format)
    m = get_or_create(("resnet_model", model_name),
                      lambda: DeepLabResNet(model_name=model_name, in_channels=x.shape[3],
                                            output_stride=output_stride, base_depth=base_depth,
                                            input_shape=tuple(input_shape),
                                            n_blocks=tuple(n_blocks), block_type=block_type,
                                            batch_norm_decay=batch_norm_decay,
                                            batch_norm_epsilon=batch_norm_epsilon,
                                            batch_norm_scale=batch_norm_scale,
                                            weight_decay=weight_decay),
                      device_of(x))
    m.train(bool(is_training))
    return from_nhwc(m(x), data_format)
