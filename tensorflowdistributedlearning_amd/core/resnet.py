"""core.resnet — reference API (core/resnet.py) on :mod:`models.deeplab`.

Reference functions and where they map:
  channel_dimension / _get_dimension (resnet.py:16-54)      → shape helpers
  resnet_arg_scope (:357-395)                               → dict of layer defaults
  bottleneck / basic_block (:57-152)                        → :class:`models.deeplab.BetaUnit`
  root_block_fn_for_beta_variant (:155-168)                 → beta stem (3 × conv+BN+ReLU)
  resnet_v2_beta_block (:260-281), resnet_v2 (:284-354),
  resnet_v2_beta (:171-257)                                 → block specs / encoder
  resnet_model (:398-496)                                   → :class:`models.deeplab.DeepLabResNet`
Tensors are NHWC (``data_format="NCHW"`` inputs are transposed at the boundary).
"""
from __future__ import annotations

import collections

import torch.nn as nn

from ..models.deeplab import DeepLabResNet, BetaUnit
from ..models.layers import ConvBN
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


def resnet_arg_scope(weight_decay=0.0001, batch_norm_decay=0.997, batch_norm_epsilon=1e-5,
                     batch_norm_scale=True):
    """Defaults applied to every conv of the ResNet (L2 decay, He init, BN+ReLU, SAME pooling)."""
    return {"weight_decay": weight_decay, "batch_norm_decay": batch_norm_decay,
            "batch_norm_epsilon": batch_norm_epsilon, "batch_norm_scale": batch_norm_scale,
            "initializer": "variance_scaling(2.0, fan_in, truncated_normal)",
            "normalizer": "batch_norm", "activation": "relu", "max_pool_padding": "SAME"}


def bottleneck(depth_in, depth, depth_bottleneck, stride, unit_rate=1, rate=1,
               batch_norm_decay=0.997, batch_norm_epsilon=1e-5, batch_norm_scale=True):
    """Hybrid pre/post-activation bottleneck unit module (core/resnet.py:94-152)."""
    return BetaUnit(depth_in, depth, depth_bottleneck, stride, rate * unit_rate, "bottleneck",
                    dict(decay=batch_norm_decay, eps=batch_norm_epsilon, scale=batch_norm_scale))


def basic_block(depth_in, depth, depth_bottleneck, stride, unit_rate=1, rate=1,
                batch_norm_decay=0.997, batch_norm_epsilon=1e-5, batch_norm_scale=True):
    """basic_block unit module (core/resnet.py:57-91)."""
    return BetaUnit(depth_in, depth, depth_bottleneck, stride, rate * unit_rate, "basic_block",
                    dict(decay=batch_norm_decay, eps=batch_norm_epsilon, scale=batch_norm_scale))


def root_block_fn_for_beta_variant(in_channels=2, batch_norm_decay=0.997, batch_norm_epsilon=1e-5):
    """3×3/s2 64 → 3×3 64 → 3×3 128, each conv+BN+ReLU (core/resnet.py:155-168)."""
    kw = dict(bn_decay=batch_norm_decay, bn_eps=batch_norm_epsilon)
    return nn.Sequential(ConvBN(in_channels, 64, 3, 2, "SAME", relu=True, pad_cin_to=8, **kw),
                         ConvBN(64, 64, 3, 1, "SAME", relu=True, **kw),
                         ConvBN(64, 128, 3, 1, "SAME", relu=True, **kw))


def resnet_v2_beta_block(scope, base_depth, num_units, stride, block_fn=bottleneck):
    """Block spec: num_units-1 units of stride 1 + a final unit with ``stride``."""
    unit = {"depth": base_depth * 4, "depth_bottleneck": base_depth, "stride": 1, "unit_rate": 1}
    return Block(scope, block_fn, [dict(unit)] * (num_units - 1) + [dict(unit, stride=stride)])


def resnet_v2(inputs=None, n_blocks=(3, 4, 6), block_type="bottleneck", num_classes=None,
              is_training=None, global_pool=False, output_stride=None, multi_grid=None,
              reuse=None, scope="resnet_v2_34", data_format="NHWC", **kw):
    """Block specs of the reference encoder (core/resnet.py:284-354); when ``inputs`` is given,
    builds (or reuses) the encoder and returns (net, end_points)."""
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
    m = get_or_create(("resnet_v2", scope, tuple(n_blocks), block_type, output_stride,
                       tuple(multi_grid), x.shape[1], x.shape[2], x.shape[3]),
                      lambda: DeepLabResNet(model_name=scope, in_channels=min(x.shape[3], 8),
                                            output_stride=output_stride,
                                            input_shape=(x.shape[1], x.shape[2]),
                                            n_blocks=n_blocks, block_type=block_type,
                                            multi_grid=tuple(multi_grid), **kw),
                      device_of(x))
    m.train(bool(is_training) if is_training is not None else m.training)
    _, ep = m(x, return_end_points=True)
    key = f"{scope}/resnet_v2/block4"
    return from_nhwc(ep[key], data_format), ep


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
                      lambda: DeepLabResNet(model_name=model_name, in_channels=min(x.shape[3], 8),
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
