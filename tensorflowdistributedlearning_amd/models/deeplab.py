"""The reference's trained model: DeepLabv3+-style ResNet-v2-beta encoder + ASPP + decoder
(core/resnet.py:398-496), NHWC.

Structure (exact replay of the reference):
  root (beta stem, core/resnet.py:155-168): 3×3/s2 64 → 3×3 64 → 3×3 128 (conv+BN+ReLU each,
    TF 'SAME' padding) → max-pool 3×3/s2 SAME → ``postnorm`` BN+ReLU (core/resnet.py:240-242);
  4 blocks of hybrid pre/post-activation units (``bottleneck`` core/resnet.py:94-152 or
    ``basic_block`` :57-91) with widths 128 / 258 / 512 / (1024, 256) and ``stack_blocks_dense``
    atrous control: once the running stride reaches ``output_stride/4`` further strides become
    dilation (multi-grid (1, 2, 1) in block4);
  ASPP ("assp", :440-472): 1×1 | 3 × split-separable 3×3 at rates 2/4/8 | image pooling → concat →
    1×1;  ``_upsample`` to the block1 resolution (D11 fixed: derived, not hard-coded 26×26);
  decoder (:476-496): 1×1 on ``block1/unit_1/bottleneck_v2/conv{3|2}`` → concat → 3×3 → 1 logit
    (bias, no BN) → ``_upsample`` to the input size.

The 3×3 conv followed by ``resnet_utils.subsample`` (core/resnet.py:137-140) is computed as one
stride-s conv with symmetric padding — identical math, 1/s² of the FLOPs.

``tf_names()`` maps every parameter/buffer to the reference's TF variable name
so checkpoints use the reference layout.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .layers import ConvBN, Conv2d, BNAct, MaxPool, DepthwiseConv2d, BatchNorm
from ..ops.pool import max_pool2d, global_avg_pool
from ..ops.upsample import upsample, upsample_into
from ..ops.elementwise import add_relu
from ..ops import gradjoin
from ..ops.bn import ResidualLink
from ..ops.common import export_impl


class _Subsample(nn.Module):
    def __init__(self, stride):
        super().__init__()
        self.stride = stride

    def forward(self, x):
        if self.stride == 1:
            return x
        return max_pool2d(x, 1, self.stride, (0, 0, 0, 0))


class BetaUnit(nn.Module):
    """``bottleneck`` / ``basic_block`` unit of core/resnet.py (hybrid pre/post activation)."""

    def __init__(self, cin, depth, depth_bottleneck, stride, rate, block_type, bn_kw, align=None):
        """``align``: channel counts that are not a multiple of it (the reference's 258-wide
        block2 bottleneck, defect D7) are carried physically padded with zero channels, so every conv of the unit
        runs on the aligned LDS-DMA kernels; parameters keep their logical shapes."""
        super().__init__()
        self.block_type = block_type
        self.stride = stride
        pad = dict(pad_cin_to=align, pad_cout_to=align)
        self.preact = BNAct(cin, relu=True, c_phys=_round_up(cin, align), **bn_kw)
        out_c = depth if block_type == "bottleneck" else depth_bottleneck
        self.out_channels = out_c
        if out_c == cin:
            self.shortcut = None
            self.subsample = _Subsample(stride)
        else:
            self.shortcut = Conv2d(cin, out_c, 1, stride, 0, bias=True, **pad)
            self.subsample = None
        cbn = dict(bn_decay=bn_kw["decay"], bn_eps=bn_kw["eps"], bn_scale=bn_kw["scale"], **pad)
        if block_type == "bottleneck":
            self.conv1 = ConvBN(cin, depth_bottleneck, 1, 1, 0, relu=True, **cbn)
            # 3×3 (rate) at stride 1 + subsample(stride) == stride-s conv, symmetric padding
            self.conv2 = ConvBN(depth_bottleneck, depth_bottleneck, 3, stride, "sym", rate,
                                relu=True, **cbn)
            self.conv3 = Conv2d(depth_bottleneck, depth, 1, 1, 0, bias=True, **pad)
        else:
            self.conv1 = ConvBN(cin, depth_bottleneck, 3, stride, "sym", 1, relu=True, **cbn)
            self.conv2 = None
            self.conv3 = Conv2d(depth_bottleneck, depth_bottleneck, 3, 1, "sym", rate, bias=True,
                                **pad)

    def forward(self, x, end_points=None, name=None):
        return self._run(x, end_points, name, None, False)[0]

    def forward_fused(self, x, stats=None):
        """The unit with its output ``relu(conv3 + bias + shortcut)`` computed in conv3's
        epilogue, which also accumulates the BN sums of that output for the next unit's
        pre-activation BN (training).  ``stats``: those sums for this unit's input.  Returns
        ``(y, stats_of_y)``; the conv3 end point (the pre-add conv3 output) is not produced."""
        return self._run(x, None, None, stats, True)

    def _run(self, x, end_points, name, stats, fuse_out):
        # identity shortcut of a fused unit: x feeds the pre-activation BN and conv3's residual
        # epilogue — the BN backward adds the residual gradient to its dx (ops/bn.ResidualLink)
        link = (ResidualLink() if fuse_out and self.shortcut is None and self.stride == 1
                and torch.is_grad_enabled() and x.requires_grad else None)
        preact = self.preact(x, stats=stats, link=link)
        if self.shortcut is None:
            sc, join = self.subsample(x), None
        else:
            # preact feeds the projection shortcut and conv1: both dgrads write one gradient
            # buffer (the second accumulates in its epilogue and applies the preact BN's ReLU
            # mask, ops/gradjoin.py) instead of autograd summing two tensors
            join = gradjoin.make(2, preact) if self.training else None
            sc = self.shortcut(preact, join=join)
        r = self.conv1(preact, join=join)
        if self.conv2 is not None:
            r = self.conv2(r)
        if fuse_out:
            if self.training:
                return self.conv3(r, want_stats=True, residual=sc, relu=True, res_link=link)
            return self.conv3(r, residual=sc, relu=True, res_link=link), None
        r = self.conv3(r)
        if end_points is not None and name is not None:
            last = "conv3" if self.block_type == "bottleneck" else "conv2"
            end_points[f"{name}/bottleneck_v2/{last}"] = _logical(r, self.out_channels)
        return add_relu(sc, r), None


def _round_up(c, multiple):
    return c if not multiple else (c + multiple - 1) // multiple * multiple


def _logical(t, c):
    """The logical channels of a (possibly channel-padded) NHWC tensor."""
    return t if t.shape[-1] == c else t[..., :c]


class SplitSeparableConv(nn.Module):
    """core/layers.py:6-49: depthwise 3×3 (rate, bias + ReLU, σ=0.33) → pointwise 1×1 +BN+ReLU
    (σ=0.06)."""

    def __init__(self, cin, filters, rate, bn_kw):
        super().__init__()
        self.depthwise = DepthwiseConv2d(cin, 3, 1, "SAME", rate, bias=True, relu=True,
                                         init_std=0.33)
        self.pointwise = ConvBN(cin, filters, 1, 1, 0, relu=True, init="trunc_normal",
                                init_std=0.06, bn_decay=bn_kw["decay"], bn_eps=bn_kw["eps"],
                                bn_scale=bn_kw["scale"])

    def forward(self, x, into=None, join=None):
        return self.pointwise(self.depthwise(x, join=join), into=into)


class DeepLabResNet(nn.Module):
    """``resnet_model`` (core/resnet.py:398) as an nn.Module; returns logits [N, H, W, 1]."""

    def __init__(self, model_name="model", in_channels=2, output_stride=8, base_depth=256,
                 input_shape=(101, 101), n_blocks=(3, 4, 6), block_type="bottleneck",
                 batch_norm_decay=0.99, batch_norm_epsilon=0.001, batch_norm_scale=True,
                 weight_decay=0.001, multi_grid=(1, 2, 1), block_widths=(128, 258, 512),
                 channel_align=8):
        super().__init__()
        if len(n_blocks) != 3:
            raise ValueError("Expect n_blocks to have length 3.")
        if output_stride is not None and output_stride % 4 != 0:
            raise ValueError("The output_stride needs to be a multiple of 4.")
        if len(multi_grid) != 3:
            raise ValueError("Expect multi_grid to have length 3.")
        self.model_name = model_name
        self.block_type = block_type
        self.input_shape = tuple(input_shape)
        self.weight_decay = weight_decay
        bn_kw = dict(decay=batch_norm_decay, eps=batch_norm_epsilon, scale=batch_norm_scale)
        cbn = dict(bn_decay=batch_norm_decay, bn_eps=batch_norm_epsilon, bn_scale=batch_norm_scale)
        self.in_channels = in_channels
        # root block (beta variant)
        self.conv1_1 = ConvBN(in_channels, 64, 3, 2, "SAME", relu=True, pad_cin_to=8, **cbn)
        self.conv1_2 = ConvBN(64, 64, 3, 1, "SAME", relu=True, **cbn)
        self.conv1_3 = ConvBN(64, 128, 3, 1, "SAME", relu=True, **cbn)
        self.pool1 = MaxPool(3, 2, "SAME")
        self.postnorm = BNAct(128, relu=True, **bn_kw)
        # block specs
        specs = []
        for bi, (base, n) in enumerate(zip(block_widths, n_blocks)):
            units = [dict(depth=base * 4, depth_bottleneck=base, stride=1, unit_rate=1)
                     for _ in range(n - 1)]
            units.append(dict(depth=base * 4, depth_bottleneck=base, stride=2, unit_rate=1))
            specs.append((f"block{bi + 1}", units))
        specs.append(("block4", [dict(depth=1024, depth_bottleneck=256, stride=1, unit_rate=r)
                                 for r in multi_grid]))
        # stack_blocks_dense atrous control (slim resnet_utils; output_stride /= 4 at :239)
        target = None if output_stride is None else output_stride // 4
        current_stride, rate = 1, 1
        self.blocks = nn.ModuleList()
        self.block_names = []
        cin = 128
        for bname, units in specs:
            mods = nn.ModuleList()
            for u in units:
                if target is not None and current_stride == target:
                    unit = BetaUnit(cin, u["depth"], u["depth_bottleneck"], 1, rate * u["unit_rate"],
                                    block_type, bn_kw, channel_align)
                    rate *= u["stride"]
                else:
                    unit = BetaUnit(cin, u["depth"], u["depth_bottleneck"], u["stride"],
                                    u["unit_rate"], block_type, bn_kw, channel_align)
                    current_stride *= u["stride"]
                cin = unit.out_channels
                mods.append(unit)
            self.blocks.append(mods)
            self.block_names.append(bname)
        if target is not None and current_stride != target:
            raise ValueError("The target output_stride cannot be reached.")
        self.encoder_channels = cin
        # ASPP
        self.assp_conv_1x1 = ConvBN(cin, base_depth, 1, 1, 0, relu=True, **cbn)
        self.assp_conv_3x3_1 = SplitSeparableConv(cin, base_depth, 2, bn_kw)
        self.assp_conv_3x3_2 = SplitSeparableConv(cin, base_depth, 4, bn_kw)
        self.assp_conv_3x3_3 = SplitSeparableConv(cin, base_depth, 8, bn_kw)
        self.assp_pool_conv = ConvBN(cin, base_depth, 1, 1, 0, relu=True, **cbn)
        self.assp_out = ConvBN(5 * base_depth, base_depth, 1, 1, 0, relu=True, **cbn)
        # decoder
        b1_out = block_widths[0] * 4 if block_type == "bottleneck" else block_widths[0]
        self.decoder_conv_1x1 = ConvBN(b1_out, base_depth, 1, 1, 0, relu=True, **cbn)
        # one logit channel: computed as 8 (zero weights / bias beyond the first) so the conv runs
        # on the aligned kernels instead of the per-element generic path
        self.decoder_conv_3x3 = Conv2d(2 * base_depth, 1, 3, 1, "SAME", bias=True,
                                       pad_cout_to=channel_align)

    # residual add + ReLU of every unit in its conv3 epilogue, with the next unit's pre-activation
    # BN statistics accumulated there too (BetaUnit.forward_fused) — not for units whose conv3 end
    # point is wanted (the decoder's block1/unit_1; all of them with return_end_points)
    fuse_residual = os.environ.get("TDL_DL_FUSE_RES", "1") == "1"

    def forward_encoder(self, x, all_end_points=True):
        """The ResNet-v2-beta encoder alone (``resnet_v2_beta`` without the ASPP / decoder,
        core/resnet.py:171-257): returns (block4 features, end_points).  ``all_end_points``
        False: only the block outputs and the decoder's block1/unit_1 conv end point (the other
        units then run with the fused residual epilogue)."""
        if x.shape[-1] != self.conv1_1.conv._cin_store:
            if x.shape[-1] > self.conv1_1.conv._cin_store:  # never crop input channels
                raise ValueError(f"input has {x.shape[-1]} channels, the stem takes "
                                 f"{self.conv1_1.conv.cin}")
            x = nn.functional.pad(x, (0, self.conv1_1.conv._cin_store - x.shape[-1]))
        end_points = {}
        root = f"{self.model_name}/resnet_v2"
        net = self.conv1_3(self.conv1_2(self.conv1_1(x)))
        net = self.postnorm(self.pool1(net))
        fuse = self.fuse_residual and not all_end_points
        st = None
        for bi, (bname, mods) in enumerate(zip(self.block_names, self.blocks)):
            for ui, unit in enumerate(mods):
                if fuse and not (bi == 0 and ui == 0):
                    net, st = unit.forward_fused(net, st)
                else:
                    net, st = unit._run(net, end_points, f"{root}/{bname}/unit_{ui + 1}", st,
                                        False)
            end_points[f"{root}/{bname}"] = _logical(net, mods[-1].out_channels)
        return end_points[f"{root}/block4"], end_points

    # ASPP / decoder concatenations written in place: every branch's BN(+ReLU) apply (and the
    # upsample of the pooled / ASPP features) stores straight into its channel slice of the
    # consumer conv's input, and each backward reads its slice of the concat gradient in place
    # (ops/bn.batch_norm_act_into, ops/upsample.upsample_into) — no torch.cat / split passes
    concat_free = os.environ.get("TDL_CONCAT_FREE", "1") == "1"
    aspp_join = os.environ.get("TDL_ASPP_JOIN", "1") == "1"

    def forward(self, x, return_end_points=False):
        root = f"{self.model_name}/resnet_v2"
        _, end_points = self.forward_encoder(x, all_end_points=return_end_points)
        atrous = end_points[f"{root}/block4"].contiguous()  # a copy only for unaligned widths
        last = 3 if self.block_type == "bottleneck" else 2
        b1 = end_points[f"{root}/block1/unit_1/bottleneck_v2/conv{last}"].contiguous()
        # (a serving trace takes the torch.cat head: the in-place concat writers are training
        # fusions with no functional form)
        if self.concat_free and export_impl() is None and self._concat_free_ok(atrous):
            out = self._head_concat_free(atrous, b1)
            return (out, end_points) if return_end_points else out
        size = (atrous.shape[1], atrous.shape[2])
        a1 = self.assp_conv_1x1(atrous)
        a2 = self.assp_conv_3x3_1(atrous)
        a3 = self.assp_conv_3x3_2(atrous)
        a4 = self.assp_conv_3x3_3(atrous)
        a5 = global_avg_pool(atrous, keepdims=True)
        a5 = self.assp_pool_conv(a5)
        a5 = upsample(a5, size)
        assp = self.assp_out(torch.cat([a1, a2, a3, a4, a5], dim=-1))
        assp_up = upsample(assp, (b1.shape[1], b1.shape[2]))
        dec = self.decoder_conv_1x1(b1)
        dec = torch.cat([dec, assp_up], dim=-1)
        dec = _logical(self.decoder_conv_3x3(dec), 1).contiguous()
        out = upsample(dec, self.input_shape)
        return (out, end_points) if return_end_points else out

    def _concat_free_ok(self, atrous):
        """Every writer's output is exactly its logical slice (no channel padding) and the
        consumers read the concatenation unpadded."""
        d = self.assp_out.bn.c
        writers = (self.assp_conv_1x1, self.assp_conv_3x3_1.pointwise,
                   self.assp_conv_3x3_2.pointwise, self.assp_conv_3x3_3.pointwise,
                   self.assp_pool_conv, self.decoder_conv_1x1)
        return (d % 8 == 0 and all(m.conv._cout_store == d for m in writers) and
                self.assp_out.conv._cin_store == 5 * d and
                self.decoder_conv_3x3._cin_store == 2 * d)

    def _head_concat_free(self, atrous, b1):
        d = self.assp_out.bn.c
        N, h, w = atrous.shape[:3]
        # the five ASPP branches read the encoder output: their input gradients meet in one
        # buffer (the first branch backward writes it, the others add in their epilogues —
        # conv dgrad accumulate, depthwise / avg-pool dadd; ops/gradjoin.py) instead of four
        # autograd adds
        join = (gradjoin.GradJoin(5) if self.aspp_join and torch.is_grad_enabled()
                and atrous.requires_grad and atrous.shape[-1] % 8 == 0 else None)
        cat = atrous.new_empty((N, h, w, 5 * d))
        cat = self.assp_conv_1x1(atrous, into=(cat, 0), join=join)
        cat = self.assp_conv_3x3_1(atrous, into=(cat, d), join=join)
        cat = self.assp_conv_3x3_2(atrous, into=(cat, 2 * d), join=join)
        cat = self.assp_conv_3x3_3(atrous, into=(cat, 3 * d), join=join)
        a5 = self.assp_pool_conv(global_avg_pool(atrous, keepdims=True, join=join))
        cat = upsample_into(cat, 4 * d, a5)
        assp = self.assp_out(cat)
        dec = b1.new_empty((b1.shape[0], b1.shape[1], b1.shape[2], 2 * d))
        dec = self.decoder_conv_1x1(b1, into=(dec, 0))
        dec = upsample_into(dec, d, assp)
        dec = _logical(self.decoder_conv_3x3(dec), 1).contiguous()
        return upsample(dec, self.input_shape)

    # ------------------------------------------------------------------------------------------
    def tf_names(self):
        """Map of torch state_dict key -> reference TF variable name."""
        M = self.model_name
        R = f"{M}/resnet_v2"
        m = {}

        def bn(prefix, tfp):
            m[f"{prefix}.gamma"] = f"{tfp}/gamma"
            m[f"{prefix}.beta"] = f"{tfp}/beta"
            m[f"{prefix}.running_mean"] = f"{tfp}/moving_mean"
            m[f"{prefix}.running_var"] = f"{tfp}/moving_variance"

        def convbn(prefix, tfp):
            m[f"{prefix}.conv.weight"] = f"{tfp}/weights"
            bn(f"{prefix}.bn", f"{tfp}/BatchNorm")

        def conv(prefix, tfp):
            m[f"{prefix}.weight"] = f"{tfp}/weights"
            m[f"{prefix}.bias"] = f"{tfp}/biases"

        for n in ("conv1_1", "conv1_2", "conv1_3"):
            convbn(n, f"{R}/{n}")
        bn("postnorm.bn", f"{R}/postnorm")
        for bi, (bname, mods) in enumerate(zip(self.block_names, self.blocks)):
            for ui, unit in enumerate(mods):
                p = f"blocks.{bi}.{ui}"
                t = f"{R}/{bname}/unit_{ui + 1}/bottleneck_v2"
                bn(f"{p}.preact.bn", f"{t}/preact")
                if unit.shortcut is not None:
                    conv(f"{p}.shortcut", f"{t}/shortcut")
                if self.block_type == "bottleneck":
                    convbn(f"{p}.conv1", f"{t}/conv1")
                    convbn(f"{p}.conv2", f"{t}/Conv")
                    conv(f"{p}.conv3", f"{t}/conv3")
                else:
                    convbn(f"{p}.conv1", f"{t}/Conv")
                    conv(f"{p}.conv3", f"{t}/conv2")
        convbn("assp_conv_1x1", f"{M}/assp/conv/conv_1x1")
        for i in (1, 2, 3):
            p = f"assp_conv_3x3_{i}"
            t = f"{M}/assp/conv/conv_3x3_{i}"
            m[f"{p}.depthwise.weight"] = f"{t}_depthwise/depthwise_weights"
            m[f"{p}.depthwise.bias"] = f"{t}_depthwise/biases"
            convbn(f"{p}.pointwise", f"{t}_pointwise")
        convbn("assp_pool_conv", f"{M}/assp/pooling/conv_1x1")
        convbn("assp_out", f"{M}/assp/conv_1x1")
        convbn("decoder_conv_1x1", f"{M}/decoder/conv_1x1")
        conv("decoder_conv_3x3", f"{M}/decoder/conv_3x3")
        sd = self.state_dict()
        return {k: v for k, v in m.items() if k in sd}

    def regularization_loss(self):
        """Σ weight_decay·½‖w‖² over the L2-regularised weights (slim l2_regularizer) — the term
        the reference creates but never adds to its loss (defect D5); opt-in here."""
        tot = 0.0
        for name, p in self.named_parameters():
            if name.endswith("weight") and "depthwise" not in name:
                tot = tot + 0.5 * (p.float() ** 2).sum()
        return self.weight_decay * tot
