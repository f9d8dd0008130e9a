"""Model families: standard ResNets (18/34/50/101/152), the reference DeepLab ResNet-v2-beta
segmentation net, and Xception-41."""
from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152
from .deeplab import DeepLabResNet
from .xception import Xception41, xception_41
from .params import FlatParams

_REGISTRY = {
    "resnet18": resnet18,
    "resnet34": resnet34,
    "resnet50": resnet50,
    "resnet101": resnet101,
    "resnet152": resnet152,
    "xception41": xception_41,
    "deeplab_resnet": DeepLabResNet,
}


def enable_fp8(model, fuse_bn=True, dgrad=None, bf16_stages=None, wgrad=None):
    """fp8 GEMMs for every bias-free conv whose input channels are a multiple of 16 (the
    3-channel stem and biased heads stay bf16): the forward on e4m3 activations × e4m3 weights
    and — with ``dgrad`` — the input gradient on e5m2 output gradients × e4m3 weights (convs with
    K % 128 == 0 output channels that feed a BN; the weight gradient stays bf16).  With
    ``fuse_bn`` the BN layers whose output feeds an fp8 conv write the e4m3 copy of it in the same
    pass (scale from the previous step's |y|max), so those conv inputs need no separate
    quantisation pass; the BN after an fp8 conv likewise writes the e5m2 copy of its input
    gradient in the backward apply.  Returns the fp8 conv count.

    ``bf16_stages`` (ResNets; default ``TDL_FP8_BF16_STAGES`` or 2): the first residual stages
    keep bf16 GEMMs.  On the memorisation curve (dev/tools/fp8_policy_sweep.py,
    profiles/r05_fp8_numerics.txt) their quantisation noise dominates: last-10-step loss tail
    bf16 0.0088, every stage fp8 0.057 (6.5×), stage 1 bf16 0.025 (2.8×), stages 1–2 bf16
    0.015 (1.7×, fp8 dgrad included).  ResNet-152 keeps 39 of its 50 blocks on fp8.

    The fp8 dgrad defaults on (``TDL_FP8_DGRAD=0`` or ``dgrad=False`` turns it off), and so does
    the fp8 weight gradient (``TDL_FP8_WGRAD=0`` / ``wgrad=False``): e5m2 output gradients × the
    forward's e4m3 input, which the conv then keeps for its backward instead of the bf16 one."""
    import os
    from .layers import Conv2d, BatchNorm, ConvBN
    if dgrad is None:
        dgrad = os.environ.get("TDL_FP8_DGRAD", "1") == "1"
    if wgrad is None:
        wgrad = os.environ.get("TDL_FP8_WGRAD", "1") == "1"
    if bf16_stages is None:
        bf16_stages = int(os.environ.get("TDL_FP8_BF16_STAGES", "2"))
    n = 0
    for m in model.modules():
        if isinstance(m, Conv2d) and m.bias is None and m._cin_store % 16 == 0:
            m.fp8 = True
            n += 1
        elif isinstance(m, BatchNorm) and fuse_bn:
            m.emit_fp8 = True  # conv inputs arrive pre-quantised (delayed scaling, ops/bn.py)
    stages = [getattr(model, f"layer{i}", None) for i in (1, 2, 3, 4)]
    if isinstance(model, ResNet) and all(s is not None for s in stages):
        n = _resnet_fp8_plan(model, stages, bf16_stages, fuse_bn)
    for m in model.modules():
        if isinstance(m, Conv2d) and getattr(m, "fp8", False):
            m.fp8_dgrad, m.fp8_wgrad = bool(dgrad), bool(wgrad)
    from ..ops.conv import FP8_WGRAD
    if wgrad and FP8_WGRAD and fuse_bn and isinstance(model, ResNet) \
            and all(s is not None for s in stages):
        # a block's inner BNs (bn1 → conv2, bn2 → conv3) have one consumer each; when it is an
        # fp8 conv with an fp8 weight gradient, nothing reads their bf16 output: write e4m3 only
        for _, b in [(si, b) for si, st in enumerate(stages) for b in st]:
            inner = _block_convbns(b)
            for j in range(len(inner) - 1):
                nxt = inner[j + 1].conv
                inner[j].bn.fp8_only = bool(
                    inner[j].bn.emit_fp8 and getattr(nxt, "fp8_wgrad", False) and nxt.bias is None
                    and not nxt.grad_needs_unpad() and nxt.cin % 16 == 0 and nxt.cout % 16 == 0)
    if dgrad or wgrad:
        bwd_only = os.environ.get("TDL_FP8_BWD_ONLY", "1") == "1"
        for m in model.modules():
            if isinstance(m, ConvBN) and getattr(m.conv, "fp8", False):
                m.bn.emit_fp8_bwd = True  # e5m2 dy for the conv's fp8 dgrad / wgrad (ops/conv.py)
                # … and only that copy when both of the conv's backward GEMMs read it
                # (ops/conv.fp8_dgrad_eligible / fp8_wgrad_eligible on the conv's static shape)
                c = m.conv
                (sh, sw), (dh, dw) = c.stride, c.dilation
                m.bn.fp8_bwd_only = bool(
                    dgrad and wgrad and FP8_WGRAD and bwd_only and c.bias is None and not c.relu
                    and not c.grad_needs_unpad() and c.cout % 128 == 0 and c._cin_store % 16 == 0
                    and not ((sh > 1 and dh > 1) or (sw > 1 and dw > 1)))
    return n


def _resnet_fp8_plan(model, stages, bf16_stages, fuse_bn):
    """fp8 convs from stage ``bf16_stages`` on; a BN emits its e4m3 copy only where an fp8 conv
    reads it (inside a block: the next conv; a block's output BN: the next block's conv1 and
    shortcut conv; never the shortcut BN, whose output is the residual of a bf16 add, nor the
    stem's, which max-pool consumes)."""
    blocks = [(si, b) for si, st in enumerate(stages) for b in st]
    n = 0
    for si, b in blocks:
        on = si >= bf16_stages
        for cb in _block_convbns(b) + ([b.downsample] if b.downsample is not None else []):
            cb.conv.fp8 = on and getattr(cb.conv, "fp8", False)
            n += int(cb.conv.fp8)
    model.stem.bn.emit_fp8 = False
    if not fuse_bn:
        return n
    for i, (si, b) in enumerate(blocks):
        inner = _block_convbns(b)
        for j in range(len(inner) - 1):
            inner[j].bn.emit_fp8 = bool(getattr(inner[j + 1].conv, "fp8", False))
        nxt = blocks[i + 1][1] if i + 1 < len(blocks) else None
        inner[-1].bn.emit_fp8 = nxt is not None and bool(getattr(nxt.conv1.conv, "fp8", False))
        if b.downsample is not None:
            b.downsample.bn.emit_fp8 = False
    return n


def _block_convbns(b):
    return [b.conv1, b.conv2] + ([b.conv3] if hasattr(b, "conv3") else [])


def build(name, **kw):
    if name not in _REGISTRY:
        raise KeyError(f"unknown model {name}; have {sorted(_REGISTRY)}")
    return _REGISTRY[name](**kw)


__all__ = ["enable_fp8", "ResNet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
           "DeepLabResNet", "Xception41", "xception_41", "FlatParams", "build"]
