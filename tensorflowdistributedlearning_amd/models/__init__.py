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


def enable_fp8(model, fuse_bn=True, dgrad=None):
    """fp8 GEMMs for every bias-free conv whose input channels are a multiple of 16 (the
    3-channel stem and biased heads stay bf16): the forward on e4m3 activations × e4m3 weights
    and — with ``dgrad`` — the input gradient on e5m2 output gradients × e4m3 weights (convs with
    K % 128 == 0 output channels that feed a BN; the weight gradient stays bf16).  With
    ``fuse_bn`` the BN layers write the e4m3 copy of their output in the same pass (scale from the
    previous step's |y|max), so those conv inputs need no separate quantisation pass; the BN after
    an fp8 conv likewise writes the e5m2 copy of its input gradient in the backward apply.
    Returns the conv count.

    The fp8 dgrad is opt-in (``dgrad=True`` or ``TDL_FP8_DGRAD=1``): the forward-only mode is the
    one whose loss curve is pinned against bf16 (tests/test_train_gpu.py::test_fp8_loss_curve_*)."""
    import os
    from .layers import Conv2d, BatchNorm, ConvBN
    if dgrad is None:
        dgrad = os.environ.get("TDL_FP8_DGRAD", "0") == "1"
    n = 0
    for m in model.modules():
        if isinstance(m, Conv2d) and m.bias is None and m._cin_store % 16 == 0:
            m.fp8 = True
            n += 1
        elif isinstance(m, BatchNorm) and fuse_bn:
            m.emit_fp8 = True  # conv inputs arrive pre-quantised (delayed scaling, ops/bn.py)
    if dgrad:
        for m in model.modules():
            if isinstance(m, ConvBN) and getattr(m.conv, "fp8", False):
                m.bn.emit_fp8_bwd = True  # e5m2 dy for the conv's fp8 dgrad (ops/conv.py)
    return n


def build(name, **kw):
    if name not in _REGISTRY:
        raise KeyError(f"unknown model {name}; have {sorted(_REGISTRY)}")
    return _REGISTRY[name](**kw)


__all__ = ["enable_fp8", "ResNet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
           "DeepLabResNet", "Xception41", "xception_41", "FlatParams", "build"]
