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


def enable_fp8(model, fuse_bn=True):
    """fp8 (e4m3) forward GEMMs for every bias-free conv whose input channels are a multiple of 16
    (the 3-channel stem and biased heads stay bf16); backward stays bf16.  With ``fuse_bn`` the BN
    layers write the e4m3 copy of their output in the same pass (scale from the previous step's
    |y|max), so those conv inputs need no separate quantisation pass.  Returns the conv count."""
    from .layers import Conv2d, BatchNorm
    n = 0
    for m in model.modules():
        if isinstance(m, Conv2d) and m.bias is None and m._cin_store % 16 == 0:
            m.fp8 = True
            n += 1
        elif isinstance(m, BatchNorm) and fuse_bn:
            m.emit_fp8 = True  # conv inputs arrive pre-quantised (delayed scaling, ops/bn.py)
    return n


def build(name, **kw):
    if name not in _REGISTRY:
        raise KeyError(f"unknown model {name}; have {sorted(_REGISTRY)}")
    return _REGISTRY[name](**kw)


__all__ = ["enable_fp8", "ResNet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
           "DeepLabResNet", "Xception41", "xception_41", "FlatParams", "build"]
