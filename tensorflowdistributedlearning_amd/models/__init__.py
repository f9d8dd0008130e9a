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


def build(name, **kw):
    if name not in _REGISTRY:
        raise KeyError(f"unknown model {name}; have {sorted(_REGISTRY)}")
    return _REGISTRY[name](**kw)


__all__ = ["ResNet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
           "DeepLabResNet", "Xception41", "xception_41", "FlatParams", "build"]
