"""Reference-compatible functional API (core.resnet / core.xception / core.layers / core.losses /
core.metric of gf712/TensorflowDistributedLearning), implemented on the NHWC modules and HIP ops
of this package.  TF's variable scopes become a module cache keyed by scope name, so calling a
builder twice with the same scope reuses the same weights (``reuse=True`` semantics)."""
from . import resnet, xception, layers, losses, metric  # noqa: F401
