"""Hot ops: hand-written gfx950 HIP kernels (GPU) with PyTorch fp32 oracles (CPU)."""
from .conv import ConvGeom, conv2d, conv_fwd, conv_dgrad, conv_wgrad, same_padding
from .bn import batch_norm_act
from .pool import max_pool2d, global_avg_pool
from .loss import softmax_cross_entropy, lovasz_hinge
from .dwconv import depthwise_conv2d, laplace
from .upsample import upsample as upsample_bilinear_tf1
from .elementwise import add_relu, relu, add, sigmoid_threshold
from .metrics import seg_scores, StreamingMean, IOU_THRESHOLDS
from . import optim

__all__ = ["ConvGeom", "conv2d", "conv_fwd", "conv_dgrad", "conv_wgrad", "same_padding",
           "batch_norm_act", "max_pool2d", "global_avg_pool", "softmax_cross_entropy",
           "lovasz_hinge", "depthwise_conv2d", "laplace", "upsample_bilinear_tf1", "add_relu", "relu", "add",
           "sigmoid_threshold", "seg_scores", "StreamingMean", "IOU_THRESHOLDS", "optim"]
