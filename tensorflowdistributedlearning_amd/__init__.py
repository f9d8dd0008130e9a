"""tensorflowdistributedlearning_amd — an MI355X-native (gfx950 / CDNA4) multi-GPU CNN training
framework with the capabilities of gf712/TensorflowDistributedLearning.

Layout
  ops/          hot ops: hand-written HIP kernels (GPU) + PyTorch fp32 oracles (CPU)
  models/       NHWC layers, ResNet-18/34/50/101/152, DeepLab ResNet-v2-beta, Xception-41, flat params
  core/         reference-compatible API (core.resnet / xception / layers / losses / metric)
  parallel/     one-process-per-GPU data parallelism, bucketed RCCL all-reduce overlapped w/ backward
  engine/       trainer, fused optimizers, checkpoints, summaries, k-fold driver
  data/         synthetic data, native (C++) image pipeline wrapper
  preprocessing/ reference-compatible preprocessing API
  model.py      ``Model`` — the reference's entry point (k-fold train / eval / export / predict)
"""
__version__ = "0.1.0"

from . import experimental  # noqa: E402,F401  (TDL_EXPERIMENTAL knobs, before any module reads them)
