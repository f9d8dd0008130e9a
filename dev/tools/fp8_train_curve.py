"""Loss curves of the same ResNet on a fixed batch: bf16, fp8 forward, fp8 forward + fp8 dgrad.
  python dev/tools/fp8_train_curve.py [--depth 50] [--batch 64] [--size 128] [--steps 12] [--lr 0.01]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--lr", type=float, default=0.01)
    a = ap.parse_args()
    gpu = torch.device("cuda")
    x, y = imagenet_batch(a.batch, a.size, num_classes=10, device=gpu)
    for name, fp8, dgrad in (("bf16", False, False), ("fp8-fwd", True, False),
                             ("fp8-fwd+dgrad", True, True)):
        torch.manual_seed(0)
        m = models.build(f"resnet{a.depth}", num_classes=10)
        if fp8:
            models.enable_fp8(m, dgrad=dgrad)
        tr = Trainer(m, softmax_cross_entropy, gpu, "sgd", dict(lr=a.lr, momentum=0.9,
                                                              weight_decay=0.0))
        ls = [float(tr.train_step(x, y)[0]) for _ in range(a.steps)]
        print(f"{name:14s} " + " ".join(f"{l:.3f}" for l in ls), flush=True)


if __name__ == "__main__":
    main()
