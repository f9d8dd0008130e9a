#!/usr/bin/env python3
"""fp8 numerics sweep on the memorisation task of tests/test_train_gpu.py::test_fp8_loss_curve_*
(ResNet-50, 64x64, 4 fixed batches of 32, SGD-momentum lr 0.003): loss-curve tails (mean of the
last 10 steps) of bf16 and of fp8 variants — delayed-scaling margin / amax-history decay
(ext().fp8_set_policy), e5m2 gradient margin, and which stages stay bf16.

  python dev/tools/fp8_policy_sweep.py [--steps 80] [--variants name,...]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402

# name: (fp8, dgrad, (margin_e4m3, margin_e5m2, decay), bf16 stages)
VARIANTS = {
    "bf16": (False, False, None, ()),
    "bf16b": (False, False, None, ()),
    "f8": (True, False, (1.0, 4.0, 0.0), ()),
    "f8m2": (True, False, (2.0, 4.0, 0.0), ()),
    "f8d9": (True, False, (1.0, 4.0, 0.9), ()),
    "f8m2d9": (True, False, (2.0, 4.0, 0.9), ()),
    "f8L4": (True, False, (1.0, 4.0, 0.0), ("layer4",)),
    "f8L1": (True, False, (1.0, 4.0, 0.0), ("layer1",)),
    "f8d": (True, True, (1.0, 4.0, 0.0), ()),
    "f8d_e1": (True, True, (1.0, 1.0, 0.0), ()),
    "f8d_e16": (True, True, (1.0, 16.0, 0.0), ()),
    "f8d_d9": (True, True, (1.0, 4.0, 0.9), ()),
    "f8L1d9": (True, False, (1.0, 4.0, 0.9), ("layer1",)),
    "f8L12": (True, False, (1.0, 4.0, 0.0), ("layer1", "layer2")),
    "f8L1d9_dg": (True, True, (1.0, 4.0, 0.9), ("layer1",)),
    "f8L1d9_dg16": (True, True, (1.0, 16.0, 0.9), ("layer1",)),
    "f8L1_dg16": (True, True, (1.0, 16.0, 0.0), ("layer1",)),
    "f8L1_dg": (True, True, (1.0, 4.0, 0.0), ("layer1",)),
    "f8L1_dg64": (True, True, (1.0, 64.0, 0.0), ("layer1",)),
    "f8L12_dg16": (True, True, (1.0, 16.0, 0.0), ("layer1", "layer2")),
    "default": (True, None, None, None),  # models.enable_fp8 defaults
}


def curve(fp8, dgrad, policy, keep, steps, lr):
    ext().fp8_set_policy(*(policy or (-1.0, -1.0, -1.0)))
    torch.manual_seed(0)
    net = models.build("resnet50", num_classes=10)
    if fp8 and keep is None:
        models.enable_fp8(net)
    elif fp8:
        models.enable_fp8(net, dgrad=dgrad, bf16_stages=0)
        for name, m in net.named_modules():
            if keep and any(name.startswith(k) for k in keep) and hasattr(m, "fp8"):
                m.fp8 = False
    tr = Trainer(net, softmax_cross_entropy, torch.device("cuda", 0), "sgd",
                 dict(lr=lr, momentum=0.9, weight_decay=0.0))
    data = [imagenet_batch(32, 64, num_classes=10, device="cuda", seed=s) for s in range(4)]
    out = [float(tr.train_step(*data[i % 4])[0]) for i in range(steps)]
    ext().fp8_set_policy(-1.0, -1.0, -1.0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=80)
    ap.add_argument("--lr", type=float, default=0.003)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args()
    for name in a.variants.split(",") * a.repeat:
        fp8, dgrad, pol, keep = VARIANTS[name]
        c = curve(fp8, dgrad, pol, keep, a.steps, a.lr)
        tail = sum(c[-10:]) / 10
        print(f"{name:8s} tail {tail:.4f}  first {c[0]:.3f}  " +
              " ".join(f"{v:.3f}" for v in c[::8]), flush=True)


if __name__ == "__main__":
    main()
