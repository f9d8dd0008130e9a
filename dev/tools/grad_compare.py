#!/usr/bin/env python3
"""Per-parameter gradient agreement between the GPU native path (bf16 HIP kernels) and the CPU
fp32 oracle path for one training step.  Localises a wrong backward kernel: a bug shows up as one
layer with low cosine, bf16 noise as a smooth degradation towards the input.

  python dev/tools/grad_compare.py --model resnet18 --size 64 --batch 16
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, lovasz_hinge  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch, segmentation_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--eval-bn", action="store_true", help="BN in inference mode (no batch-stat "
                    "cancellation in backward: isolates conv/pool/loss kernels)")
    ap.add_argument("--cpu-bf16", action="store_true", help="CPU oracle with bf16 storage")
    a = ap.parse_args()
    torch.manual_seed(0)
    if a.model == "deeplab":
        mk = lambda: models.DeepLabResNet(model_name="m", input_shape=(a.size, a.size))  # noqa: E731
        x, y = segmentation_batch(a.batch, (a.size, a.size), dtype=torch.float32)
        lossf = lovasz_hinge
    else:
        mk = lambda: models.build(a.model, num_classes=10)  # noqa: E731
        x, y = imagenet_batch(a.batch, a.size, num_classes=10, dtype=torch.float32)
        lossf = softmax_cross_entropy
    mc, mg = mk(), mk()
    mg.load_state_dict(mc.state_dict())
    x = x.bfloat16().float()  # same rounded input for both
    tc = Trainer(mc, lossf, "cpu", "sgd", dict(lr=0.0, momentum=0.0, weight_decay=0.0),
                 lowp_dtype=torch.bfloat16 if a.cpu_bf16 else None)
    # round CPU master weights to bf16 so both paths see identical weights
    with torch.no_grad():
        tc.flat.master.copy_(tc.flat.master.bfloat16().float())
        tc.flat.sync_lowp()
    dev = torch.device("cuda", 0)
    tg = Trainer(mg, lossf, dev, "sgd", dict(lr=0.0, momentum=0.0, weight_decay=0.0))
    with torch.no_grad():
        tg.flat.master.copy_(tc.flat.master.to(dev))
        tg.flat.sync_lowp()
    if a.eval_bn:
        tc.train_mode = tg.train_mode = False
    lc, oc = tc.train_step(x.bfloat16() if a.cpu_bf16 else x, y)
    lg, og = tg.train_step(x.to(dev, torch.bfloat16), y.to(dev))
    print(f"loss cpu {float(lc):.5f} gpu {float(lg):.5f}; out cos "
          f"{torch.nn.functional.cosine_similarity(oc.flatten().float(), og.cpu().flatten().float(), 0).item():.5f}")
    worst = []
    for name, pc, pg in zip(tc.flat.names, tc.flat.params, tg.flat.params):
        gc, gg = pc.grad.flatten(), pg.grad.cpu().flatten()
        cos = torch.nn.functional.cosine_similarity(gc, gg, 0).item()
        rel = ((gc - gg).norm() / (gc.norm() + 1e-12)).item()
        worst.append((cos, name))
        print(f"{cos:8.5f} {rel:8.4f} {gc.norm().item():10.4e}  {name}")
    worst.sort()
    print("WORST:", worst[:5])
    allc = torch.nn.functional.cosine_similarity(tc.flat.grad, tg.flat.grad.cpu(), 0).item()
    print(f"ALL cos {allc:.5f}")


if __name__ == "__main__":
    main()
