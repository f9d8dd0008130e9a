"""Pre-masked residual joins (ops/gradjoin.py) vs the BN applying its ReLU mask: gradient
agreement per parameter, against the run-to-run noise floor of the baseline path itself.

  python dev/tools/premask_check.py [--depth 18] [--batch 8] [--size 64] [--eval-bn]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.ops import gradjoin  # noqa: E402


def run(m, x, enabled):
    gradjoin.MASK_ENABLED = enabled
    for p in m.parameters():
        p.grad = None
    xi = x.clone().requires_grad_(True)
    y = m(xi)
    (y.float() * torch.linspace(-1, 1, y.shape[-1], device=x.device)).sum().backward()
    gradjoin.MASK_ENABLED = True
    return {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}, \
        xi.grad.float().clone()


def cos(a, b):
    return torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--eval-bn", action="store_true")
    a = ap.parse_args()
    torch.manual_seed(7)
    dev = torch.device("cuda")
    m = models.build(f"resnet{a.depth}", num_classes=10).to(dev)
    m.train()
    if a.eval_bn:
        for mod in m.modules():
            if mod.__class__.__name__ == "BatchNorm":
                mod.train(False)
    x = torch.randn(a.batch, a.size, a.size, 8, device=dev, dtype=torch.bfloat16)
    g0, x0 = run(m, x, False)
    g1, x1 = run(m, x, False)
    g2, x2 = run(m, x, True)
    print(f"x grad: off/off {cos(x0, x1):.6f}  off/on {cos(x0, x2):.6f}")
    for n in g0:
        c01, c02 = cos(g0[n], g1[n]), cos(g0[n], g2[n])
        flag = "  <--" if c02 < c01 - 1e-3 else ""
        print(f"{n:50s} off/off {c01:.6f} off/on {c02:.6f}{flag}")


if __name__ == "__main__":
    main()
