#!/usr/bin/env python3
"""Diagnose a HIP-graph-captured training step against an eager twin: after each replay, report
the parameters whose gradient / master weight differ (or are non-finite).

  python tools/graph_debug.py --model resnet18 --opt sgd --steps 3
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402


def report(tag, ta, tb, limit=12):
    bad = []
    for name, pa, pb in zip(ta.flat.names, ta.flat.params, tb.flat.params):
        for kind, a, b in (("grad", pa.grad, pb.grad), ("param", pa.data, pb.data)):
            fin = bool(torch.isfinite(b).all())
            d = (a - b).abs().max().item() if fin else float("nan")
            if not fin or d > 0:
                bad.append((name, kind, tuple(a.shape), d, fin))
    print(f"[{tag}] {len(bad)} mismatching tensors", flush=True)
    for b in bad[:limit]:
        print("   ", b, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--opt", default="sgd")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--train-mode", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(7)
    nets = [models.build(a.model, num_classes=10) for _ in range(2)]
    nets[1].load_state_dict(nets[0].state_dict())
    okw = dict(lr=1e-3) if a.opt == "adam" else dict(lr=0.05, momentum=0.9)
    ta, tb = [Trainer(n, softmax_cross_entropy, dev, a.opt, dict(okw)) for n in nets]
    ta.train_mode = tb.train_mode = a.train_mode
    x, y = imagenet_batch(8, 32, num_classes=10, device=dev)
    tb.capture(x, y, warmup=2)
    for _ in range(2):
        ta.train_step(x, y)
    torch.cuda.synchronize()
    report("after warm-up", ta, tb)
    for i in range(a.steps):
        la, _ = ta.train_step(x, y)
        lb, _ = tb.replay()
        torch.cuda.synchronize()
        print(f"step {i}: loss eager {float(la):.6f} graph {float(lb):.6f}", flush=True)
        report(f"replay {i}", ta, tb)
        for (na, ma), mb in zip(ta.model.named_modules(), tb.model.modules()):
            pa, pb = getattr(ma, "_padded", None), getattr(mb, "_padded", None)
            if pa is not None and pb is not None:
                print(f"    padded weight copy {na}: max |eager - graph| = "
                      f"{(pa.float() - pb.float()).abs().max().item():.3g}", flush=True)


if __name__ == "__main__":
    main()
