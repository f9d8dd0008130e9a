#!/usr/bin/env python3
"""Host-side cost of an eager training step: time for the Python / launch path to return from
``Trainer.train_step`` (no device sync) vs the wall time per step, plus a cProfile of a few steps.
If the issue time approaches the wall time the step is launch-bound (HIP graphs remove it).

  python dev/tools/host_overhead.py [--model deeplab_ref|resnet50|xception41] [--batch B] [--profile]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, lovasz_hinge  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch, segmentation_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="deeplab_ref")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    if a.model == "deeplab_ref":
        m = models.DeepLabResNet(model_name="model", input_shape=(101, 101))
        tr = Trainer(m, lovasz_hinge, dev, "adam", dict(lr=1e-3))
        x, y = segmentation_batch(a.batch or 64, device=dev)
    else:
        m = models.build(a.model, num_classes=1000)
        tr = Trainer(m, softmax_cross_entropy, dev, "sgd", dict(lr=0.1, momentum=0.9))
        size = 299 if a.model.startswith("xception") else 224
        x, y = imagenet_batch(a.batch or 64, size, device=dev)
    for _ in range(5):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    issue = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s = time.perf_counter()
        tr.train_step(x, y)
        issue.append(time.perf_counter() - s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    issue.sort()
    print(f"{a.model} batch {x.shape[0]}: wall {wall * 1e3:.2f} ms/step, host issue median "
          f"{issue[len(issue) // 2] * 1e3:.2f} ms/step (min {issue[0] * 1e3:.2f})", flush=True)
    if a.profile:
        # backward on the calling thread, so cProfile sees the Python backward functions
        torch.autograd.set_multithreading_enabled(False)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(5):
            tr.train_step(x, y)
        pr.disable()
        torch.cuda.synchronize()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
        print(s.getvalue())


if __name__ == "__main__":
    main()
