#!/usr/bin/env python3
"""Which conv route rows (csrc/kernels/conv_route.hip) one eager training step of a model ran,
with the measurement behind each row — the dispatch table in action.

  python tools/route_report.py [--model resnet50] [--batch 256] [--image 224]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = getattr(models, a.model)(num_classes=1000)
    x, y = imagenet_batch(a.batch, a.image, num_classes=1000, device=dev)
    tr = Trainer(m, softmax_cross_entropy, dev, "sgd", dict(lr=0.01, momentum=0.9))
    tr.train_step(x, y)  # warm (workspaces, flipped filters)
    torch.cuda.synchronize()
    ext().conv_route_counts(True)
    tr.train_step(x, y)
    torch.cuda.synchronize()
    counts = ext().conv_route_counts(False)
    rows = {r["name"]: r for r in ext().conv_route_table()}
    print(f"# conv route rows of one {a.model} training step, batch {a.batch}, {a.image}x{a.image}")
    for op in ("fwd", "dgrad", "wgrad"):
        tot = sum(v for k, v in counts.items() if rows[k]["op"] == op)
        print(f"\n{op}: {tot} launches")
        for name, r in rows.items():
            if r["op"] == op and name in counts:
                print(f"  {counts[name]:4d}  {name:28s} cfg {r['cfg']:<3d} {r['evidence']}")


if __name__ == "__main__":
    main()
