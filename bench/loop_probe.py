#!/usr/bin/env python3
"""Where the Model.train fold loop's time goes beyond the bare graph-replayed step (bench.py
--graph): the same DeepLab preset trainer at batch B, timed as (a) graph replays alone, (b) replays
fed from the native loader (next batch + static-input copies), (c) plus the per-step metric
updates of Model._train_fold, (d) the loader alone.

  python bench/loop_probe.py --batch 32 --steps 100
"""
import argparse
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model_loop import write_dataset  # noqa: E402  (same synthetic PNG set)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--threads", type=int, default=4)
    args = ap.parse_args()
    from tensorflowdistributedlearning_amd.model import Model, _lovasz_loss, _logit
    from tensorflowdistributedlearning_amd.data.pipeline import SegmentationPipeline
    from tensorflowdistributedlearning_amd.ops.metrics import seg_scores, StreamingMean
    from tensorflowdistributedlearning_amd.parallel.dist import get_context
    dev = torch.device("cuda", 0)
    with tempfile.TemporaryDirectory() as td:
        X, _ = write_dataset(os.path.join(td, "data"), 640)
        imgs = [os.path.join(td, "data", "images", f"{i}.png") for i in X]
        masks = [os.path.join(td, "data", "masks", f"{i}.png") for i in X]
        m = Model(os.path.join(td, "run", "tgs"), os.path.join(td, "data"), n_gpus=1, n_fold=5)
        ctx = get_context()
        net = m.build_network()
        tr = m._make_trainer(net, _lovasz_loss, dev, ctx, 10 ** 6, None)
        pipe = SegmentationPipeline(imgs, masks, args.batch, augment=True, shuffle=True,
                                    repeat=True, seed=1, device=dev, threads=args.threads,
                                    aug=m.augmentation)
        x, y = next(pipe)
        tr.train_step(x, y)
        tr.capture(x, y, warmup=1)
        iou, acc_m = StreamingMean(dev), StreamingMean(dev)

        def timed(name, body):
            for _ in range(5):
                body()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                body()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            print(f"{name:44s} {ms:7.3f} ms/step  ({args.batch * 1e3 / ms:7.0f} img/s)", flush=True)

        timed("(a) graph replay only", lambda: tr.replay())

        def fed():
            xb, yb = next(pipe)
            return tr.replay(xb, yb), yb
        timed("(b) replay fed by the loader", fed)

        def full():
            (loss, out), yb = fed()
            pred = (out.float() > _logit(0.5)).float()
            s, a = seg_scores(yb, pred)
            iou.update(s)
            acc_m.update(a)
        timed("(c) + per-step metrics (the fold loop)", full)
        timed("(d) loader alone", lambda: next(pipe))


if __name__ == "__main__":
    main()
