"""Command line: ``python -m tensorflowdistributedlearning_amd <command> …``.

  train    k-fold training of the reference DeepLab model on a TGS-style directory
           (``<data>/images/*.png`` + ``<data>/masks/*.png``), stratified on mask-coverage class
           exactly like the reference notebook (coverage = Σmask / (H·W), class = ⌈10·coverage⌉,
           Test.ipynb) — i.e. ``Model(...).train(ids, classes, batch_size, steps)``; or, with
           ``--arch resnet18|…|resnet152|xception41 --synthetic``, a north-star classifier on the
           learnable synthetic dataset (``--num-samples`` ids, ``--num-classes``): softmax-CE +
           SGD-momentum, LR schedule, checkpoints / resume / eval / summaries, e.g. BASELINE
           config 1: ``train --arch resnet18 --image-size 32 --synthetic --device cpu``;
  predict  TTA-averaged probabilities of every ``*.png`` in a directory → ``.npz`` (+ optional CSV
           with run-length-encoded masks, the Kaggle submission format);
  export   the servable program of a trained fold (its latest checkpoint) → ``.pt2``
           (engine/serving.py: ``--kind native`` tdl:: operators on the gfx950 kernels, or
           ``portable`` stock ATen that any PyTorch loads);
  bench    the training benchmark (same as ``python bench.py``);
  config   print the default configuration (JSON) to start a config file from.

Configuration comes from ``--config file.{json,yaml}`` and is overridden by flags.
"""
from __future__ import annotations

import argparse
import dataclasses
import glob
import json
import math
import os
import sys

import numpy as np

from .config import ModelConfig, load, from_dict


def coverage_classes(data_dir, ids):
    """Reference notebook stratification label: class = smallest i with 10·coverage ≤ i."""
    from . import _native
    ext = _native.load()
    classes = []
    for i in ids:
        m = ext.png_decode_gray(os.path.join(data_dir, "masks", f"{i}.png")).numpy()
        cov = float((m > 0.5).sum()) / m.size
        classes.append(int(math.ceil(cov * 10 - 1e-9)) if cov > 0 else 0)
    return np.array(classes)


def rle_encode(mask):
    """Kaggle TGS run-length encoding (column-major, 1-indexed)."""
    pixels = np.concatenate([[0], mask.T.flatten(), [0]])
    runs = np.where(pixels[1:] != pixels[:-1])[0] + 1
    runs[1::2] -= runs[::2]
    return " ".join(str(r) for r in runs)


def _model_cfg(args):
    cfg = load(args.config) if args.config else ModelConfig()
    over = {k: v for k, v in vars(args).items()
            if k in {f.name for f in dataclasses.fields(ModelConfig)} and v is not None}
    d = dataclasses.asdict(cfg)
    d.update(over)
    return from_dict(ModelConfig, d).validate()


def cmd_train(args):
    from .model import Model
    cfg = _model_cfg(args)
    if cfg.arch != "deeplab_ref":
        if not cfg.synthetic:
            raise SystemExit(f"--arch {cfg.arch} from the command line trains on --synthetic data "
                             "(image arrays: Model(...).train(images, labels, ...) in Python)")
        m = Model(**cfg.model_kwargs())
        res = m.train(args.num_samples, None, args.batch_size, args.steps)
        print(json.dumps({"params": m.params, "folds": res}, default=float))
        return
    ids = sorted(os.path.splitext(os.path.basename(p))[0]
                 for p in glob.glob(os.path.join(cfg.data_directory, "images", "*.png")))
    if not ids:
        raise SystemExit(f"no images under {cfg.data_directory}/images")
    y = coverage_classes(cfg.data_directory, ids)
    m = Model(**cfg.model_kwargs())
    res = m.train(np.array(ids), y, args.batch_size, args.steps)
    print(json.dumps({"params": m.params, "folds": res}, default=float))


def cmd_predict(args):
    from .model import Model
    cfg = _model_cfg(args)
    m = Model(**cfg.model_kwargs())
    out = m.predict(args.test_dir, args.batch_size, tti=args.tta)
    np.savez_compressed(args.out, ids=np.array(out["ids"]), probabilities=out["probabilities"])
    if args.csv:
        with open(args.csv, "w") as f:
            f.write("id,rle_mask\n")
            for i, mk in zip(out["ids"], out["mask"]):
                f.write(f"{i},{rle_encode(mk)}\n")
    print(f"wrote {args.out}" + (f" and {args.csv}" if args.csv else ""))


def cmd_export(args):
    from .model import Model
    cfg = _model_cfg(args)
    m = Model(**cfg.model_kwargs())
    path = m.export(args.out, args.fold, args.kind, args.checkpoint, batch=2)
    print(f"wrote {path}")


def cmd_bench(rest):
    sys.argv = ["bench.py"] + rest
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, here)
    import bench
    bench.main()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] == "bench":
        return cmd_bench(argv[1:])
    ap = argparse.ArgumentParser(prog="python -m tensorflowdistributedlearning_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)

    def common(p):
        p.add_argument("--config")
        p.add_argument("--model-dir", dest="model_dir")
        p.add_argument("--data-dir", dest="data_directory")
        p.add_argument("--n-gpus", dest="n_gpus", type=int)
        p.add_argument("--n-fold", dest="n_fold", type=int)
        p.add_argument("--lr", type=float)
        p.add_argument("--seed", type=int)
        p.add_argument("--device")
        p.add_argument("--block-type", dest="block_type")
        p.add_argument("--precision", choices=("bf16", "fp32"),
                       help="GPU compute precision (fp32: the reference's own precision)")
        p.add_argument("--batch-size", dest="batch_size", type=int, default=64)
        p.add_argument("--arch", help="deeplab_ref (default) | resnet18/34/50/101/152 | xception41")
        p.add_argument("--num-classes", dest="num_classes", type=int)
        p.add_argument("--image-size", dest="image_size", type=int)
        p.add_argument("--loss", choices=("lovasz", "softmax_ce"))
        p.add_argument("--optimizer", choices=("adam", "sgd_momentum"))
        p.add_argument("--momentum", type=float)
        p.add_argument("--lr-schedule", dest="lr_schedule",
                       choices=("exponential", "cosine", "step", "constant"))
        p.add_argument("--lr-decay-steps", dest="lr_decay_steps", type=int)
        p.add_argument("--lr-decay-rate", dest="lr_decay_rate", type=float)
        p.add_argument("--lr-warmup-steps", dest="lr_warmup_steps", type=int)
        p.add_argument("--weight-decay", dest="weight_decay", type=float)
        p.add_argument("--use-regularization", dest="use_regularization", action="store_true",
                       default=None)
        p.add_argument("--synthetic", action="store_true", default=None,
                       help="classifiers: the learnable synthetic dataset (data/classification.py)")
        p.add_argument("--num-samples", dest="num_samples", type=int, default=1024)
        p.add_argument("--max-folds", dest="max_folds", type=int)
        p.add_argument("--fp8", action="store_true", default=None)
        p.add_argument("--hip-graph", dest="hip_graph", choices=("auto", "off"))
        p.add_argument("--save-checkpoints-steps", dest="save_checkpoints_steps", type=int)
        p.add_argument("--save-summary-steps", dest="save_summary_steps", type=int)
        p.add_argument("--eval-batches", dest="eval_batches", type=int)
        p.add_argument("--export-format", dest="export_format",
                       choices=("native", "portable", "both", "none"))

    t = sub.add_parser("train")
    common(t)
    t.add_argument("--steps", type=int, default=100)
    p = sub.add_parser("predict")
    common(p)
    p.add_argument("--test-dir", required=True)
    p.add_argument("--tta", action="store_true")
    p.add_argument("--out", default="predictions.npz")
    p.add_argument("--csv")
    e = sub.add_parser("export")
    common(e)
    e.add_argument("--fold", type=int, default=0)
    e.add_argument("--kind", choices=("native", "portable"), default="native")
    e.add_argument("--checkpoint")
    e.add_argument("--out", default="model.pt2")
    sub.add_parser("config")
    args = ap.parse_args(argv)
    if args.cmd == "train":
        cmd_train(args)
    elif args.cmd == "predict":
        cmd_predict(args)
    elif args.cmd == "export":
        cmd_export(args)
    elif args.cmd == "config":
        print(json.dumps(dataclasses.asdict(ModelConfig()), indent=1))


if __name__ == "__main__":
    main()
