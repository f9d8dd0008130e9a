#!/usr/bin/env python3
"""The reference's own training entry point, timed: ``Model(...).train`` (k-fold driver, native
PNG loader with augmentation, Lovász loss, Adam, metrics, summaries) on a synthetic TGS-style
PNG dataset written to a temporary directory, one fold, with and without the per-fold HIP-graph
capture — to compare with ``bench.py --model deeplab_ref --batch B --graph`` (the bare step).

  python bench/model_loop.py --batch 32 --steps 120 --out gpurun_out/model_loop.json
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def write_dataset(root, n, hw=101, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "images"))
    os.makedirs(os.path.join(root, "masks"))
    ids, cls = [], []
    for i in range(n):
        img = (rng.random((hw, hw)) * 255).astype(np.uint8)
        m = np.zeros((hw, hw), np.uint8)
        r = int(rng.integers(0, 40))
        if r:
            c = int(rng.integers(r, hw - r))
            m[c - r:c + r, c - r:c + r] = 255
        Image.fromarray(img, "L").save(os.path.join(root, "images", f"s{i:05d}.png"))
        Image.fromarray(m, "L").save(os.path.join(root, "masks", f"s{i:05d}.png"))
        ids.append(f"s{i:05d}")
        cls.append(int(np.ceil((m > 0).mean() * 10)))
    return np.array(ids), np.array(cls)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--images", type=int, default=640)
    ap.add_argument("--out", default=None)
    ap.add_argument("--modes", default="off,auto",
                    help="comma list of hip_graph modes; 'auto:T:S:P' = auto with T loader "
                         "threads, summaries every S steps (0: none), device prefetch P (1/0)")
    args = ap.parse_args()
    from tensorflowdistributedlearning_amd.model import Model
    res = {}
    with tempfile.TemporaryDirectory() as td:
        X, y = write_dataset(os.path.join(td, "data"), args.images)
        for spec in args.modes.split(","):
            mode, *rest = spec.split(":")
            threads = int(rest[0]) if rest else 4
            summ = int(rest[1]) if len(rest) > 1 else 20
            pf = bool(int(rest[2])) if len(rest) > 2 else True
            m = Model(os.path.join(td, f"run_{spec.replace(':', '_')}", "tgs"),
                      os.path.join(td, "data"), n_gpus=1, n_fold=5, max_folds=1, save_best=0,
                      save_checkpoints_steps=10 ** 9, save_summary_steps=summ, hip_graph=mode,
                      loader_threads=threads, device_prefetch=pf)
            mode = spec
            r = m.train(X, y, args.batch, args.steps)[0]
            res[mode] = {"steady_ms_per_step": r["steady_ms_per_step"], "hip_graph": r["hip_graph"],
                         "img_per_s": args.batch * 1e3 / r["steady_ms_per_step"]}
            print(f"Model.train hip_graph={mode}: {r['steady_ms_per_step']:.3f} ms/step "
                  f"({res[mode]['img_per_s']:.0f} img/s, batch {args.batch})", flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
