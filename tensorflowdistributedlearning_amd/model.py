"""High-level k-fold training driver — the reference's ``Model`` (model.py:27-514).

What the reference does with ``tf.estimator.train_and_evaluate`` + ``MirroredStrategy`` towers in
one process, this does with one process per GPU (RCCL all-reduce, bucketed and overlapped with
backward) around the native engine:

* ``Model(model_dir, data_directory, data_format, lr, n_gpus, n_fold, seed, save_best, **kw)``
  (model.py:29-136): hyper-parameters from ``kw`` (weight_decay, batch_norm_decay — D2 fixed, the
  reference reads ``weight_decay`` here —, batch_norm_epsilon, batch_norm_scale, output_stride,
  base_depth, input_shape, n_blocks, block_type); ``_prepare_directory`` + StratifiedKFold.
* ``train(X, y, batch_size, steps)`` (model.py:138-227): per fold, symlink the split, train to
  ``steps`` global steps (resuming from the fold's latest checkpoint, Estimator semantics) with
  Adam + ``exponential_decay(lr, step, 10000, 0.5)`` on the per-image Lovász hinge, checkpoint
  every ``save_checkpoints_steps`` (500), train summaries every ``save_summary_steps`` (20),
  evaluate after every checkpoint and at the end (metrics/mean_iou, metrics/mean_acc,
  loss/lovasz_loss), BestExporter on metrics/mean_iou (D4 comparator fixed).
  ``batch_size`` is global and must divide by ``n_gpus`` (per-tower batch, model.py:152-155).
* ``predict(test_dir, batch_size, tti)`` (model.py:230-255, unfinished upstream — D6/D7): loads
  each fold's latest checkpoint, runs the test set under each TTA transformation (all four when
  ``tti``), undoes the transformation and averages probabilities over transformations and folds.
* ``params`` (model.py:507-513): parameter count once a model has been built.

Block type: the reference passes ``params['block_type']="basic_block"`` to the model_fn but the
model reads ``self.block_type`` (default "bottleneck") — D19; ``block_type`` kw is honoured here.
"""
from __future__ import annotations

import functools
import json
import math
import os
import time

import numpy as np
import torch

from .engine.kfold import StratifiedKFold
from .engine import checkpoint as ckpt
from .engine.summary import SummaryWriter
from .engine.exporter import BestExporter
from .engine.trainer import Trainer
from .models.deeplab import DeepLabResNet
from .models.params import FlatParams
from .ops.loss import lovasz_hinge
from .ops.metrics import seg_scores, StreamingMean
from .ops.optim import exponential_decay
from .preprocessing.preprocessing import _prepare_directory, create_symlinks, TRAIN, EVAL
from .data.pipeline import SegmentationPipeline, TestPipeline, fold_files, TRAIN_AUG
from .utils import metric_comparisson, get_available_gpus

WEIGHT_DECAY = 0.001
BATCH_NORM_DECAY = 0.99
BATCH_NORM_EPSILON = 0.001
BATCH_NORM_SCALE = True
OUTPUT_STRIDE = 8
INPUT_SHAPE = (101, 101)
BASE_DEPTH = 256

_TTA = ["vertical", "horizontal", "transpose", "none"]


def _undo_transform(t, transformation):
    """Self-inverse TTA transforms on [N, H, W, C] (model.py:384-387)."""
    if transformation == "vertical":
        return t.flip(1)
    if transformation == "horizontal":
        return t.flip(2)
    if transformation == "transpose":
        return t.transpose(1, 2)
    return t


class Model:
    def __init__(self, model_dir, data_directory, data_format="NHWC", lr=0.001, n_gpus=2,
                 n_fold=5, seed=42, save_best=5, **kwargs):
        if data_format not in ("NCHW", "NHWC"):
            raise ValueError(f"Unknown data format {data_format}. Has to be either NCHW or NHWC")
        # every kernel runs NHWC; NCHW is accepted for API parity (layout is internal)
        self.data_format = data_format
        self.weight_decay = kwargs.get("weight_decay", WEIGHT_DECAY)
        self.batch_norm_decay = kwargs.get("batch_norm_decay", BATCH_NORM_DECAY)
        self.batch_norm_epsilon = kwargs.get("batch_norm_epsilon", BATCH_NORM_EPSILON)
        self.batch_norm_scale = kwargs.get("batch_norm_scale", BATCH_NORM_SCALE)
        self.output_stride = kwargs.get("output_stride", OUTPUT_STRIDE)
        self.base_depth = kwargs.get("base_depth", BASE_DEPTH)
        self.input_shape = tuple(kwargs.get("input_shape", INPUT_SHAPE))
        self.n_blocks = tuple(kwargs.get("n_blocks", (3, 4, 6)))
        self.block_type = kwargs.get("block_type", "bottleneck")
        # engine knobs (the reference's RunConfig / hooks, model.py:117-121,470-480)
        self.save_checkpoints_steps = kwargs.get("save_checkpoints_steps", 500)
        self.save_summary_steps = kwargs.get("save_summary_steps", 20)
        self.keep_checkpoint_max = kwargs.get("keep_checkpoint_max", 5)
        self.threshold = kwargs.get("threshold", 0.5)
        self.use_regularization = kwargs.get("use_regularization", False)  # D5: opt-in
        self.kaggle_metric = kwargs.get("kaggle_metric", False)  # D16: reference formula default
        self.loader_threads = kwargs.get("loader_threads", 4)
        # read_and_preprocess knobs of the training input (model.py:315-317: crop_probability=0,
        # the function's other defaults); e.g. augmentation={"brightness_range": 0.1}
        self.augmentation = dict(TRAIN_AUG, **kwargs.get("augmentation", {}))
        self.device = kwargs.get("device", None)
        self.backend = kwargs.get("backend", None)
        # GPU compute precision: bf16 (default; fp32 accumulation, statistics, optimizer state and
        # master weights) or fp32 (the reference's precision — no dtype option exists in
        # /root/reference/model.py: every op on fp32 operands, csrc/kernels/f32.hip)
        self.precision = kwargs.get("precision", "bf16")
        if self.precision not in ("bf16", "fp32"):
            raise ValueError(f"unknown precision {self.precision} (bf16 or fp32)")

        self.model_name = model_dir.rstrip("/").split("/")[-1]
        self.model_dir = model_dir
        self.data_dir = data_directory
        self.n_gpus = n_gpus
        self.n_folds = n_fold
        self.seed = seed
        self.lr = lr
        self.save_best = save_best
        _prepare_directory(self.model_dir, self.n_folds)
        self.skf = StratifiedKFold(n_splits=self.n_folds, shuffle=True, random_state=self.seed)

    # ------------------------------------------------------------------------------------------
    def config(self):
        return {"model_name": self.model_name, "weight_decay": self.weight_decay,
                "batch_norm_decay": self.batch_norm_decay,
                "batch_norm_epsilon": self.batch_norm_epsilon,
                "batch_norm_scale": self.batch_norm_scale, "output_stride": self.output_stride,
                "base_depth": self.base_depth, "input_shape": list(self.input_shape),
                "n_blocks": list(self.n_blocks), "block_type": self.block_type,
                "lr": self.lr, "seed": self.seed, "precision": self.precision}

    def build_network(self):
        return DeepLabResNet(model_name=self.model_name, in_channels=2,
                             output_stride=self.output_stride, base_depth=self.base_depth,
                             input_shape=self.input_shape, n_blocks=self.n_blocks,
                             block_type=self.block_type, batch_norm_decay=self.batch_norm_decay,
                             batch_norm_epsilon=self.batch_norm_epsilon,
                             batch_norm_scale=self.batch_norm_scale,
                             weight_decay=self.weight_decay)

    def _cast(self, x):
        """The network input in the compute precision (the loaders deliver bf16 images)."""
        return x.float() if self.precision == "fp32" and x.dtype != torch.float32 else x

    def _world(self):
        """Processes to launch: one per GPU when enough GPUs exist; ``device='cpu'`` with
        ``n_gpus>1`` runs that many gloo ranks (DP rehearsal on the host)."""
        if self.device == "cpu":
            return self.n_gpus
        n = len(get_available_gpus())  # device_count(): does not initialise HIP in the parent
        return max(1, min(self.n_gpus, n))

    # ------------------------------------------------------------------------------------------
    def train(self, X, y, batch_size, steps=100):
        X = np.asarray(X)
        y = np.asarray(y)
        splits = [(tr, te) for tr, te in self.skf.split(X, y)]
        if batch_size % self.n_gpus != 0:
            raise ValueError("Batch size must be a multiple of n_gpus")
        per_tower = batch_size // self.n_gpus
        world = self._world()
        results = []
        for i, (tr, te) in enumerate(splits):
            print(f"[Model] Processing fold {i}", flush=True)
            create_symlinks(self.data_dir, self.model_dir, TRAIN, X[tr], i)
            create_symlinks(self.data_dir, self.model_dir, EVAL, X[te], i)
            # keep the global batch when fewer processes than towers are available
            local_batch = per_tower * self.n_gpus // world
            if world > 1:
                from .parallel.launcher import spawn
                out = os.path.join(self.model_dir, f"fold{i}", "result.json")
                spawn(_fold_worker, world, args=(self._state(), i, local_batch, steps))
                with open(out) as f:
                    res = json.load(f)
            else:
                res = self._train_fold(i, local_batch, steps)
            self.n_params = res["n_params"]
            results.append(res)
            print(f"[Model] Finished training fold {i}: {res['eval']}", flush=True)
        return results

    def _state(self):
        d = dict(self.__dict__)
        d.pop("skf", None)
        return d

    @classmethod
    def _from_state(cls, st):
        m = cls.__new__(cls)
        m.__dict__.update(st)
        m.skf = StratifiedKFold(n_splits=m.n_folds, shuffle=True, random_state=m.seed)
        return m

    def _device(self, ctx):
        if self.device is not None and self.device != "cuda":
            return torch.device(self.device)
        return ctx.device if ctx.device.type == "cuda" else (
            torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))

    def _train_fold(self, fold, batch, steps, ctx=None):
        from .parallel.dist import get_context
        ctx = ctx or get_context()
        device = self._device(ctx)
        fold_dir = os.path.join(self.model_dir, f"fold{fold}")
        torch.manual_seed(self.seed + fold)
        net = self.build_network()
        self.n_params = sum(p.numel() for p in net.parameters()) + sum(
            b.numel() for n, b in net.named_buffers() if "running" in n)
        schedule = functools.partial(exponential_decay, self.lr, decay_steps=10000,
                                     decay_rate=0.5, staircase=False)
        extra = ((lambda m: m.regularization_loss()) if self.use_regularization else None)
        trainer = Trainer(net, lambda out, yy: lovasz_hinge(out, yy), device, optimizer="adam",
                          opt_kwargs=dict(lr=self.lr, lr_schedule=schedule), ctx=ctx,
                          extra_loss_fn=extra,
                          lowp_dtype=None if self.precision == "fp32" else torch.bfloat16)
        start = 0
        latest = ckpt.latest_checkpoint(fold_dir)
        if latest is not None:
            start = ckpt.restore(latest, net, trainer.optimizer, trainer.flat)
            trainer.global_step = start
            if ctx.is_distributed:
                trainer.broadcast_state()
        tr_imgs, tr_masks = fold_files(self.model_dir, TRAIN, fold)
        ev_imgs, ev_masks = fold_files(self.model_dir, EVAL, fold)
        pipe = SegmentationPipeline(tr_imgs, tr_masks, batch, augment=True, shuffle=True,
                                    repeat=True, seed=self.seed + 7919 * fold + start,
                                    device=device, rank=ctx.rank, world=ctx.world_size,
                                    threads=self.loader_threads, aug=self.augmentation)
        main = ctx.is_main
        tw = SummaryWriter(os.path.join(fold_dir, "train"), enabled=main)
        ew = SummaryWriter(os.path.join(fold_dir, "eval"), enabled=main)
        exporter = None
        if self.save_best > 0 and main:
            exporter = BestExporter(
                os.path.join(fold_dir, "export"),
                functools.partial(metric_comparisson, key="metrics/mean_iou",
                                  greater_is_better=True),
                exports_to_keep=self.save_best,
                serving_shape=[None, self.input_shape[0], self.input_shape[1], 2],
                model_config=self.config())
        iou_m, acc_m = StreamingMean(device), StreamingMean(device)
        eval_result = {}
        step = start
        t0 = time.time()
        while step < steps:
            x, yy = next(pipe)
            x = self._cast(x)
            loss, out = trainer.train_step(x, yy)
            step = trainer.global_step
            pred = (out.float() > _logit(self.threshold)).float()
            score, acc = seg_scores(yy, pred, self.kaggle_metric)
            iou_m.update(score)
            acc_m.update(acc)
            if self.save_summary_steps and step % self.save_summary_steps == 0 and main:
                tw.scalars({"metrics/mean_acc": float(acc_m.result()),
                            "metrics/mean_iou": float(iou_m.result()),
                            "loss/lovasz_loss": float(loss),
                            "learning_rate": trainer.optimizer.lr_at(step - 1),
                            "global_step/sec": (step - start) / max(time.time() - t0, 1e-9)},
                           step)
                _image_summaries(tw, "train", x, yy, out, self.threshold, step)
            if step % self.save_checkpoints_steps == 0 or step == steps:
                if main:
                    ckpt.save(fold_dir, step, net, trainer.optimizer, self.keep_checkpoint_max,
                              {"config": self.config()})
                eval_result = self._evaluate(net, ev_imgs, ev_masks, batch * 2, device, ctx,
                                             ew if main else None, step)
                eval_result["global_step"] = step
                if main:
                    ew.scalars({k: v for k, v in eval_result.items() if k != "global_step"}, step)
                    if exporter is not None:
                        exporter.maybe_export(net, eval_result, step)
        if step == start and start > 0:  # already trained: evaluate the restored model
            eval_result = self._evaluate(net, ev_imgs, ev_masks, batch * 2, device, ctx)
            eval_result["global_step"] = step
        tw.close()
        ew.close()
        res = {"fold": fold, "n_params": self.n_params, "eval": eval_result, "steps": step}
        if main:
            with open(os.path.join(fold_dir, "result.json"), "w") as f:
                json.dump(res, f)
        return res

    @torch.no_grad()
    def _evaluate(self, net, images, masks, batch, device, ctx, writer=None, step=0):
        """One pass over the fold's held-out split (each rank its shard; sums all-reduced)."""
        net.eval()
        pipe = SegmentationPipeline(images, masks, batch, augment=False, shuffle=False,
                                    repeat=False, device=device, rank=ctx.rank,
                                    world=ctx.world_size, threads=self.loader_threads)
        sums = torch.zeros(4, dtype=torch.float64, device=device)  # iou, acc, loss, count
        first = True
        for x, yy in pipe:
            x = self._cast(x)
            out = net(x)
            if first and writer is not None:
                _image_summaries(writer, "eval", x, yy, out, self.threshold, step)
            first = False
            loss = lovasz_hinge(out, yy)
            pred = (out.float() > _logit(self.threshold)).float()
            score, acc = seg_scores(yy, pred, self.kaggle_metric)
            n = x.shape[0]
            sums += torch.stack([score.double().sum(), acc.double().sum(),
                                 loss.double() * n, torch.tensor(float(n), dtype=torch.float64,
                                                                 device=device)])
        if ctx.is_distributed:
            s = sums.to(ctx.device) if ctx.native is not None else sums.cpu()
            ctx.all_reduce_sum_(s)
            sums = s
        sums = sums.cpu()
        n = max(float(sums[3]), 1.0)
        net.train()
        return {"metrics/mean_iou": float(sums[0]) / n, "metrics/mean_acc": float(sums[1]) / n,
                "loss/lovasz_loss": float(sums[2]) / n}

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def predict(self, test_dir, batch_size, tti=False):
        """Returns {"ids": [...], "probabilities": float32 [N, H, W], "mask": uint8 [N, H, W]}."""
        import glob
        images = sorted(glob.glob(os.path.join(test_dir, "*.png")))
        if not images:
            raise ValueError(f"no *.png files under {test_dir}")
        device = torch.device(self.device) if self.device else (
            torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
        transforms = _TTA if tti else ["none"]
        acc, ids, n_models = None, None, 0
        for i in range(self.n_folds):
            path = ckpt.latest_checkpoint(os.path.join(self.model_dir, f"fold{i}"))
            if path is None:
                continue
            net = self.build_network().to(device)
            ckpt.restore(path, net)
            if device.type == "cuda" and self.precision != "fp32":
                # bf16 compute copies of the weights once per fold (not per batch); in eval mode
                # under no_grad every conv+BN runs BN-folded (models/layers.ConvBN)
                FlatParams(net, device, lowp_dtype=torch.bfloat16)
            net.eval()
            for tf in transforms:
                probs, fold_ids = [], []
                for x, b_ids in TestPipeline(images, batch_size, tf, device=device,
                                             threads=self.loader_threads):
                    p = torch.sigmoid(net(self._cast(x)).float())
                    probs.append(_undo_transform(p, tf)[..., 0].cpu())
                    fold_ids += b_ids
                p = torch.cat(probs)
                acc = p if acc is None else acc + p
                ids = fold_ids
                n_models += 1
        if n_models == 0:
            raise ValueError("no trained fold checkpoints found; call train first")
        prob = (acc / n_models).numpy()
        return {"ids": ids, "probabilities": prob,
                "mask": (prob > self.threshold).astype(np.uint8)}

    # ------------------------------------------------------------------------------------------
    # reference-surface helpers (model.py:257-505): the pieces train()/predict() are built from
    def build_model_fn_optimizer(self):
        """Returns ``model_fn(mode, device, ctx=None) -> spec`` (model.py:326-505): for "train" a
        dict with the network, loss function, :class:`engine.trainer.Trainer` (Adam +
        exponential_decay(lr, step, 10000, 0.5)) and the threshold; for "eval"/"predict" the
        network in inference mode."""
        def model_fn(mode, device=None, ctx=None):
            from .parallel.dist import get_context
            ctx = ctx or get_context()
            device = torch.device(device) if device is not None else self._device(ctx)
            net = self.build_network()
            loss_fn = (lambda out, yy: lovasz_hinge(out, yy))
            spec = {"mode": mode, "network": net, "loss": loss_fn, "threshold": self.threshold}
            if mode == TRAIN:
                schedule = functools.partial(exponential_decay, self.lr, decay_steps=10000,
                                             decay_rate=0.5, staircase=False)
                spec["trainer"] = Trainer(net, loss_fn, device, optimizer="adam",
                                          opt_kwargs=dict(lr=self.lr, lr_schedule=schedule),
                                          ctx=ctx, lowp_dtype=None if self.precision == "fp32"
                                          else torch.bfloat16)
            else:
                net.to(device).eval()
            return spec
        return model_fn

    def _make_input_fn(self, mode, fold, batch_size, augment, shuffle, device="cpu", rank=0,
                       world=1):
        """model.py:285-324: returns ``input_fn() -> iterator of (x, y)`` over the fold's
        symlinked split (repeating for training, one pass for evaluation)."""
        def input_fn():
            imgs, masks = fold_files(self.model_dir, mode, fold)
            return SegmentationPipeline(imgs, masks, batch_size, augment=augment, shuffle=shuffle,
                                        repeat=(mode == TRAIN), seed=self.seed + fold,
                                        device=device, rank=rank, world=world,
                                        threads=self.loader_threads, aug=self.augmentation)
        return input_fn

    def _make_test_input(self, batch_size, test_directory, tti="none", device="cpu"):
        """model.py:257-283: returns ``test_input_fn() -> iterator of (x, ids)`` over
        ``test_directory/*.png`` with one TTA ``transformation`` (the reference's ``tti``
        argument is the transformation name)."""
        import glob
        transformation = tti if isinstance(tti, str) else "none"

        def test_input_fn():
            images = sorted(glob.glob(os.path.join(test_directory, "*.png")))
            return TestPipeline(images, batch_size, transformation, device=device,
                                threads=self.loader_threads)
        return test_input_fn

    @property
    def params(self):
        try:
            return self.n_params
        except AttributeError:
            raise ValueError("No model has been defined at this point! Call train method first.")


def _image_summaries(writer, mode, x, y, logits, threshold, step):
    """``tf.summary.image`` of the first sample's input / label / probability / prediction
    (model.py:405-440); the input is min-max scaled like TF's float image summary."""
    img = x[0, :, :, 0].float().cpu()
    img = (img - img.min()) / (img.max() - img.min()).clamp_min(1e-12)
    prob = torch.sigmoid(logits[0, :, :, 0].float()).cpu()
    writer.image(f"{mode}/{mode}_image", img.numpy(), step)
    writer.image(f"{mode}/{mode}_label", y[0, :, :, 0].float().cpu().numpy(), step)
    writer.image(f"{mode}/{mode}_prob", prob.numpy(), step)
    writer.image(f"{mode}/{mode}_prediction", (prob > threshold).float().numpy(), step)


def _logit(p):
    """sigmoid(z) > p  ⇔  z > logit(p) (threshold applied to logits; no sigmoid pass)."""
    p = min(max(p, 1e-7), 1 - 1e-7)
    return math.log(p / (1 - p))


def _fold_worker(rank, state, fold, batch, steps):
    from .parallel.dist import init_distributed, shutdown
    m = Model._from_state(state)
    dev = "cpu" if m.device == "cpu" else None
    ctx = init_distributed(device_type=dev, backend=m.backend)
    try:
        m._train_fold(fold, batch, steps, ctx)
    finally:
        shutdown()
