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

North-star workloads train through the same class: ``arch`` selects the
network (``"deeplab_ref"`` — the reference's DeepLab-ResNet, default — or ``resnet18/34/50/101/
152`` / ``xception41``, the classifiers the reference reaches through its ``resnet_v2`` logits head,
/root/reference/core/resnet.py:246-256, and /root/reference/model.py:356-370).  Classifiers train
with softmax cross-entropy + SGD-momentum by default (``loss`` / ``optimizer`` override), an LR
schedule (``lr_schedule``: exponential — the reference's —, cosine, step, constant), the same
k-fold / checkpoint / resume / eval (top-1 accuracy) / summaries / best-export cadence, on
``X`` = an image array [N, H, W, C] or, with ``synthetic=True``, sample ids of a learnable
synthetic dataset (data/classification.py).  ``hip_graph`` (default on for GPU runs) captures the
training step of each fold as one HIP graph after the first step and replays it
(engine/trainer.Trainer.capture) — the reference's per-step session loop without per-kernel host
launches.

Block type: the reference passes ``params['block_type']="basic_block"`` to the model_fn but the
model reads ``self.block_type`` (default "bottleneck") — D19; ``block_type`` kw is honoured here.
"""
from __future__ import annotations

import contextlib
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
from .engine import schedules
from .models.deeplab import DeepLabResNet
from . import models as _models
from .models.params import FlatParams
from .ops.loss import lovasz_hinge, softmax_cross_entropy, softmax_eval
from .ops.metrics import seg_scores, StreamingMean
from .ops.optim import exponential_decay
from .preprocessing.preprocessing import _prepare_directory, create_symlinks, TRAIN, EVAL
from .data.pipeline import SegmentationPipeline, TestPipeline, fold_files, TRAIN_AUG
from .data.prefetch import DevicePrefetcher
from .data.classification import ClassificationPipeline, SyntheticImages, ArrayImages
from .utils import metric_comparisson, get_available_gpus

WEIGHT_DECAY = 0.001
BATCH_NORM_DECAY = 0.99
BATCH_NORM_EPSILON = 0.001
BATCH_NORM_SCALE = True
OUTPUT_STRIDE = 8
INPUT_SHAPE = (101, 101)
BASE_DEPTH = 256

_TTA = ["vertical", "horizontal", "transpose", "none"]

from .config import SEGMENTATION_ARCHS, CLASSIFIER_ARCHS  # noqa: E402  (re-exported)


def _undo_transform(t, transformation):
    """Self-inverse TTA transforms on [N, H, W, C] (model.py:384-387)."""
    if transformation == "vertical":
        return t.flip(1)
    if transformation == "horizontal":
        return t.flip(2)
    if transformation == "transpose":
        return t.transpose(1, 2)
    return t


def network_from_config(cfg):
    """Rebuild the network a :meth:`Model.config` dict describes (export bundles' config.json)."""
    arch = cfg.get("arch", "deeplab_ref")
    if arch in CLASSIFIER_ARCHS:
        return _models.build(arch, num_classes=cfg["num_classes"],
                             in_channels=cfg.get("image_channels", 3))
    return DeepLabResNet(model_name=cfg["model_name"], in_channels=2,
                         output_stride=cfg["output_stride"], base_depth=cfg["base_depth"],
                         input_shape=tuple(cfg["input_shape"]), n_blocks=tuple(cfg["n_blocks"]),
                         block_type=cfg["block_type"], batch_norm_decay=cfg["batch_norm_decay"],
                         batch_norm_epsilon=cfg["batch_norm_epsilon"],
                         batch_norm_scale=cfg["batch_norm_scale"],
                         weight_decay=cfg["weight_decay"])


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
        # H2D copies of the next batches on a copy stream, fed by a worker thread
        # (data/prefetch.py); False: the loader's batch is copied in line on the step's stream
        self.device_prefetch = bool(kwargs.get("device_prefetch", True))
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
        # north-star workloads: network, objective, optimizer, schedule
        self.arch = kwargs.get("arch", "deeplab_ref")
        if self.arch not in SEGMENTATION_ARCHS + CLASSIFIER_ARCHS:
            raise ValueError(f"unknown arch {self.arch}; have {SEGMENTATION_ARCHS + CLASSIFIER_ARCHS}")
        seg = self.arch in SEGMENTATION_ARCHS
        self.num_classes = kwargs.get("num_classes", 1000)
        self.image_size = kwargs.get("image_size", 299 if self.arch == "xception41" else 224)
        self.image_channels = kwargs.get("image_channels", 3)
        self.loss = kwargs.get("loss", "lovasz" if seg else "softmax_ce")
        if self.loss not in ("lovasz", "softmax_ce"):
            raise ValueError(f"unknown loss {self.loss} (lovasz or softmax_ce)")
        if (self.loss == "lovasz") != seg:
            raise ValueError(f"loss {self.loss} does not fit arch {self.arch}")
        self.optimizer = kwargs.get("optimizer", "adam" if seg else "sgd_momentum")
        if self.optimizer not in ("adam", "sgd_momentum"):
            raise ValueError(f"unknown optimizer {self.optimizer} (adam or sgd_momentum)")
        self.momentum = kwargs.get("momentum", 0.9)
        self.lr_schedule = kwargs.get("lr_schedule", "exponential")
        if self.lr_schedule not in schedules.SCHEDULES:
            raise ValueError(f"unknown lr_schedule {self.lr_schedule}; have {schedules.SCHEDULES}")
        self.lr_decay_steps = kwargs.get("lr_decay_steps", 10000)   # model.py:457-459
        self.lr_decay_rate = kwargs.get("lr_decay_rate", 0.5)
        self.lr_warmup_steps = kwargs.get("lr_warmup_steps", 0)
        self.synthetic = kwargs.get("synthetic", False)
        self.fp8 = kwargs.get("fp8", False)
        # HIP-graph capture of each fold's training step ("auto": GPU runs whose collectives, if
        # any, are on the native RCCL communicator)
        self.hip_graph = kwargs.get("hip_graph", "auto")
        self.eval_batches = kwargs.get("eval_batches", None)  # cap on eval batches per pass
        self.max_folds = kwargs.get("max_folds", None)  # train only the first k folds
        # servable program written with every best export (engine/serving.py; the reference's
        # SavedModel): native (tdl:: ops) | portable (stock ATen) | both | none
        self.export_format = kwargs.get("export_format", "native")
        if self.export_format not in ("native", "portable", "both", "none"):
            raise ValueError(f"unknown export_format {self.export_format}")

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
    @property
    def segmentation(self):
        return self.arch in SEGMENTATION_ARCHS

    def config(self):
        if not self.segmentation:
            return {"model_name": self.model_name, "arch": self.arch,
                    "num_classes": self.num_classes, "image_size": self.image_size,
                    "image_channels": self.image_channels, "loss": self.loss,
                    "optimizer": self.optimizer, "lr": self.lr, "lr_schedule": self.lr_schedule,
                    "weight_decay": self.weight_decay, "seed": self.seed,
                    "precision": self.precision, "fp8": self.fp8}
        return {"model_name": self.model_name, "weight_decay": self.weight_decay,
                "batch_norm_decay": self.batch_norm_decay,
                "batch_norm_epsilon": self.batch_norm_epsilon,
                "batch_norm_scale": self.batch_norm_scale, "output_stride": self.output_stride,
                "base_depth": self.base_depth, "input_shape": list(self.input_shape),
                "n_blocks": list(self.n_blocks), "block_type": self.block_type,
                "lr": self.lr, "seed": self.seed, "precision": self.precision}

    def build_network(self):
        net = network_from_config(self.config())
        if not self.segmentation and self.fp8:
            _models.enable_fp8(net)
        return net

    def export(self, path, fold=0, kind="native", checkpoint=None, device=None, batch=2):
        """Write the servable program of fold ``fold`` (its latest checkpoint, or ``checkpoint``)
        to ``path`` — engine/serving.py; ``kind`` native | portable.  Returns the path."""
        from .engine import serving
        dev = torch.device(device or self.device or ("cuda" if torch.cuda.is_available()
                                                      else "cpu"))
        net = self.build_network().to(dev)
        ck = checkpoint or ckpt.latest_checkpoint(os.path.join(self.model_dir, f"fold{fold}"))
        if ck is None:
            raise FileNotFoundError(f"no checkpoint for fold {fold} under {self.model_dir}")
        ckpt.restore(ck, net)
        if dev.type == "cuda" and self.precision == "bf16":
            net._tdl_flat = FlatParams(net, dev, lowp_dtype=torch.bfloat16, with_grad=False)
        shape = self._serving_shape()
        example = torch.zeros([batch] + shape[1:], device=dev)
        serving.export_serving(net, example, path, "segmentation" if self.segmentation
                               else "classification", kind, self._serving_dtype(dev))
        return path

    def _serving_shape(self):
        if self.segmentation:
            return [None, self.input_shape[0], self.input_shape[1], 2]
        return [None, self.image_size, self.image_size, self.image_channels]

    def _serving_dtype(self, device):
        if torch.device(device).type != "cuda" or self.precision == "fp32":
            return torch.float32
        return torch.bfloat16

    def _cast(self, x):
        """The network input in the compute precision (the loaders deliver bf16 images, or fp32
        ones for precision="fp32" — then this is a no-op)."""
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
        """k-fold training (model.py:138-227).  Segmentation (``arch="deeplab_ref"``): ``X`` =
        image ids under ``data_directory/images``, ``y`` = the stratification classes.
        Classifiers: ``X`` = images [N, H, W, C] (uint8 or float) and ``y`` = class labels, or with
        ``synthetic=True`` ``X`` = sample ids (or a sample count) of the synthetic dataset and
        ``y`` = their labels (None: seeded random labels)."""
        if not self.segmentation:
            self._set_cls_data(X, y)
            X, y = self._cls_ids, self._cls_labels
        X = np.asarray(X)
        y = np.asarray(y)
        splits = [(tr, te) for tr, te in self.skf.split(X, y)]
        splits = splits[:self.max_folds or len(splits)]
        if batch_size % self.n_gpus != 0:
            raise ValueError("Batch size must be a multiple of n_gpus")
        per_tower = batch_size // self.n_gpus
        world = self._world()
        results = []
        for i, (tr, te) in enumerate(splits):
            print(f"[Model] Processing fold {i}", flush=True)
            if self.segmentation:
                create_symlinks(self.data_dir, self.model_dir, TRAIN, X[tr], i)
                create_symlinks(self.data_dir, self.model_dir, EVAL, X[te], i)
            else:
                self._cls_split = (tr, te)
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
            self.last_results = results
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

    def _use_graph(self, device, ctx):
        if self.hip_graph in (False, "off", 0) or device.type != "cuda":
            return False
        return not ctx.is_distributed or getattr(ctx, "native", None) is not None

    def _schedule(self, steps):
        return schedules.make(self.lr_schedule, self.lr, total_steps=steps,
                              decay_steps=self.lr_decay_steps, decay_rate=self.lr_decay_rate,
                              warmup_steps=self.lr_warmup_steps)

    def _make_trainer(self, net, loss_fn, device, ctx, steps, extra=None):
        opt = "adam" if self.optimizer == "adam" else "sgd"
        kw = dict(lr=self.lr, lr_schedule=self._schedule(steps))
        if opt == "sgd":
            kw.update(momentum=self.momentum,
                      weight_decay=self.weight_decay if self.use_regularization else 0.0)
        return Trainer(net, loss_fn, device, optimizer=opt, opt_kwargs=kw, ctx=ctx,
                       extra_loss_fn=extra,
                       lowp_dtype=None if self.precision == "fp32" else torch.bfloat16)

    def _train_fold(self, fold, batch, steps, ctx=None):
        from .parallel.dist import get_context
        ctx = ctx or get_context()
        if not self.segmentation:
            return self._train_fold_cls(fold, batch, steps, ctx)
        device = self._device(ctx)
        fold_dir = os.path.join(self.model_dir, f"fold{fold}")
        torch.manual_seed(self.seed + fold)
        net = self.build_network()
        self.n_params = sum(p.numel() for p in net.parameters()) + sum(
            b.numel() for n, b in net.named_buffers() if "running" in n)
        extra = ((lambda m: m.regularization_loss()) if self.use_regularization else None)
        trainer = self._make_trainer(net, _lovasz_loss, device, ctx, steps, extra)
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
                                    threads=self.loader_threads, aug=self.augmentation,
                                    fp32=self.precision == "fp32")
        batches, quiet = pipe, None
        if device.type == "cuda" and self.device_prefetch:
            batches = DevicePrefetcher(pipe.next_host, device, depth=2, cast=self._cast)
            quiet = batches.quiesced
        stepper = _Stepper(trainer, self._use_graph(device, ctx), quiet)
        main = ctx.is_main
        tw = SummaryWriter(os.path.join(fold_dir, "train"), enabled=main)
        ew = SummaryWriter(os.path.join(fold_dir, "eval"), enabled=main)
        exporter = None
        if self.save_best > 0 and main:
            exporter = BestExporter(
                os.path.join(fold_dir, "export"),
                functools.partial(metric_comparisson, key="metrics/mean_iou",
                                  greater_is_better=True),
                exports_to_keep=self.save_best, serving_shape=self._serving_shape(),
                model_config=self.config(), serving=self.export_format, task="segmentation",
                compute_dtype=self._serving_dtype(device))
        iou_m, acc_m = StreamingMean(device), StreamingMean(device)
        saver = ckpt.AsyncSaver()  # D2H on a copy stream, file write on a worker thread
        eval_result = {}
        step = start
        t0 = time.time()
        clock = _StepClock(device, start)
        lt = _LoopTimer()
        while step < steps:
            lt.mark()
            x, yy = next(batches)
            if batches is pipe:
                x = self._cast(x)
            lt.mark("loader")
            loss, out = stepper(x, yy)
            step = trainer.global_step
            clock.tick(step)
            lt.mark("step")
            pred = (out.float() > _logit(self.threshold)).float()
            score, acc = seg_scores(yy, pred, self.kaggle_metric)
            iou_m.update(score)
            acc_m.update(acc)
            lt.mark("metrics")
            if self.save_summary_steps and step % self.save_summary_steps == 0 and main:
                # one device→host transfer for the scalars and the four images; PNG encoding
                # and the event write happen on the writer's thread
                vals, imgs = _summary_fetch([acc_m.result(), iou_m.result(), loss], x, yy, out,
                                            self.threshold)
                tw.scalars({"metrics/mean_acc": vals[0], "metrics/mean_iou": vals[1],
                            "loss/lovasz_loss": vals[2],
                            "learning_rate": trainer.optimizer.lr_at(step - 1),
                            "global_step/sec": (step - start) / max(time.time() - t0, 1e-9)},
                           step)
                tw.images_async([(f"train/train_{k}", im) for k, im in imgs.items()], step)
            if step % self.save_checkpoints_steps == 0 or step == steps:
                with clock.paused():
                    if main:
                        saver.save(fold_dir, step, net, trainer.optimizer,
                                   self.keep_checkpoint_max, {"config": self.config()})
                    eval_result = self._evaluate(net, ev_imgs, ev_masks, batch * 2, device, ctx,
                                                 ew if main else None, step)
                eval_result["global_step"] = step
                if main:
                    ew.scalars({k: v for k, v in eval_result.items() if k != "global_step"}, step)
                    if exporter is not None:
                        with clock.paused():
                            exporter.maybe_export(net, eval_result, step)
        if step == start and start > 0:  # already trained: evaluate the restored model
            eval_result = self._evaluate(net, ev_imgs, ev_masks, batch * 2, device, ctx)
            eval_result["global_step"] = step
        saver.wait()
        if batches is not pipe:
            batches.close()
        tw.close()
        ew.close()
        res = {"fold": fold, "n_params": self.n_params, "eval": eval_result, "steps": step,
               "hip_graph": stepper.graph, "steady_ms_per_step": clock.result(step)}
        lt.report()
        if main:
            with open(os.path.join(fold_dir, "result.json"), "w") as f:
                json.dump(res, f)
        return res

    # ---- classification (north-star workloads) -----------------------------------------------
    def _set_cls_data(self, X, y):
        """(source, ids, labels) of a classifier's training set (data/classification.py)."""
        if self.synthetic:
            ids = np.arange(int(X)) if np.isscalar(X) else np.asarray(X)
            if y is None:
                y = np.random.default_rng(self.seed).integers(0, self.num_classes, len(ids))
            self._cls_source = SyntheticImages(self.num_classes, self.image_size,
                                               self.image_channels, seed=self.seed)
        else:
            arr = np.asarray(X)
            if arr.ndim not in (3, 4):
                raise ValueError(f"arch {self.arch}: X must be images [N, H, W, C] "
                                 "(or pass synthetic=True with sample ids)")
            if y is None:
                raise ValueError("class labels y are required")
            self._cls_source = ArrayImages(arr)
            self.image_size = arr.shape[1]
            self.image_channels = self._cls_source.channels
            ids = np.arange(len(arr))
        self._cls_ids = ids
        self._cls_labels = np.asarray(y, dtype=np.int64)
        if self._cls_labels.min() < 0 or self._cls_labels.max() >= self.num_classes:
            raise ValueError(f"labels must lie in [0, {self.num_classes})")

    def _train_fold_cls(self, fold, batch, steps, ctx):
        """One fold of classifier training: softmax-CE + SGD-momentum (or Adam), the LR schedule,
        checkpoint every ``save_checkpoints_steps`` with resume, evaluation (top-1 accuracy,
        loss/softmax_cross_entropy) after every checkpoint, train summaries every
        ``save_summary_steps``, BestExporter on metrics/accuracy."""
        device = self._device(ctx)
        fold_dir = os.path.join(self.model_dir, f"fold{fold}")
        torch.manual_seed(self.seed + fold)
        net = self.build_network()
        self.n_params = sum(p.numel() for p in net.parameters()) + sum(
            b.numel() for n, b in net.named_buffers() if "running" in n)
        extra = ((lambda m: m.regularization_loss())
                 if self.use_regularization and hasattr(net, "regularization_loss") and
                 self.optimizer == "adam" else None)
        trainer = self._make_trainer(net, softmax_cross_entropy, device, ctx, steps, extra)
        start = 0
        latest = ckpt.latest_checkpoint(fold_dir)
        if latest is not None:
            start = ckpt.restore(latest, net, trainer.optimizer, trainer.flat)
            trainer.global_step = start
            if ctx.is_distributed:
                trainer.broadcast_state()
        stepper = _Stepper(trainer, self._use_graph(device, ctx))
        tr, te = self._cls_split
        dtype = torch.float32 if self.precision == "fp32" or device.type != "cuda" \
            else torch.bfloat16
        pipe = ClassificationPipeline(self._cls_source, self._cls_ids[tr], self._cls_labels[tr],
                                      batch, shuffle=True, repeat=True, seed=self.seed + fold,
                                      device=device, rank=ctx.rank, world=ctx.world_size,
                                      dtype=dtype, start_step=start)
        main = ctx.is_main
        tw = SummaryWriter(os.path.join(fold_dir, "train"), enabled=main)
        ew = SummaryWriter(os.path.join(fold_dir, "eval"), enabled=main)
        exporter = None
        if self.save_best > 0 and main:
            exporter = BestExporter(
                os.path.join(fold_dir, "export"),
                functools.partial(metric_comparisson, key="metrics/accuracy",
                                  greater_is_better=True),
                exports_to_keep=self.save_best, serving_shape=self._serving_shape(),
                model_config=self.config(), serving=self.export_format, task="classification",
                compute_dtype=self._serving_dtype(device))
        correct = StreamingMean(device)
        saver = ckpt.AsyncSaver()  # D2H on a copy stream, file write on a worker thread
        eval_result = {}
        # per-step losses land in one preallocated device buffer (no per-step allocation or host
        # sync; read once when the fold ends)
        history = torch.zeros(max(steps - start, 0), dtype=torch.float32, device=device) \
            if main else None
        n_hist = 0
        step = start
        t0 = time.time()
        clock = _StepClock(device, start)
        while step < steps:
            x, yy = next(pipe)
            loss, out = stepper(x, yy)
            step = trainer.global_step
            clock.tick(step)
            _, top1, _ = softmax_eval(out, yy)  # top-1 count in one HIP launch
            correct.update_sum(top1, yy.shape[0])
            if main and n_hist < history.numel():
                history[n_hist].copy_(loss.detach().reshape(()))
                n_hist += 1
            if self.save_summary_steps and step % self.save_summary_steps == 0 and main:
                tw.scalars({"metrics/accuracy": float(correct.result()),
                            "loss/softmax_cross_entropy": float(loss),
                            "learning_rate": trainer.optimizer.lr_at(step - 1),
                            "global_step/sec": (step - start) / max(time.time() - t0, 1e-9)},
                           step)
            if step % self.save_checkpoints_steps == 0 or step == steps:
                with clock.paused():
                    if main:
                        saver.save(fold_dir, step, net, trainer.optimizer,
                                   self.keep_checkpoint_max, {"config": self.config()})
                    eval_result = self._evaluate_cls(net, te, batch * 2, device, ctx, dtype)
                eval_result["global_step"] = step
                if main:
                    ew.scalars({k: v for k, v in eval_result.items() if k != "global_step"}, step)
                    if exporter is not None:
                        with clock.paused():
                            exporter.maybe_export(net, eval_result, step)
        if step == start and start > 0:
            eval_result = self._evaluate_cls(net, te, batch * 2, device, ctx, dtype)
            eval_result["global_step"] = step
        saver.wait()
        tw.close()
        ew.close()
        res = {"fold": fold, "n_params": self.n_params, "eval": eval_result, "steps": step,
               "train_loss": history[:n_hist].cpu().tolist() if history is not None else [],
               "hip_graph": stepper.graph,
               "steady_ms_per_step": clock.result(step)}
        if main:
            with open(os.path.join(fold_dir, "result.json"), "w") as f:
                json.dump(res, f)
        return res

    @torch.no_grad()
    def _evaluate_cls(self, net, te, batch, device, ctx, dtype):
        net.eval()
        pipe = ClassificationPipeline(self._cls_source, self._cls_ids[te], self._cls_labels[te],
                                      batch, shuffle=False, repeat=False, seed=self.seed + 1,
                                      device=device, rank=ctx.rank, world=ctx.world_size,
                                      dtype=dtype)
        sums = torch.zeros(3, dtype=torch.float64, device=device)  # correct, loss·n, count
        for i, (x, yy) in enumerate(pipe):
            if self.eval_batches is not None and i >= self.eval_batches:
                break
            n = x.shape[0]
            # loss sum and top-1 count in one HIP launch (ops/loss.softmax_eval)
            loss_sum, correct, _ = softmax_eval(net(x), yy)
            sums += torch.stack([correct.double(), loss_sum.double(),
                                 torch.tensor(float(n), dtype=torch.float64, device=device)])
        if ctx.is_distributed:
            s = sums.to(ctx.device) if ctx.native is not None else sums.cpu()
            ctx.all_reduce_sum_(s)
            sums = s
        sums = sums.cpu()
        n = max(float(sums[2]), 1.0)
        net.train()
        return {"metrics/accuracy": float(sums[0]) / n,
                "loss/softmax_cross_entropy": float(sums[1]) / n}

    @torch.no_grad()
    def predict_classes(self, X, batch_size):
        """Class probabilities [N, num_classes] of images ``X`` (or synthetic sample ids),
        averaged over every trained fold's latest checkpoint."""
        if self.synthetic:
            ids = np.arange(int(X)) if np.isscalar(X) else np.asarray(X)
            src = SyntheticImages(self.num_classes, self.image_size, self.image_channels,
                                  seed=self.seed)
        else:
            src = getattr(self, "_cls_source", None)
            src = ArrayImages(X, src.mean, src.std) if isinstance(src, ArrayImages) \
                else ArrayImages(X)
            ids = np.arange(len(src.images))
        device = torch.device(self.device) if self.device else (
            torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
        dtype = torch.bfloat16 if device.type == "cuda" and self.precision != "fp32" \
            else torch.float32
        acc, n_models = None, 0
        for i in range(self.n_folds):
            path = ckpt.latest_checkpoint(os.path.join(self.model_dir, f"fold{i}"))
            if path is None:
                continue
            net = self.build_network().to(device)
            ckpt.restore(path, net)
            if device.type == "cuda" and self.precision != "fp32":
                net._tdl_flat = FlatParams(net, device, lowp_dtype=torch.bfloat16, with_grad=False)
            net.eval()
            labels = np.zeros(len(ids), dtype=np.int64)  # unused by the image sources
            probs = [softmax_eval(net(x), probs=True)[2].cpu() for x, _ in ClassificationPipeline(
                src, ids, labels, batch_size, shuffle=False, repeat=False, device=device,
                dtype=dtype)]
            p = torch.cat(probs)
            acc = p if acc is None else acc + p
            n_models += 1
        if n_models == 0:
            raise ValueError("no trained fold checkpoints found; call train first")
        return (acc / n_models).numpy()

    @torch.no_grad()
    def _evaluate(self, net, images, masks, batch, device, ctx, writer=None, step=0):
        """One pass over the fold's held-out split (each rank its shard; sums all-reduced)."""
        net.eval()
        pipe = SegmentationPipeline(images, masks, batch, augment=False, shuffle=False,
                                    repeat=False, device=device, rank=ctx.rank,
                                    world=ctx.world_size, threads=self.loader_threads,
                                    fp32=self.precision == "fp32")
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
                # bf16 compute copies of the weights once per fold (not per batch; no gradient
                # buffer), kept with the network; in eval mode under no_grad every conv+BN runs
                # BN-folded (models/layers.ConvBN)
                net._tdl_flat = FlatParams(net, device, lowp_dtype=torch.bfloat16, with_grad=False)
            net.eval()
            for tf in transforms:
                probs, fold_ids = [], []
                for x, b_ids in TestPipeline(images, batch_size, tf, device=device,
                                             threads=self.loader_threads,
                                             fp32=self.precision == "fp32"):
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
                                        threads=self.loader_threads, aug=self.augmentation,
                                    fp32=self.precision == "fp32")
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
                                threads=self.loader_threads, fp32=self.precision == "fp32")
        return test_input_fn

    @property
    def params(self):
        try:
            return self.n_params
        except AttributeError:
            raise ValueError("No model has been defined at this point! Call train method first.")


def _summary_fetch(scalars, x, y, logits, threshold):
    """The train-summary values in ONE device→host copy: ([float scalars], {name: [H, W] array})
    — input (min-max scaled like TF's float image summary), label, probability, prediction of
    the first sample (model.py:405-440)."""
    img = x[0, :, :, 0].float()
    img = (img - img.min()) / (img.max() - img.min()).clamp_min(1e-12)
    prob = torch.sigmoid(logits[0, :, :, 0].float())
    ims = torch.stack([img, y[0, :, :, 0].float(), prob, (prob > threshold).float()])
    sc = torch.stack([torch.as_tensor(s, device=ims.device).float().reshape(()) for s in scalars])
    host = torch.cat([sc, ims.reshape(-1)]).cpu().numpy()
    n = len(scalars)
    ims_h = host[n:].reshape(ims.shape)
    return ([float(v) for v in host[:n]],
            {"image": ims_h[0], "label": ims_h[1], "prob": ims_h[2], "prediction": ims_h[3]})


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


def _lovasz_loss(out, yy):
    return lovasz_hinge(out, yy)


class _Stepper:
    """The fold loop's training step: eager for the first step, then (``graph``) one warm-up
    step that also records the step as a HIP graph (engine/trainer.Trainer.capture) and graph
    replays from there on — the loader's batch is copied into the static inputs.  The returned
    (loss, out) are the graph's static outputs, valid until the next step.  ``quiet``: a context
    that keeps other threads off the device during the capture (the device prefetcher)."""

    def __init__(self, trainer, graph, quiet=None):
        self.trainer = trainer
        self.graph = bool(graph)
        self.eager_steps = 0
        self.quiet = quiet if quiet is not None else contextlib.nullcontext

    def __call__(self, x, y):
        tr = self.trainer
        if not self.graph:
            return tr.train_step(x, y)
        if tr.graph is None:
            if self.eager_steps < 1:
                self.eager_steps += 1
                return tr.train_step(x, y)
            with self.quiet():
                tr.capture(x, y, warmup=1)  # the warm-up step trains on (x, y)
            return tr.warmup_out
        return tr.replay(x, y)


class _LoopTimer:
    """TDL_LOOP_PROFILE=1: host time of each phase of the fold loop (where the training thread
    waits), printed per fold — a host-bound loop shows up as one phase holding the step time."""

    def __init__(self):
        self.on = os.environ.get("TDL_LOOP_PROFILE", "0") == "1"
        self.acc = {}
        self.t = None
        self.n = 0

    def mark(self, phase=None):
        if not self.on:
            return
        now = time.perf_counter()
        if phase is None:
            self.n += 1
        elif self.t is not None:
            self.acc[phase] = self.acc.get(phase, 0.0) + now - self.t
        self.t = now

    def report(self):
        if self.on and self.n:
            print("[Model] loop host ms/step: " + ", ".join(
                f"{k} {v * 1e3 / self.n:.3f}" for k, v in self.acc.items()), flush=True)


class _StepClock:
    """Steady-state step time of a fold loop: wall clock between the end of step start+10 (after
    the graph capture and the caches warmed up) and the last step, with one device sync at
    each end — everything the loop does per step (loader, step, metrics, summaries) included,
    the checkpoint + evaluation passes (:meth:`paused`; reported by their own metrics) not."""

    WARM = 10

    def __init__(self, device, start):
        self.device = device
        self.mark = start + self.WARM
        self.t0 = None
        self.off = 0.0

    @contextlib.contextmanager
    def paused(self):
        if self.t0 is None:
            yield
            return
        self._sync()
        t = time.perf_counter()
        try:
            yield
        finally:
            self._sync()
            self.off += time.perf_counter() - t

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def tick(self, step):
        if step == self.mark:
            self._sync()
            self.t0 = time.perf_counter()

    def result(self, step):
        if self.t0 is None or step <= self.mark:
            return None
        self._sync()
        return (time.perf_counter() - self.t0 - self.off) * 1e3 / (step - self.mark)
