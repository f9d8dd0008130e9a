"""Typed configuration.

* :class:`ModelConfig` mirrors the reference ``Model`` constructor knobs and their defaults
  (model.py:13-24,29-136) plus the engine knobs that the reference hard-codes (checkpoint every
  500 steps, summaries every 20, …) — ``Model(**cfg.model_kwargs())`` builds the same model.
* :class:`BenchConfig` holds the north-star additions (architecture preset, dtype, optimizer,
  loss, synthetic data, DP bucket sizes).

Both load from / dump to plain dicts, JSON or YAML (``yaml.safe_load``) and are what the CLI
(``python -m tensorflowdistributedlearning_amd …``) fills from flags.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from typing import Optional, Tuple

# network presets: the reference's segmentation net and the north-star classifiers
SEGMENTATION_ARCHS = ("deeplab_ref",)
CLASSIFIER_ARCHS = ("resnet18", "resnet34", "resnet50", "resnet101", "resnet152", "xception41")


@dataclass
class ModelConfig:
    model_dir: str = "runs/model"
    data_directory: str = "data"
    data_format: str = "NHWC"
    lr: float = 0.001
    n_gpus: int = 2
    n_fold: int = 5
    seed: int = 42
    save_best: int = 5
    # reference kwargs (model.py:63-106) — D1/D2 fixed: each reads its own name
    weight_decay: float = 0.001
    batch_norm_decay: float = 0.99
    batch_norm_epsilon: float = 0.001
    batch_norm_scale: bool = True
    output_stride: int = 8
    base_depth: int = 256
    input_shape: Tuple[int, int] = (101, 101)
    n_blocks: Tuple[int, int, int] = (3, 4, 6)
    block_type: str = "bottleneck"
    # hard-coded in the reference (RunConfig / hooks / model_fn params)
    save_checkpoints_steps: int = 500
    save_summary_steps: int = 20
    keep_checkpoint_max: int = 5
    threshold: float = 0.5
    # extensions
    use_regularization: bool = False  # D5: opt-in L2 term
    kaggle_metric: bool = False       # D16: reference formula by default
    loader_threads: int = 4
    device: Optional[str] = None
    # GPU compute precision: "bf16" (fused bf16 kernels, fp32 accumulation / master weights) or
    # "fp32" (the reference's own precision: fp32 operands on the fp32 kernels end to end)
    precision: str = "bf16"
    # north-star workloads through Model; None = the arch's default
    arch: str = "deeplab_ref"         # or resnet18/34/50/101/152, xception41
    num_classes: int = 1000
    image_size: Optional[int] = None  # classifiers: 224 (xception41: 299)
    image_channels: int = 3
    loss: Optional[str] = None        # lovasz (deeplab_ref) | softmax_ce (classifiers)
    optimizer: Optional[str] = None   # adam (deeplab_ref) | sgd_momentum (classifiers)
    momentum: float = 0.9
    lr_schedule: str = "exponential"  # exponential (the reference's) | cosine | step | constant
    lr_decay_steps: int = 10000
    lr_decay_rate: float = 0.5
    lr_warmup_steps: int = 0
    synthetic: bool = False           # classifiers: learnable synthetic dataset (sample ids)
    fp8: bool = False                 # classifiers: fp8 forward GEMMs
    hip_graph: str = "auto"           # capture each fold's step as a HIP graph (GPU)
    eval_batches: Optional[int] = None
    max_folds: Optional[int] = None   # train only the first k folds
    export_format: str = "native"     # servable program per best export: native|portable|both|none

    def validate(self):
        if self.data_format not in ("NCHW", "NHWC"):
            raise ValueError(f"Unknown data format {self.data_format}. Has to be either NCHW or NHWC")
        if self.output_stride is not None and self.output_stride % 4:
            raise ValueError("The output_stride needs to be a multiple of 4.")
        if len(self.n_blocks) != 3:
            raise ValueError("Expect n_blocks to have length 3.")
        if self.block_type not in ("bottleneck", "basic_block"):
            raise ValueError(f"unknown block_type {self.block_type}")
        if self.precision not in ("bf16", "fp32"):
            raise ValueError(f"unknown precision {self.precision} (bf16 or fp32)")
        if self.arch not in SEGMENTATION_ARCHS + CLASSIFIER_ARCHS:
            raise ValueError(f"unknown arch {self.arch}")
        if self.export_format not in ("native", "portable", "both", "none"):
            raise ValueError(f"unknown export_format {self.export_format}")
        return self

    def model_kwargs(self):
        d = dataclasses.asdict(self)
        d["input_shape"] = tuple(d["input_shape"])
        d["n_blocks"] = tuple(d["n_blocks"])
        d["n_fold"] = d.pop("n_fold")
        for k in ("image_size", "loss", "optimizer"):  # None: the arch's default
            if d[k] is None:
                d.pop(k)
        return d


@dataclass
class BenchConfig:
    """What ``bench.py`` runs (it builds one from its flags, or from ``--config``): the
    architecture preset, precision, objective, optimizer, data source and DP bucket sizes."""
    arch: str = "resnet50"            # resnet18/34/50/101/152, xception41, deeplab_ref
    dtype: str = "bf16"               # bf16 | fp32 | fp8 (fp8 forward GEMMs, bf16 backward)
    optimizer: Optional[str] = None   # sgd_momentum (classifiers) | adam (deeplab_ref)
    loss: Optional[str] = None        # softmax_ce (classifiers) | lovasz (deeplab_ref)
    synthetic: bool = True            # the only data source of the benchmark
    batch: Optional[int] = None       # per GPU (None: 1024 for classifiers, 64/N deeplab_ref)
    image_size: Optional[int] = None  # None: 299 for xception41 (BASELINE config 4), else 224
    steps: int = 20
    warmup: int = 5
    lr: Optional[float] = None        # None: 0.1 (SGD) / 1e-3 (Adam)
    momentum: float = 0.9
    weight_decay: float = 5e-5
    bucket_mb: float = 32.0
    first_bucket_mb: float = 4.0
    grad_dtype: str = "fp32"          # dtype of the bucketed gradient all-reduces (fp32 | bf16)
    fp8_dgrad: bool = False
    graph: bool = False
    extra: dict = field(default_factory=dict)

    def validate(self):
        if self.grad_dtype not in ("fp32", "bf16"):
            raise ValueError(f"unknown gradient bucket dtype {self.grad_dtype}")
        if self.arch not in SEGMENTATION_ARCHS + CLASSIFIER_ARCHS:
            raise ValueError(f"unknown arch {self.arch}")
        seg = self.arch in SEGMENTATION_ARCHS
        self.optimizer = self.optimizer or ("adam" if seg else "sgd_momentum")
        self.loss = self.loss or ("lovasz" if seg else "softmax_ce")
        if self.lr is None:
            self.lr = 1e-3 if self.optimizer == "adam" else 0.1
        if self.image_size is None:
            self.image_size = 299 if self.arch == "xception41" else 224
        if self.dtype not in ("bf16", "fp32", "fp8"):
            raise ValueError(f"unknown dtype {self.dtype}")
        if self.optimizer not in ("adam", "sgd_momentum"):
            raise ValueError(f"unknown optimizer {self.optimizer}")
        if self.loss not in ("lovasz", "softmax_ce") or (self.loss == "lovasz") != seg:
            raise ValueError(f"loss {self.loss} does not fit arch {self.arch}")
        if not self.synthetic:
            raise ValueError("the benchmark runs on synthetic data only")
        if self.dtype == "fp8" and seg:
            raise ValueError("fp8 is for the ImageNet models")
        return self


def _coerce(cls, d):
    names = {f.name: f for f in dataclasses.fields(cls)}
    unknown = set(d) - set(names)
    if unknown:
        raise ValueError(f"unknown {cls.__name__} keys: {sorted(unknown)}")
    out = {}
    for k, v in d.items():
        if isinstance(v, list):
            v = tuple(v)
        out[k] = v
    return cls(**out)


def from_dict(cls, d):
    return _coerce(cls, dict(d))


def load(path, cls=ModelConfig):
    """JSON or YAML (safe loader) file → config."""
    with open(path) as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml
        d = yaml.safe_load(text) or {}
    else:
        d = json.loads(text)
    return from_dict(cls, d)


def dump(cfg, path):
    d = dataclasses.asdict(cfg)
    with open(path, "w") as f:
        if path.endswith((".yaml", ".yml")):
            import yaml
            yaml.safe_dump(d, f, sort_keys=False)
        else:
            json.dump(d, f, indent=1)
