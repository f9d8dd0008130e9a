"""Best-model exporter (the reference's ``tf.estimator.BestExporter(name="best_exporter",
exports_to_keep=save_best, compare_fn=metric_comparisson(key="metrics/mean_iou"))``,
model.py:189-204).

Each export is an inference bundle under ``fold{i}/export/best_exporter/<timestamp>/``:
``variables.safetensors`` (weights + BN moving statistics, reference TF names when available),
``config.json`` (model config + serving signature: input key ``images`` [None, H, W, C] — the
reference's serving key mismatch D3 is fixed), ``eval_result.json`` and — the SavedModel part —
the servable program ``model.pt2`` (+ ``model.json``; ``model_portable.pt2`` for the stock-ATen
lowering), see engine/serving.py.  At most ``exports_to_keep`` bundles are kept (oldest removed
first, like TF's exporter GC).
"""
from __future__ import annotations

import json
import os
import shutil
import time
import warnings

import torch
from safetensors.torch import save_file


class BestExporter:
    def __init__(self, export_dir, compare_fn, exports_to_keep=5, name="best_exporter",
                 serving_shape=None, model_config=None, serving="native", task="segmentation",
                 compute_dtype=None):
        """``serving``: servable program(s) written with each bundle — "native" (tdl:: ops,
        gfx950 kernels), "portable" (stock ATen), "both" or None (weights only)."""
        if serving not in (None, "none", "native", "portable", "both"):
            raise ValueError(f"unknown serving export {serving!r}")
        self.serving = None if serving == "none" else serving
        self.task = task
        self.compute_dtype = compute_dtype
        self.dir = os.path.join(export_dir, name)
        self.compare_fn = compare_fn
        self.keep = exports_to_keep
        self.best = None
        self.serving_shape = serving_shape
        self.model_config = model_config or {}
        os.makedirs(self.dir, exist_ok=True)
        self._load_best()

    def _load_best(self):
        for d in sorted(os.listdir(self.dir)):
            p = os.path.join(self.dir, d, "eval_result.json")
            if os.path.exists(p):
                with open(p) as f:
                    r = json.load(f)
                if self.best is None or self.compare_fn(self.best, r):
                    self.best = r

    def maybe_export(self, model, eval_result, step):
        """Export if ``eval_result`` beats the best so far; returns the bundle path or None."""
        if self.best is not None and not self.compare_fn(self.best, eval_result):
            return None
        self.best = dict(eval_result)
        ts = str(int(time.time() * 1000))
        out = os.path.join(self.dir, ts)
        os.makedirs(out, exist_ok=True)
        names = model.tf_names() if hasattr(model, "tf_names") else {}
        tensors = {names.get(k, k): v.detach().to("cpu").contiguous()
                   for k, v in model.state_dict().items()}
        save_file(tensors, os.path.join(out, "variables.safetensors"))
        served = self._serving(model, out) if self.serving and self.serving_shape else {}
        outputs = (["probabilities", "mask"] if self.task == "segmentation"
                   else ["logits", "probabilities", "classes"])
        with open(os.path.join(out, "config.json"), "w") as f:
            json.dump({"model": self.model_config, "global_step": int(step),
                       "signature": {"inputs": {"images": self.serving_shape},
                                     "outputs": outputs}, "serving": served}, f)
        with open(os.path.join(out, "eval_result.json"), "w") as f:
            json.dump({k: float(v) for k, v in eval_result.items()}, f)
        self._gc()
        return out

    def _serving(self, model, out):
        """Write the servable program(s); a tracing failure is reported in config.json (and
        warned) instead of ending the training run that produced the weights."""
        from . import serving as sv
        p = next(iter(model.parameters()))
        example = torch.zeros([2] + list(self.serving_shape[1:]), device=p.device)
        kinds = ("native", "portable") if self.serving == "both" else (self.serving,)
        res = {}
        for kind in kinds:
            name = "model.pt2" if kind == "native" else "model_portable.pt2"
            try:
                sv.export_serving(model, example, os.path.join(out, name), self.task, kind,
                                  self.compute_dtype)
                res[kind] = name
            except Exception as e:  # noqa: BLE001 — keep the weights bundle
                warnings.warn(f"serving export ({kind}) failed: {e!r}")
                res[kind] = f"error: {e!r}"
        return res

    def _gc(self):
        exports = sorted(d for d in os.listdir(self.dir) if d.isdigit())
        while self.keep and len(exports) > self.keep:
            shutil.rmtree(os.path.join(self.dir, exports.pop(0)), ignore_errors=True)


def load_export(path, model):
    """Load an exported bundle's weights into ``model`` (inverse name map)."""
    from safetensors.torch import load_file
    tensors = load_file(os.path.join(path, "variables.safetensors"))
    names = model.tf_names() if hasattr(model, "tf_names") else {}
    with torch.no_grad():
        for k, v in model.state_dict().items():
            key = names.get(k, k)
            if key in tensors:
                v.copy_(tensors[key].to(v.device, v.dtype))
    return model
