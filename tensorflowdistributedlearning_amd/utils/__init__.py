"""Utilities (reference utils.py).

* :func:`get_available_gpus` — names of the visible HIP devices (reference: TF ``device_lib``
  filtered to GPUs, utils.py:6-8).  Uses ``torch.cuda.device_count()``, which on this ROCm image
  does not initialise the GPU.
* :func:`metric_comparisson` — BestExporter comparator.  The reference returns ``best > current``
  for ``greater_is_better`` (utils.py:23-28), i.e. the inverse of what BestExporter expects
  (defect D4); here it returns True when ``current`` is better than ``best``.  The misspelt name is
  kept for API parity.
"""
from __future__ import annotations

LOSS_KEY = "loss"


def get_available_gpus():
    import torch
    n = torch.cuda.device_count()
    return [f"/device:GPU:{i}" for i in range(n)]


def metric_comparisson(best_eval_result, current_eval_result, key=LOSS_KEY,
                       greater_is_better=True):
    if not best_eval_result or key not in best_eval_result:
        raise ValueError("best_eval_result cannot be empty or no loss is found in it.")
    if not current_eval_result or key not in current_eval_result:
        raise ValueError("current_eval_result cannot be empty or no loss is found in it.")
    if greater_is_better:
        return current_eval_result[key] > best_eval_result[key]
    return current_eval_result[key] < best_eval_result[key]


__all__ = ["get_available_gpus", "metric_comparisson"]
