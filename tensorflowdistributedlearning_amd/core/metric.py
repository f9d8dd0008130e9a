"""core.metric — reference API (core/metric.py:3-71).

``mIOU`` / ``mean_accuracy`` return ``(value, update)`` with ``tf.metrics.mean`` semantics
(core/metric.py:42-50): the streaming state (total, count) lives on the device under ``name``
(tf's local metric variables); ``value`` reads the running mean as it stands — creating the metric
does not fold the batch in — and ``update()`` (the update op) folds this batch's per-image scores
into the state and returns the new mean.  Calling ``update()`` twice folds the batch twice, as
running the update op twice would; the mean of an empty state is 0 (tf's ``div_no_nan``).
Per-image scores come from the fused seg-metrics kernel on the GPU.
"""
from __future__ import annotations

from ..ops.metrics import IOU_THRESHOLDS, StreamingMean, seg_scores

_STATE = {}


def _stream(name, device):
    s = _STATE.get(name)
    if s is None or s.total.device != device:
        s = StreamingMean(device)
        _STATE[name] = s
    return s


def reset(name=None):
    if name is None:
        _STATE.clear()
    else:
        _STATE.pop(name, None)


def _metric(y_true, y_pred, which, name, kaggle=False):
    s = _stream(name, y_pred.device)
    value = s.result()  # the current state: this batch is not folded in yet

    def update():
        score, acc = seg_scores(y_true, y_pred, kaggle)
        return s.update(score if which == "iou" else acc)
    return value, update


def result(name):
    """The running mean of metric ``name`` (0 when empty)."""
    s = _STATE.get(name)
    return None if s is None else s.result()


def mIOU(y_true, y_pred, metrics_collections=None, updates_collections=None, name="iou",
         kaggle=False):
    """Reference formula mean_t(IoU·[IoU>t]) (D16, parity) or the Kaggle score if ``kaggle``."""
    v, u = _metric(y_true, y_pred, "iou", name, kaggle)
    if metrics_collections is not None:
        metrics_collections.append(v)
    if updates_collections is not None:
        updates_collections.append(u)
    return v, u


def mean_accuracy(y_true, y_pred, metrics_collections=None, updates_collections=None, name="acc"):
    v, u = _metric(y_true, y_pred, "acc", name)
    if metrics_collections is not None:
        metrics_collections.append(v)
    if updates_collections is not None:
        updates_collections.append(u)
    return v, u


__all__ = ["IOU_THRESHOLDS", "mIOU", "mean_accuracy", "reset", "result"]
