"""core.metric — reference API (core/metric.py:3-71).

``mIOU`` / ``mean_accuracy`` return ``(value, update)`` like ``tf.metrics.mean``: ``update`` is a
callable that folds the current batch into a device-resident streaming mean stored under
``name`` (tf's local metric variables); ``value`` is the running mean *after* this batch.
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
    score, acc = seg_scores(y_true, y_pred, kaggle)
    vals = score if which == "iou" else acc
    s = _stream(name, vals.device)
    value = s.update(vals)

    def update():
        return s.result()
    return value, update


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


__all__ = ["IOU_THRESHOLDS", "mIOU", "mean_accuracy", "reset"]
