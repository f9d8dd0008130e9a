"""Segmentation metrics (per image), computed on device.

``seg_scores(labels, predictions)`` returns per-image (iou_score, pixel_accuracy) in one kernel
(``csrc/kernels/metrics.hip``: one workgroup per image counts TP/FP/FN/TN with a block reduction,
then applies the threshold formula).

* reference ``mIOU`` formula (core/metric.py:14-33): IoU = TP/(TP+FP+FN) (1 if the denominator is
  0), score = mean_t(IoU·[IoU > t]) over IOU_THRESHOLDS — defect D16 reproduced for parity;
* ``kaggle=True`` gives the intended Kaggle score mean_t([IoU > t]);
* accuracy = mean(labels == predictions) (core/metric.py:53-71).
"""
from __future__ import annotations

import torch

from .common import on_gpu, ext

IOU_THRESHOLDS = [0.5, 0.55, 0.6, 0.65, 0.7, 0.75, 0.8, 0.85, 0.9, 0.95]


def ref_seg_scores(labels, preds, kaggle=False):
    B = labels.shape[0]
    lab = labels.reshape(B, -1).float() > 0.5
    pr = preds.reshape(B, -1).float() > 0.5
    tp = (lab & pr).sum(1).float()
    fp = (~lab & pr).sum(1).float()
    fn = (lab & ~pr).sum(1).float()
    den = tp + fp + fn
    iou = torch.where(den > 0, tp / den.clamp_min(1), torch.ones_like(den))
    th = torch.tensor(IOU_THRESHOLDS, device=iou.device)
    hit = (iou.view(-1, 1) > th.view(1, -1)).float()
    score = hit.mean(1) if kaggle else (iou.view(-1, 1) * hit).mean(1)
    acc = (lab == pr).float().mean(1)
    return score, acc


def seg_scores(labels, preds, kaggle=False):
    if on_gpu(preds):
        B = labels.shape[0]
        score = torch.empty(B, device=preds.device, dtype=torch.float32)
        acc = torch.empty_like(score)
        ext().seg_metrics(labels.reshape(B, -1).contiguous(), preds.reshape(B, -1).contiguous(),
                          score, acc, bool(kaggle))
        return score, acc
    return ref_seg_scores(labels, preds, kaggle)


class StreamingMean:
    """Device-resident streaming mean (tf.metrics.mean semantics, core/metric.py:42-50)."""

    def __init__(self, device=None):
        self.total = torch.zeros((), dtype=torch.float64, device=device)
        self.count = torch.zeros((), dtype=torch.float64, device=device)

    def update(self, values):
        v = values.detach().reshape(-1)
        self.total += v.double().sum()
        self.count += v.numel()
        return self.result()

    def update_sum(self, total, count):
        """Fold in a pre-reduced batch: ``total`` (device scalar) over ``count`` values."""
        self.total += total.detach().double()
        self.count += float(count)
        return self.result()

    def result(self):
        return self.total / self.count.clamp_min(1)

    def reset(self):
        self.total.zero_()
        self.count.zero_()
