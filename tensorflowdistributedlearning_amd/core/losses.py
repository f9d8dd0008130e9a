"""core.losses — reference API (core/losses.py:5-92).

``lovasz_loss`` / ``lovasz_hinge(per_image=True, ignore=None)`` run the fused HIP Lovász kernel
on the GPU (one workgroup per image: LDS bitonic sort, scans, loss and gradient — the reference's
CPU ``tf.map_fn`` + ``top_k`` path, D17).  ``per_image=False`` and ``ignore`` masks use the
PyTorch reference implementation (same math, differentiable).
"""
from __future__ import annotations

import torch

from ..ops import loss as _L

lovasz_grad = _L.lovasz_grad


def flatten_binary_scores(scores, labels, ignore=None):
    scores = scores.reshape(-1)
    labels = labels.reshape(-1)
    if ignore is None:
        return scores, labels
    valid = labels != ignore
    return scores[valid], labels[valid]


def lovasz_hinge_flat(logits, labels):
    """Differentiable reference form (gradient flows through the sorted errors only)."""
    if logits.numel() == 0:
        return logits.sum() * 0.0
    labelsf = labels.float()
    signs = 2.0 * labelsf - 1.0
    errors = 1.0 - logits.float() * signs.detach()
    errors_sorted, perm = torch.sort(errors, descending=True, stable=True)
    grad = lovasz_grad(labelsf[perm]).detach()
    return torch.dot(torch.relu(errors_sorted), grad)


def lovasz_hinge(logits, labels, per_image=True, ignore=None):
    if per_image and ignore is None:
        return _L.lovasz_hinge(logits, labels)
    if per_image:
        losses = [lovasz_hinge_flat(*flatten_binary_scores(l, y, ignore))
                  for l, y in zip(logits, labels)]
        return torch.stack(losses).mean()
    return lovasz_hinge_flat(*flatten_binary_scores(logits, labels, ignore))


def lovasz_loss(y_true, y_pred, data_format="NHWC"):
    """Squeeze the channel axis and apply per-image Lovász hinge (losses.py:83-92)."""
    ax = -1 if data_format == "NHWC" else 1
    return lovasz_hinge(y_pred.squeeze(ax), y_true.squeeze(ax), per_image=True, ignore=None)
