"""Loss functions with fused forward+gradient kernels.

* ``softmax_cross_entropy`` — classification loss of the north-star workloads (BASELINE.json:
  ResNet-50/152, Xception).  One HIP kernel computes the per-row log-softmax loss and the gradient
  (softmax − onehot)/N in a single pass over the logits (``csrc/kernels/loss.hip``).  Not present
  in the reference (its classification head, core/resnet.py:249-256, has no loss) — SURVEY §2.7.
* ``lovasz_hinge`` — the reference's binary Lovász hinge, per image (core/losses.py:5-92).  The
  reference runs it on the CPU with ``tf.map_fn`` + ``tf.nn.top_k`` full sort (model.py:391,
  SURVEY K16/D17); here one workgroup per image sorts the P errors in LDS (bitonic), scans the
  Jaccard gradient and emits loss and ∂loss/∂logit without leaving the GPU.
"""
from __future__ import annotations

import torch

from .common import on_gpu, ext


# ----------------------------------------------------------------------------------------------
# softmax cross entropy
# ----------------------------------------------------------------------------------------------

def ref_softmax_xent(logits, labels, label_smoothing=0.0):
    lf = logits.float()
    logp = torch.log_softmax(lf, dim=-1)
    N, K = lf.shape
    onehot = torch.zeros_like(lf).scatter_(1, labels.view(-1, 1).long(), 1.0)
    if label_smoothing:
        onehot = onehot * (1 - label_smoothing) + label_smoothing / K
    loss_rows = -(onehot * logp).sum(-1)
    grad = (torch.softmax(lf, -1) - onehot) / N
    return loss_rows.mean(), grad


class _SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, label_smoothing):
        logits = logits.contiguous()
        if on_gpu(logits):
            loss = torch.zeros((), device=logits.device, dtype=torch.float32)
            grad = torch.empty_like(logits)
            ext().softmax_xent(logits, labels, loss, grad, float(label_smoothing))
        else:
            loss, grad = ref_softmax_xent(logits, labels, label_smoothing)
            grad = grad.to(logits.dtype)
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (grad,) = ctx.saved_tensors
        if on_gpu(grad):
            out = torch.empty_like(grad)
            ext().scale_by_scalar(grad, dloss.float().reshape(1).contiguous(), out)
            return out, None, None
        return (grad.float() * dloss.float()).to(grad.dtype), None, None


def softmax_cross_entropy(logits, labels, label_smoothing=0.0):
    """Mean softmax cross-entropy over the batch. logits [N, K]; labels int [N]."""
    return _SoftmaxXentFn.apply(logits, labels, label_smoothing)


def softmax_eval(logits, labels=None, probs=False):
    """Forward-only classification head (evaluation / prediction, no gradient): returns
    ``(loss_sum, correct, p)`` — the summed softmax cross-entropy and the number of rows whose
    argmax is the label (fp32 device scalars, None without ``labels``) and the fp32 softmax
    probabilities [N, K] when ``probs``.  GPU: one HIP launch (``loss.hip`` softmax_eval_kernel);
    CPU: the fp32 reference ops."""
    logits = logits.contiguous()
    if logits.dim() != 2:
        raise ValueError(f"softmax_eval: logits [N, K], got {tuple(logits.shape)}")
    if on_gpu(logits) and logits.dtype in (torch.bfloat16, torch.float32):
        dev = logits.device
        ls = torch.zeros(1, device=dev) if labels is not None else None
        cr = torch.zeros(1, device=dev) if labels is not None else None
        p = torch.empty(logits.shape, device=dev, dtype=torch.float32) if probs else None
        lab = labels.to(device=dev, dtype=torch.int64).contiguous() if labels is not None else None
        ext().softmax_eval(logits, lab, ls, cr, p)
        return (ls[0] if ls is not None else None), (cr[0] if cr is not None else None), p
    lf = logits.float()
    p = torch.softmax(lf, -1) if probs else None
    if labels is None:
        return None, None, p
    lab = labels.long().view(-1)
    ls = (torch.logsumexp(lf, -1) - lf.gather(1, lab.view(-1, 1)).view(-1)).sum()
    cr = (lf.argmax(-1) == lab).float().sum()
    return ls, cr, p


# ----------------------------------------------------------------------------------------------
# Lovász hinge (binary, per image)
# ----------------------------------------------------------------------------------------------

def lovasz_grad(gt_sorted):
    """Gradient of the Lovász extension w.r.t. sorted errors (core/losses.py:5-15)."""
    gts = gt_sorted.sum()
    intersection = gts - gt_sorted.cumsum(0)
    union = gts + (1.0 - gt_sorted).cumsum(0)
    jaccard = 1.0 - intersection / union
    if gt_sorted.numel() > 1:
        jaccard = torch.cat([jaccard[:1], jaccard[1:] - jaccard[:-1]])
    return jaccard


def ref_lovasz_hinge_flat(logits, labels):
    """Per-image loss and d loss / d logits (core/losses.py:40-65)."""
    if logits.numel() == 0:
        return logits.sum() * 0.0, torch.zeros_like(logits)
    labelsf = labels.float()
    signs = 2.0 * labelsf - 1.0
    errors = 1.0 - logits.float() * signs
    errors_sorted, perm = torch.sort(errors, descending=True, stable=True)
    gt_sorted = labelsf[perm]
    g = lovasz_grad(gt_sorted)
    loss = torch.dot(torch.relu(errors_sorted), g)
    dsorted = g * (errors_sorted > 0).float()
    derr = torch.empty_like(errors)
    derr[perm] = dsorted
    return loss, -signs * derr


def ref_lovasz_hinge(logits, labels):
    """logits, labels: [B, P] (flattened per image). Returns mean loss and grad [B, P]."""
    B = logits.shape[0]
    losses, grads = [], []
    for i in range(B):
        li, gi = ref_lovasz_hinge_flat(logits[i].float(), labels[i])
        losses.append(li)
        grads.append(gi)
    return torch.stack(losses).mean(), torch.stack(grads) / B


class _LovaszFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        shape = logits.shape
        B = shape[0]
        lg = logits.reshape(B, -1).contiguous()
        lb = labels.reshape(B, -1).contiguous()
        if on_gpu(lg):
            loss = torch.zeros((), device=lg.device, dtype=torch.float32)
            grad = torch.empty(lg.shape, device=lg.device, dtype=torch.float32)
            ext().lovasz_hinge(lg, lb, loss, grad)
        else:
            loss, grad = ref_lovasz_hinge(lg, lb)
        ctx.shape = shape
        ctx.dtype = logits.dtype
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (grad,) = ctx.saved_tensors
        g = (grad * dloss.float()).to(ctx.dtype).reshape(ctx.shape)
        return g, None


def lovasz_hinge(logits, labels):
    """Binary Lovász hinge, per image, mean over the batch.  logits [B, ...], labels {0,1}."""
    return _LovaszFn.apply(logits, labels)
