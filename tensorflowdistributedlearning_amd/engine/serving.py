"""Servable export: the inference network as a ``torch.export`` program (the reference's
``BestExporter`` SavedModel with a ``serving_input_receiver_fn`` signature, model.py:189-204).

A SavedModel is a self-contained graph + variables that a server runs without the Python that
built it.  The equivalent here is an ``ExportedProgram`` (``.pt2``): the eval-mode network with
every BN folded into its conv (models/layers.ConvBN), traced once, saved with its constants, and
reloaded with ``torch.export.load`` — no model classes, configs or builders needed.  Two lowerings:

* ``native`` (default): every layer primitive is a registered PyTorch operator of the ``tdl``
  namespace (``torch.ops.tdl.conv2d``, ``dwconv2d``, ``max_pool2d``, ``avg_pool``,
  ``upsample``, ``add_act``, ``row_pack``, ``bn_act``, ``sigmoid_threshold``) whose GPU
  implementation is the hand-written gfx950 kernel and whose CPU implementation is the fp32
  reference.  Loading needs ``import tensorflowdistributedlearning_amd.engine.serving`` (it
  registers the operators — the way a SavedModel needs the TF ops it names).
* ``portable``: the same graph lowered to stock ATen operators (``aten.convolution``, …), so the
  artifact runs on any PyTorch build and device with nothing of this package installed — slower,
  but servable anywhere.

Signature (D3 fixed — the reference's receiver declared ``image`` but its model read
``images``): input ``images`` float [batch, H, W, C] (batch dynamic); outputs
``probabilities`` + ``mask`` (segmentation, sigmoid + 0.5 threshold as model.py:479-495 PREDICT)
or ``logits`` + ``probabilities`` + ``classes`` (classifiers).

Tracing: the model code stays as it is; while :func:`export_serving` traces, the ops layer
(``ops/common.export_impl``) hands each primitive to the active lowering instead of launching a
kernel on a fake tensor.
"""
from __future__ import annotations

import contextlib
import json
import os
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F

from ..ops import common as _common

Tensor = torch.Tensor


@contextlib.contextmanager
def _suspended():
    """Run an operator's eager implementation with export routing off (the kernels proper)."""
    prev = _common._EXPORT[0]
    _common._EXPORT[0] = None
    try:
        yield
    finally:
        _common._EXPORT[0] = prev


def _geom(stride, padding, dilation):
    from ..ops.conv import ConvGeom
    return ConvGeom(tuple(stride), tuple(padding), tuple(dilation))


def _out_hw(H, W, R, S, stride, padding, dilation):
    Ho = (H + padding[0] + padding[1] - dilation[0] * (R - 1) - 1) // stride[0] + 1
    Wo = (W + padding[2] + padding[3] - dilation[1] * (S - 1) - 1) // stride[1] + 1
    return Ho, Wo


# ----------------------------------------------------------------------------------------------
# tdl:: operators (eager implementation = the ops layer: HIP kernel on the GPU, fp32 reference on
# the CPU; fake implementation = output metadata for tracing)
# ----------------------------------------------------------------------------------------------

@torch.library.custom_op("tdl::conv2d", mutates_args=())
def conv2d_op(x: Tensor, w: Tensor, bias: Optional[Tensor], residual: Optional[Tensor],
              stride: List[int], padding: List[int], dilation: List[int], relu: bool) -> Tensor:
    """act(conv(x, w) + bias [+ residual]), NHWC x, KRSC w, fp32 bias."""
    from ..ops.conv import conv_fwd
    with _suspended():
        return conv_fwd(x, w, _geom(stride, padding, dilation), bias=bias, relu=relu,
                        residual=residual)


@conv2d_op.register_fake
def _(x, w, bias, residual, stride, padding, dilation, relu):
    Ho, Wo = _out_hw(x.shape[1], x.shape[2], w.shape[1], w.shape[2], stride, padding, dilation)
    return x.new_empty((x.shape[0], Ho, Wo, w.shape[0]))


@torch.library.custom_op("tdl::dwconv2d", mutates_args=())
def dwconv2d_op(x: Tensor, w: Tensor, bias: Optional[Tensor], stride: List[int],
                padding: List[int], dilation: List[int], relu: bool, relu_in: bool) -> Tensor:
    """Depthwise k×k conv, weight [R, S, C], optional fused input / output ReLU."""
    from ..ops.dwconv import depthwise_conv2d
    with _suspended():
        return depthwise_conv2d(x, w, bias, _geom(stride, padding, dilation), relu, relu_in)


@dwconv2d_op.register_fake
def _(x, w, bias, stride, padding, dilation, relu, relu_in):
    Ho, Wo = _out_hw(x.shape[1], x.shape[2], w.shape[0], w.shape[1], stride, padding, dilation)
    return x.new_empty((x.shape[0], Ho, Wo, x.shape[3]))


@torch.library.custom_op("tdl::max_pool2d", mutates_args=())
def max_pool2d_op(x: Tensor, k: int, s: int, padding: List[int]) -> Tensor:
    from ..ops.pool import max_pool2d
    with _suspended():
        return max_pool2d(x, k, s, tuple(padding))


@max_pool2d_op.register_fake
def _(x, k, s, padding):
    Ho, Wo = _out_hw(x.shape[1], x.shape[2], k, k, (s, s), padding, (1, 1))
    return x.new_empty((x.shape[0], Ho, Wo, x.shape[3]))


@torch.library.custom_op("tdl::avg_pool", mutates_args=())
def avg_pool_op(x: Tensor, keepdims: bool) -> Tensor:
    """Global average pool over H, W."""
    from ..ops.pool import global_avg_pool
    with _suspended():
        return global_avg_pool(x, keepdims).clone()


@avg_pool_op.register_fake
def _(x, keepdims):
    return x.new_empty((x.shape[0], 1, 1, x.shape[3]) if keepdims else (x.shape[0], x.shape[3]))


@torch.library.custom_op("tdl::upsample", mutates_args=())
def upsample_op(x: Tensor, out_h: int, out_w: int) -> Tensor:
    """TF1 ``resize_bilinear`` (align_corners=False, legacy half-pixel off) of the reference's
    ``_upsample``."""
    from ..ops.upsample import upsample
    with _suspended():
        return upsample(x, (out_h, out_w))


@upsample_op.register_fake
def _(x, out_h, out_w):
    return x.new_empty((x.shape[0], out_h, out_w, x.shape[3]))


@torch.library.custom_op("tdl::add_act", mutates_args=())
def add_act_op(a: Tensor, b: Optional[Tensor], relu: bool) -> Tensor:
    from ..ops.elementwise import _AddReluFn
    with _suspended():
        return _AddReluFn.apply(a, b, relu)


@add_act_op.register_fake
def _(a, b, relu):
    return torch.empty_like(a)


@torch.library.custom_op("tdl::row_pack", mutates_args=())
def row_pack_op(x: Tensor, creal: int, S: int, sw: int, pl: int, Wo: int, Cp: int) -> Tensor:
    from ..ops.conv import _row_pack
    with _suspended():
        return _row_pack(x, creal, S, sw, pl, Wo, Cp)


@row_pack_op.register_fake
def _(x, creal, S, sw, pl, Wo, Cp):
    return x.new_empty((x.shape[0], x.shape[1], Wo, Cp))


@torch.library.custom_op("tdl::bn_act", mutates_args=())
def bn_act_op(x: Tensor, coef: Tensor, residual: Optional[Tensor], relu: bool) -> Tensor:
    """act(x·coef[0] + coef[1] [+ residual]) — an eval-mode BN (+ReLU) no conv absorbed."""
    from ..ops.bn import bn_apply
    with _suspended():
        return bn_apply(x, coef, residual, relu)


@bn_act_op.register_fake
def _(x, coef, residual, relu):
    return torch.empty_like(x)


@torch.library.custom_op("tdl::sigmoid_threshold", mutates_args=())
def sigmoid_threshold_op(logits: Tensor, threshold: float) -> Tuple[Tensor, Tensor]:
    from ..ops.elementwise import sigmoid_threshold
    with _suspended():
        return sigmoid_threshold(logits.contiguous(), threshold)


@sigmoid_threshold_op.register_fake
def _(logits, threshold):
    return (logits.new_empty(logits.shape, dtype=torch.float32),
            logits.new_empty(logits.shape, dtype=torch.float32))


# ----------------------------------------------------------------------------------------------
# lowerings the ops layer calls while a model is traced
# ----------------------------------------------------------------------------------------------

class _Native:
    """Every primitive as its ``tdl::`` operator (gfx950 kernels at run time)."""
    kind = "native"

    def conv2d(self, x, w, geom, bias, relu, residual):
        return torch.ops.tdl.conv2d(x, w, bias, residual, list(geom.stride), list(geom.padding),
                                    list(geom.dilation), bool(relu))

    def dwconv2d(self, x, w, bias, geom, relu, relu_in):
        return torch.ops.tdl.dwconv2d(x, w, bias, list(geom.stride), list(geom.padding),
                                      list(geom.dilation), bool(relu), bool(relu_in))

    def max_pool2d(self, x, k, s, pad):
        return torch.ops.tdl.max_pool2d(x, int(k), int(s), list(pad))

    def avg_pool(self, x, keepdims):
        return torch.ops.tdl.avg_pool(x, bool(keepdims))

    def upsample(self, x, out_h, out_w):
        return torch.ops.tdl.upsample(x, int(out_h), int(out_w))

    def add_act(self, a, b, relu):
        return torch.ops.tdl.add_act(a, b, bool(relu))

    def row_pack(self, x, creal, S, sw, pl, Wo, Cp):
        return torch.ops.tdl.row_pack(x, int(creal), int(S), int(sw), int(pl), int(Wo), int(Cp))

    def bn_act(self, x, coef, residual, relu):
        return torch.ops.tdl.bn_act(x, coef, residual, bool(relu))

    def sigmoid_threshold(self, logits, threshold):
        return torch.ops.tdl.sigmoid_threshold(logits, float(threshold))


def _interp_const(in_size, out_size):
    """The bilinear interpolation matrix as a real constant (built in numpy, so the tracer
    records one tensor instead of the per-tap element updates)."""
    import numpy as np
    from ..ops.upsample import _taps
    i0, i1, w0, w1 = _taps(in_size, out_size)
    A = np.zeros((out_size, in_size), dtype=np.float32)
    for o in range(out_size):
        A[o, i0[o]] += w0[o]
        A[o, i1[o]] += w1[o]
    return torch.tensor(A)


class _Portable:
    """Every primitive in stock ATen operators (the fp32 references of the ops layer), output
    cast back to the activation dtype like the kernels' bf16 stores."""
    kind = "portable"

    def conv2d(self, x, w, geom, bias, relu, residual):
        from ..ops.conv import ref_conv_fwd
        y = ref_conv_fwd(x, w, geom, bias)
        if residual is not None:
            y = y + residual.float()
        return (torch.relu(y) if relu else y).to(x.dtype)

    def dwconv2d(self, x, w, bias, geom, relu, relu_in):
        from ..ops.dwconv import ref_dw_fwd
        y = ref_dw_fwd(torch.relu(x) if relu_in else x, w, geom, bias)
        return (torch.relu(y) if relu else y).to(x.dtype)

    def max_pool2d(self, x, k, s, pad):
        from ..ops.pool import ref_max_pool
        return ref_max_pool(x, k, s, pad).to(x.dtype)

    def avg_pool(self, x, keepdims):
        y = x.float().mean(dim=(1, 2), keepdim=bool(keepdims))
        return y.to(x.dtype)

    def upsample(self, x, out_h, out_w):
        Ah = _interp_const(int(x.shape[1]), int(out_h)).to(x.device)
        Aw = _interp_const(int(x.shape[2]), int(out_w)).to(x.device)
        return torch.einsum("ia,jb,nabc->nijc", Ah, Aw, x.float()).to(x.dtype)

    def add_act(self, a, b, relu):
        y = a.float() + (b.float() if b is not None else 0.0)
        return (torch.relu(y) if relu else y).to(a.dtype)

    def row_pack(self, x, creal, S, sw, pl, Wo, Cp):
        N, H, W, _ = x.shape
        xp = F.pad(x[..., :creal], (0, 0, pl, max(0, (Wo - 1) * sw + S - W - pl)))
        cols = xp.unfold(2, S, sw)[:, :, :Wo]
        t = cols.permute(0, 1, 2, 4, 3).reshape(N, H, Wo, S * creal)
        return F.pad(t, (0, Cp - S * creal)).contiguous()

    def bn_act(self, x, coef, residual, relu):
        y = x.float() * coef[0] + coef[1]
        if residual is not None:
            y = y + residual.float()
        return (torch.relu(y) if relu else y).to(x.dtype)

    def sigmoid_threshold(self, logits, threshold):
        p = torch.sigmoid(logits.float())
        return p, (p > threshold).float()


LOWERINGS = {"native": _Native, "portable": _Portable}


@contextlib.contextmanager
def export_mode(kind="native"):
    """Route the ops layer to a lowering (``native`` / ``portable``) while tracing."""
    prev = _common._EXPORT[0]
    _common._EXPORT[0] = LOWERINGS[kind]()
    try:
        yield
    finally:
        _common._EXPORT[0] = prev


# ----------------------------------------------------------------------------------------------
# serving signature + export / load
# ----------------------------------------------------------------------------------------------

class ServingModule(torch.nn.Module):
    """The serving signature around an eval-mode network: ``images`` float NHWC in, a dict of
    named outputs (see the module docstring) out."""

    def __init__(self, net, task="segmentation", compute_dtype=torch.bfloat16, threshold=0.5):
        super().__init__()
        if task not in ("segmentation", "classification"):
            raise ValueError(f"unknown serving task {task!r}")
        # not a registered submodule: the tracer then sees the network's tensors as constants
        # and keeps only those the inference graph reads (folded weights, not the raw
        # parameters / moving statistics they were folded from)
        self.__dict__["net"] = net
        self.task = task
        self.compute_dtype = compute_dtype
        self.threshold = float(threshold)

    def forward(self, images):
        logits = self.net(images.to(self.compute_dtype))
        if self.task == "segmentation":
            from ..ops.elementwise import sigmoid_threshold
            prob, mask = sigmoid_threshold(logits, self.threshold)
            return {"probabilities": prob, "mask": mask}
        lf = logits.float()
        return {"logits": lf, "probabilities": torch.softmax(lf, dim=-1),
                "classes": torch.argmax(lf, dim=-1)}


def _freeze(net, dtype, device):
    """Materialise every derived inference tensor the trace would otherwise recompute per call
    (bf16 weight copies of the unfolded convs, eval BN coefficients) as real tensors stashed on
    the modules (``_serve``), read by the ops layer's export paths."""
    from ..models.layers import Conv2d, DepthwiseConv2d, BatchNorm
    from ..ops.bn import eval_coef
    from ..ops.common import compute_weight
    for m in net.modules():
        if isinstance(m, Conv2d):
            m.__dict__["_serve"] = (m.compute_weight(dtype).detach().clone(),
                                    None if m.bias is None else m.compute_bias().float().clone())
        elif isinstance(m, DepthwiseConv2d):
            m.__dict__["_serve"] = (compute_weight(m.weight, dtype).detach().clone(),
                                    None if m.bias is None else m.bias.detach().float().clone())
        elif isinstance(m, BatchNorm):
            m.__dict__["_serve"] = eval_coef(m, device)


def _unfreeze(net):
    for m in net.modules():
        m.__dict__.pop("_serve", None)


def default_dtype(device):
    return torch.bfloat16 if torch.device(device).type == "cuda" else torch.float32


def export_serving(net, example, path, task="segmentation", kind="native", compute_dtype=None,
                   dynamic_batch=True, max_batch=1 << 16, threshold=0.5):
    """Trace ``net`` (eval mode, BN folded) behind the serving signature and save the program to
    ``path`` (``.pt2``); ``example``: a float [n, H, W, C] batch on the serving device.  Returns
    the ``ExportedProgram``.  The network's train/eval mode is restored afterwards."""
    if kind not in LOWERINGS:
        raise ValueError(f"unknown export kind {kind!r} (native | portable)")
    dtype = compute_dtype or default_dtype(example.device)
    was_training = net.training
    net.eval()
    wrapper = ServingModule(net, task, dtype, threshold)
    try:
        with torch.no_grad():
            _freeze(net, dtype, example.device)
            dyn = None
            if dynamic_batch:
                dyn = ({0: torch.export.Dim("batch", min=1, max=max_batch)},)
            with export_mode(kind):
                # one eager pass through the same lowering first: the folded weights (and other
                # per-version derived copies) are materialised as real tensors, so the trace
                # captures them as constants instead of re-folding BN on every call
                wrapper(example)
                ep = torch.export.export(wrapper, (example,), dynamic_shapes=dyn, strict=False)
    finally:
        _unfreeze(net)
        net.train(was_training)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.export.save(ep, path)
    meta = {"kind": kind, "task": task, "compute_dtype": str(dtype).replace("torch.", ""),
            "inputs": {"images": [None] + list(example.shape[1:])},
            "outputs": (["probabilities", "mask"] if task == "segmentation"
                        else ["logits", "probabilities", "classes"]),
            "device": str(example.device)}
    with open(os.path.splitext(path)[0] + ".json", "w") as f:
        json.dump(meta, f, indent=1)
    return ep


def load_serving(path, device=None):
    """Load an exported program and return its callable module (``images`` → dict).  ``device``
    moves it (e.g. a portable program exported on the GPU, served on the CPU)."""
    ep = torch.export.load(path)
    if device is not None:
        from torch.export.passes import move_to_device_pass
        ep = move_to_device_pass(ep, device)
    return ep.module()
