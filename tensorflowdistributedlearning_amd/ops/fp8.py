"""fp8 (OCP e4m3fn) per-tensor quantisation for the fp8 forward convolution.

``quantize_e4m3(x)`` → ``(x8, scale)`` with ``scale = amax(|x|) / 448`` kept on the device (a [1]
fp32 tensor: no host synchronisation) and ``x8 = sat(x / scale)`` in ``torch.float8_e4m3fn``.
GPU: ``csrc/kernels/fp8.hip`` (amax reduction + vectorised ``v_cvt_pk_fp8_f32`` quantiser).
CPU: the same math in PyTorch (the reference for the tests).
"""
from __future__ import annotations

import torch

from .common import on_gpu, ext

E4M3 = torch.float8_e4m3fn
E4M3_MAX = 448.0


def quantize_e4m3(x):
    if on_gpu(x):
        amax = torch.zeros(1, device=x.device, dtype=torch.float32)
        scale = torch.empty(1, device=x.device, dtype=torch.float32)
        y8 = torch.empty(x.shape, device=x.device, dtype=E4M3)
        xc = x.contiguous()
        ext().fp8_amax(xc, amax)
        ext().fp8_quantize(xc, amax, scale, y8)
        return y8, scale
    xf = x.float()
    amax = xf.abs().max().clamp_min(1e-12)
    scale = (amax / E4M3_MAX).reshape(1)
    y8 = (xf / scale).clamp(-E4M3_MAX, E4M3_MAX).to(E4M3)
    return y8, scale


def dequantize(y8, scale):
    if on_gpu(y8):
        out = torch.empty(y8.shape, device=y8.device, dtype=torch.float32)
        ext().fp8_dequantize(y8.contiguous(), scale, out)
        return out
    return y8.float() * scale
