"""Module cache standing in for TF variable scopes (``reuse`` semantics)."""
import torch

_CACHE = {}


def get_or_create(key, factory, device=None):
    m = _CACHE.get(key)
    if m is None:
        m = factory()
        _CACHE[key] = m
    if device is not None:
        m = m.to(device)
        _CACHE[key] = m
    return m


def clear():
    _CACHE.clear()


def to_nhwc(x, data_format):
    if data_format == "NCHW":
        return x.permute(0, 2, 3, 1).contiguous()
    if data_format != "NHWC":
        raise ValueError(f"Unknown data format {data_format}. Has to be either NCHW or NHWC")
    return x


def from_nhwc(x, data_format):
    return x.permute(0, 3, 1, 2).contiguous() if data_format == "NCHW" else x


def device_of(x):
    return x.device if isinstance(x, torch.Tensor) else None
