"""Checkpoints in the reference's directory layout.

Layout per fold directory (``model_dir/fold{i}``):
  checkpoint                       TF-style pointer file (model_checkpoint_path / all_model_checkpoint_paths)
  model.ckpt-{step}.safetensors    flat, self-describing tensor file (no pickle), names =
                                   the reference's TF variable names when the model provides
                                   ``tf_names()`` (DeepLab preset: ``M/resnet_v2/block1/...``)
  model.ckpt-{step}.json           metadata (step, names map, optimizer kind, config)

Contents: every parameter and buffer (BN moving statistics), ``global_step``, optimizer slots
(``<var>/Adam``, ``<var>/Adam_1`` or ``<var>/Momentum``), ``beta1_power`` / ``beta2_power`` for
Adam — the TF1 variable set [TF-internal naming].  Saving copies the flat buffers to host once
(device → host of one contiguous buffer per state tensor) and writes on rank 0 only.
Resume: :func:`latest_checkpoint` + :func:`restore` reproduce TF's "continue from the latest
checkpoint of the fold" behaviour; ``keep_max`` (default 5) old checkpoints are retained.
"""
from __future__ import annotations

import glob
import json
import os
import re

import torch
from safetensors.torch import save_file, load_file


def _names(model):
    fn = getattr(model, "tf_names", None)
    sd = model.state_dict()
    if fn is None:
        return {k: k for k in sd}
    m = fn()
    return {k: m.get(k, k) for k in sd}


def save(directory, step, model, optimizer=None, keep_max=5, extra_meta=None):
    os.makedirs(directory, exist_ok=True)
    names = _names(model)
    tensors = {}
    for k, v in model.state_dict().items():
        tensors[names[k]] = v.detach().to("cpu", copy=True).contiguous()
    tensors["global_step"] = torch.tensor([step], dtype=torch.int64)
    opt_kind = None
    if optimizer is not None:
        opt_kind = type(optimizer).__name__
        flat = optimizer.flat
        slots = optimizer.state_tensors()
        host_slots = {s: t.detach().to("cpu") for s, t in slots.items()}
        pname = {id(p): n for n, p in model.named_parameters()}
        for p in flat.params:
            o, e = flat.slice_of(p)
            base = names.get(pname[id(p)], pname[id(p)])
            for sname, st in host_slots.items():
                tensors[f"{base}/{sname}"] = st[o:e].reshape(p.shape).clone()
        if hasattr(optimizer, "beta1"):
            t = optimizer.step_count
            tensors["beta1_power"] = torch.tensor([optimizer.beta1 ** (t + 1)], dtype=torch.float32)
            tensors["beta2_power"] = torch.tensor([optimizer.beta2 ** (t + 1)], dtype=torch.float32)
    prefix = f"model.ckpt-{step}"
    path = os.path.join(directory, prefix + ".safetensors")
    tmp = path + ".tmp"
    save_file(tensors, tmp)
    os.replace(tmp, path)
    meta = {"step": int(step), "names": names, "optimizer": opt_kind}
    if extra_meta:
        meta.update(extra_meta)
    with open(os.path.join(directory, prefix + ".json"), "w") as f:
        json.dump(meta, f)
    _update_pointer(directory, prefix, keep_max)
    return path


def _all_steps(directory):
    steps = []
    for p in glob.glob(os.path.join(directory, "model.ckpt-*.safetensors")):
        m = re.search(r"model\.ckpt-(\d+)\.safetensors$", p)
        if m:
            steps.append(int(m.group(1)))
    return sorted(steps)


def _update_pointer(directory, latest_prefix, keep_max):
    steps = _all_steps(directory)
    while keep_max and len(steps) > keep_max:
        old = steps.pop(0)
        for ext in (".safetensors", ".json"):
            try:
                os.remove(os.path.join(directory, f"model.ckpt-{old}{ext}"))
            except FileNotFoundError:
                pass
    lines = [f'model_checkpoint_path: "{latest_prefix}"']
    lines += [f'all_model_checkpoint_paths: "model.ckpt-{s}"' for s in steps]
    with open(os.path.join(directory, "checkpoint"), "w") as f:
        f.write("\n".join(lines) + "\n")


def latest_checkpoint(directory):
    ptr = os.path.join(directory, "checkpoint")
    if os.path.exists(ptr):
        with open(ptr) as f:
            for line in f:
                m = re.match(r'model_checkpoint_path: "(.+)"', line.strip())
                if m:
                    p = os.path.join(directory, m.group(1) + ".safetensors")
                    if os.path.exists(p):
                        return p
    steps = _all_steps(directory)
    return os.path.join(directory, f"model.ckpt-{steps[-1]}.safetensors") if steps else None


class CheckpointMismatchError(KeyError):
    """A checkpoint lacks variables the model (or optimizer) needs — TF's Saver raises
    ``NotFoundError`` in the same situation; training must not continue silently from a partial
    random init (e.g. a checkpoint of another preset, or a renamed ``tf_names()`` mapping)."""


def restore(path, model, optimizer=None, flat=None, strict=True):
    """Load a checkpoint written by :func:`save`; returns the global step.

    ``strict`` (default): every model variable — and, with ``optimizer``, every slot variable —
    must be present with a matching element count, else :class:`CheckpointMismatchError` lists
    them and nothing is loaded.  ``strict=False`` loads what matches and warns about the rest."""
    tensors = load_file(path)
    names = _names(model)
    sd = model.state_dict()
    missing = [names[k] for k, v in sd.items()
               if names[k] not in tensors or tensors[names[k]].numel() != v.numel()]
    slot_plan = []
    if optimizer is not None:
        pname = {id(p): n for n, p in model.named_parameters()}
        slots = optimizer.state_tensors()
        for p in optimizer.flat.params:
            o, e = optimizer.flat.slice_of(p)
            base = names.get(pname[id(p)], pname[id(p)])
            for sname, st in slots.items():
                key = f"{base}/{sname}"
                if key in tensors and tensors[key].numel() == e - o:
                    slot_plan.append((key, st, o, e))
                else:
                    missing.append(key)
    if missing:
        msg = (f"{path}: {len(missing)} variable(s) missing or of another size, e.g. "
               f"{missing[:5]}")
        if strict:
            raise CheckpointMismatchError(msg)
        import warnings
        warnings.warn("partial restore — " + msg)
    with torch.no_grad():
        for k, v in sd.items():
            key = names[k]
            if key in tensors and tensors[key].numel() == v.numel():
                v.copy_(tensors[key].to(v.device, v.dtype).reshape(v.shape))
        for key, st, o, e in slot_plan:
            st[o:e].copy_(tensors[key].reshape(-1).to(st.device))
    if flat is not None:
        flat.sync_lowp()
    step = int(tensors["global_step"][0]) if "global_step" in tensors else 0
    if optimizer is not None:
        optimizer.step_count = step
    return step
