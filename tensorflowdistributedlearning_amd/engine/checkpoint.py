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
(device → host of one contiguous buffer per state tensor) and writes on rank 0 only;
:class:`AsyncSaver` does the copies on a copy stream into pinned buffers and the file write on a
worker thread, so the training loop never waits for the host.
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


def _collect(model, optimizer, step, to_host):
    """(tensors, slot plan, optimizer kind): every variable copied to the host by ``to_host``
    (synchronous, or into pinned buffers on a copy stream); the optimizer slots as whole flat
    buffers, split per variable by :func:`_finish` once the copies have landed."""
    names = _names(model)
    tensors = {}
    for k, v in model.state_dict().items():
        tensors[names[k]] = to_host("v/" + k, v.detach())
    tensors["global_step"] = torch.tensor([step], dtype=torch.int64)
    opt_kind, plan = None, None
    if optimizer is not None:
        opt_kind = type(optimizer).__name__
        flat = optimizer.flat
        host_slots = {s: to_host("s/" + s, t.detach()) for s, t in optimizer.state_tensors().items()}
        pname = {id(p): n for n, p in model.named_parameters()}
        plan = (host_slots, [(names.get(pname[id(p)], pname[id(p)]), flat.slice_of(p), p.shape)
                             for p in flat.params])
        if hasattr(optimizer, "beta1"):
            t = optimizer.step_count
            tensors["beta1_power"] = torch.tensor([optimizer.beta1 ** (t + 1)], dtype=torch.float32)
            tensors["beta2_power"] = torch.tensor([optimizer.beta2 ** (t + 1)], dtype=torch.float32)
    return names, tensors, plan, opt_kind


def _finish(tensors, plan):
    if plan is not None:
        host_slots, vars_ = plan
        for base, (o, e), shape in vars_:
            for sname, st in host_slots.items():
                tensors[f"{base}/{sname}"] = st[o:e].reshape(shape).clone()
    return {k: v.contiguous() for k, v in tensors.items()}


def save(directory, step, model, optimizer=None, keep_max=5, extra_meta=None):
    os.makedirs(directory, exist_ok=True)
    names, tensors, plan, opt_kind = _collect(
        model, optimizer, step, lambda key, t: t.to("cpu", copy=True))
    return _write(directory, step, names, _finish(tensors, plan), opt_kind, keep_max, extra_meta)


class AsyncSaver:
    """Checkpoint writes off the training thread (SURVEY §5.4 "rank 0 writes after async D2H").

    ``save`` copies every device tensor into pinned host buffers (reused across saves) on a
    dedicated copy stream ordered after the work queued so far, makes the caller's stream wait
    for those copies only (the next optimizer step cannot overwrite a variable before it is
    copied; the host never blocks), and returns; a worker thread waits for the copies, then
    writes the safetensors file and moves the ``checkpoint`` pointer.  At most one save is in
    flight (a second waits for the first); :meth:`wait` joins — called before anything reads
    the directory (fold end, restore)."""

    def __init__(self):
        self._thread = None
        self._error = None
        self._pinned = {}
        self._stream = None

    def _to_host(self, key, t):
        if not t.is_cuda:
            return t.to("cpu", copy=True)
        buf = self._pinned.get(key)
        if buf is None or buf.shape != t.shape or buf.dtype != t.dtype:
            buf = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            self._pinned[key] = buf
        with torch.cuda.stream(self._stream):
            buf.copy_(t, non_blocking=True)
        return buf

    def save(self, directory, step, model, optimizer=None, keep_max=5, extra_meta=None):
        self.wait()
        os.makedirs(directory, exist_ok=True)
        dev = next((p.device for p in model.parameters() if p.is_cuda), None)
        if dev is None:  # host model: nothing to overlap
            return save(directory, step, model, optimizer, keep_max, extra_meta)
        if self._stream is None:
            self._stream = torch.cuda.Stream(dev)
        cur = torch.cuda.current_stream(dev)
        self._stream.wait_stream(cur)
        names, tensors, plan, opt_kind = _collect(model, optimizer, step, self._to_host)
        done = torch.cuda.Event()
        done.record(self._stream)
        cur.wait_event(done)  # the device waits for the copies, the host does not

        def work():
            try:
                done.synchronize()
                _write(directory, step, names, _finish(tensors, plan), opt_kind, keep_max,
                       extra_meta)
            except BaseException as e:  # surfaced by wait()
                self._error = e

        import threading
        self._thread = threading.Thread(target=work, name="tdl-ckpt", daemon=True)
        self._thread.start()
        return os.path.join(directory, f"model.ckpt-{step}.safetensors")

    def wait(self):
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise e


def _write(directory, step, names, tensors, opt_kind, keep_max, extra_meta):
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
