"""Side HIP stream for weight gradients (default on; ``TDL_WGRAD_STREAM=0`` disables).

A conv's wgrad and dgrad both read only dy; the rest of the backward chain (the BN backward of the
layer below, its dgrad, …) needs only dgrad.  With the side stream the wgrad (+ bias colsum)
runs concurrently with that chain, so the memory-bound BN kernels can overlap the MFMA-bound
wgrads.  Ordering: the side stream waits for the compute stream before each wgrad (dy ready);
the compute stream joins the side stream before any gradient bucket is all-reduced
(parallel/bucketer.py) and after backward (engine/trainer.py), so no collective or optimizer
reads a gradient that is still being written.

Under HIP-graph capture the side stream is forked into the capture by that same event wait (a
captured cross-stream dependency) and joined back before the capture ends, so a captured training
step keeps the wgrad overlap (``TDL_WGRAD_IN_GRAPH=0``: wgrads on the capturing stream instead).

Measured on one MI355X (bench.py, eager): ResNet-50 b256 9646 → 9925 img/s, Xception-41 b128
2551 → 2650, reference DeepLab preset b64 4685 → 4814."""
from __future__ import annotations

import os

import torch

_ENABLED = os.environ.get("TDL_WGRAD_STREAM", "1") == "1"
IN_GRAPH = os.environ.get("TDL_WGRAD_IN_GRAPH", "1") == "1"
_FORKED: set = set()  # devices whose side stream joined the capture in progress
# Tensors the side stream reads (a conv's dy and x), held until the caller's stream next joins
# the side stream.  Dropped then, their blocks return to the caching allocator with every later
# use on the joined stream ordered after the side stream's reads.  (record_stream instead
# defers each block's reuse to an event poll; with the side stream a few layers behind, the
# allocator kept carving new segments: ResNet-50 b512 reserved 108 GiB for 21 GiB allocated.)
_KEEP: dict = {}
KEEP_ALIVE = os.environ.get("TDL_SIDE_KEEPALIVE", "1") == "1"


def current(device):
    """``torch.cuda.current_stream(device)`` without its Python-level device normalisation (this
    runs several times per conv backward; the public helper cost ≈5 µs per call, ≈1.4 ms of host
    time per step of the reference DeepLab preset — dev/tools/host_overhead.py)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    sid, di, dt = torch._C._cuda_getCurrentStream(idx)
    return torch.cuda.Stream(stream_id=sid, device_index=di, device_type=dt)


def capturing() -> bool:
    """Is the current stream capturing a HIP graph (raw query, no lazy-init wrapper)?"""
    return torch._C._cuda_isCurrentStreamCapturing()


class on:
    """``with on(stream):`` — make ``stream`` current on its device, restore the previous one on
    exit (a lean ``torch.cuda.stream`` for the per-conv side-stream switch)."""
    __slots__ = ("s", "prev")

    def __init__(self, stream):
        self.s = stream

    def __enter__(self):
        self.prev = torch._C._cuda_getCurrentStream(self.s.device_index)
        torch._C._cuda_setStream(stream_id=self.s.stream_id, device_index=self.s.device_index,
                                 device_type=self.s.device_type)
        return self.s

    def __exit__(self, *exc):
        sid, di, dt = self.prev
        torch._C._cuda_setStream(stream_id=sid, device_index=di, device_type=dt)
        return False


def keep_alive(device, *tensors):
    """Keep ``tensors`` (read by side-stream work; allocated on the caller's stream) alive until
    the caller's stream next joins the side stream (:func:`join`)."""
    if KEEP_ALIVE:
        dev = torch.device(device)
        cur = current(dev)
        _KEEP.setdefault((dev, cur.stream_id), []).extend(tensors)
    else:
        s = _SIDE[torch.device(device)]
        for t in tensors:
            t.record_stream(s)
_ORIGIN: dict = {}    # device -> the stream that last forked work onto the side stream
# Record the side stream's wait on dy before the conv's dgrad is launched (the wgrad overlaps that
# dgrad too); TDL_WGRAD_EARLY=0 records it after the dgrad launch (the previous ordering, for A/B).
EARLY_WAIT = os.environ.get("TDL_WGRAD_EARLY", "1") == "1"
_SIDE: dict = {}
# HIP stream priority of the side stream (A/B knob; torch.cuda.Stream.priority_range(): lower is
# more urgent)
SIDE_PRIO = int(os.environ.get("TDL_SIDE_PRIO", "0"))


def enabled() -> bool:
    return _ENABLED


def set_enabled(flag: bool):
    global _ENABLED
    _ENABLED = bool(flag)


def side(device):
    """The side stream for ``device`` when enabled, else None.  During a graph capture the
    caller's ``side.wait_stream(current)`` forks it into the capture; :func:`join` merges it
    back."""
    if not _ENABLED or device.type != "cuda":
        return None
    if capturing():
        if not IN_GRAPH:
            return None
        _FORKED.add(torch.device(device))
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device=device, priority=SIDE_PRIO)
    cur = current(device)
    if cur != s:
        _ORIGIN[torch.device(device)] = cur
    return s


def side_if_active(device):
    """The side stream of ``device`` if it exists and may take work now (outside a capture, or
    forked into the capture in progress), else None.  Unlike :func:`side` it does not create
    the stream or fork it into a capture."""
    dev = torch.device(device)
    s = _SIDE.get(dev)
    if s is None or not _ENABLED:
        return None
    if capturing() and dev not in _FORKED:
        return None
    return s


def is_side(stream, device) -> bool:
    """Is ``stream`` the side stream of ``device``?"""
    s = _SIDE.get(torch.device(device))
    return s is not None and stream == s


def origin(device):
    """The stream that forks work onto the side stream (the compute / capturing stream)."""
    return _ORIGIN.get(torch.device(device), current(torch.device(device)))


def end_capture(capture_stream=None):
    """Forget the capture's forked side streams and the tensors its side-stream work read (call
    once the capture has ended: the graph's private pool keeps their memory for its replays)."""
    _FORKED.clear()
    if capture_stream is not None:
        for key in [k for k in _KEEP if k[1] == capture_stream.stream_id]:
            del _KEEP[key]


_JOIN_QUEUED: dict = {}  # device -> autograd graph-task id whose final callback joins it


def join_at_backward_end(device):
    """Make the running autograd pass end with the caller's stream joined to the side stream.

    Called by every backward that queues work on the side stream.  The first call of a pass
    registers an autograd final callback; the engine runs final callbacks on the streams that
    were current around the user's ``backward()`` call (after syncing them with the leaf
    streams), so ``loss.backward()`` returns with every gradient the side stream writes ordered
    before anything the caller queues next — also outside :class:`Trainer`, which joins
    explicitly as well.  Parameters' ``.grad`` tensors are therefore safe to read on the
    caller's stream without a manual :func:`join`.  Keyed by the graph-task id, so a pass that
    died before its callbacks ran cannot suppress the next pass's registration."""
    dev = torch.device(device)
    task = torch._C._current_graph_task_id()
    if task < 0:  # not inside a backward pass (a direct call of the backward function):
        join(dev)  # called after the side-stream work was queued, so join right away
        return
    if _JOIN_QUEUED.get(dev) == task:
        return

    def _cb():
        if _JOIN_QUEUED.get(dev) == task:
            del _JOIN_QUEUED[dev]
        join(dev)

    torch.autograd.Variable._execution_engine.queue_callback(_cb)
    _JOIN_QUEUED[dev] = task


def join(device=None):
    """Make the current stream wait for all work queued on the side stream(s).  While a HIP graph
    is being captured only side streams forked into that capture are joined (a wait on an event
    of a stream outside the capture must not enter the graph)."""
    cap = torch.cuda.is_available() and capturing()
    for dev, s in _SIDE.items():
        if device is None or dev == torch.device(device):
            if cap and dev not in _FORKED:
                continue
            cur = current(dev)
            cur.wait_stream(s)
            if cur != s and not cap:
                # everything queued on `cur` from here on runs after the side stream's reads
                _KEEP.pop((dev, cur.stream_id), None)
