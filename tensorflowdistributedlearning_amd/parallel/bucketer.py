"""Bucketed gradient all-reduce overlapped with backward.

The reference concatenates ALL gradients into one NCCL pack after the full backward
(``num_packs=1``, Test.ipynb:200 — SURVEY §2.4/§2.6: 167 MB, no overlap).  Here:

* gradients already live in one flat fp32 buffer (models/params.py) laid out in forward order, so a
  bucket is just a contiguous slice — no pack/unpack copies;
* buckets are cut walking the parameters *backwards* (the order backward produces them); each of
  our autograd Functions calls ``p._grad_hook(p)`` right after its wgrad kernel is enqueued; when
  the last parameter of a bucket lands, the bucket's all-reduce is issued immediately on the
  native RCCL communicator (parallel/rccl.py orders it after the producing kernels with an event
  and runs it on its own high-priority comm stream, so it overlaps the rest of backward on the
  compute stream; the optimizer's stream waits on the bucket's completion event only);
* buckets are always launched in index order (identical on every rank, as RCCL requires);
* the first-issued bucket is kept small so communication starts early, later ones are large
  (``bucket_mb``, default 32 MB) — fewer, larger collectives suit xGMI's per-link ring bandwidth
  (7 links × ≈153 GB/s per MI355X);
* the last-issued bucket (the network's first layers, whose gradients arrive when backward
  ends) is also kept small: it is the one collective nothing overlaps, so its size is exposed
  step time — the remainder is split off the bucket before it;
* the 1/world averaging is fused into the optimizer kernel (no extra pass);
* with side-stream weight gradients (ops/streams.py) a collective is issued from the side stream
  after it waited for the compute stream, so the comm stream follows both producers and the
  compute stream is never made to wait at a bucket boundary (:meth:`GradBucketer.issue_stream`).

Delivery accounting: a bucket is launched when each of its parameters has delivered its *final*
contribution of the step, not when the hook has fired ``len(params)`` times.  ``deliver_grad``
fires the hook on every contribution; a parameter that legitimately receives several (a weight
used twice in the forward) declares it with ``p._tdl_contribs = n``.  A delivery beyond that
raises — a second delivery after the bucket was launched would mean the collective read a
gradient that was still changing — and :meth:`finish` records parameters that delivered nothing
(unused ones, zero-filled by ``FlatParams.finish_grads``) in ``last_missing`` (an error with
``strict=True``).  ``early_launches`` counts the collectives issued from the hooks, i.e. while
backward was still running (the overlap), as opposed to those forced by :meth:`finish`.

bf16 gradient buckets (``comm_dtype=torch.bfloat16``, SURVEY §5.8 "bf16/fp32 gradient buckets"):
each bucket's fp32 gradients are packed into a bf16 mirror of the flat gradient buffer on the
issuing stream (``ext().convert``, one pass over the slice), the collective runs on the bf16
slice — half the bytes on xGMI — and :meth:`finish` unpacks the whole mirror back into the fp32
buffer in one pass after the collectives, so the optimizer still accumulates in fp32.  The RCCL /
gloo reduction itself sums in bf16 (an option for communication-bound runs, off by default).

A ``comm_hook`` can replace the collective (used by tests to record launch order with a fake
communicator, or to snapshot each bucket in stream order: tests/test_bucket_order_gpu.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import streams


class Bucket:
    __slots__ = ("index", "lo", "hi", "params", "pending", "launched", "work")

    def __init__(self, index, lo, hi, params):
        self.index, self.lo, self.hi, self.params = index, lo, hi, params
        self.pending = len(params)
        self.launched = False
        self.work = None

    @property
    def nbytes(self):
        return (self.hi - self.lo) * 4  # (fp32 slice; a bf16 bucket moves half)

    @staticmethod
    def hi_of(p, flat):
        lo, _ = flat.slice_of(p)
        return lo + ((p.numel() + 63) // 64) * 64


class GradBucketer:
    def __init__(self, flat, ctx=None, bucket_mb=32.0, first_bucket_mb=4.0, comm_hook=None,
                 group=None, strict=False, comm_dtype=torch.float32):
        self.flat = flat
        self.strict = strict
        if comm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"gradient bucket dtype: float32 or bfloat16, not {comm_dtype}")
        self.comm_dtype = comm_dtype
        # the bf16 mirror of the flat gradient buffer the collectives run on (bf16 buckets)
        self.comm16 = (torch.zeros(flat.grad.numel(), dtype=torch.bfloat16,
                                   device=flat.grad.device)
                       if comm_dtype == torch.bfloat16 else None)
        self._seen = {}          # id(param) -> contributions delivered this step
        self.early_launches = 0  # collectives issued from hooks in the last finished step
        self._early = 0
        self.last_missing = []   # parameters that delivered nothing in the last finished step
        self.ctx = ctx
        self.group = group
        self.comm_hook = comm_hook
        self.buckets = []
        self.bucket_of = {}
        cap_first = int(first_bucket_mb * 2 ** 20 / 4)
        cap = int(bucket_mb * 2 ** 20 / 4)
        params = list(flat.params)
        cur, cur_lo, cur_hi = [], None, None
        limit = cap_first
        for p in reversed(params):
            lo, _ = flat.slice_of(p)
            hi = lo + ((p.numel() + 63) // 64) * 64
            if cur_hi is None:
                cur_hi = hi
            cur.append(p)
            cur_lo = lo
            if (cur_hi - cur_lo) >= limit:
                self._add_bucket(cur_lo, cur_hi, cur)
                cur, cur_lo, cur_hi = [], None, None
                limit = cap
        if cur:
            self._add_bucket(cur_lo, cur_hi, cur)
        self._shrink_tail(cap_first)
        self.next_launch = 0
        for p in params:
            p._grad_hook = self._on_ready

    def _shrink_tail(self, cap):
        """Split the last bucket so that its trailing part (the earliest parameters) holds at
        most ~``cap`` elements: all but that part goes into its own bucket before it."""
        last = self.buckets[-1]
        if len(last.params) < 2 or last.hi - last.lo <= cap:
            return
        # last.params runs from high to low offsets; keep the lowest-offset params ≤ cap
        keep = []
        for p in reversed(last.params):
            if keep and last.hi_of(p, self.flat) - last.lo > cap:
                break
            keep.append(p)
        head = last.params[: len(last.params) - len(keep)]
        if not head:
            return
        split = self.flat.slice_of(keep[-1])[0] + ((keep[-1].numel() + 63) // 64) * 64
        self.buckets.pop()
        self._add_bucket(split, last.hi, head)
        self._add_bucket(last.lo, split, list(reversed(keep)))

    def _add_bucket(self, lo, hi, ps):
        b = Bucket(len(self.buckets), lo, hi, list(ps))
        self.buckets.append(b)
        for p in ps:
            self.bucket_of[id(p)] = b

    # ------------------------------------------------------------------------------------------
    def _on_ready(self, p):
        b = self.bucket_of.get(id(p))
        if b is None:
            return
        k = id(p)
        n = self._seen.get(k, 0) + 1
        self._seen[k] = n
        need = getattr(p, "_tdl_contribs", 1)
        if n > need:
            raise RuntimeError(
                f"GradBucketer: gradient of parameter {tuple(p.shape)} (bucket {b.index}) "
                f"delivered {n} times in one step, expected {need}"
                + (" — its bucket's collective was already issued" if b.launched else "")
                + "; declare extra contributions with p._tdl_contribs")
        if n < need:
            return
        b.pending -= 1
        before = self.next_launch
        self._launch_ready()
        self._early += self.next_launch - before

    def _launch_ready(self, force=False):
        while self.next_launch < len(self.buckets):
            b = self.buckets[self.next_launch]
            if b.pending > 0 and not force:
                break
            self._launch(b)
            self.next_launch += 1

    def _launch(self, b):
        view = self.flat.grad[b.lo:b.hi]
        issuer = self.issue_stream(view.device) if view.is_cuda else None
        if issuer is None:
            self._issue(b, self._pack(b, view))
        else:
            with streams.on(issuer):
                self._issue(b, self._pack(b, view))
        b.launched = True

    def _pack(self, b, view):
        """The tensor the collective runs on: the fp32 slice, or its bf16 copy (packed on the
        current stream, i.e. after the bucket's producers)."""
        if self.comm16 is None:
            return view
        v16 = self.comm16[b.lo:b.hi]
        if view.is_cuda:
            from ..ops.common import ext
            ext().convert(view, v16)
        else:
            v16.copy_(view)
        return v16

    def _unpack(self):
        """bf16 buckets: the reduced bf16 mirror back into the fp32 gradient buffer (one pass, on
        the current stream, after every collective was waited for)."""
        if self.comm16 is None:
            return
        if self.flat.grad.is_cuda:
            from ..ops.common import ext
            ext().convert(self.comm16, self.flat.grad)
        else:
            self.flat.grad.copy_(self.comm16)

    @staticmethod
    def issue_stream(device):
        """The stream a bucket's collective is ordered after: the side stream, made to wait for
        the compute stream's position first, when side-stream weight gradients are in use — the
        bucket's gradients come from both streams (conv weights on the side stream, BN γ/β and
        biases on the compute stream), and the comm stream then waits on one event that follows
        both.  The compute stream never waits: a join at a bucket boundary would stall the
        dgrad / BN chain behind every weight gradient still queued on the side stream.  None:
        no side stream (or one outside the capture in progress) — issue from the current
        stream."""
        dev = torch.device(device)
        s = streams.side_if_active(dev)
        if s is None:
            return None
        cur = streams.current(dev)
        if cur != s:
            s.wait_stream(cur)
        else:
            # the hook fired inside a side-stream section (a weight gradient's delivery): the
            # bucket may also hold gradients written on the compute stream before it (BN γ/β of
            # the folded depthwise BN, ops/bnfold.py), which the side stream has not waited for
            s.wait_stream(streams.origin(dev))
        return s

    def _issue(self, b, view):
        if self.comm_hook is not None:
            b.work = self.comm_hook(b, view)
        elif self.ctx is not None and self.ctx.is_distributed:
            if getattr(self.ctx, "native", None) is not None:
                b.work = self.ctx.all_reduce_async(view)  # native RCCL (parallel/rccl.py)
            else:
                b.work = dist.all_reduce(view, async_op=True, group=self.group)

    def finish(self):
        """After backward: launch any bucket still pending (unused parameters — their grads were
        zeroed by ``FlatParams.finish_grads``), wait for all collectives, reset for next step."""
        missing = [p for b in self.buckets for p in b.params
                   if self._seen.get(id(p), 0) < getattr(p, "_tdl_contribs", 1)]
        self._launch_ready(force=True)
        self.last_missing = missing
        self.early_launches = self._early
        self._early = 0
        self._seen = {}
        for b in self.buckets:
            if b.work is not None and hasattr(b.work, "wait"):
                b.work.wait()
            b.work = None
            b.launched = False
            b.pending = len(b.params)
        self.next_launch = 0
        self._unpack()
        if self.ctx is not None and hasattr(self.ctx, "check"):
            self.ctx.check()  # native comm watchdog: fail fast on timeout / RCCL error
        if missing and self.strict:
            raise RuntimeError(f"GradBucketer: {len(missing)} parameter(s) delivered no final "
                               f"gradient this step: {[tuple(p.shape) for p in missing[:8]]}")

    def standalone_ms(self, reps=3):
        """Milliseconds of the step's collectives alone — every bucket issued back to back on an
        idle device, then waited for — the yardstick for how much of the communication the
        overlapped backward hides (bench.py reports exposed / standalone for N > 1)."""
        import time
        cuda = self.flat.grad.is_cuda
        times = []
        for _ in range(reps):
            if cuda:
                torch.cuda.synchronize(self.flat.grad.device)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
            t0 = time.perf_counter()
            for b in self.buckets:
                self._issue(b, self._pack(b, self.flat.grad[b.lo:b.hi]))
            for b in self.buckets:
                if b.work is not None and hasattr(b.work, "wait"):
                    b.work.wait()
                b.work = None
            if cuda:
                e1.record()
                torch.cuda.synchronize(self.flat.grad.device)
                times.append(e0.elapsed_time(e1))
            else:
                times.append((time.perf_counter() - t0) * 1e3)
        return sorted(times)[len(times) // 2]

    def describe(self):
        return [(b.index, len(b.params), b.nbytes) for b in self.buckets]

    @property
    def comm_bytes(self):
        """Bytes one step's collectives move per rank (before the ring's 2·(n−1)/n factor)."""
        per = 2 if self.comm16 is not None else 4
        return sum((b.hi - b.lo) * per for b in self.buckets)
