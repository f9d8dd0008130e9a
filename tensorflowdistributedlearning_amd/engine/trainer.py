"""The per-process training step (the reference's MonitoredTrainingSession loop body,
SURVEY §3.2/§3.5): forward → loss → backward with bucketed all-reduce overlap → fused optimizer.

Nothing in ``train_step`` synchronises with the host: the loss comes back as a device tensor and is
read only when the caller asks (summaries every N steps, like the reference's SummarySaverHook
every 20 steps, model.py:470-473).
"""
from __future__ import annotations

import time

import torch

from ..models import params as _params
from ..models.params import FlatParams
from ..parallel.bucketer import GradBucketer
from ..parallel.dist import get_context
from .optimizer import build_optimizer
from ..ops import workspace, streams
from ..ops.fp8 import RingRoller


class PhaseTimer:
    """Per-phase step timing with device events: forward, backward (incl. the
    bucketed all-reduces launched from the gradient hooks), comm_wait (waiting for the last
    buckets), optimizer.  Events are read lazily — ``summary()`` synchronises once."""

    PHASES = ("forward", "backward", "comm_wait", "optimizer")

    def __init__(self, device):
        self.cuda = device.type == "cuda"
        self.steps = []
        self.cur = {}

    def mark(self, name):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.cur[name] = e
        else:
            self.cur[name] = time.perf_counter()

    def end_step(self):
        self.steps.append(self.cur)
        self.cur = {}

    def summary(self, reset=True):
        """Mean milliseconds per phase over the recorded steps."""
        if not self.steps:
            return {}
        if self.cuda:
            torch.cuda.synchronize()
        tot = {p: 0.0 for p in self.PHASES}
        order = ("start",) + self.PHASES
        for st in self.steps:
            for a, b in zip(order[:-1], order[1:]):
                if self.cuda:
                    tot[b] += st[a].elapsed_time(st[b])
                else:
                    tot[b] += (st[b] - st[a]) * 1e3
        n = len(self.steps)
        if reset:
            self.steps = []
        res = {k: v / n for k, v in tot.items()}
        res["step"] = sum(res.values())
        return res


class Trainer:
    def __init__(self, model, loss_fn, device, optimizer="sgd", opt_kwargs=None, ctx=None,
                 bucket_mb=32.0, first_bucket_mb=4.0, lowp_dtype=torch.bfloat16,
                 broadcast_init=True, extra_loss_fn=None, profile_phases=False,
                 grad_comm_dtype=torch.float32):
        self.device = torch.device(device)
        self.model = model.to(self.device)
        self.loss_fn = loss_fn
        self.extra_loss_fn = extra_loss_fn
        self.ctx = ctx or get_context()
        self.flat = FlatParams(self.model, self.device, lowp_dtype=lowp_dtype)
        if self.ctx.is_distributed and broadcast_init:
            self.broadcast_state()
        self.optimizer = build_optimizer(optimizer, self.flat, **(opt_kwargs or {}))
        # grad_comm_dtype: the dtype the bucketed all-reduces move (bf16: half the bytes; the
        # optimizer still accumulates into fp32, parallel/bucketer.py)
        self.bucketer = (GradBucketer(self.flat, self.ctx, bucket_mb, first_bucket_mb,
                                      comm_dtype=grad_comm_dtype)
                         if self.ctx.is_distributed else None)
        self.global_step = 0
        self.train_mode = True  # False: BN uses moving statistics while training (frozen BN)
        self.timer = PhaseTimer(self.device) if profile_phases else None
        self.graph = None  # HIP graph of one whole step (capture / replay)
        # fp8 delayed scaling: one end-of-step device roll of every amax ring (ops/fp8.py)
        # (a no-op until the model's first fp8 scaler exists)
        self.fp8_roller = RingRoller(self.model)
        self._comm_marks = []  # (backward end, collectives done) per eager DP step

    # ------------------------------------------------------------------------------------------
    def broadcast_state(self):
        """rank-0 → all broadcast of parameters and buffers (MirroredVariable init)."""
        self.ctx.broadcast_(self.flat.master, 0)
        for b in self.model.buffers():
            self.ctx.broadcast_(b, 0)
        self.flat.sync_lowp()

    def train_step(self, x, y):
        if self.graph is not None:
            raise RuntimeError("this Trainer runs a captured graph: use replay()")
        return self._step(x, y)

    def _step(self, x, y):
        t = self.timer
        if self.model.training != self.train_mode:  # (the recursive set is ~0.8 ms of host time)
            self.model.train(self.train_mode)
        workspace.reset(self.device)
        self.flat.begin_step()
        if t:
            t.mark("start")
        out = self.model(x)
        loss = self.loss_fn(out, y)
        if self.extra_loss_fn is not None:
            loss = loss + self.extra_loss_fn(self.model)
        if t:
            t.mark("forward")
        loss.backward()
        if self.device.type == "cuda":
            streams.join(self.device)  # side-stream wgrads (ops/streams.py)
        self.flat.finish_grads()
        if t:
            t.mark("backward")
        world = 1
        if self.bucketer is not None:
            mark = self._comm_mark()
            self.bucketer.finish()
            if mark is not None:
                self._comm_marks.append((mark, self._comm_mark()))
                del self._comm_marks[:-256]
            world = self.ctx.world_size
        if t:
            t.mark("comm_wait")
        self.optimizer.step(grad_scale=1.0 / world)
        self.fp8_roller.roll(self.device)
        if t:
            t.mark("optimizer")
            t.end_step()
        self.global_step += 1
        return loss.detach(), out.detach()

    def _comm_mark(self):
        if self.device.type == "cuda":
            if streams.capturing():
                return None
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def comm_wait_ms(self, last=None):
        """Mean exposed communication per eager step: from the end of backward to the last
        bucket's completion on the compute stream (the collectives backward did not hide)."""
        marks = self._comm_marks[-last:] if last else self._comm_marks
        if not marks:
            return None
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
            return sum(a.elapsed_time(b) for a, b in marks) / len(marks)
        return sum((b - a) * 1e3 for a, b in marks) / len(marks)

    # ------------------------------------------------------------------------------------------
    def capture(self, x, y, warmup=3):
        """Record one whole training step — forward, backward, gradient delivery, the fused
        optimizer update — as a HIP graph over static copies of ``x``/``y``; :meth:`replay` then
        runs a step with a single graph launch instead of ~10³ host-side kernel launches (the
        launch-bound small-batch configs, e.g. the reference preset at 32 images per GPU).

        The step must be host-synchronisation-free (it is: losses stay on the device) and its
        Python-side choices static across steps; the learning rate moves to a device scalar
        (optimizer ``set_device_lr``).  Data parallel: with the native RCCL communicator
        (every GPU run with world > 1) the bucketed all-reduces are captured into the graph too
        (csrc/runtime/comm.cpp forks its comm stream into the capture) and overlap backward at
        every replay; each replay is registered with the communicator's watchdog, so a replay
        whose collectives hang is timed out like an eager collective.  fp8 models capture too:
        their delayed-scaling state has fixed slot roles and is rolled on the device once per
        step (ops/fp8.RingRoller), so no kernel argument changes between steps."""
        if self.device.type != "cuda":
            raise RuntimeError("graph capture needs a GPU")
        if (self.bucketer is not None and self.bucketer.comm_hook is None
                and getattr(self.ctx, "native", None) is None):
            raise RuntimeError("data-parallel graph capture needs the native RCCL communicator "
                               "(GPU ranks; not the TDL_SHARE_GPU gloo rehearsal)")
        self.timer = None
        self.static_x = x.detach().clone()
        self.static_y = y.detach().clone()
        self.graph_arena = workspace.ZeroArena()  # private: its addresses are baked in
        # the warm-up runs on the stream the capture then records on: per-stream state sized by
        # the warm-up (deterministic mode's reduction slabs, csrc/kernels/det.hip) exists at
        # capture time, where it must not be allocated
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with workspace.use_arena(self.graph_arena):
            with torch.cuda.stream(side):  # warm-up: caches, arena size, kernel attributes
                for _ in range(warmup):
                    # real training steps on (x, y); the last one's (loss, out) is kept for a
                    # caller that counts the warm-up as its step (model.Model's loop)
                    self.warmup_out = self._step(self.static_x, self.static_y)
            torch.cuda.current_stream(self.device).wait_stream(side)
            torch.cuda.synchronize(self.device)
            self.optimizer.set_device_lr(True)
            step_count, global_step = self.optimizer.step_count, self.global_step
            rolls = self.fp8_roller.rolls  # the captured roll() counts one that never ran
            _params.bump_version()  # derived weight copies (channel padding) refresh in-graph
            g = torch.cuda.CUDAGraph()
            cap_stream = None
            try:
                # thread_local: the native communicator's watchdog thread keeps polling its
                # eager collectives' events during the capture (a global-mode capture would be
                # invalidated by that)
                with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                    # wgrads fork onto the side stream inside the capture and are joined back
                    # after backward (ops/streams.py), as in eager steps
                    cap_stream = torch.cuda.current_stream(self.device)
                    self.graph_out = self._step(self.static_x, self.static_y)
            finally:
                streams.end_capture(cap_stream)
        # capture records without executing: the host-side counters did not really advance
        self.optimizer.step_count, self.global_step = step_count, global_step
        self.fp8_roller.rolls = rolls
        self.graph = g
        return self

    def replay(self, x=None, y=None):
        """One captured training step (``x``/``y`` are copied into the static inputs if given).
        Returns the static (loss, output) tensors, overwritten by the next replay."""
        if x is not None:
            self.static_x.copy_(x, non_blocking=True)
        if y is not None:
            self.static_y.copy_(y, non_blocking=True)
        self.optimizer.prepare_replay()
        self.graph.replay()
        nc = getattr(self.ctx, "native", None)
        if nc is not None and hasattr(nc, "track_current"):
            nc.track_current("graph_replay")  # watchdog covers the captured collectives
        self.optimizer.step_count += 1
        self.global_step += 1
        self.fp8_roller.note_replay()  # the captured step rolled the fp8 amax rings on the device
        _params.bump_version()
        return self.graph_out

    def release_graph(self):
        """Back to eager steps after :meth:`capture`: drop the graph (and its private arena) and
        let the update kernel read the host learning rate again.  Counters carry on from the
        replays."""
        if self.graph is None:
            return
        torch.cuda.synchronize(self.device)
        self.graph = None
        self.graph_out = None
        self.graph_arena = None
        self.optimizer.set_device_lr(False)

    @torch.no_grad()
    def eval_step(self, x):
        self.model.eval()
        return self.model(x)

    def timed_steps(self, batches, n):
        """Run n steps over an iterator of (x, y); returns seconds (device-synchronised)."""
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        for _ in range(n):
            x, y = next(batches)
            self.train_step(x, y)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return time.perf_counter() - t0
