"""The per-process training step (the reference's MonitoredTrainingSession loop body,
SURVEY §3.2/§3.5): forward → loss → backward with bucketed all-reduce overlap → fused optimizer.

Nothing in ``train_step`` synchronises with the host: the loss comes back as a device tensor and is
read only when the caller asks (summaries every N steps, like the reference's SummarySaverHook
every 20 steps, model.py:470-473).
"""
from __future__ import annotations

import time

import torch

from ..models.params import FlatParams
from ..parallel.bucketer import GradBucketer
from ..parallel.dist import get_context
from .optimizer import build_optimizer
from ..ops import workspace


class Trainer:
    def __init__(self, model, loss_fn, device, optimizer="sgd", opt_kwargs=None, ctx=None,
                 bucket_mb=32.0, first_bucket_mb=4.0, lowp_dtype=torch.bfloat16,
                 broadcast_init=True, extra_loss_fn=None):
        self.device = torch.device(device)
        self.model = model.to(self.device)
        self.loss_fn = loss_fn
        self.extra_loss_fn = extra_loss_fn
        self.ctx = ctx or get_context()
        self.flat = FlatParams(self.model, self.device, lowp_dtype=lowp_dtype)
        if self.ctx.is_distributed and broadcast_init:
            self.broadcast_state()
        self.optimizer = build_optimizer(optimizer, self.flat, **(opt_kwargs or {}))
        self.bucketer = (GradBucketer(self.flat, self.ctx, bucket_mb, first_bucket_mb)
                         if self.ctx.is_distributed else None)
        self.global_step = 0
        self.train_mode = True  # False: BN uses moving statistics while training (frozen BN)

    # ------------------------------------------------------------------------------------------
    def broadcast_state(self):
        """rank-0 → all broadcast of parameters and buffers (MirroredVariable init)."""
        self.ctx.broadcast_(self.flat.master, 0)
        for b in self.model.buffers():
            self.ctx.broadcast_(b, 0)
        self.flat.sync_lowp()

    def train_step(self, x, y):
        self.model.train(self.train_mode)
        workspace.reset(self.device)
        self.flat.begin_step()
        out = self.model(x)
        loss = self.loss_fn(out, y)
        if self.extra_loss_fn is not None:
            loss = loss + self.extra_loss_fn(self.model)
        loss.backward()
        self.flat.finish_grads()
        world = 1
        if self.bucketer is not None:
            self.bucketer.finish()
            world = self.ctx.world_size
        self.optimizer.step(grad_scale=1.0 / world)
        self.global_step += 1
        return loss.detach(), out.detach()

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
