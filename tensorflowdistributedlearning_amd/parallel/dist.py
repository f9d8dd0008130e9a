"""Process-group setup: one process per GPU (RCCL over xGMI via torch.distributed 'nccl'),
gloo on CPU.

Replaces the reference's single-process in-graph towers
(``tf.contrib.distribute.MirroredStrategy(devices=gpus[:n_gpus])``, model.py:114-116) with the
idiomatic ROCm layout: N processes, rank r drives GPU ``LOCAL_RANK``; rendezvous through the
env:// store (MASTER_ADDR=127.0.0.1 by default; the container hostname may not resolve).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    native: object = None  # parallel.rccl.NativeComm when comm="rccl" (GPU collectives)

    @property
    def is_distributed(self):
        return self.world_size > 1

    @property
    def is_main(self):
        return self.rank == 0

    def barrier(self):
        if self.is_distributed:
            if self.native is not None:
                self.native.barrier()
            elif self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def all_reduce_max(self, value: float) -> float:
        if not self.is_distributed:
            return value
        if self.native is not None:
            t = torch.tensor([value], dtype=torch.float64, device=self.device)
            self.native.all_reduce(t, "max")
            return float(t.item())
        t = torch.tensor([value], dtype=torch.float64,
                         device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_reduce_sum_(self, t):
        if self.is_distributed:
            if self.native is not None and t.is_cuda:
                self.native.all_reduce(t)
            else:
                dist.all_reduce(t)
        return t

    def broadcast_(self, t, src=0):
        if self.is_distributed:
            if self.native is not None and t.is_cuda:
                self.native.broadcast(t, src)
            else:
                dist.broadcast(t, src)
        return t

    def all_reduce_async(self, t):
        """Sum-all-reduce ``t`` in place without blocking; returns a handle with ``wait()``
        (native RCCL: stream-ordered; torch: ProcessGroup work)."""
        if self.native is not None:
            return self.native.all_reduce(t, async_op=True)
        return dist.all_reduce(t, async_op=True)

    def check(self):
        """Raise if the native communicator's watchdog latched an error."""
        if self.native is not None and not self.native.ok:
            from .rccl import CommError
            raise CommError(self.native.error)


_CTX = None


def init_distributed(device_type=None, backend=None, timeout_s=600, comm="torch") -> DistContext:
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).
    Single process when WORLD_SIZE is unset or 1.

    ``comm="rccl"`` (GPU, world > 1): GPU collectives go through the native RCCL communicator
    (parallel/rccl.py — dedicated comm stream + watchdog); torch.distributed runs gloo only for
    the rendezvous and host-side barriers."""
    global _CTX
    if _CTX is not None:
        return _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        # TDL_SHARE_GPU=1 (rehearsal only): ranks share the visible devices round-robin, so the
        # multi-rank path can be exercised on a one-GPU box (with TDL_DIST_BACKEND=gloo)
        dev_idx = local_rank
        if os.environ.get("TDL_SHARE_GPU") == "1":
            dev_idx = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    be = "none"
    native = comm == "rccl" and device_type == "cuda" and world > 1
    if world > 1:
        be = backend or os.environ.get("TDL_DIST_BACKEND") or \
            ("nccl" if device_type == "cuda" and not native else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        import datetime
        kw = {}
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(be, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _CTX = DistContext(rank, world, local_rank, device, be)
    if native:
        from .rccl import NativeComm
        _CTX.native = NativeComm(rank, world, device, timeout_s=timeout_s)
    return _CTX


def get_context() -> DistContext:
    return _CTX if _CTX is not None else DistContext()


def shutdown():
    global _CTX
    if _CTX is not None and _CTX.native is not None:
        _CTX.native.synchronize()
        _CTX.native = None
    if _CTX is not None and _CTX.is_distributed and dist.is_initialized():
        dist.destroy_process_group()
    _CTX = None
