"""Process-group setup: one process per GPU, GPU collectives on the native RCCL communicator
over xGMI (parallel/rccl.py), gloo for the rendezvous store and for CPU runs.

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
    native: object = None  # parallel.rccl.NativeComm: every GPU collective when world > 1

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
            else:
                dist.barrier()

    def all_reduce_max(self, value: float) -> float:
        if not self.is_distributed:
            return value
        if self.native is not None:
            t = torch.tensor([value], dtype=torch.float64, device=self.device)
            self.native.all_reduce(t, "max")
            return float(t.item())
        t = torch.tensor([value], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_reduce_sum_(self, t):
        if self.is_distributed:
            if self.native is not None and t.is_cuda:
                self.native.all_reduce(t)
            elif t.is_cuda:  # TDL_SHARE_GPU rehearsal: gloo through host memory
                h = t.cpu()
                dist.all_reduce(h)
                t.copy_(h)
            else:
                dist.all_reduce(t)
        return t

    @property
    def rccl_ranks(self):
        """Rank count RCCL itself reports (None without a native communicator)."""
        return self.native.rccl_count if self.native is not None else None

    def broadcast_(self, t, src=0):
        if self.is_distributed:
            if self.native is not None and t.is_cuda:
                self.native.broadcast(t, src)
            else:
                dist.broadcast(t, src)
        return t

    def all_reduce_async(self, t):
        """Sum-all-reduce ``t`` in place without blocking; returns a handle with ``wait()``
        (native RCCL: stream-ordered; CPU / shared-GPU rehearsal: gloo work)."""
        if self.native is not None:
            return self.native.all_reduce(t, async_op=True)
        return dist.all_reduce(t, async_op=True)

    def check(self):
        """Raise if the native communicator's watchdog latched an error."""
        if self.native is not None and not self.native.ok:
            from .rccl import CommError
            raise CommError(self.native.error)


_CTX = None


def init_distributed(device_type=None, backend=None, timeout_s=600, comm=None) -> DistContext:
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).
    Single process when WORLD_SIZE is unset or 1.

    GPU runs with world > 1 do every collective on the native RCCL communicator
    (parallel/rccl.py: dedicated comm stream, watchdog, graph-capturable) — there is no second GPU
    collective backend.  torch.distributed is initialised with gloo beside it, only for the
    rendezvous store (the ncclUniqueId exchange) and host-side barriers.  CPU runs use gloo.

    ``TDL_SHARE_GPU=1`` is a rehearsal mode for one-GPU boxes: the ranks share the visible
    device(s) round-robin, which RCCL refuses ("Duplicate GPU"), so its GPU tensors are reduced
    through gloo instead.  ``comm`` is accepted for API compatibility ("rccl" or None)."""
    global _CTX
    if _CTX is not None:
        return _CTX
    if comm not in (None, "rccl"):
        raise ValueError(f"comm={comm!r}: the GPU collective backend is the native RCCL "
                         "communicator (comm='rccl')")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    share = os.environ.get("TDL_SHARE_GPU") == "1"
    if device_type == "cuda":
        ndev = torch.cuda.device_count()
        dev_idx = local_rank
        if share:
            dev_idx = local_rank % max(1, ndev)
        elif dev_idx >= ndev:
            raise RuntimeError(f"local rank {local_rank} needs GPU {dev_idx} but only {ndev} "
                               "visible (one process per GPU)")
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    be = "none"
    native = device_type == "cuda" and world > 1 and not share
    if world > 1:
        be = backend or "gloo"
        if be != "gloo":
            raise ValueError(f"backend={be!r}: torch.distributed runs gloo only (rendezvous, CPU "
                             "collectives); GPU collectives are native RCCL")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        import datetime
        dist.init_process_group(be, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    _CTX = DistContext(rank, world, local_rank, device, be)
    if native:
        from .rccl import NativeComm
        _CTX.native = NativeComm(rank, world, device, timeout_s=timeout_s)
        n = _CTX.native.rccl_count
        if n != world or _CTX.native.rccl_rank != rank:
            raise RuntimeError(f"RCCL reports {n} ranks / rank {_CTX.native.rccl_rank}, "
                               f"expected {world} / {rank}")
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
