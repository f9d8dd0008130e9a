"""Native RCCL communicator (csrc/runtime/comm.cpp) — the direct C++ RCCL backend of SURVEY §5.8
(N14 ``NcclAllReduce`` / N15 init broadcast of the reference's MirroredStrategy,
model.py:114-116, Test.ipynb:197-200) with the failure detection of §5.3.

* rank 0 creates the 128-byte ``ncclUniqueId``; it reaches the other ranks through the
  torch.distributed store (gloo process group — torch is used only for rendezvous here);
* collectives are enqueued on a dedicated high-priority HIP stream after an event recorded on the
  compute stream, and return a ticket; ``wait(ticket)`` makes the compute stream wait on the
  collective's completion event (no host synchronisation);
* a C++ watchdog thread polls outstanding collectives and ``ncclCommGetAsyncError``; a collective
  older than ``timeout_s`` or an async RCCL error aborts the communicator and every later call
  raises :class:`CommError` (fail fast instead of hanging the job).

This is the only GPU collective path: ``init_distributed`` creates it for every GPU run with
world > 1 (torch.distributed runs gloo beside it for the rendezvous store and host barriers only).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import _native


class CommError(RuntimeError):
    pass


class Work:
    """Handle of an enqueued collective: ``wait()`` orders the current stream after it."""
    __slots__ = ("comm", "ticket")

    def __init__(self, comm, ticket):
        self.comm, self.ticket = comm, ticket

    def wait(self):
        self.comm.wait(self.ticket)


class NativeComm:
    def __init__(self, rank, world, device, timeout_s=600.0, uid=None):
        ext = _native.load()
        if uid is None:
            uid = _exchange_uid(ext, rank, world)
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        self._c = ext.RcclComm(uid, rank, world, self.device.index or 0, float(timeout_s))

    # --------------------------------------------------------------------------------------
    def _check(self):
        if not self._c.ok:
            raise CommError(self._c.error)

    def all_reduce(self, t, op="sum", async_op=False):
        self._check()
        w = Work(self, self._c.all_reduce(t, op))
        if not async_op:
            w.wait()
            return None
        return w

    def broadcast(self, t, root=0, async_op=False):
        self._check()
        w = Work(self, self._c.broadcast(t, root))
        if not async_op:
            w.wait()
            return None
        return w

    def reduce_scatter(self, inp, out, op="sum", async_op=False):
        self._check()
        w = Work(self, self._c.reduce_scatter(inp, out, op))
        if not async_op:
            w.wait()
            return None
        return w

    def all_gather(self, inp, out, async_op=False):
        self._check()
        w = Work(self, self._c.all_gather(inp, out))
        if not async_op:
            w.wait()
            return None
        return w

    def wait(self, ticket):
        self._check()
        self._c.wait(ticket)

    def synchronize(self):
        try:
            self._c.synchronize()
        except RuntimeError as e:
            raise CommError(str(e)) from None

    def barrier(self):
        t = torch.zeros(1, device=self.device)
        self.all_reduce(t)
        torch.cuda.current_stream(self.device).synchronize()
        self._check()

    @property
    def ok(self):
        return self._c.ok

    @property
    def error(self):
        return self._c.error

    @property
    def outstanding(self):
        return self._c.outstanding

    @property
    def rccl_count(self):
        """Rank count as RCCL reports it (``ncclCommCount``)."""
        return self._c.rccl_count

    @property
    def rccl_rank(self):
        return self._c.rccl_rank

    @property
    def rccl_device(self):
        return self._c.rccl_device

    def track_current(self, name="graph_replay"):
        """Watch everything queued so far on the current stream like a collective (the watchdog
        times it out): a HIP-graph replay's captured collectives are covered this way."""
        self._check()
        return Work(self, self._c.track_current(name))

    def abort(self, why="aborted by user"):
        self._c.abort(why)

    def debug_delay(self, ms, track=False):
        """Fault injection: stall the comm stream for ``ms`` milliseconds (``track``: watch the
        stall like a collective, so the watchdog times it out with no RCCL op in flight)."""
        return Work(self, self._c.debug_delay(float(ms), bool(track)))


def _exchange_uid(ext, rank, world):
    if world == 1:
        return ext.rccl_unique_id()
    if not dist.is_initialized():
        raise RuntimeError("NativeComm with world > 1 needs torch.distributed (gloo) for rendezvous")
    obj = [ext.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]
