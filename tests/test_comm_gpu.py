"""Native RCCL communicator (csrc/runtime/comm.cpp, parallel/rccl.py) on one GPU: collectives,
stream ordering, the bucketed DP path through it, and the watchdog's timeout → abort → raise
(SURVEY §5.3 failure detection).  Multi-rank correctness of the same calls is RCCL's; the
multi-process DP logic is rehearsed with gloo in tests/test_dist_cpu.py."""
import time

import pytest
import torch

from tensorflowdistributedlearning_amd.parallel.rccl import NativeComm, CommError

pytestmark = pytest.mark.gpu


@pytest.fixture
def comm(gpu):
    c = NativeComm(0, 1, gpu, timeout_s=30)
    yield c
    c.synchronize()


def test_rccl_shares_torch_library():
    from tensorflowdistributedlearning_amd import _native
    v = _native.load().rccl_version()
    assert v >= 22000, v


def test_collectives_world1(comm, gpu):
    x = torch.randn(1000, device=gpu)
    ref = x.clone()
    comm.all_reduce(x)
    assert torch.equal(x, ref)
    comm.all_reduce(x, "max")
    comm.all_reduce(x, "avg")
    assert torch.equal(x, ref)
    b = torch.arange(10, device=gpu, dtype=torch.float32).bfloat16()
    comm.broadcast(b, 0)
    assert torch.equal(b.float().cpu(), torch.arange(10.0))
    out = torch.empty(1000, device=gpu)
    comm.reduce_scatter(x, out)
    assert torch.equal(out, ref)
    g = torch.empty(1000, device=gpu)
    comm.all_gather(x, g)
    assert torch.equal(g, ref)


def test_async_ticket_orders_compute_stream(comm, gpu):
    """A delayed collective: the consumer kernel after wait() must see its result."""
    x = torch.ones(1 << 20, device=gpu)
    comm.debug_delay(200)              # comm stream busy for 0.2 s
    w = comm.all_reduce(x, async_op=True)
    w.wait()                           # compute stream waits on the completion event
    y = x * 2                          # enqueued behind the wait
    assert float(y.sum()) == 2.0 * (1 << 20)
    assert comm.ok


def test_bucketer_through_native_comm(gpu):
    from types import SimpleNamespace
    from tensorflowdistributedlearning_amd.models.params import FlatParams
    from tensorflowdistributedlearning_amd.parallel.bucketer import GradBucketer
    nc = NativeComm(0, 1, gpu)
    ctx = SimpleNamespace(is_distributed=True, native=nc,
                          all_reduce_async=lambda t: nc.all_reduce(t, async_op=True),
                          check=lambda: None)
    m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.Linear(64, 8))
    fp = FlatParams(m, gpu)
    bk = GradBucketer(fp, ctx=ctx, bucket_mb=0.01, first_bucket_mb=0.001)
    fp.grad.normal_()
    ref = fp.grad.clone()
    for p in reversed(fp.params):
        p._grad_hook(p)
    assert all(b.launched for b in bk.buckets) and len(bk.buckets) >= 2
    bk.finish()
    torch.cuda.synchronize()
    assert torch.equal(fp.grad, ref)  # world 1: sum = identity, in order, no corruption
    nc.synchronize()


def test_watchdog_times_out_and_aborts(gpu):
    c = NativeComm(0, 1, gpu, timeout_s=0.5)
    x = torch.ones(16, device=gpu)
    c.debug_delay(2500, track=True)    # a "collective" that cannot complete for 2.5 s
    t0 = time.time()
    while c.ok and time.time() - t0 < 5:
        time.sleep(0.05)
    assert not c.ok
    assert "not complete" in c.error
    with pytest.raises(CommError):
        c.all_reduce(x)
    torch.cuda.synchronize()           # the bounded spin drains; the GPU stays usable
    assert float((x + 1).sum()) == 32.0
