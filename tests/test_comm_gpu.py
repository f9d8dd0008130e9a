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


def test_collective_captured_in_hip_graph(comm, gpu):
    """A native-RCCL all-reduce issued while the compute stream captures a HIP graph is captured
    with it (comm stream forked in by an event wait, joined back by the ticket wait) and runs at
    every replay; it is not left outstanding for the watchdog."""
    x = torch.ones(4096, device=gpu)
    s = torch.cuda.Stream(gpu)
    s.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(s):  # warm-up outside capture
        y = x * 2
        comm.all_reduce(y)
        z = y + 1
    torch.cuda.current_stream(gpu).wait_stream(s)
    torch.cuda.synchronize()
    before = comm.outstanding  # the eager warm-up until the watchdog retires it
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):  # watchdog threads keep polling
        y = x * 2
        w = comm.all_reduce(y, async_op=True)
        w.wait()
        z = y + 1
    assert comm.outstanding <= before  # the captured collective is not watched as pending
    for k in range(3):
        x.fill_(float(k))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(z, torch.full_like(z, 2.0 * k + 1)), k
    assert comm.ok


@pytest.mark.parametrize("side", [False, True])
def test_dp_graph_capture_matches_eager(gpu, side):
    """Data-parallel step captured as a HIP graph with its bucketed all-reduces (native RCCL,
    world 1 standing in for the collectives; the bucketer / hook / join / fork logic is the DP
    one): same trajectory as the eager DP steps, with and without the side-stream wgrads."""
    from types import SimpleNamespace
    from tensorflowdistributedlearning_amd import models
    from tensorflowdistributedlearning_amd.engine.trainer import Trainer
    from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, streams
    from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch
    nc = NativeComm(0, 1, gpu)

    def make_ctx():
        return SimpleNamespace(is_distributed=True, world_size=2, rank=0, is_main=True, native=nc,
                               all_reduce_async=lambda t: nc.all_reduce(t, async_op=True),
                               broadcast_=lambda t, src=0: t, check=lambda: None,
                               barrier=lambda: None)
    old = streams.enabled()
    streams.set_enabled(side)
    try:
        torch.manual_seed(11)
        nets = [models.resnet18(num_classes=10) for _ in range(2)]
        nets[1].load_state_dict(nets[0].state_dict())
        ta, tb = [Trainer(n, softmax_cross_entropy, gpu, "sgd", dict(lr=0.05, momentum=0.9),
                          ctx=make_ctx(), bucket_mb=1.0, first_bucket_mb=0.25) for n in nets]
        assert ta.bucketer is not None and len(ta.bucketer.buckets) > 2
        ta.train_mode = tb.train_mode = False  # frozen BN: no float atomics in the comparison
        x, y = imagenet_batch(8, 32, num_classes=10, device=gpu)
        tb.capture(x, y, warmup=2)
        for _ in range(2):
            ta.train_step(x, y)
        torch.cuda.synchronize()
        m0 = ta.flat.master.clone()
        torch.testing.assert_close(m0, tb.flat.master, rtol=1e-5, atol=1e-7)
        for _ in range(3):
            la, _ = ta.train_step(x, y)
            lb, _ = tb.replay()
        torch.cuda.synchronize()
        ua, ub = ta.flat.master - m0, tb.flat.master - m0
        assert ua.norm() > 0 and torch.isfinite(ub).all()
        # fp32 atomics in the BN backward sums: summation order varies run to run
        cos = torch.nn.functional.cosine_similarity(ua, ub, dim=0).item()
        assert cos > 0.9999, cos
        assert ((ua - ub).norm() / ua.norm()).item() < 0.01
        torch.testing.assert_close(float(lb), float(la), rtol=1e-3, atol=1e-4)
        assert nc.ok
    finally:
        streams.set_enabled(old)
        nc.synchronize()
