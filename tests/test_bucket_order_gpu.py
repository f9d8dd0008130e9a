"""Data-parallel ordering on ONE GPU (stream/event ordering bugs are
invisible at world 1, where an all-reduce is the identity).

A fake communicator (``GradBucketer(comm_hook=...)``) behaves like the real one: its collective
stream waits on whatever stream the bucketer issued from and snapshots the bucket there — the
bytes a real all-reduce would read.  For every fused model path (ResNet-50; ResNet-152 with fp8
GEMMs; Xception-41 with the depthwise-BN → pointwise fold, the pointwise-BN → depthwise fold and
the deferred BNs; the reference DeepLab preset with its gradient joins and concat-free ASPP),
eager and HIP-graph, side-stream weight gradients on and off (with the side stream stalled so a
missing wait reads stale data):

  * every parameter delivers its final gradient exactly once per step (``strict`` bucketer:
    a duplicate or missing delivery raises);
  * every snapshot equals the bucket's final gradient bit for bit (no collective ordered before
    a producer of its bytes);
  * at least (buckets − 1) collectives were issued from gradient hooks, i.e. during backward
    (the overlap is real, not everything forced at the end).

Reference: the gradients the reference all-reduces in one NCCL pack after backward,
/root/reference/model.py:114-116, Test.ipynb:197,200."""
import pytest
import torch

from tensorflowdistributedlearning_amd import models
from tensorflowdistributedlearning_amd.engine.trainer import Trainer
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, lovasz_hinge, streams
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch, segmentation_batch
from tensorflowdistributedlearning_amd.parallel.bucketer import GradBucketer

pytestmark = pytest.mark.gpu


def _stall(stream, cycles=20_000_000):
    with torch.cuda.stream(stream):
        torch.cuda._sleep(cycles)


def _build(name, gpu):
    torch.manual_seed(3)
    if name == "resnet50":
        m = models.resnet50(num_classes=10)
        x, y = imagenet_batch(8, 64, num_classes=10, device=gpu)
        return m, softmax_cross_entropy, x, y, "sgd", dict(lr=0.0, momentum=0.0)
    if name == "resnet152_fp8":
        m = models.resnet152(num_classes=10)
        models.enable_fp8(m, dgrad=True)
        x, y = imagenet_batch(8, 64, num_classes=10, device=gpu)
        return m, softmax_cross_entropy, x, y, "sgd", dict(lr=0.0, momentum=0.0)
    if name == "xception41":
        m = models.xception_41(num_classes=10)
        x, y = imagenet_batch(4, 96, num_classes=10, device=gpu)
        return m, softmax_cross_entropy, x, y, "sgd", dict(lr=0.0, momentum=0.0)
    m = models.DeepLabResNet(model_name="m", input_shape=(101, 101))
    x, y = segmentation_batch(4, device=gpu)
    return m, lovasz_hinge, x, y, "adam", dict(lr=0.0)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("side", [True, False])
@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("name", ["resnet50", "resnet152_fp8", "xception41", "deeplab_ref"])
def test_bucket_collectives_read_final_gradients(gpu, name, graph, side):
    old = streams.enabled()
    streams.set_enabled(side)
    try:
        m, lossf, x, y, opt, okw = _build(name, gpu)
        tr = Trainer(m, lossf, gpu, opt, okw)
        comm = torch.cuda.Stream(gpu)
        snaps, issued_from = {}, set()

        class Work:
            def __init__(self, ev):
                self.ev = ev

            def wait(self):
                torch.cuda.current_stream(gpu).wait_event(self.ev)

        def hook(b, view):
            cur = torch.cuda.current_stream(gpu)
            issued_from.add(cur.stream_id)
            comm.wait_stream(cur)
            with torch.cuda.stream(comm):
                snaps[b.index] = view.clone()
                ev = torch.cuda.Event()
                ev.record(comm)
            return Work(ev)

        tr.bucketer = GradBucketer(tr.flat, None, bucket_mb=2.0, first_bucket_mb=0.5,
                                   comm_hook=hook, strict=True)
        nb = len(tr.bucketer.buckets)
        assert nb > 4
        if graph:
            tr.capture(x, y)
            if side:
                _stall(streams.side(gpu))
            tr.replay()
        else:
            tr.train_step(x, y)  # (warm: workspace arenas, fp8 scales)
            if side:
                _stall(streams.side(gpu))
            tr.train_step(x, y)
        torch.cuda.synchronize()
        assert tr.bucketer.last_missing == []
        assert len(snaps) == nb
        for b in tr.bucketer.buckets:
            assert torch.equal(snaps[b.index], tr.flat.grad[b.lo:b.hi]), \
                f"bucket {b.index} ({len(b.params)} params) launched before its gradients landed"
        if not graph:  # (during a capture the hooks run once, at record time)
            assert tr.bucketer.early_launches >= nb - 1, (tr.bucketer.early_launches, nb)
        if side and not graph:
            assert streams.side(gpu).stream_id in issued_from
    finally:
        streams.set_enabled(old)


def test_bf16_bucket_collectives_read_final_gradients(gpu):
    """bf16 gradient buckets: each collective reads the bf16 pack of its bucket's
    final gradients, packed on the issuing stream after every producer; finish() unpacks the
    reduced mirror so the optimizer sees fp32(bf16(grad))."""
    old = streams.enabled()
    streams.set_enabled(True)
    try:
        m, lossf, x, y, opt, okw = _build("resnet50", gpu)
        tr = Trainer(m, lossf, gpu, opt, okw)
        comm = torch.cuda.Stream(gpu)
        snaps = {}

        class Work:
            def __init__(self, ev):
                self.ev = ev

            def wait(self):
                torch.cuda.current_stream(gpu).wait_event(self.ev)

        def hook(b, view):
            assert view.dtype == torch.bfloat16
            comm.wait_stream(torch.cuda.current_stream(gpu))
            with torch.cuda.stream(comm):
                snaps[b.index] = view.clone()
                ev = torch.cuda.Event()
                ev.record(comm)
            return Work(ev)

        tr.bucketer = GradBucketer(tr.flat, None, bucket_mb=2.0, first_bucket_mb=0.5,
                                   comm_hook=hook, strict=True, comm_dtype=torch.bfloat16)
        tr.train_step(x, y)
        _stall(streams.side(gpu))
        tr.train_step(x, y)
        torch.cuda.synchronize()
        for b in tr.bucketer.buckets:
            g = tr.flat.grad[b.lo:b.hi]
            assert torch.equal(snaps[b.index], g.bfloat16())
            assert torch.equal(g, g.bfloat16().float())  # unpacked from the bf16 mirror
        assert tr.bucketer.comm_bytes * 2 == sum((b.hi - b.lo) * 4 for b in tr.bucketer.buckets)
    finally:
        streams.set_enabled(old)
