"""Data-parallel logic on the CPU (SURVEY §7.5 "Dist logic"): bucket layout, launch order with a
fake communicator, and real multi-process gloo training equivalence (world_size 2 and 4), and
the driver's own ``torch.distributed.run`` launch of bench.py."""
import os

import pytest
import torch
import torch.nn as nn

from tensorflowdistributedlearning_amd.models.params import FlatParams
from tensorflowdistributedlearning_amd.parallel.bucketer import GradBucketer
from tensorflowdistributedlearning_amd.parallel import launcher
from tensorflowdistributedlearning_amd.models.layers import Conv2d, Linear
from tensorflowdistributedlearning_amd.ops.pool import global_avg_pool
from tensorflowdistributedlearning_amd.ops.elementwise import relu


class TinyNet(nn.Module):
    """conv-only net (no BN: per-rank BN statistics would make DP != large-batch)."""

    def __init__(self):
        super().__init__()
        self.c1 = Conv2d(8, 16, 3, 2, "sym", bias=True)
        self.c2 = Conv2d(16, 32, 3, 1, "sym", bias=True)
        self.c3 = Conv2d(32, 32, 1, 1, 0)
        self.fc = Linear(32, 5)

    def forward(self, x):
        x = relu(self.c1(x))
        x = relu(self.c2(x))
        x = relu(self.c3(x))
        return self.fc(global_avg_pool(x))


def test_flat_params_layout_and_views():
    m = TinyNet()
    f = FlatParams(m, "cpu", lowp_dtype=None)
    assert f.total % 64 == 0
    for p in f.params:
        o = p._flat_offset
        assert o % 64 == 0
        assert p.data.data_ptr() == f.master[o:].data_ptr()
        assert p.grad.data_ptr() == f.grad[o:].data_ptr()
    # biases flagged no-decay, weights decay
    assert f.decay_flags[m.c1.bias._flat_offset // 64] == 0
    assert f.decay_flags[m.c1.weight._flat_offset // 64] == 1


def test_bucketer_fills_in_backward_order_and_launches_in_index_order():
    torch.manual_seed(0)
    m = TinyNet()
    f = FlatParams(m, "cpu", lowp_dtype=None)
    log = []
    b = GradBucketer(f, ctx=None, bucket_mb=0.004, first_bucket_mb=0.001,
                     comm_hook=lambda bk, view: log.append((bk.index, view.numel())))
    assert len(b.buckets) >= 3
    # contiguous, covering, in reverse flat order
    cov = sorted((bk.lo, bk.hi) for bk in b.buckets)
    assert cov[0][0] == 0
    for (lo0, hi0), (lo1, hi1) in zip(cov, cov[1:]):
        assert hi0 == lo1
    assert b.buckets[0].hi == max(h for _, h in cov)  # first bucket = last params (fc)
    f.begin_step()
    out = m(torch.randn(2, 8, 8, 8))
    out.sum().backward()
    f.finish_grads()
    b.finish()
    assert [i for i, _ in log] == list(range(len(b.buckets)))
    # readiness order: the fc bucket must be complete before the first conv's bucket
    assert sum(n for _, n in log) == sum(bk.hi - bk.lo for bk in b.buckets)


def test_bucketer_reset_between_steps():
    m = TinyNet()
    f = FlatParams(m, "cpu", lowp_dtype=None)
    log = []
    b = GradBucketer(f, None, 0.004, 0.001, comm_hook=lambda bk, v: log.append(bk.index))
    for _ in range(2):
        f.begin_step()
        m(torch.randn(2, 8, 8, 8)).sum().backward()
        f.finish_grads()
        b.finish()
    assert log == list(range(len(b.buckets))) * 2


def test_bucketer_counts_final_deliveries_not_hook_calls():
    """A parameter's extra contribution raises instead of silently completing another
    parameter's bucket (the collective would read a gradient still being written)."""
    from tensorflowdistributedlearning_amd.ops.common import deliver_grad
    m = TinyNet()
    f = FlatParams(m, "cpu", lowp_dtype=None)
    log = []
    b = GradBucketer(f, None, 0.004, 0.001, comm_hook=lambda bk, v: log.append(bk.index),
                     strict=True)
    f.begin_step()
    m(torch.randn(2, 8, 8, 8)).sum().backward()
    assert b.early_launches == 0 and b._early >= len(b.buckets) - 1  # launched during backward
    with pytest.raises(RuntimeError, match="delivered 2 times"):
        deliver_grad(m.fc.conv.weight, torch.zeros_like(m.fc.conv.weight))
    f.finish_grads()
    b.finish()
    assert b.early_launches >= len(b.buckets) - 1 and b.last_missing == []
    # declared double contribution: the bucket waits for the second one
    w = m.c3.weight
    w._tdl_contribs = 2
    try:
        log.clear()
        f.begin_step()
        bk = b.bucket_of[id(w)]
        deliver_grad(w, torch.ones_like(w))
        assert bk.index not in log
        deliver_grad(w, torch.ones_like(w))
        assert bk.pending == len(bk.params) - 1
    finally:
        del w._tdl_contribs
    # a parameter that delivered nothing is reported (strict: raised after the reset)
    with pytest.raises(RuntimeError, match="delivered no final gradient"):
        f.finish_grads()
        b.finish()
    assert len(b.last_missing) == len(f.params) - 1 and b.next_launch == 0


def _dp_worker(rank, tmpdir, world=2, grad_dtype="fp32"):
    import torch
    from tensorflowdistributedlearning_amd.parallel.dist import init_distributed, shutdown
    from tensorflowdistributedlearning_amd.engine.trainer import Trainer
    from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy
    ctx = init_distributed(device_type="cpu")
    torch.manual_seed(123)  # same init on all ranks is NOT assumed: rank 0 broadcasts
    if rank == 1:
        torch.manual_seed(999)
    m = TinyNet()
    tr = Trainer(m, softmax_cross_entropy, "cpu", "sgd", dict(lr=0.1, momentum=0.9,
                                                              weight_decay=1e-4),
                 ctx=ctx, bucket_mb=0.004, first_bucket_mb=0.001, lowp_dtype=None,
                 grad_comm_dtype=torch.bfloat16 if grad_dtype == "bf16" else torch.float32)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 8, 8, 8, generator=g)
    y = torch.randint(0, 5, (8,), generator=g)
    per = 8 // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    for _ in range(3):
        tr.train_step(xs, ys)
    torch.save(tr.flat.master.clone(), os.path.join(tmpdir, f"rank{rank}.pt"))
    shutdown()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world,grad_dtype", [(2, "fp32"), (4, "fp32"), (2, "bf16")])
def test_gloo_dp_equals_large_batch(tmp_path, world, grad_dtype):
    """W ranks × batch 8/W with mean-gradient all-reduce == 1 process × batch 8 (rank 0's
    parameters broadcast at start: rank 1 starts from different weights).  bf16 gradient buckets
    (parallel/bucketer.py): the replicas stay bit-identical and track fp32 to bf16 rounding."""
    launcher.spawn(_dp_worker, world, args=(str(tmp_path), world, grad_dtype))
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    for r in range(1, world):  # replicas stay identical
        assert torch.equal(r0, torch.load(tmp_path / f"rank{r}.pt", weights_only=True))
    from tensorflowdistributedlearning_amd.engine.trainer import Trainer
    from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy
    torch.manual_seed(123)
    m = TinyNet()
    tr = Trainer(m, softmax_cross_entropy, "cpu", "sgd", dict(lr=0.1, momentum=0.9,
                                                              weight_decay=1e-4), lowp_dtype=None)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 8, 8, 8, generator=g)
    y = torch.randint(0, 5, (8,), generator=g)
    for _ in range(3):
        tr.train_step(x, y)
    if grad_dtype == "bf16":  # gradients rounded to 8 mantissa bits before the reduction
        rel = ((r0 - tr.flat.master).norm() / tr.flat.master.norm()).item()
        assert rel < 2e-3, rel
        assert not torch.equal(r0, tr.flat.master)  # the bf16 path really ran
    else:
        assert torch.allclose(r0, tr.flat.master, atol=1e-5, rtol=1e-4)


def test_phase_timer_cpu():
    import torch
    from tensorflowdistributedlearning_amd import models
    from tensorflowdistributedlearning_amd.engine.trainer import Trainer
    from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy
    from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch
    torch.manual_seed(0)
    m = models.build("resnet18", num_classes=4, width=8)
    tr = Trainer(m, softmax_cross_entropy, "cpu", "sgd", dict(lr=0.01), lowp_dtype=None,
                 profile_phases=True)
    x, y = imagenet_batch(2, 32, num_classes=4, dtype=torch.float32)
    for _ in range(2):
        tr.train_step(x, y)
    s = tr.timer.summary()
    assert set(s) == {"forward", "backward", "comm_wait", "optimizer", "step"}
    assert s["forward"] > 0 and s["backward"] > 0 and abs(s["step"] - sum(
        s[k] for k in ("forward", "backward", "comm_wait", "optimizer"))) < 1e-6


def test_native_comm_selector_cpu():
    """comm="rccl" only engages the native communicator for GPU runs with world > 1."""
    from tensorflowdistributedlearning_amd.parallel import dist as D
    from tensorflowdistributedlearning_amd.parallel import rccl  # importable without a GPU
    D.shutdown()
    ctx = D.init_distributed(device_type="cpu", comm="rccl")
    try:
        assert ctx.native is None and not ctx.is_distributed
        ctx.check()
        assert issubclass(rccl.CommError, RuntimeError)
    finally:
        D.shutdown()


def test_bucketer_last_bucket_is_small():
    """The bucket launched last (earliest layers, exposed after backward) is split down to about
    the first-bucket size; buckets still tile the flat buffer contiguously."""
    from tensorflowdistributedlearning_amd import models
    m = models.resnet18(num_classes=10)
    f = FlatParams(m, "cpu", lowp_dtype=None)
    b = GradBucketer(f, None, bucket_mb=8.0, first_bucket_mb=0.5,
                     comm_hook=lambda bk, v: None)
    cap = int(0.5 * 2 ** 20 / 4)
    assert b.buckets[-1].hi - b.buckets[-1].lo <= cap
    assert b.buckets[-1].lo == 0
    cov = sorted((bk.lo, bk.hi) for bk in b.buckets)
    for (lo0, hi0), (lo1, hi1) in zip(cov, cov[1:]):
        assert hi0 == lo1
    assert cov[-1][1] == f.total or cov[-1][1] == sum(((p.numel() + 63) // 64) * 64
                                                       for p in f.params)
    seen = [id(p) for bk in b.buckets for p in bk.params]
    assert sorted(seen) == sorted(id(p) for p in f.params)
    for bk in b.buckets:  # every param lies inside its bucket's range
        for p in bk.params:
            lo, hi = f.slice_of(p)
            assert bk.lo <= lo and hi <= bk.hi


def _bench_env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    return env


@pytest.mark.timeout(300)
def test_bench_self_spawns_ranks_cpu(tmp_path):
    """`python bench.py --gpus 2` with no launcher environment starts two worker processes of
    itself (gloo on the CPU here, native RCCL on GPUs), times them barrier-bracketed and prints
    exactly one JSON line from rank 0 with n_gpus = 2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--model", "resnet18",
           "--image-size", "32", "--batch", "2", "--steps", "1", "--warmup", "1"]
    r = subprocess.run(cmd, env=_bench_env(), cwd=str(tmp_path), capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["comm"] == "gloo" and out["config"]["global_batch"] == 4
    assert out["value"] > 0 and out["steps"] == 1 and out["warmup"] == 1
    co = out["config"]["comm_overlap"]  # exposed vs standalone collective time (N > 1)
    assert co["standalone_ms"] > 0 and co["exposed_ms"] >= 0 and co["buckets"] >= 1
    assert co["overlap"] is None or 0.0 <= co["overlap"] <= 1.0


@pytest.mark.timeout(300)
def test_bench_under_torchrun_driver_form_cpu(tmp_path):
    """The driver's exact multi-GPU launch (`python -m torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...`) with
    N = 4 gloo ranks: bench.py takes the launcher's ranks (no self-spawn), the barrier-bracketed
    timing covers every rank and only rank 0 prints the JSON line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(launcher.free_port()),
           os.path.join(root, "bench.py"), "--gpus", "4", "--model", "resnet18",
           "--image-size", "32", "--batch", "2", "--steps", "2", "--warmup", "1"]
    env = _bench_env()
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["config"]["parallelism"] == "dp4"
    assert out["config"]["global_batch"] == 8 and out["steps"] == 2 and out["warmup"] == 1
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert abs(out["value"] - 8 * 1e3 / out["ms_per_step"]) / out["value"] < 0.01


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model", ["resnet18", "deeplab_ref"])
def test_bench_infer_mode_cpu(tmp_path, model):
    """`bench.py --mode infer` (eval forward, folded BN): one JSON line with no training
    baseline attached."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--mode", "infer", "--model", model,
           "--image-size", "32", "--batch", "2", "--steps", "1", "--warmup", "1"]
    r = subprocess.run(cmd, env=_bench_env(), cwd=str(tmp_path), capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["metric"].startswith("inference images/sec") and "folded" in out["metric"]
    assert out["config"]["mode"] == "infer" and out["vs_baseline"] is None and out["value"] > 0


@pytest.mark.timeout(300)
def test_bench_self_spawn_propagates_worker_failure(tmp_path):
    """A failing worker makes the launcher exit non-zero (and stops its peers)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--model",
           "no_such_model", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, env=_bench_env(), cwd=str(tmp_path), capture_output=True, text=True,
                       timeout=280)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_init_distributed_rejects_second_gpu_backend():
    """There is one GPU collective backend (native RCCL); torch.distributed is gloo-only."""
    from tensorflowdistributedlearning_amd.parallel import dist as D
    D.shutdown()
    with pytest.raises(ValueError):
        D.init_distributed(device_type="cpu", comm="torch")
    D.shutdown()


def test_bucket_launch_never_joins_the_compute_stream(monkeypatch):
    """A bucket's collective is ordered after BOTH producers by issuing it from the side stream
    once that stream waited for the compute stream — the compute stream itself never waits on
    the side stream at a bucket boundary (that stalled the dgrad / BN chain behind every queued
    weight gradient).  Fake streams record the waits; a compute-stream join raises."""
    from tensorflowdistributedlearning_amd.ops import streams
    from tensorflowdistributedlearning_amd.parallel import bucketer as bmod
    import inspect

    class FakeStream:
        def __init__(self, name):
            self.name, self.waited = name, []

        def wait_stream(self, other):
            self.waited.append(other.name)

        def __eq__(self, o):
            return isinstance(o, FakeStream) and o.name == self.name

    side, comp = FakeStream("side"), FakeStream("compute")

    def no_join(*a, **k):
        raise AssertionError("bucket launch joined the compute stream to the side stream")

    monkeypatch.setattr(streams, "join", no_join)
    monkeypatch.setattr(streams, "side_if_active", lambda dev: side)
    monkeypatch.setattr(streams, "current", lambda dev: comp)
    s = GradBucketer.issue_stream(torch.device("cpu"))
    assert s is side and side.waited == ["compute"] and comp.waited == []
    # hook fired on the side stream itself (a wgrad's gradient-ready hook): the side stream still
    # waits for the compute (origin) stream — the bucket can hold γ/β gradients written there
    # before the side-stream section (the folded depthwise BN's γ/β)
    monkeypatch.setattr(streams, "current", lambda dev: side)
    monkeypatch.setattr(streams, "origin", lambda dev: comp)
    side.waited.clear()
    assert GradBucketer.issue_stream(torch.device("cpu")) is side and side.waited == ["compute"]
    assert comp.waited == []
    # no side stream: issue from the current stream
    monkeypatch.setattr(streams, "side_if_active", lambda dev: None)
    assert GradBucketer.issue_stream(torch.device("cpu")) is None
    # the launch path has no join left in it
    assert "streams.join" not in inspect.getsource(bmod.GradBucketer._launch)
