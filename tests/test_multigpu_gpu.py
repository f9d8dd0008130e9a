"""Multi-GPU data parallelism on real devices (SURVEY §7.5 "Dist real"): one process per GPU, every
collective on the native RCCL communicator over xGMI.  These run only where at least two GPUs are
visible (skipped on a one-GPU box; RCCL refuses two ranks on one device, so the one-GPU rehearsal
of the multi-rank bench path is tests/test_train_gpu.py::test_bench_two_ranks_share_one_gpu).

* collectives: all-reduce (sum / max / avg, fp32 and bf16), broadcast, reduce-scatter,
  all-gather, with RCCL's own rank count checked (ncclCommCount);
* DP training equivalence: N ranks × batch b == 1 rank × batch N·b (frozen BN — per-rank batch
  statistics are the reference's MirroredStrategy semantics too, /root/reference/model.py:114-121,
  so only frozen BN makes the two runs the same function);
* ``bench.py --gpus N`` without a launcher: N self-spawned ranks, RCCL-confirmed.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from tensorflowdistributedlearning_amd.parallel import launcher

pytestmark = pytest.mark.gpu

NDEV = torch.cuda.device_count() if torch.cuda.is_available() else 0
need2 = pytest.mark.skipif(NDEV < 2, reason="needs >= 2 visible GPUs")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _collectives_worker(rank, outdir):
    import torch
    from tensorflowdistributedlearning_amd.parallel.dist import init_distributed, shutdown
    ctx = init_distributed()
    n, dev = ctx.world_size, ctx.device
    res = {"rank": rank, "rccl_count": ctx.native.rccl_count, "rccl_rank": ctx.native.rccl_rank,
           "device": ctx.native.rccl_device}
    # sum of rank-dependent values
    x = torch.full((1 << 16,), float(rank + 1), device=dev)
    ctx.native.all_reduce(x)
    res["sum_ok"] = bool(torch.all(x == n * (n + 1) / 2).item())
    y = torch.full((4097,), float(rank), device=dev)
    ctx.native.all_reduce(y, "max")
    res["max_ok"] = bool(torch.all(y == n - 1).item())
    z = torch.full((1000,), float(2 * rank), device=dev)
    ctx.native.all_reduce(z, "avg")
    res["avg_ok"] = bool(torch.allclose(z, torch.full_like(z, float(n - 1))))
    b = torch.full((777,), float(rank + 1), device=dev, dtype=torch.bfloat16)
    ctx.native.all_reduce(b)
    res["bf16_ok"] = bool(torch.all(b.float() == n * (n + 1) / 2).item())
    c = torch.arange(513, device=dev, dtype=torch.float32) * (rank + 3)
    ctx.native.broadcast(c, 0)
    res["bcast_ok"] = bool(torch.equal(c, torch.arange(513, device=dev, dtype=torch.float32) * 3))
    # reduce-scatter: rank r's output = Σ_ranks of chunk r
    inp = torch.arange(n * 64, device=dev, dtype=torch.float32) + rank
    out = torch.empty(64, device=dev)
    ctx.native.reduce_scatter(inp, out)
    ref = (torch.arange(rank * 64, (rank + 1) * 64, device=dev, dtype=torch.float32) * n +
           n * (n - 1) / 2)
    res["rs_ok"] = bool(torch.equal(out, ref))
    g = torch.empty(n * 32, device=dev)
    ctx.native.all_gather(torch.full((32,), float(rank), device=dev), g)
    res["ag_ok"] = bool(torch.equal(g, torch.arange(n, device=dev).float().repeat_interleave(32)))
    # async ticket ordering across many collectives on the comm stream
    ws = [ctx.native.all_reduce(torch.ones(1 << 18, device=dev) * (i + 1), async_op=True)
          for i in range(8)]
    for w in ws:
        w.wait()
    res["async_ok"] = ctx.native.ok
    ctx.barrier()
    res["max_time"] = ctx.all_reduce_max(float(rank))
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    shutdown()


@need2
@pytest.mark.timeout(180)
@pytest.mark.parametrize("n", sorted({2, min(NDEV, 8)}) if NDEV >= 2 else [2])
def test_rccl_collectives_n_ranks(tmp_path, n):
    launcher.spawn(_collectives_worker, n, args=(str(tmp_path),))
    for r in range(n):
        res = json.load(open(tmp_path / f"r{r}.json"))
        assert res["rccl_count"] == n and res["rccl_rank"] == r and res["device"] == r, res
        for k in ("sum_ok", "max_ok", "avg_ok", "bf16_ok", "bcast_ok", "rs_ok", "ag_ok",
                  "async_ok"):
            assert res[k], (r, k)
        assert res["max_time"] == n - 1


def _frozen_resnet_trainer(dev, ctx=None):
    from tensorflowdistributedlearning_amd import models
    from tensorflowdistributedlearning_amd.engine.trainer import Trainer
    from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy
    torch.manual_seed(21)
    m = models.resnet18(num_classes=10)
    tr = Trainer(m, softmax_cross_entropy, dev, "sgd", dict(lr=0.05, momentum=0.9), ctx=ctx,
                 bucket_mb=2.0, first_bucket_mb=0.5)
    tr.train_mode = False  # frozen BN: the DP run and the large batch compute the same function
    return tr


def _global_batch(n, per):
    from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch
    return imagenet_batch(n * per, 32, num_classes=10, seed=5)


def _dp_worker(rank, outdir, per, steps):
    import torch
    from tensorflowdistributedlearning_amd.parallel.dist import init_distributed, shutdown
    ctx = init_distributed()
    tr = _frozen_resnet_trainer(ctx.device, ctx)
    assert tr.bucketer is not None and len(tr.bucketer.buckets) > 2
    x, y = _global_batch(ctx.world_size, per)
    xs = x[rank * per:(rank + 1) * per].to(ctx.device)
    ys = y[rank * per:(rank + 1) * per].to(ctx.device)
    for _ in range(steps):
        tr.train_step(xs, ys)
    torch.cuda.synchronize()
    torch.save(tr.flat.master.cpu(), os.path.join(outdir, f"m{rank}.pt"))
    shutdown()


@need2
@pytest.mark.timeout(240)
def test_dp_ranks_equal_large_batch(tmp_path, gpu):
    """2 GPUs × 8 images with bucketed RCCL all-reduce overlapped with backward == 1 GPU × 16."""
    n, per, steps = 2, 8, 3
    launcher.spawn(_dp_worker, n, args=(str(tmp_path), per, steps))
    ms = [torch.load(tmp_path / f"m{r}.pt", weights_only=True) for r in range(n)]
    assert torch.equal(ms[0], ms[1])  # replicas bit-identical after the all-reduce
    tr = _frozen_resnet_trainer(gpu)
    m0 = tr.flat.master.detach().cpu().clone()
    x, y = _global_batch(n, per)
    x, y = x.to(gpu), y.to(gpu)
    for _ in range(steps):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    ref = tr.flat.master.detach().cpu()
    ua, ub = ms[0] - m0, ref - m0
    assert ub.norm() > 0
    cos = torch.nn.functional.cosine_similarity(ua, ub, dim=0).item()
    assert cos > 0.999, cos
    assert ((ua - ub).norm() / ub.norm()).item() < 0.03


def _dp_graph_worker(rank, outdir, per, steps):
    """One rank of the DP step captured as a HIP graph with its bucketed RCCL all-reduces."""
    import torch
    from tensorflowdistributedlearning_amd.parallel.dist import init_distributed, shutdown
    ctx = init_distributed()
    tr = _frozen_resnet_trainer(ctx.device, ctx)
    x, y = _global_batch(ctx.world_size, per)
    xs = x[rank * per:(rank + 1) * per].to(ctx.device)
    ys = y[rank * per:(rank + 1) * per].to(ctx.device)
    tr.capture(xs, ys, warmup=1)  # the warm-up step trains too
    for _ in range(steps - 1):
        tr.replay()
    torch.cuda.synchronize()
    assert ctx.native.ok
    torch.save(tr.flat.master.cpu(), os.path.join(outdir, f"g{rank}.pt"))
    shutdown()


@need2
@pytest.mark.timeout(300)
def test_dp_graph_capture_n_ranks_matches_eager(tmp_path, gpu):
    """The data-parallel step captured as one HIP graph per rank — the bucket all-reduces forked
    into the capture on the comm stream (engine/trainer.py, parallel/bucketer.py) — replayed on
    2 real ranks: the replicas stay bit-identical and follow the eager DP trajectory (which
    test_dp_ranks_equal_large_batch ties to the single-GPU large batch)."""
    n, per, steps = 2, 8, 3
    launcher.spawn(_dp_graph_worker, n, args=(str(tmp_path), per, steps))
    launcher.spawn(_dp_worker, n, args=(str(tmp_path), per, steps))
    g = [torch.load(tmp_path / f"g{r}.pt", weights_only=True) for r in range(n)]
    e = torch.load(tmp_path / "m0.pt", weights_only=True)
    assert torch.equal(g[0], g[1])
    m0 = _frozen_resnet_trainer(gpu).flat.master.detach().cpu()
    ug, ue = g[0] - m0, e - m0
    cos = torch.nn.functional.cosine_similarity(ug, ue, dim=0).item()
    assert cos > 0.9999, cos
    assert ((ug - ue).norm() / ue.norm()).item() < 0.01


@need2
@pytest.mark.timeout(300)
def test_bench_self_spawn_gpus(tmp_path):
    n = min(NDEV, 8)
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "TDL_SHARE_GPU")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--model",
           "resnet18", "--image-size", "64", "--batch", "16", "--steps", "3", "--warmup", "2"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["config"]["rccl_ranks"] == n
    assert out["config"]["comm"] == "rccl" and out["value"] > 0
