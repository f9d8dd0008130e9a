#!/usr/bin/env python3
"""Flagship benchmark: ResNet-50, 224×224, bf16, synthetic data, SGD+momentum, softmax-CE,
data-parallel over N MI355X GPUs (one process per GPU, RCCL all-reduce overlapped with backward).

  python bench.py --gpus 1 --steps 20 --warmup 5
  python bench.py --gpus 8                 # self-launches 8 worker processes (one per GPU)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

With ``--gpus N > 1`` and no launcher environment (WORLD_SIZE unset) the process starts N fresh
worker processes of itself with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 set and
relays their exit status; it never touches the GPU itself.  Under torchrun it is one of the
workers.  Every GPU rank count > 1 runs its collectives on the native RCCL communicator, and the
run fails unless RCCL itself (``ncclCommCount``) reports N ranks; the JSON line carries that
count as ``config.rccl_ranks``.

Metric (BASELINE.json): images/sec for the whole node (weak scaling: per-GPU batch fixed).
Timing: W untimed warmup steps, then barrier + device sync, K timed steps, device sync + barrier;
the step time is the MAX over ranks; rank 0 prints one JSON line.

``--model deeplab_ref`` runs the reference's own trained config instead (DeepLab ResNet-v2-beta,
101×101×2, Lovász loss, Adam, global batch 64) — comparable with the reference's measured
90.7 img/s on 2 GPUs (Test.ipynb:212-213).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import signal
import socket
import subprocess

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node), ResNet-50 224x224 bf16 at 1/2/4/8 MI355X"
REF_PER_GPU_DERIVED = 86.0   # ResNet-50-equivalent at the reference's FLOP rate
REF_DEEPLAB_2GPU = 90.7      # measured, 2 GPUs, global batch 64


def launch_workers(n: int, argv) -> int:
    """Start ``n`` worker processes of this script (one per GPU) and relay their exit status.

    The parent imports nothing that touches the GPU.  Rank 0's stdout (the JSON line) and every
    rank's stderr are inherited.  If any worker fails, the others are terminated (SIGTERM, then
    SIGKILL after 15 s) so a dead rank cannot leave its peers blocked in a collective."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env, cwd=os.getcwd(), start_new_session=False))
    def forward(sig, _frame):  # a signal to the launcher (e.g. `timeout`) reaches every worker
        for q in procs:
            if q.poll() is None:
                q.send_signal(sig)
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            r = p.poll()
            if r is None:
                continue
            alive.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                print(f"[bench] worker pid {p.pid} exited with {r}; stopping the others",
                      file=sys.stderr, flush=True)
                for q in alive:
                    q.send_signal(signal.SIGTERM)
                t0 = time.time()
                while any(q.poll() is None for q in alive) and time.time() - t0 < 15:
                    time.sleep(0.2)
                for q in alive:
                    if q.poll() is None:
                        q.kill()
                        q.wait()
                alive = []
        time.sleep(0.05)
    return rc


def _opt(name):
    return "sgd" if name == "sgd_momentum" else name


def _opt_kw(bc):
    if bc.optimizer == "adam":
        return dict(lr=bc.lr)
    return dict(lr=bc.lr, momentum=bc.momentum, weight_decay=bc.weight_decay)


def bench_config(args):
    """The run's :class:`config.BenchConfig`: ``--config`` file (or the defaults), then every
    flag that was given."""
    from tensorflowdistributedlearning_amd.config import BenchConfig, load
    cfg = load(args.config, BenchConfig) if args.config else BenchConfig()
    over = {"arch": args.model, "batch": args.batch, "image_size": args.image_size,
            "steps": args.steps, "warmup": args.warmup, "lr": args.lr,
            "bucket_mb": args.bucket_mb, "first_bucket_mb": args.first_bucket_mb,
            "optimizer": args.optimizer, "dtype": args.dtype, "grad_dtype": getattr(args, "grad_dtype", None)}
    for k, v in over.items():
        if v is not None:
            setattr(cfg, k, v)
    if args.fp8:
        cfg.dtype = "fp8"
    cfg.fp8_dgrad = cfg.fp8_dgrad or args.fp8_dgrad
    cfg.graph = cfg.graph or args.graph
    return cfg.validate()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", help="BenchConfig JSON / YAML (config.BenchConfig); flags override")
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 20)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed warm-up steps (default 5)")
    ap.add_argument("--model", default=None, help="arch preset (default resnet50)")
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (default 1024 for the ImageNet models, 64/N for deeplab_ref)")
    ap.add_argument("--image-size", type=int, default=None)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--first-bucket-mb", type=float, default=None)
    ap.add_argument("--grad-dtype", choices=("fp32", "bf16"), default=None,
                    help="dtype of the bucketed gradient all-reduces (bf16: half the xGMI bytes, "
                         "fp32 accumulation in the optimizer; default fp32)")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--optimizer", choices=("sgd_momentum", "adam"), default=None)
    ap.add_argument("--fp8", action="store_true",
                    help="fp8 GEMMs on the CDNA4 16x16x128 f8f6f4 MFMA for every eligible conv: "
                         "forward e4m3 activations x e4m3 weights; weight and input gradients "
                         "stay bf16")
    ap.add_argument("--fp8-dgrad", action="store_true",
                    help="with --fp8: the input gradients on fp8 too (e5m2 x e4m3) — the default "
                         "unless TDL_FP8_DGRAD=0")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole training step as a HIP graph and replay it (removes "
                         "host launch overhead in launch-bound configs; with N>1 the bucketed "
                         "all-reduces are captured too, on the native RCCL communicator)")
    ap.add_argument("--dtype", choices=("bf16", "fp32"), default=None,
                    help="GPU compute precision: bf16 (fused bf16 kernels, fp32 accumulation / "
                         "master weights) or fp32 (fp32 operands on the fp32 MFMA end to end — the "
                         "reference's own precision, for the like-for-like deeplab_ref comparison)")
    ap.add_argument("--mode", choices=("train", "infer"), default="train",
                    help="train (the headline: full training step) or infer (serving: eval-mode "
                         "forward under no_grad with every BatchNorm folded into its conv, "
                         "models/layers.ConvBN; images/sec of forward passes)")
    ap.add_argument("--no-fold", action="store_true",
                    help="with --mode infer: keep the unfolded conv + BN-apply eval path (A/B)")
    ap.add_argument("--profile-phases", action="store_true",
                    help="also print per-phase step times (forward/backward/comm_wait/optimizer, "
                         "device events) to stderr")
    args = ap.parse_args()
    if args.no_fold:
        os.environ["TDL_BN_FOLD"] = "0"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_workers(args.gpus, sys.argv[1:]))
    bc = bench_config(args)  # in the workers: a bad preset fails a rank (launcher relays it)

    import torch
    from tensorflowdistributedlearning_amd.parallel.dist import init_distributed, shutdown
    from tensorflowdistributedlearning_amd.ops import streams
    from tensorflowdistributedlearning_amd.engine.trainer import Trainer
    from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, lovasz_hinge
    from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch, segmentation_batch
    from tensorflowdistributedlearning_amd import models

    ctx = init_distributed()
    n = ctx.world_size
    if n != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {n}")
    dev = ctx.device
    if dev.type == "cuda" and os.environ.get("TDL_COMPUTE_PRIO"):
        # A/B knob: run the step on a stream of the given HIP priority (lower = more urgent)
        torch.cuda.set_stream(torch.cuda.Stream(dev, priority=int(os.environ["TDL_COMPUTE_PRIO"])))
    rccl_ranks = ctx.rccl_ranks
    if dev.type == "cuda" and n > 1 and os.environ.get("TDL_SHARE_GPU") != "1" \
            and rccl_ranks != args.gpus:
        raise SystemExit(f"RCCL reports {rccl_ranks} ranks, --gpus {args.gpus}")
    comm = "rccl" if ctx.native is not None else ("gloo" if n > 1 else "none")
    # CPU (plumbing runs, tests): fp32 storage, the PyTorch reference ops; GPU --dtype fp32: fp32
    # activations + the fp32 master weights read directly by the fp32 kernels (no compute copy)
    gpu_bf16 = dev.type == "cuda" and bc.dtype in ("bf16", "fp8")
    lowp = torch.bfloat16 if gpu_bf16 else None
    ddt = torch.bfloat16 if gpu_bf16 else torch.float32
    dtype_name = "bf16" if gpu_bf16 else "fp32" if dev.type == "cuda" else "fp32 (CPU plumbing run)"
    if bc.dtype == "fp8" and not gpu_bf16:
        raise SystemExit("--fp8 runs on the bf16 GPU path")
    torch.manual_seed(1234)
    fp8_desc = None
    if bc.arch == "deeplab_ref" and bc.dtype == "fp8":
        raise SystemExit("--fp8 is for the ImageNet models")

    if bc.arch == "deeplab_ref":
        per_gpu = bc.batch or max(64 // n, 1)
        model = models.DeepLabResNet(model_name="model", input_shape=(101, 101))
        tr = Trainer(model, lovasz_hinge, dev, _opt(bc.optimizer), _opt_kw(bc), ctx=ctx,
                     bucket_mb=bc.bucket_mb, first_bucket_mb=bc.first_bucket_mb,
                     profile_phases=args.profile_phases, lowp_dtype=lowp,
                     grad_comm_dtype=torch.bfloat16 if bc.grad_dtype == "bf16" else torch.float32)
        x, y = segmentation_batch(per_gpu, device=dev, seed=ctx.rank, dtype=ddt)
        metric = ("images/sec (whole node), reference DeepLab-ResNet 101x101x2 "
                  + ("bf16" if gpu_bf16 else "fp32"))
        cfg = {"model": "deeplab_resnet_v2_beta(3,4,6) os8", "global_batch": per_gpu * n,
               "image": "101x101x2", "parallelism": f"dp{n}", "comm": comm, "rccl_ranks": rccl_ranks, "optimizer": bc.optimizer,
               "loss": "lovasz_hinge", "hip_graph": bc.graph, "grad_comm_dtype": bc.grad_dtype,
               "wgrad_side_stream": streams.enabled()}
        base = REF_DEEPLAB_2GPU / 2 * n
    else:
        # 1024 images per GPU by default (ResNet-50: 49 GiB reserved of the 288 GB HBM): +2.9 %
        # img/s over 512 and +15 % over 256 on the same box (bigger GEMM M, fixed per-layer costs
        # amortised; profiles/r02_resnet50_batch_sweep.txt)
        per_gpu = bc.batch or 1024
        model = models.build(bc.arch, num_classes=1000)
        if bc.dtype == "fp8":
            models.enable_fp8(model, dgrad=bc.fp8_dgrad or None)
            dg = any(getattr(m, "emit_fp8_bwd", False) for m in model.modules())
            wg = any(getattr(m, "fp8_wgrad", False) for m in model.modules())
            st = int(os.environ.get("TDL_FP8_BF16_STAGES", "2"))
            fp8_desc = (("fp8 (e4m3 fwd, e5m2 x e4m3 dgrad + wgrad GEMMs, bf16 BN" if dg and wg
                         else "fp8 (e4m3 fwd, e5m2 x e4m3 dgrad GEMMs, bf16 wgrad + BN" if dg
                         else "fp8 (e4m3 x e4m3 forward GEMMs, bf16 dgrad / wgrad + BN")
                        + (f"; stages 1-{st} bf16)" if st > 0 else ")"))
        tr = Trainer(model, softmax_cross_entropy, dev, _opt(bc.optimizer), _opt_kw(bc), ctx=ctx,
                     bucket_mb=bc.bucket_mb, first_bucket_mb=bc.first_bucket_mb,
                     profile_phases=args.profile_phases, lowp_dtype=lowp,
                     grad_comm_dtype=torch.bfloat16 if bc.grad_dtype == "bf16" else torch.float32)
        x, y = imagenet_batch(per_gpu, bc.image_size, device=dev, seed=ctx.rank, dtype=ddt)
        metric = METRIC if bc.arch == "resnet50" and bc.image_size == 224 and gpu_bf16 \
            else (f"images/sec (whole node), {bc.arch} {bc.image_size}x{bc.image_size} "
                  f"{fp8_desc if bc.dtype == 'fp8' else 'bf16' if gpu_bf16 else 'fp32'}")
        cfg = {"model": bc.arch, "global_batch": per_gpu * n, "seq_len": None,
               "image": f"{bc.image_size}x{bc.image_size}x3", "per_gpu_batch": per_gpu,
               "parallelism": f"dp{n}", "comm": comm, "rccl_ranks": rccl_ranks,
               "optimizer": bc.optimizer,
               "loss": "softmax_ce", "hip_graph": bc.graph, "grad_comm_dtype": bc.grad_dtype,
               "wgrad_side_stream": streams.enabled()}
        base = REF_PER_GPU_DERIVED * n

    def step():
        tr.train_step(x, y)

    if args.mode == "infer":
        if bc.dtype == "fp8":
            raise SystemExit("--mode infer: bf16 / fp32")
        model.eval()
        shape = ("101x101x2 (the reference's Model.predict workload)" if bc.arch == "deeplab_ref"
                 else f"{bc.image_size}x{bc.image_size}")
        metric = ("inference images/sec (whole node), " + bc.arch + f" {shape} "
                  + ("bf16" if gpu_bf16 else "fp32")
                  + (" (BN unfolded)" if args.no_fold else " (BN folded into the convs)"))
        cfg.update(optimizer=None, loss=None, mode="infer", bn_folded=not args.no_fold)
        base = None

        @torch.no_grad()
        def step():
            model(x)

    if bc.graph and args.mode == "infer":
        step()
        torch.cuda.synchronize(dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream(dev).wait_stream(s)
        gr = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(gr):
            model(x)
        step = gr.replay
        for _ in range(bc.warmup):
            step()
    elif bc.graph:
        tr.capture(x, y, warmup=bc.warmup)  # W eager warm-up steps, then the capture
        step = tr.replay
        step()  # first replay (graph upload) stays untimed
        print(f"[bench] step captured as a HIP graph ({bc.arch}, batch {per_gpu}/gpu)",
              file=sys.stderr, flush=True)
    else:
        for i in range(bc.warmup):
            step()
            if ctx.is_main and i == 0:
                print(f"[bench] first step done ({bc.arch}, batch {per_gpu}/gpu, n={n})",
                      file=sys.stderr, flush=True)
    ctx.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(bc.steps):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    ctx.barrier()
    el = time.perf_counter() - t0
    el = ctx.all_reduce_max(el)
    ms = el / bc.steps * 1e3
    comm_stats = None
    if n > 1 and tr.bucketer is not None and not bc.graph and args.mode == "train":
        # exposed communication (backward end → last bucket done, compute stream) vs the same
        # collectives run alone: overlap = the fraction backward hid
        exposed = ctx.all_reduce_max(tr.comm_wait_ms(last=bc.steps) or 0.0)
        alone = ctx.all_reduce_max(tr.bucketer.standalone_ms())
        comm_stats = {"exposed_ms": round(exposed, 3), "standalone_ms": round(alone, 3),
                      "overlap": round(max(0.0, 1.0 - exposed / alone), 3) if alone > 0 else None,
                      "buckets": len(tr.bucketer.buckets),
                      "comm_mb_per_step": round(tr.bucketer.comm_bytes / 2 ** 20, 1)}
    value = per_gpu * n * bc.steps / el
    if ctx.is_main:
        if dev.type == "cuda":
            print(f"[bench] peak device memory {torch.cuda.max_memory_allocated(dev) / 2**30:.1f} "
                  f"GiB allocated, {torch.cuda.max_memory_reserved(dev) / 2**30:.1f} GiB reserved",
                  file=sys.stderr, flush=True)
        if tr.timer is not None:
            ph = tr.timer.summary()
            print("[bench] phases ms/step (timed + warmup steps): " +
                  " ".join(f"{k}={v:.2f}" for k, v in ph.items()), file=sys.stderr)
        if comm_stats is not None:
            cfg["comm_overlap"] = comm_stats
        print(json.dumps({
            "metric": metric, "value": round(value, 2), "unit": "images/sec", "n_gpus": n,
            "steps": bc.steps, "warmup": bc.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / base, 3) if base else None,
            "baseline": (None if base is None else
                         "BASELINE.md derived ResNet-50-equivalent 86 img/s/GPU (no published "
                         "ResNet-50 number)" if bc.arch != "deeplab_ref" else
                         "BASELINE.md measured 90.7 img/s on 2 GPUs, scaled per GPU"),
            "dtype": fp8_desc if bc.dtype == "fp8" else dtype_name,
            "data": "synthetic (device-resident random batch, random-init weights)",
            "config": cfg}), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
