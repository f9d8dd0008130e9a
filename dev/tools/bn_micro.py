"""Microbenchmark of the BN kernels at the ResNet-50 (default) or ResNet-152 layer shapes:
µs and TB/s per kernel and shape, plus the per-step total weighted by how often each shape occurs.

  python dev/tools/bn_micro.py [--model resnet50|resnet152] [--batch 256] [--iters 30]

Per-step classes (ResNet bottleneck, training): "apply" = BN+ReLU (bn1/bn2/stem), "apply_res" =
BN + residual + ReLU with the 1-bit mask (bn3), "apply_ds" = BN without ReLU (downsample branch);
backward "red2/bwd2" (mask from x), "red3/bwd3" (bit mask, dres written), "red0/bwd0" (no ReLU)."""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import bn as B  # noqa: E402


def timeit(fn, it):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def resnet_shapes(blocks):
    """(H, C, kind) -> count per training step for a torchvision-style (v1.5) bottleneck ResNet."""
    cnt = collections.Counter()
    cnt[(112, 64, "relu")] += 1
    hw, width = 56, 64
    for si, nb in enumerate(blocks):
        for b in range(nb):
            h_in = hw * 2 if (b == 0 and si > 0) else hw
            cnt[(h_in, width, "relu")] += 1        # bn1 (conv1 is at the input resolution)
            cnt[(hw, width, "relu")] += 1          # bn2
            cnt[(hw, width * 4, "res")] += 1       # bn3 + residual + relu
            if b == 0:
                cnt[(hw, width * 4, "ds")] += 1    # downsample BN (no relu)
        hw //= 2
        width *= 2
    return cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--tag", default=os.environ.get("BN_TAG", ""))
    a = ap.parse_args()
    blocks = {"resnet50": (3, 4, 6, 3), "resnet152": (3, 8, 36, 3)}[a.model]
    shapes = resnet_shapes(blocks)
    dev = "cuda"
    tot = collections.Counter()
    for (hw, C, kind), n in sorted(shapes.items(), key=lambda kv: (-kv[0][0], kv[0][1])):
        M = a.batch * hw * hw
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(M, C, device=dev, generator=g).bfloat16()
        dy = torch.randn(M, C, device=dev, generator=g).bfloat16()
        res = torch.randn(M, C, device=dev, generator=g).bfloat16() if kind == "res" else None
        coef = torch.stack([torch.rand(C) + .5, torch.randn(C), torch.randn(C) * .1,
                            torch.rand(C) + .5]).to(dev)
        gam = torch.ones(C, device=dev)
        S = M * C * 2 / 1e6  # MB per bf16 tensor
        if kind == "res":
            mask = torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
            B.bn_apply(x, coef, res, True, None, mask)
            ta = timeit(lambda: B.bn_apply(x, coef, res, True, None, mask), a.iters)
            red = B.bn_bwd_reduce(dy, mask, x, coef, 3)
            tr = timeit(lambda: B.bn_bwd_reduce(dy, mask, x, coef, 3), a.iters)
            tb = timeit(lambda: B.bn_bwd_apply(dy, mask, x, coef, red, gam, M, 3, True), a.iters)
            ba, br, bb = 3 * S + S / 16, 2 * S + S / 16, 4 * S + S / 16
        else:
            relu = kind == "relu"
            mode = 2 if relu else 0
            ta = timeit(lambda: B.bn_apply(x, coef, None, relu), a.iters)
            red = B.bn_bwd_reduce(dy, None, x, coef, mode)
            tr = timeit(lambda: B.bn_bwd_reduce(dy, None, x, coef, mode), a.iters)
            tb = timeit(lambda: B.bn_bwd_apply(dy, None, x, coef, red, gam, M, mode, False),
                        a.iters)
            ba, br, bb = 2 * S, 2 * S, 3 * S
        tot["apply"] += n * ta
        tot["reduce"] += n * tr
        tot["bwd_apply"] += n * tb
        print(f"{a.tag} {hw:3d}x{hw:<3d} C={C:5d} {kind:4s} x{n:2d} {S:7.1f}MB | apply {ta:7.1f}us "
              f"{ba / ta:5.2f}TB/s | reduce {tr:7.1f}us {br / tr:5.2f}TB/s | bwd {tb:7.1f}us "
              f"{bb / tb:5.2f}TB/s", flush=True)
        del x, dy, res
    print(json.dumps({"tag": a.tag, "model": a.model, "batch": a.batch,
                      **{k: round(v / 1e3, 3) for k, v in tot.items()},
                      "total_ms": round(sum(tot.values()) / 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
