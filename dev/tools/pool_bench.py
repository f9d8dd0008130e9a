"""Stand-alone timing of the ResNet stem's fused pool kernels at the bench shape (batch 256,
112×112×64 → 56×56×64): bn_maxpool_fwd and maxpool_bn_bwd (sums + apply), against a plain copy
of the 112² tensor as the bandwidth yardstick.  ``--only fwd|bwd|copy`` runs one of them (for
rocprofv3 --pmc passes)."""
import argparse
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from tensorflowdistributedlearning_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--heat", action="store_true",
                    help="run bf16 GEMMs for ~0.3 s before each timed call (the bench's power state)")
    a = ap.parse_args()
    ext = _native.load()
    dev = torch.device("cuda", 0)
    N, H, C, Ho = a.n, 112, 64, 56
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, H, C, device=dev, generator=g).bfloat16()
    coef = torch.zeros(4, C, device=dev)
    coef[0] = 1.3
    coef[1] = -0.1
    coef[3] = 1.0
    y = torch.empty(N, Ho, Ho, C, device=dev, dtype=torch.bfloat16)
    zarg = torch.empty_like(y)
    idx = torch.empty(N, Ho, Ho, C, device=dev, dtype=torch.uint8)
    dy = torch.randn(N, Ho, Ho, C, device=dev, generator=g).bfloat16()
    dx = torch.empty_like(x)
    red = torch.zeros(2, C, device=dev)
    gamma = torch.ones(C, device=dev)
    dg = torch.empty(C, device=dev)
    db = torch.empty(C, device=dev)
    cp = torch.empty_like(x)

    def fwd():
        ext.bn_maxpool_fwd(x, coef, y, idx, 3, 2, 1, 1, zarg=zarg)

    def bwd():
        red.zero_()
        ext.maxpool_bn_bwd(dy, idx, zarg, x, coef, red, gamma, dx, dg, db, float(N * H * H), 3, 2,
                           1, 1)

    def copy():
        cp.copy_(x)

    ha = torch.randn(8192, 8192, device=dev).bfloat16()
    hb, hc = ha.clone(), torch.empty_like(ha)
    xb = x.numel() * 2
    yb = y.numel() * 2
    cases = {"fwd": (fwd, xb + 2 * yb + yb // 2), "bwd": (bwd, 2 * xb + 2 * yb + yb // 2 + yb + yb // 2),
             "copy": (copy, 2 * xb)}
    fwd()
    bwd()
    torch.cuda.synchronize()
    # checksum of dx for cross-build / cross-knob exactness checks (same inputs every run)
    print(f"dx checksum {dx.double().sum().item():.10e} {dx.float().abs().sum().item():.10e}", flush=True)
    for name, (fn, nbytes) in cases.items():
        if a.only and name != a.only:
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        if a.heat:
            tot = 0.0
            for _ in range(a.iters):
                for _ in range(30):
                    torch.matmul(ha, hb, out=hc)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                tot += e0.elapsed_time(e1)
            us = tot * 1e3 / a.iters
        else:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(f"{name:5s} {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s (min bytes {nbytes / 1e6:.0f} MB)",
              flush=True)


if __name__ == "__main__":
    main()
