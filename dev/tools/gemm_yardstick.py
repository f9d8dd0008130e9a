"""hipBLASLt (torch.mm) bf16 yardstick at the implicit-GEMM shapes of the ResNet-50 convs.

A measurement only (never the product path): what the vendor GEMM library reaches on the same
M/N/K as each conv's forward, input gradient and weight gradient, so the conv kernels' TF/s can be
read against a same-box number instead of the 2.5 PF marketing peak.

  fwd   : y[M,K]  = x[M,C]  · W[C,K]       (1x1: exactly the conv; 3x3: K-dim C*9, im2col'd)
  dgrad : dx[M,C] = dy[M,K] · W[K,C]
  wgrad : dW[K,C] = dy[M,K]ᵀ · x[M,C]      (reduction over M = batch·H·W)

python dev/tools/gemm_yardstick.py --batch 1024 > profiles/r06_gemm_yardstick.txt
"""
import argparse

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
B = args.batch

convs = [  # (name, H*W, C_in, K_out, taps)
    ("56x56 1x1 64->256", 3136, 64, 256, 1),
    ("56x56 1x1 256->64", 3136, 256, 64, 1),
    ("56x56 3x3 64->64", 3136, 64, 64, 9),
    ("28x28 1x1 128->512", 784, 128, 512, 1),
    ("28x28 1x1 512->128", 784, 512, 128, 1),
    ("28x28 3x3 128->128", 784, 128, 128, 9),
    ("14x14 1x1 256->1024", 196, 256, 1024, 1),
    ("14x14 1x1 1024->256", 196, 1024, 256, 1),
    ("14x14 3x3 256->256", 196, 256, 256, 9),
    ("7x7 1x1 512->2048", 49, 512, 2048, 1),
    ("7x7 1x1 2048->512", 49, 2048, 512, 1),
    ("7x7 3x3 512->512", 49, 512, 512, 9),
]


def time_mm(a, b, trans_a=False):
    def run():
        return (a.t() @ b) if trans_a else (a @ b)
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(args.iters):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / args.iters * 1e3


print(f"# hipBLASLt bf16 torch.mm yardstick, ResNet-50 conv GEMM shapes at batch {B} "
      f"({torch.cuda.get_device_name(0)}, torch {torch.__version__})")
print(f"{'conv':22s} {'op':5s} {'M':>8s} {'N':>5s} {'K':>8s} {'us':>9s} {'TF/s':>7s}")
for name, hw, c, k, taps in convs:
    M = B * hw
    kc = c * taps
    x = torch.randn(M, kc, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(kc, k, device="cuda", dtype=torch.bfloat16)
    us = time_mm(x, w)
    print(f"{name:22s} fwd   {M:8d} {k:5d} {kc:8d} {us:9.1f} {2 * M * k * kc / us / 1e6:7.1f}", flush=True)
    dy = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
    wt = torch.randn(k, kc, device="cuda", dtype=torch.bfloat16)
    us = time_mm(dy, wt)
    print(f"{name:22s} dgrad {M:8d} {kc:5d} {k:8d} {us:9.1f} {2 * M * k * kc / us / 1e6:7.1f}", flush=True)
    us = time_mm(dy, x, trans_a=True)
    print(f"{name:22s} wgrad {k:8d} {kc:5d} {M:8d} {us:9.1f} {2 * M * k * kc / us / 1e6:7.1f}", flush=True)
    del x, w, dy, wt
    torch.cuda.empty_cache()
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
us = time_mm(a, a)
print(f"{'square 8192':22s} mm    {8192:8d} {8192:5d} {8192:8d} {us:9.1f} {2 * 8192**3 / us / 1e6:7.1f}")
