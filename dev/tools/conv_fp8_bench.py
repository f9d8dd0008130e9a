#!/usr/bin/env python3
"""fp8 vs bf16 forward conv on ResNet-152 shapes: GEMM time with pre-quantised operands, and the
cost of quantising the activation (amax + quantize passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops import fp8 as F8  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402


def t(fn, it=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


def main():
    dev = torch.device("cuda")
    N = 128
    for H, Cin, Cout, k, s in [(56, 64, 64, 3, 1), (28, 128, 128, 3, 1), (14, 256, 256, 3, 1),
                               (7, 512, 512, 3, 1), (14, 1024, 256, 1, 1), (14, 256, 1024, 1, 1)]:
        p = k // 2
        g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
        x = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16) * 0.05
        x8, sx = F8.quantize_e4m3(x)
        w8, sw = F8.quantize_e4m3(w)
        flop = 2.0 * N * H * H * Cout * Cin * k * k
        ext().conv_set_glds_mode(2)
        tb = t(lambda: C.conv_fwd(x, w, g))
        ext().conv_set_glds_mode(-1)
        tf = t(lambda: C.conv_fwd_fp8(x8, sx, w8, sw, g))
        tq = t(lambda: F8.quantize_e4m3(x))
        print(f"{H:3d}x{H:<3d} {Cin:4d}->{Cout:4d} k{k}: bf16 {tb:7.1f}us ({flop / tb / 1e6:5.0f}TF)"
              f"  fp8 {tf:7.1f}us ({flop / tf / 1e6:5.0f}TF)  quantize(x) {tq:6.1f}us", flush=True)


if __name__ == "__main__":
    main()
