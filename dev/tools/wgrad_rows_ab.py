"""Weight-gradient route rows forced one at a time on the ResNet-50 b1024 shapes that default to
the register-staged kernel (wgrad.gemm): us per call (CUDA events), for a same-box choice."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402

N = int(os.environ.get("N", "1024"))
# (H, Cin, Cout, k, stride)
SHAPES = [(56, 64, 64, 3, 1), (7, 512, 512, 3, 1), (14, 256, 256, 3, 1), (28, 128, 128, 3, 1),
          (56, 256, 64, 1, 1), (28, 512, 128, 1, 1), (56, 64, 64, 1, 1), (56, 256, 128, 1, 1)]
ROWS = ["wgrad.gemm", "wgrad.halo.aligned", "wgrad.glds.aligned.m128", "wgrad.glds.aligned",
        "wgrad.glds.1x1", "wgrad.halo.wide3x3"]


def t(fn, it=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


e = ext()
for (H, ci, co, k, st) in SHAPES:
    p = (k - 1) // 2
    Ho = (H + 2 * p - k) // st + 1
    x = torch.randn(N, H, H, ci, device="cuda").bfloat16()
    dy = torch.randn(N, Ho, Ho, co, device="cuda").bfloat16()
    out = torch.empty(co, k, k, ci, device="cuda")
    line = f"{H}x{H}x{ci}->{co} k{k} s{st}:"
    ref = None
    for r in ROWS:
        e.conv_route_force(2, r)
        try:
            f = lambda: e.conv_wgrad(dy, x, out, None, st, st, p, p, 1, 1, False, None)
            us = t(f)
            if ref is None:
                ref = out.clone()
            err = ((out - ref).abs().max() / (ref.abs().max() + 1e-6)).item()
            line += f"  {r.split('wgrad.')[1]} {us:7.1f}" + (" (!)" if err > 1e-3 else "")
        except RuntimeError:
            pass
        finally:
            e.conv_route_force(2, "")
    print(line, flush=True)
