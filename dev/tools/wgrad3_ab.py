"""3x3 stride-1 weight gradients at the ResNet-50 b1024 shapes on each route row that takes them
(forced): median CUDA-event times."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402


def timeit(fn, reps=15):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    e = ext()
    dev = torch.device("cuda")
    for H, C in ((56, 64), (28, 128), (14, 256), (7, 512)):
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        dy = torch.randn(N, H, H, C, device=dev).bfloat16()
        out = torch.empty(C, 3, 3, C, device=dev)
        flop = 2.0 * N * H * H * C * 9 * C
        for r in ("wgrad.halo.aligned", "wgrad.gemm", "wgrad.glds.aligned.m128", "wgrad.glds.aligned"):
            e.conv_route_force(2, r)
            try:
                us = timeit(lambda: e.conv_wgrad(dy, x, out, None, 1, 1, 1, 1, 1, 1, False, None))
                print(f"wgrad {r:26s} N{N} {H}x{H}x{C} 3x3: {us:8.1f} us  {flop / us / 1e6:7.1f} TF/s",
                      flush=True)
            except RuntimeError as err:
                print(f"wgrad {r:26s} {H}x{H}x{C}: {str(err)[:80]}", flush=True)
            finally:
                e.conv_route_force(2, "")


if __name__ == "__main__":
    main()
