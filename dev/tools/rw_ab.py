"""Resident-filter 3x3 64->64 conv (route rows fwd.halo.rw64 / dgrad.asfwd.rw64) vs the rows it
replaced, at the ResNet-50 layer-1 shape: forward with fused BN sums, input gradient (as the
forward conv of dy) with the ReLU bit mask and the BN-backward sums — median of CUDA-event times."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402
from tensorflowdistributedlearning_amd.ops import bn as B  # noqa: E402


def timeit(fn, reps=20):
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
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 56
    e = ext()
    dev = torch.device("cuda")
    x = torch.randn(N, H, H, 64, device=dev).bfloat16()
    w = (torch.randn(64, 3, 3, 64, device=dev) / 24).bfloat16()
    y = torch.empty_like(x)
    st = torch.zeros(2, 64, device=dev)
    dy = torch.randn(N, H, H, 64, device=dev).bfloat16()
    coef = torch.zeros(4, 64, device=dev)
    coef[0].uniform_(0.3, 2.0)
    coef[1].normal_(0, 0.6)
    mask = torch.empty(x.numel() // 8, device=dev, dtype=torch.uint8)
    B.bn_apply(x, coef, None, True, mask=mask)
    wf = torch.empty_like(w)
    e.conv_flip_weight(w, wf)
    dx = torch.empty_like(x)
    red = torch.zeros(2, 64, device=dev)
    flop = 2.0 * N * H * H * 64 * 576
    for op, rows in ((0, ["fwd.halo.rw64", "fwd.halo.narrow", "fwd.glds.aligned.n64"]),
                     (1, ["dgrad.asfwd.rw64", "dgrad.asfwd.glds.n64", "dgrad.asfwd.halo"])):
        for r in rows:
            e.conv_route_force(op, r)
            try:
                if op == 0:
                    f = lambda: e.conv_fwd(x, w, y, None, st, 1, 1, 1, 1, 1, 1, False)
                else:
                    # (the halo dgrad row takes no statistics: plain mask form there)
                    sx = None if r == "dgrad.asfwd.halo" else x
                    sr = None if r == "dgrad.asfwd.halo" else red
                    f = lambda: e.conv_dgrad(dy, w, dx, 1, 1, 1, 1, 1, 1, False, mask, None, sx, sr,
                                             None, wf)
                us = timeit(f)
                print(f"{'fwd  ' if op == 0 else 'dgrad'} {r:24s} N{N} {H}x{H}x64 3x3: "
                      f"{us:8.1f} us  {flop / us / 1e6:7.1f} TF/s", flush=True)
            except RuntimeError as err:
                print(f"{r}: {str(err)[:100]}", flush=True)
            finally:
                e.conv_route_force(op, "")


if __name__ == "__main__":
    main()
