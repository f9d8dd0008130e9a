#!/usr/bin/env python3
"""Same-box A/B of the halo-tiled direct conv (csrc/kernels/conv_halo.hip) against the default
implicit-GEMM selection on the stride-1 3×3 convs of ResNet-50 and the reference DeepLab preset:
forward with BN statistics and the input gradient with the ReLU mask + BN-backward statistics
(the bottleneck conv2 pattern).  Interleaved rounds in one process (guide §5.4 rule 24); prints a
table and writes JSON.

  python bench/halo_ab.py --batch 1024 --out gpurun_out/halo_ab.json
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops import bn as BN  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402

# (name, batch multiplier, H, W, Cin, Cout, dilation, count per step)
SHAPES = {
    "resnet50": [("l1.conv2 56x56x64", 1, 56, 56, 64, 64, 1, 3),
                 ("l2.conv2 28x28x128", 1, 28, 28, 128, 128, 1, 3),
                 ("l3.conv2 14x14x256", 1, 14, 14, 256, 256, 1, 5),
                 ("l4.conv2 7x7x512", 1, 7, 7, 512, 512, 1, 2)],
    "deeplab": [("conv1_2 51x51x64", 1, 51, 51, 64, 64, 1, 1),
                ("conv1_3 51x51x64->128", 1, 51, 51, 64, 128, 1, 1),
                ("block1 26x26x128", 1, 26, 26, 128, 128, 1, 2),
                ("block3 13x13x512 d2", 1, 13, 13, 512, 512, 2, 6),
                ("block4 13x13x256 d4", 1, 13, 13, 256, 256, 4, 2)],
}


def timeit(fn, iters):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--deeplab-batch", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows = []
    for net, shapes in SHAPES.items():
        B0 = args.batch if net == "resnet50" else args.deeplab_batch
        for name, mult, H, W, Cin, K, dil, cnt in shapes:
            N = B0 * mult
            g = C.ConvGeom((1, 1), (dil, dil, dil, dil), (dil, dil))
            torch.manual_seed(0)
            x = (torch.randn(N, H, W, Cin, device=dev) * 1.2).bfloat16()
            w = (torch.randn(K, 3, 3, Cin, device=dev) / math.sqrt(9 * Cin)).bfloat16()
            dy = torch.randn(N, H, W, K, device=dev).bfloat16()
            gam = torch.rand(Cin, device=dev) + 0.5
            bet = torch.randn(Cin, device=dev) * 0.3
            coef = BN.bn_finalize(BN.bn_stats(x), N * H * W, gam, bet,
                                  torch.zeros(Cin, device=dev), torch.ones(Cin, device=dev),
                                  0.9, 1e-3, True)
            mask = torch.empty(x.numel() // 8, device=dev, dtype=torch.uint8)
            BN.bn_apply(x, coef, None, True, mask=mask)
            stats = torch.zeros(2, K, device=dev)

            def fwd():
                stats.zero_()
                C.conv_fwd(x, w, g, stats=stats)

            def dgrad():
                C.conv_dgrad_bnstat(dy, w, x.shape, g, x, mask=mask)

            dwb = torch.empty(K, 3, 3, Cin, device=dev)

            def wgrad():
                C.conv_wgrad(dy, x, tuple(w.shape), g, out=dwb)

            res = {}
            outs = {}
            for mode in (0, 2):  # correctness cross-check of the two paths first
                ext().conv_set_halo_mode(mode)
                stats.zero_()
                y = C.conv_fwd(x, w, g, stats=stats)
                dx, _ = C.conv_dgrad_bnstat(dy, w, x.shape, g, x, mask=mask)
                dwv = C.conv_wgrad(dy, x, tuple(w.shape), g)
                outs[mode] = (y.float(), dx.float(), dwv.float())
            ey = ((outs[0][0] - outs[2][0]).abs().max() / outs[0][0].abs().max()).item()
            ed = ((outs[0][1] - outs[2][1]).abs().max() / outs[0][1].abs().max()).item()
            ew = ((outs[0][2] - outs[2][2]).abs().max() / outs[0][2].abs().max()).item()
            for r in range(args.rounds):
                for mode in (0, 2):
                    ext().conv_set_halo_mode(mode)
                    fwd(); dgrad(); wgrad()
                    torch.cuda.synchronize()
                    res.setdefault((mode, "fwd"), []).append(timeit(fwd, args.iters))
                    res.setdefault((mode, "dgrad"), []).append(timeit(dgrad, args.iters))
                    res.setdefault((mode, "wgrad"), []).append(timeit(wgrad, args.iters))
            ext().conv_set_halo_mode(-1)
            fl = 2.0 * N * H * W * K * Cin * 9
            row = {"net": net, "shape": name, "batch": N, "count": cnt, "rel_diff_fwd": ey,
                   "rel_diff_dgrad": ed, "rel_diff_wgrad": ew}
            for mode, tag in ((0, "gemm"), (2, "halo")):
                for p in ("fwd", "dgrad", "wgrad"):
                    t = sorted(res[(mode, p)])[len(res[(mode, p)]) // 2]
                    row[f"{tag}_{p}_us"] = round(t, 1)
                    row[f"{tag}_{p}_tf"] = round(fl / t / 1e6, 1)
            rows.append(row)
            print(f"{net:9s} {name:24s} N={N:5d}  fwd {row['gemm_fwd_us']:8.1f} -> "
                  f"{row['halo_fwd_us']:8.1f} us ({row['halo_fwd_tf']:6.1f} TF)   dgrad "
                  f"{row['gemm_dgrad_us']:8.1f} -> {row['halo_dgrad_us']:8.1f} us "
                  f"({row['halo_dgrad_tf']:6.1f} TF)   wgrad {row['gemm_wgrad_us']:8.1f} -> "
                  f"{row['halo_wgrad_us']:8.1f} us ({row['halo_wgrad_tf']:6.1f} TF)  x{cnt}  "
                  f"diff {ey:.1e}/{ed:.1e}/{ew:.1e}", flush=True)
            del x, w, dy, mask, dwb
            torch.cuda.empty_cache()
    for net in SHAPES:
        for p in ("fwd", "dgrad", "wgrad"):
            a = sum(r[f"gemm_{p}_us"] * r["count"] for r in rows if r["net"] == net)
            b = sum(r[f"halo_{p}_us"] * r["count"] for r in rows if r["net"] == net)
            print(f"{net}: stride-1 3x3 {p} per step {a / 1e3:.2f} ms -> {b / 1e3:.2f} ms")
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
