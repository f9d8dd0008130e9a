#!/usr/bin/env python3
"""Same-box A/B of the producer/consumer forward (csrc/kernels/conv_pc.hip, TDL_CONV_PC) against
the default LDS-DMA forward (conv_glds.hip) on ResNet-50's forward convs (b1024, BN statistics
epilogue as in training).  Interleaved rounds in one process; outputs and statistics compared.

  python bench/pc_ab.py --batch 1024 --out gpurun_out/pc_ab.json
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402

MODES = (0, 1, 2)  # conv_set_pc: 0 = conv_glds, 1 = 2 producer waves, 2 = 4
# (H, W, Cin, Cout, k, stride, count per ResNet-50 step)
SHAPES = [(56, 56, 64, 256, 1, 1, 4), (56, 56, 256, 128, 1, 1, 1), (56, 56, 256, 512, 1, 2, 1),
          (56, 56, 128, 128, 3, 2, 1), (28, 28, 128, 128, 3, 1, 3), (28, 28, 128, 512, 1, 1, 4),
          (28, 28, 512, 128, 1, 1, 3), (28, 28, 512, 256, 1, 1, 1), (28, 28, 512, 1024, 1, 2, 1),
          (28, 28, 256, 256, 3, 2, 1), (14, 14, 256, 256, 3, 1, 5), (14, 14, 256, 1024, 1, 1, 6),
          (14, 14, 1024, 256, 1, 1, 5), (14, 14, 1024, 512, 1, 1, 1),
          (14, 14, 1024, 2048, 1, 2, 1), (14, 14, 512, 512, 3, 2, 1), (7, 7, 512, 512, 3, 1, 2),
          (7, 7, 512, 2048, 1, 1, 3), (7, 7, 2048, 512, 1, 1, 2)]


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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows, tot = [], {m: 0.0 for m in MODES}
    for H, W, Cin, K, k, s, cnt in SHAPES:
        N = args.batch
        p = (k - 1) // 2
        g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
        torch.manual_seed(0)
        x = (torch.randn(N, H, W, Cin, device=dev)).bfloat16()
        w = (torch.randn(K, k, k, Cin, device=dev) / math.sqrt(k * k * Cin)).bfloat16()
        stats = torch.zeros(2, K, device=dev)
        outs = {}
        for mode in MODES:
            ext().conv_set_pc(mode)
            stats.zero_()
            y = C.conv_fwd(x, w, g, stats=stats)
            torch.cuda.synchronize()
            outs[mode] = (y.clone(), stats.clone())
        same = all(torch.equal(outs[0][0], outs[m][0]) for m in MODES)
        sdiff = max(((outs[0][1] - outs[m][1]).abs().max() / outs[0][1].abs().max()).item()
                    for m in MODES)
        res = {}

        def fwd():
            stats.zero_()
            C.conv_fwd(x, w, g, stats=stats)
        for _ in range(args.rounds):
            for mode in MODES:
                ext().conv_set_pc(mode)
                fwd()
                torch.cuda.synchronize()
                res.setdefault(mode, []).append(timeit(fwd, args.iters))
        ext().conv_set_pc(-1)
        Ho = (H + 2 * p - k) // s + 1
        fl = 2.0 * N * Ho * Ho * K * Cin * k * k
        t = {m: sorted(v)[len(v) // 2] for m, v in res.items()}
        for m in MODES:
            tot[m] += t[m] * cnt
        row = dict(shape=f"{H}x{W}x{Cin}->{K} k{k} s{s}", count=cnt, identical=same,
                   stats_rel_diff=sdiff)
        for m in MODES:
            row[f"mode{m}_us"] = round(t[m], 1)
            row[f"mode{m}_tf"] = round(fl / t[m] / 1e6, 1)
        rows.append(row)
        print(f"{row['shape']:28s} x{cnt}  " + "  ".join(
            f"m{m} {t[m]:7.1f} us ({fl / t[m] / 1e6:5.0f} TF)" for m in MODES) +
            f"  identical={same} stats {sdiff:.1e}", flush=True)
        del x, w, outs
        torch.cuda.empty_cache()
    print("forward convs per step: " + ", ".join(f"mode {m} {tot[m] / 1e3:.2f} ms" for m in MODES)
          + "  (0 = conv_glds, 1 = producer/consumer with 2 producers, 2 = with 4)")
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
