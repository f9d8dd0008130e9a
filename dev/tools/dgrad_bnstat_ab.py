#!/usr/bin/env python3
"""Same-box A/B: BN-backward statistics fused into the dgrad epilogue vs dgrad + BN reduce pass.

For each ResNet-50 shape (batch N) times
  A  conv_dgrad (+ join accumulate / ReLU mask where the model has them) then bn_bwd_reduce
  B  conv_dgrad_bnstat (the dgrad epilogue accumulates Σg, Σg·x)
and checks that B's sums match A's reduce (after the Σg·x → Σg·x̂ conversion) and dx is equal.

  python dev/tools/dgrad_bnstat_ab.py [--n 256] [--iters 20] [--json gpurun_out/dgrad_bnstat.jsonl]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops import bn as B  # noqa: E402
from route_ab import glds_cfg, RF_STATS, RF_JOIN  # noqa: E402

# (name, H, dx channels C, dy channels K, k, join): the BN whose output is the conv input has C
# channels; join = the block-input gradient join (accumulate into the residual gradient + mask)
SHAPES = [
    ("conv3 56 64<-256", 56, 64, 256, 1, False),
    ("conv3 28 128<-512", 28, 128, 512, 1, False),
    ("conv3 14 256<-1024", 14, 256, 1024, 1, False),
    ("conv3 7 512<-2048", 7, 512, 2048, 1, False),
    ("conv2 28 128 3x3", 28, 128, 128, 3, False),
    ("conv2 14 256 3x3", 14, 256, 256, 3, False),
    ("conv2 7 512 3x3", 7, 512, 512, 3, False),
    ("conv1 56 256<-64 join", 56, 256, 64, 1, True),
    ("conv1 28 512<-128 join", 28, 512, 128, 1, True),
    ("conv1 14 1024<-256 join", 14, 1024, 256, 1, True),
    ("conv1 7 2048<-512 join", 7, 2048, 512, 1, True),
]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default="")
    ap.add_argument("--cfgs", default="", help="comma list of fused-dgrad tile configs to time "
                    "(route_ab.glds_cfg on the statistics rows); default: the table's choice")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    out = open(a.json, "a") if a.json else None
    for name, H, Cc, K, k, join in SHAPES:
        p = (k - 1) // 2
        g = C.ConvGeom((1, 1), (p, p, p, p), (1, 1))
        x = (torch.randn(a.n, H, H, Cc, device=dev) * 1.5 + 0.3).to(torch.bfloat16)  # BN input
        w = (torch.randn(K, k, k, Cc, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(a.n, H, H, K, device=dev, dtype=torch.bfloat16)
        stats = B.bn_stats(x)
        gam = torch.rand(Cc, device=dev) + 0.5
        bet = torch.randn(Cc, device=dev) * 0.2
        coef = B.bn_finalize(stats, x.numel() // Cc, gam, bet, torch.zeros(Cc, device=dev),
                             torch.ones(Cc, device=dev), 0.9, 1e-5, True)
        mask = torch.empty(x.numel() // 8, device=dev, dtype=torch.uint8)
        y = B.bn_apply(x, coef, None, True, mask=mask)  # writes the ReLU bit mask
        prev = torch.randn_like(x) if join else None
        buf = torch.empty_like(x)

        def run_a():
            if join:
                buf.copy_(prev)
                dx = C.conv_dgrad(dy, w, x.shape, g, out=buf, accumulate=True, mask=mask)
                return dx, B.bn_bwd_reduce(dx, None, x, coef, 0)
            dx = C.conv_dgrad(dy, w, x.shape, g)
            return dx, B.bn_bwd_reduce(dx, y, x, coef, 2)

        def run_b():
            if join:
                buf.copy_(prev)
                return C.conv_dgrad_bnstat(dy, w, x.shape, g, x, out=buf, accumulate=True,
                                           mask=mask)
            return C.conv_dgrad_bnstat(dy, w, x.shape, g, x, mask=mask)

        dxa, reda = run_a()
        dxa = dxa.clone()
        reda = reda.clone()
        dxb, redb = run_b()
        fused = redb is not None
        err = {}
        if fused:
            s1 = coef[3] * (redb[1] - coef[2] * redb[0])
            ga = B._relu_mask(2, y, x, coef, Cc).reshape(dxa.shape) if not join else None
            dxa_m = dxa.float() * ga if ga is not None else dxa.float()
            err = dict(dx=float((dxb.float() - dxa_m).abs().max()),
                       s0=float((redb[0] - reda[0]).abs().max() / (reda[0].abs().max() + 1e-6)),
                       s1=float((s1 - reda[1]).abs().max() / (reda[1].abs().max() + 1e-6)))
        copy_us = timeit(lambda: buf.copy_(prev), a.iters) if join else 0.0
        cfgs = [c for c in a.cfgs.split(",") if c] or [None]
        ta, tb = 0.0, {c: 0.0 for c in cfgs}
        for _ in range(3):  # interleaved
            ta += timeit(run_a, a.iters)
            for c in cfgs:
                glds_cfg("dgrad", c, RF_STATS | (RF_JOIN if join else 0))
                tb[c] += timeit(run_b, a.iters)
        glds_cfg("dgrad", None, RF_STATS)
        ta = ta / 3 - copy_us
        tb = {c: v / 3 - copy_us for c, v in tb.items()}
        best = min(tb, key=tb.get)
        rec = dict(shape=name, n=a.n, fused=fused, a_us=round(ta, 1),
                   b_us={str(c): round(v, 1) for c, v in tb.items()}, best=str(best),
                   gain=round(1 - tb[best] / ta, 3), **{k_: round(v, 5) for k_, v in err.items()})
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
