#!/usr/bin/env python3
"""Interleaved A/B timing of conv kernel variants on one shape (guide §5.4 rule 24):
mode 0 (register-staged) and mode 2 (LDS-DMA) with ablation flags TDL_CONV_DBG
(1 = drop operand loads, 2 = skip MFMA, 4 = taps-fastest K order)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="256,14,512,512,3,2,1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--op", default="fwd")
    a = ap.parse_args()
    N, H, Cin, Cout, k, s, p = [int(v) for v in a.shape.split(",")]
    dev = torch.device("cuda")
    g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
    x = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    w = torch.randn(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16) * 0.05
    flop = 2.0 * N * g.out_hw(H, H, k, k)[0] ** 2 * Cout * Cin * k * k
    variants = [("reg", 0, 0), ("glds", 2, 0), ("glds-noload", 2, 1), ("glds-nomfma", 2, 2),
                ("nomfma-noreads", 2, 18),
                ("nomfma-nobarrier", 2, 34), ("nomfma-nodma", 2, 66), ("nomfma-nodma-noreads", 2, 82),
                ("nomfma-nodma-noreads-nobar", 2, 114), ("nodma", 2, 64), ("noreads", 2, 16)]
    res = {v[0]: [] for v in variants}
    for _ in range(a.rounds):
        for name, mode, dbg in variants:
            os.environ["TDL_CONV_DBG"] = str(dbg)
            ext().conv_set_glds_mode(mode)
            C.conv_fwd(x, w, g)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(10):
                C.conv_fwd(x, w, g)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 10 * 1e3)
    print(a.shape, " ".join(f"{n}={min(v):.1f}us({flop / min(v) / 1e6:.0f}TF)" for n, v in res.items()),
          flush=True)


if __name__ == "__main__":
    main()
