#!/usr/bin/env python3
"""Row-packed 7x7 stem (7x1 conv over [N, 224, 112, 24], 24 -> 64, stride (2, 1)) under the conv
kernel selections: register-staged (mode 0), default (1), LDS-DMA forced (2) with tile configs.
python dev/tools/stem_ab.py --batch 1024"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "bench"))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402
from route_ab import glds_cfg  # noqa: E402
from conv_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    t = torch.randn(N, 224, 112, 24, device=dev, dtype=torch.bfloat16)
    w = torch.randn(64, 7, 1, 24, device=dev, dtype=torch.bfloat16) * 0.05
    g = C.ConvGeom((2, 1), (3, 3, 0, 0), (1, 1))
    Ho, Wo = g.out_hw(224, 112, 7, 1)
    dy = torch.randn(N, Ho, Wo, 64, device=dev, dtype=torch.bfloat16)
    st = torch.zeros(2, 64, device=dev)
    flop = 2.0 * N * Ho * Wo * 64 * 147
    x = torch.randn(N, 224, 224, 8, device=dev, dtype=torch.bfloat16)
    tp = timeit(lambda: C.row_pack(x, 3, 7, 2, 3, 112, 24))
    print(f"row_pack {tp:.1f} us  ({(x.numel() + t.numel()) * 2 / tp / 1e6:.2f} TB/s)")
    ref = None
    for mode, cfgs in ((0, [None]), (1, [None]), (2, ["1", "4", "5"])):
        for cfg in cfgs:
            ext().conv_set_glds_mode(mode)
            if cfg:
                glds_cfg("fwd", cfg)
            y = C.conv_fwd(t, w, g)
            if ref is None:
                ref = y.float()
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            tf = timeit(lambda: C.conv_fwd(t, w, g, stats=st))
            tw = timeit(lambda: C.conv_wgrad(dy, t, tuple(w.shape), g))
            print(f"mode {mode} cfg {cfg}: fwd {tf:7.1f} us ({flop / tf / 1e6:4.0f} TF, "
                  f"{(t.numel() + y.numel()) * 2 / tf / 1e6:.2f} TB/s min-bytes) wgrad {tw:7.1f} us "
                  f"({flop / tw / 1e6:4.0f} TF)  err {err:.2e}", flush=True)
            glds_cfg("fwd", None)
    ext().conv_set_glds_mode(-1)
    # weight gradient: register-staged 64x128 tiles (dy read twice) vs the LDS-DMA 64x256 tile
    for v in ("0", "1", "0", "1"):
        ext().conv_route_set("wgrad.glds.stem", on=int(v))
        dw = C.conv_wgrad(dy, t, tuple(w.shape), g)
        tw = timeit(lambda: C.conv_wgrad(dy, t, tuple(w.shape), g))
        if v == "0":
            dw0 = dw.float()
        err = ((dw.float() - dw0).abs().max() / dw0.abs().max()).item()
        print(f"stem wgrad wgrad.glds.stem on={v}: {tw:7.1f} us ({flop / tw / 1e6:4.0f} TF) "
              f"err vs register-staged {err:.2e}", flush=True)
    ext().conv_route_reset()


if __name__ == "__main__":
    main()
