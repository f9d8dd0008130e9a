"""Depthwise 3×3 forward / dgrad at Xception-41 b128 shapes: µs and HBM-equivalent TB/s."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for (hw, c) in [(19, 728), (150, 128), (75, 256), (38, 728)]:
    x = torch.randn(128, hw, hw, c, device="cuda").bfloat16()
    w = (torch.randn(3, 3, c, device="cuda") * 0.3).bfloat16()
    y = torch.empty_like(x)
    f = lambda: ext().dwconv_fwd(x, w, None, y, 1, 1, 1, 1, 1, 1, False, False)
    d = lambda: ext().dwconv_dgrad(x, w, y, 1, 1, 1, 1, 1, 1, None)
    mb = x.numel() * 2 / 1e6
    tf, td = t(f), t(d)
    print(f"{hw}x{hw}x{c}: fwd {tf:7.1f} us ({2 * mb / tf:4.2f} TB/s)  dgrad {td:7.1f} us "
          f"({2 * mb / td:4.2f} TB/s)", flush=True)
    del x, y
