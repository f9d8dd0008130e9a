"""Microbenchmark of the BN kernels at ResNet-152 shapes (batch 128): GB/s per kernel."""
import sys, torch
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tensorflowdistributedlearning_amd.ops import bn as B

def t(fn, it=50):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3

dev = "cuda"
for (hw, C) in [(14, 256), (14, 1024), (7, 512), (56, 64), (28, 512), (56, 256)]:
    M = 128 * hw * hw
    x = torch.randn(M, C, device=dev).bfloat16()
    dy = torch.randn(M, C, device=dev).bfloat16()
    coef = torch.stack([torch.rand(C) + .5, torch.randn(C), torch.randn(C) * .1, torch.rand(C) + .5]).to(dev)
    gam = torch.ones(C, device=dev)
    y = B.bn_apply(x, coef, None, True)
    red = B.bn_bwd_reduce(dy, None, x, coef, 2)
    mb = M * C * 2 / 1e6
    ta = t(lambda: B.bn_apply(x, coef, None, True))
    tr = t(lambda: B.bn_bwd_reduce(dy, None, x, coef, 2))
    tb = t(lambda: B.bn_bwd_apply(dy, None, x, coef, red, gam, M, 2, False))
    tr1 = t(lambda: B.bn_bwd_reduce(dy, y, x, coef, 1))
    tb1 = t(lambda: B.bn_bwd_apply(dy, y, x, coef, red, gam, M, 1, True))
    print(f"M={M:8d} C={C:5d} {mb:7.1f}MB/tensor apply {ta:6.1f}us ({2*mb/ta:5.2f}TB/s) "
          f"reduce2 {tr:6.1f}us ({2*mb/tr:5.2f}) bwd2 {tb:6.1f}us ({3*mb/tb:5.2f}) "
          f"reduce1 {tr1:6.1f}us ({3*mb/tr1:5.2f}) bwd1 {tb1:6.1f}us ({5*mb/tb1:5.2f})", flush=True)
