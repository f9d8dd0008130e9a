"""BN apply / backward-apply bandwidth vs channel count at a fixed tensor size: do the per-thread
coefficient loads (every thread reads its channel vector's rows from the same few cache lines)
cost anything at small C?  python dev/tools/bn_hot.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from tensorflowdistributedlearning_amd.ops import bn as B  # noqa: E402


def timed(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


def main():
    dev = torch.device("cuda")
    n = 1 << 29  # elements (1 GiB bf16)
    for C in (64, 128, 256, 512, 1024, 2048):
        x = torch.randn(n // C, C, device=dev).bfloat16()
        dy = torch.randn_like(x)
        coef = torch.rand(4, C, device=dev) + 0.5
        red = torch.randn(2, C, device=dev)
        g = torch.rand(C, device=dev) + 0.5
        ta = timed(lambda: B.bn_apply(x, coef, None, True))
        tb = timed(lambda: B.bn_bwd_apply(dy, None, x, coef, red, g, n // C, 0, False))
        print(f"C={C:5d}  apply {ta:7.1f} us {2 * 2 * n / ta / 1e6:5.2f} TB/s   "
              f"bwd_apply {tb:7.1f} us {3 * 2 * n / tb / 1e6:5.2f} TB/s", flush=True)
        del x, dy


if __name__ == "__main__":
    main()
