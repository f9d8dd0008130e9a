"""Why the stem's fused pool kernels run ~3× slower inside the ResNet-50 step than stand-alone
(dev/tools/pool_bench.py): time bn_maxpool_fwd on the step's own BN input / coefficients, on a
fresh copy of that tensor (new memory, same data), and on random data in the step's tensor
(same memory, other data)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from tensorflowdistributedlearning_amd import _native, models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, pool  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ext = _native.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = models.resnet50(num_classes=1000)
    tr = Trainer(m, softmax_cross_entropy, dev, "sgd", dict(lr=0.1, momentum=0.9, weight_decay=1e-4))
    x, y = imagenet_batch(256, 224, device=dev)
    seen = {}
    orig = ext.bn_maxpool_fwd

    class Spy:
        def __getattr__(self, k):
            return getattr(ext, k)

        def bn_maxpool_fwd(self, z, coef, yy, idx, *args, **kw):
            seen.update(z=z, coef=coef.clone(), y=yy, idx=idx, args=args, kw=kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = orig(z, coef, yy, idx, *args, **kw)
            e1.record()
            seen.setdefault("ev", []).append((e0, e1))
            return r

    for _ in range(2):
        tr.train_step(x, y)
    pool.ext = lambda: Spy()  # type: ignore[attr-defined]
    for _ in range(3):
        loss, _ = tr.train_step(x, y)
    torch.cuda.synchronize()
    print("in-step bn_maxpool_fwd (events):", ["%.1f" % (a.elapsed_time(b) * 1e3) for a, b in seen["ev"]],
          flush=True)
    z, coef, yy, idx = seen["z"], seen["coef"], seen["y"], seen["idx"]
    args, kw = seen["args"], seen["kw"]
    print("z", tuple(z.shape), z.stride(), z.dtype, "ptr %x" % z.data_ptr(),
          "mem alloc GB", torch.cuda.memory_allocated() / 1e9,
          "reserved GB", torch.cuda.memory_reserved() / 1e9, flush=True)
    zs = z.float()
    print("z stats: mean %.3f std %.3f zeros %.4f; coef scale mean %.3f shift mean %.3f" % (
        zs.mean(), zs.std(), (z == 0).float().mean(), coef[0].mean(), coef[1].mean()), flush=True)
    del zs
    zarg = kw.get("zarg")
    print("step tensors        %.1f us" % timed(lambda: orig(z, coef, yy, idx, *args, **kw)), flush=True)
    zc = z.clone()
    print("fresh copy of z     %.1f us" % timed(lambda: orig(zc, coef, yy, idx, *args, **kw)), flush=True)
    zr = torch.randn_like(z, dtype=torch.float32).bfloat16()
    print("random data, new    %.1f us" % timed(lambda: orig(zr, coef, yy, idx, *args, **kw)), flush=True)
    c2 = coef.clone()
    c2[0] = 1.3
    c2[1] = -0.1
    print("step z, flat coef   %.1f us" % timed(lambda: orig(z, c2, yy, idx, *args, **kw)), flush=True)
    z.copy_(zr)
    print("step memory, random %.1f us" % timed(lambda: orig(z, coef, yy, idx, *args, **kw)), flush=True)
    print("zarg", None if zarg is None else tuple(zarg.shape))

    def after(prep, fn, iters=10):
        tot = 0.0
        for _ in range(iters):
            prep()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
        return tot * 1e3 / iters

    run = lambda: orig(z, coef, yy, idx, *args, **kw)  # noqa: E731
    big = torch.empty(1 << 30, device=dev, dtype=torch.bfloat16)
    print("after z rewritten   %.1f us" % after(lambda: z.copy_(zc), run), flush=True)
    print("after other 2 GB    %.1f us" % after(lambda: big.fill_(1.0), run), flush=True)
    print("after y/idx written %.1f us" % after(lambda: (yy.fill_(0), idx.fill_(0)), run), flush=True)
    print("after nothing       %.1f us" % after(lambda: None, run), flush=True)


if __name__ == "__main__":
    main()
