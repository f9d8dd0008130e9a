#!/usr/bin/env python3
"""Per-conv achieved TFLOP/s from a rocprofv3 kernel trace of bench.py (last training step):
forward convs are matched in forward order, dgrad/wgrad in reverse order, by kernel mode.
python tools/conv_eff.py gpurun_out/prof_r50/run_kernel_trace.csv --model resnet50 --batch 256"""
import argparse, csv, re, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def conv_list(model, batch, image):
    from tensorflowdistributedlearning_amd import models
    from tensorflowdistributedlearning_amd.models.layers import Conv2d
    if model == "deeplab_ref":
        m = models.DeepLabResNet(model_name="model", input_shape=(image, image))
        cin = 2
    else:
        m = models.build(model, num_classes=1000) if model != "xception41" else models.build(model)
        cin = 3
    out = []
    def hook(mod, inp, o):
        x = inp[0]
        y = o[0] if isinstance(o, tuple) else o
        N, H, W, C = x.shape
        _, Ho, Wo, K = y.shape
        fl = 2.0 * batch * Ho * Wo * K * C * mod.k[0] * mod.k[1]
        st = mod.stride[0] if isinstance(mod.stride, tuple) else mod.stride
        dl = mod.dilation[0]
        # minimum HBM bytes (bf16): input + output activations + weights, each touched once
        by = 2.0 * (batch * (H * W * C + Ho * Wo * K) + K * C * mod.k[0] * mod.k[1])
        # launches of its input gradient as forward convs of dy: one per parity class with taps
        g = mod._geom_cache.get((H, W))
        ncls = 1
        if g is not None and st > 1:
            from tensorflowdistributedlearning_amd.ops.conv import _classes
            ncls = sum(1 for r in _classes(st, mod.k[0], g.padding[0]) if r) * \
                sum(1 for c in _classes(st, mod.k[1], g.padding[2]) if c)
        out.append((f"{H}x{W}x{C}->{Ho}x{Wo}x{K} k{mod.k[0]} s{st}" + (f" d{dl}" if dl > 1 else ""), fl, by,
                    2.0 * batch * H * W * C, ncls))
    for mod in m.modules():
        if isinstance(mod, Conv2d):
            mod.register_forward_hook(hook)
    m.eval()
    os.environ["TDL_BN_FOLD"] = "0"  # the folded inference path bypasses Conv2d.forward (hooks)
    with torch.no_grad():
        m(torch.zeros(1, image, image, cin))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--marker", default="sgd_kernel", help="optimizer kernel delimiting steps")
    ap.add_argument("--hbm", type=float, default=5.6, help="achievable HBM TB/s")
    ap.add_argument("--mfma", type=float, default=2.3, help="achievable dense bf16 PFLOP/s")
    ap.add_argument("--fused-bytes", action="store_true",
                    help="count a fused dgrad's extra operands (BN-statistics input, residual-join "
                         "previous dx) in its minimum bytes")
    a = ap.parse_args()

    def bound_us(fl, by):
        return max(fl / (a.mfma * 1e15), by / (a.hbm * 1e12)) * 1e6
    convs = conv_list(a.model, a.batch, a.image)
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    seg = rows[idx[-2] + 1: idx[-1] + 1]
    by = {0: [], 1: [], 2: []}
    for r in seg:
        name = r["Kernel_Name"]
        mm = re.search(r"conv_(glds|gemm|halo)_kernel<(\d)", name)
        impl, mode = (mm.group(1), int(mm.group(2))) if mm else (None, None)
        if "conv_pc_kernel<" in name:  # producer/consumer forward (conv_pc.hip)
            impl, mode = "pc", 0
        elif "conv_halo_wgrad_kernel<" in name:
            impl, mode = "halo", 2
        elif "conv_rw_kernel<" in name:  # resident-filter 3x3 64->64 (first flag: DGRAD epilogue)
            impl = "rw"
            mode = 1 if re.search(r"conv_rw_kernel<\s*true", name) else 0
        # dgrad as the forward conv of dy (DEPI: the dgrad epilogue on a forward kernel)
        tp = re.search(r"conv_(glds|halo|pc)_kernel<([^>]*)>", name)
        if tp and mode == 0:
            f = [t.strip() for t in tp.group(2).split(",")]
            at = {"glds": 14, "halo": 10, "pc": 10}[tp.group(1)]
            if len(f) > at and f[at] == "true":
                mode = 1
        if impl is not None:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            # fused dgrad operands (conv_glds_kernel<1, …, STATS, …, NJ, …>): the BN-backward
            # statistics read a.bn_x and a residual join reads the previous dx — each one more
            # dx-sized tensor through HBM
            extra = 0
            tp = re.search(r"conv_glds_kernel<([^>]*)>", name)
            if mode == 1 and tp:
                f = [t.strip() for t in tp.group(1).split(",")]
                extra = (f[6] == "true") + (len(f) > 10 and f[10] == "false")
            by[mode].append((d, impl, extra))
    print(f"{len(convs)} convs; kernels fwd {len(by[0])} dgrad {len(by[1])} wgrad {len(by[2])}")
    fw = by[0]
    tot = {}
    # forward in forward order; dgrad (no stem: its input is the image) and wgrad in reverse
    lists = {0: convs, 1: [c for c in convs[1:]][::-1], 2: convs[::-1]}
    grand = [0.0, 0.0]
    # a dgrad that ran as forward convs is one launch per parity class: merge them
    ks1, i = [], 0
    for c in lists[1]:
        if i < len(by[1]):
            n = 1 if by[1][i][1] == "gemm" or c[4] == 1 else c[4]
            grp = by[1][i:i + n]
            ks1.append((sum(g[0] for g in grp), grp[0][1] + (f"/{n}" if n > 1 else ""), grp[0][2]))
            i += n
    if i == len(by[1]):
        by[1] = ks1
    for mode, nm in ((0, "forward"), (1, "dgrad"), (2, "wgrad")):
        ks, cl = by[mode], lists[mode]
        if len(ks) != len(cl):
            agg = {}
            for d, impl, _ in ks:
                e = agg.setdefault(impl, [0, 0.0])
                e[0] += 1
                e[1] += d
            print(f"{nm}: count mismatch ({len(ks)} kernels, {len(cl)} convs): " +
                  ", ".join(f"{impl} x{n} {d:.1f} us" for impl, (n, d) in sorted(agg.items())))
            continue
        print(f"{nm}:  (bound = max(FLOP / {a.mfma} PF, min bytes / {a.hbm} TB/s))")
        agg = {}
        for (d, impl, extra), (name, fl, bts, dxb, _) in zip(ks, cl):
            if a.fused_bytes:
                bts = bts + extra * dxb
            e = agg.setdefault((name, impl), [0, 0.0, fl, bts])
            e[0] += 1
            e[1] += d
        tot = [0.0, 0.0]
        for (name, impl), (n, d, fl, bts) in sorted(agg.items(), key=lambda x: -x[1][1]):
            b = bound_us(fl, bts)
            tot[0] += d
            tot[1] += b * n
            print(f"  {name:32s} {impl:7s} x{n:2d} {d / n:7.1f} us  {fl / (d / n) / 1e6:7.1f} TF/s "
                  f"{bts / (d / n) / 1e6:5.2f} TB/s  bound {b:6.1f} us ({b / (d / n) * 100:3.0f} %)  total {d:7.1f} us")
        print(f"  sum {tot[0] / 1e3:.2f} ms, bound {tot[1] / 1e3:.2f} ms ({tot[1] / tot[0] * 100:.0f} %)")
        grand[0] += tot[0]
        grand[1] += tot[1]
    if grand[0]:
        print(f"all matched convs: {grand[0] / 1e3:.2f} ms vs bound {grand[1] / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
