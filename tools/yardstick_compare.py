#!/usr/bin/env python3
"""Per-conv time of the native kernels (tools/conv_eff.py output) next to the hipBLASLt
``torch.mm`` yardstick of the same GEMM (dev/tools/gemm_yardstick.py output, same box).

The yardstick is a plain library GEMM on pre-laid-out operands (no im2col / col2im, no fused
epilogue), so it is what the vendor library reaches on that M×N×K on this part — a practical
ceiling to read the conv kernels against, instead of the 2.5 PF marketing peak.  Stride-1 convs
only (the yardstick has no strided shapes).

  python tools/yardstick_compare.py gpurun_out/prof_g_conv.txt gpurun_out/r06_yardstick.txt
"""
import re
import sys


def parse_conv(path):
    out = {}
    sec = None
    for line in open(path):
        m = re.match(r"(forward|dgrad|wgrad):", line)
        if m:
            sec = {"forward": "fwd", "dgrad": "dgrad", "wgrad": "wgrad"}[m.group(1)]
            continue
        if line.startswith("## "):
            break  # the --fused-bytes re-listing repeats the dgrad section
        m = re.match(r"\s+(\d+)x(\d+)x(\d+)->(\d+)x(\d+)x(\d+) k(\d) s(\d)\s+(\S+)\s+x\s*(\d+)\s+([\d.]+) us\s+([\d.]+) TF/s",
                     line)
        if m and sec:
            h, w, c, ho, wo, k, taps, s = (int(m.group(i)) for i in range(1, 9))
            if s != 1:
                continue
            key = (f"{h}x{w} {taps}x{taps} {c}->{k}", sec)
            out[key] = (m.group(9), int(m.group(10)), float(m.group(11)), float(m.group(12)))
    return out


def parse_yard(path):
    out = {}
    for line in open(path):
        m = re.match(r"(\d+x\d+ \dx\d \d+->\d+)\s+(fwd|dgrad|wgrad)\s+\d+\s+\d+\s+\d+\s+([\d.]+)\s+([\d.]+)",
                     line)
        if m:
            out[(m.group(1), m.group(2))] = (float(m.group(3)), float(m.group(4)))
    return out


def main():
    conv, yard = parse_conv(sys.argv[1]), parse_yard(sys.argv[2])
    print(f"{'conv (stride 1)':24s} {'op':5s} {'kernel':7s} {'n':>2s} {'ours us':>8s} {'TF/s':>7s} "
          f"{'hipBLASLt us':>12s} {'TF/s':>7s} {'ours/lib':>8s}")
    tot_o = tot_y = 0.0
    for op in ("fwd", "dgrad", "wgrad"):
        for (name, o), (kern, n, us, tf) in sorted(conv.items(), key=lambda kv: -kv[1][2] * kv[1][1]):
            if o != op or (name, op) not in yard:
                continue
            yus, ytf = yard[(name, op)]
            tot_o += us * n
            tot_y += yus * n
            print(f"{name:24s} {op:5s} {kern:7s} {n:2d} {us:8.1f} {tf:7.1f} {yus:12.1f} {ytf:7.1f} "
                  f"{yus / us * 100:7.0f}%")
    print(f"matched convs per step: ours {tot_o / 1e3:.2f} ms, hipBLASLt same GEMMs {tot_y / 1e3:.2f} ms "
          f"(ours/lib speed {tot_y / tot_o * 100:.0f} %)")


if __name__ == "__main__":
    main()
