#!/usr/bin/env python3
"""How well the side-stream weight gradients hide behind the compute stream: two rocprofv3 kernel
traces of the same bench configuration on one box — serial (TDL_WGRAD_STREAM=0) and concurrent
(the default) — matched kernel by kernel in launch order over the last training step.

Reports the step wall time of both, per kernel class the serial time, the concurrent time and the
stretch, how much of the side-stream time ran beside each compute-stream class, and the largest
individual stretches.  Kernel classes: bn_fwd (apply), bn_bwd (backward apply), bn_red (reduce
passes), conv_fwd, conv_dgrad, conv_wgrad (by kernel mode and stream), other.

  python tools/overlap_report.py SERIAL.csv CONCURRENT.csv [--marker sgd_kernel]
"""
import argparse
import collections
import csv
import re


def load_step(path, marker):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))  # launch order
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    seg = rows[idx[-2] + 1: idx[-1] + 1]
    out = []
    for r in seg:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n)
        out.append(dict(name=re.sub(r"^void ", "", n), stream=r["Stream_Id"],
                        t0=int(r["Start_Timestamp"]), t1=int(r["End_Timestamp"])))
    return out


def klass(name, side):
    if "bwd_apply" in name:
        return "bn_bwd"
    if "apply_vec" in name:
        return "bn_fwd"
    if "reduce" in name and "splitk" not in name:
        return "bn_red"
    m = re.match(r"tdl::conv_(\w+?)_kernel<(\d)", name)
    if "wgrad" in name or (m and m.group(2) == "2"):
        return "conv_wgrad"
    if m or "conv_" in name:
        # a dgrad run as the forward conv of dy is launched from the backward: the stream and
        # position tell it apart; class by the DEPI flag when visible (last template argument)
        if m and m.group(2) == "1":
            return "conv_dgrad"
        return "conv_fwd/dgrad"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("serial")
    ap.add_argument("concurrent")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    s, c = load_step(a.serial, a.marker), load_step(a.concurrent, a.marker)
    if [k["name"] for k in s] != [k["name"] for k in c]:
        raise SystemExit(f"launch sequences differ ({len(s)} vs {len(c)} kernels)")
    wall_s = max(k["t1"] for k in s) - min(k["t0"] for k in s)
    wall_c = max(k["t1"] for k in c) - min(k["t0"] for k in c)
    streams = collections.Counter(k["stream"] for k in c)
    main_stream = streams.most_common(1)[0][0]
    side_t = sum(k["t1"] - k["t0"] for k in c if k["stream"] != main_stream)
    print(f"step wall: serial {wall_s / 1e6:.2f} ms, concurrent {wall_c / 1e6:.2f} ms "
          f"(hidden {(wall_s - wall_c) / 1e6:.2f} ms of {side_t / 1e6:.2f} ms side-stream kernel time)")
    # the backward begins at the first kernel that runs on the side stream's stream, minus the
    # dgrad launched with it: report the backward window separately
    cls_s, cls_c = collections.Counter(), collections.Counter()
    for ks, kc in zip(s, c):
        side = kc["stream"] != main_stream
        key = klass(kc["name"], side) + (" (side)" if side else "")
        cls_s[key] += ks["t1"] - ks["t0"]
        cls_c[key] += kc["t1"] - kc["t0"]
    print(f"\n{'class':24s} {'serial ms':>10s} {'concurrent ms':>14s} {'stretch':>8s}")
    for key in sorted(cls_s, key=lambda k: -cls_s[k]):
        print(f"{key:24s} {cls_s[key] / 1e6:10.2f} {cls_c[key] / 1e6:14.2f} "
              f"{cls_c[key] / max(cls_s[key], 1):8.2f}x")
    # what the side-stream kernels ran beside (time-overlap with compute-stream kernels)
    beside = collections.Counter()
    alone = 0
    mains = [k for k in c if k["stream"] == main_stream]
    for k in c:
        if k["stream"] == main_stream:
            continue
        covered = 0
        for m in mains:
            ov = min(k["t1"], m["t1"]) - max(k["t0"], m["t0"])
            if ov > 0:
                beside[klass(m["name"], False)] += ov
                covered += ov
        alone += max(0, (k["t1"] - k["t0"]) - covered)
    print(f"\nside-stream kernel time beside compute-stream classes (ms): "
          + ", ".join(f"{kk} {v / 1e6:.2f}" for kk, v in beside.most_common())
          + f", alone {alone / 1e6:.2f}")
    # compute-stream idle while the side stream runs (the compute stream waits on it)
    ev = sorted([(k["t0"], 1, k["stream"] == main_stream) for k in c] +
                [(k["t1"], -1, k["stream"] == main_stream) for k in c])
    nm = ns = 0
    last = None
    only_side = 0
    for t, d, is_main in ev:
        if last is not None and nm == 0 and ns > 0:
            only_side += t - last
        if is_main:
            nm += d
        else:
            ns += d
        last = t
    print(f"time with only the side stream busy: {only_side / 1e6:.2f} ms")
    print(f"\nlargest stretches (concurrent − serial, µs):")
    rows = []
    for ks, kc in zip(s, c):
        rows.append(((kc["t1"] - kc["t0"]) - (ks["t1"] - ks["t0"]), kc, ks))
    for d, kc, ks in sorted(rows, key=lambda r: -r[0])[:a.top]:
        side = "side" if kc["stream"] != main_stream else "main"
        print(f"  {d / 1e3:8.1f}  {side}  {(ks['t1'] - ks['t0']) / 1e3:8.1f} -> "
              f"{(kc['t1'] - kc['t0']) / 1e3:8.1f}  {kc['name'][:90]}")


if __name__ == "__main__":
    main()
