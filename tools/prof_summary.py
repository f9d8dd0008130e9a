#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py: per-step wall time, kernel-busy time, host
gaps and the per-kernel breakdown of the last `--steps` training steps (steps are delimited by the
optimizer kernel).  python tools/prof_summary.py gpurun_out/prof4/run_kernel_trace.csv --steps 5"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    seg = rows[idx[-a.steps - 1] + 1: idx[-1] + 1]
    k = a.steps
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    print(f"wall {(t1 - t0) / 1e6 / k:.2f} ms/step, kernel busy {busy / 1e6 / k:.2f} ms/step, "
          f"{len(seg) / k:.0f} kernels/step")
    agg = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n)
        n = re.sub(r"^void ", "", n)[:100]
        agg[n][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[n][1] += 1
    print("ms/step  calls/step  kernel")
    for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:a.top]:
        print(f"{t / 1e6 / k:7.3f} {c / k:6.1f}  {n}")
    gaps = [int(seg[i + 1]["Start_Timestamp"]) - int(seg[i]["End_Timestamp"]) for i in range(len(seg) - 1)]
    print(f"idle between kernels {sum(g for g in gaps if g > 0) / 1e6 / k:.2f} ms/step "
          f"({sum(1 for g in gaps if g > 5000) / k:.0f} gaps > 5 us per step)")
    # With the side (wgrad) stream, launch-order gaps overstate idleness: report the time no
    # stream has a kernel running, and the kernel transitions that leave the device idle.
    idle, end, prev = 0, t0, None
    trans = collections.Counter()
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > end:
            idle += s - end
            if prev is not None and s - end > 5000:
                trans[(prev, _short(r["Kernel_Name"]))] += s - end
        if e > end:
            end, prev = e, _short(r["Kernel_Name"])
    print(f"device idle (no stream busy) {idle / 1e6 / k:.2f} ms/step; largest idle transitions:")
    for (p, n), t in trans.most_common(5):
        print(f"  {t / 1e3 / k:7.1f} us/step  {p} -> {n}")


def _short(name):
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    return re.sub(r"^void ", "", n)[:60]


if __name__ == "__main__":
    main()
