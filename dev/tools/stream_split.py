#!/usr/bin/env python3
"""Per-stream kernel time of the last N training steps of a rocprofv3 kernel trace: which kernels
sit on the compute stream (the critical path) and which on the side (weight-gradient) stream.
python dev/tools/stream_split.py gpurun_out/prof_x/run_kernel_trace.csv --steps 5"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    seg = rows[idx[-a.steps - 1] + 1: idx[-1] + 1]
    k = a.steps
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    by = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0]))
    tot = collections.defaultdict(int)
    for r in seg:
        q = r["Queue_Id"]
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n)
        n = re.sub(r"^void ", "", n)[:90]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        by[q][n][0] += d
        by[q][n][1] += 1
        tot[q] += d
    print(f"wall {(t1 - t0) / 1e6 / k:.2f} ms/step")
    for q in sorted(tot, key=lambda q: -tot[q]):
        print(f"queue {q}: busy {tot[q] / 1e6 / k:.2f} ms/step")
        for n, (t, c) in sorted(by[q].items(), key=lambda x: -x[1][0])[:a.top]:
            print(f"   {t / 1e6 / k:7.3f} {c / k:6.1f}  {n}")


if __name__ == "__main__":
    main()
