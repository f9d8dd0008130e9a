#!/usr/bin/env python3
"""Per-step kernel summary of the last N training steps from a rocprofv3 rocpd database (the
default output format): kernels per queue with time and count per step, and a list of every
kernel that is not one of ours (namespace tdl::).
python tools/rocpd_step.py gpurun_out/prof_dl/dl_results.db --steps 5 --marker adam_kernel"""
import argparse
import collections
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    qcol = "queue_id" if "queue_id" in cols else ("queue" if "queue" in cols else None)
    rows = c.execute(f"select name, start, end, {qcol or 0} from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(idx) < a.steps + 1:
        raise SystemExit(f"only {len(idx)} '{a.marker}' launches")
    seg = rows[idx[-a.steps - 1] + 1: idx[-1] + 1]
    k = a.steps
    t0, t1 = seg[0][1], seg[-1][2]
    by = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0]))
    tot = collections.defaultdict(int)
    foreign = collections.defaultdict(lambda: [0, 0])
    for name, s, e, q in seg:
        n = name.replace("(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n)
        n = re.sub(r"^void ", "", n)[:100]
        by[q][n][0] += e - s
        by[q][n][1] += 1
        tot[q] += e - s
        if not n.startswith("tdl::"):
            foreign[n][0] += e - s
            foreign[n][1] += 1
    print(f"wall {(t1 - t0) / 1e6 / k:.3f} ms/step over {k} steps")
    for q in sorted(tot, key=lambda q: -tot[q]):
        print(f"queue {q}: busy {tot[q] / 1e6 / k:.3f} ms/step")
        for n, (t, cnt) in sorted(by[q].items(), key=lambda x: -x[1][0])[:a.top]:
            print(f"   {t / 1e6 / k:8.3f} {cnt / k:6.1f}  {n}")
    print("kernels not in tdl:: per step:")
    for n, (t, cnt) in sorted(foreign.items(), key=lambda x: -x[1][0]):
        print(f"   {t / 1e6 / k:8.3f} {cnt / k:6.1f}  {n}")
    if not foreign:
        print("   (none)")


if __name__ == "__main__":
    main()
