"""Per-layer forward vs dgrad conv kernel time from a rocprofv3 kernel trace of bench.py
(ResNet bottleneck order: forward [downsample] conv1 conv2 conv3 …, backward in reverse).
  python dev/tools/fwd_dgrad_pairs.py gpurun_out/prof_X/run_kernel_trace.csv"""
import csv
import re
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
    seg = rows[idx[-2] + 1: idx[-1] + 1]

    def nm(r):
        return re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", ""))

    def dur(r):
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3

    fw = [(nm(r), dur(r)) for r in seg if re.search(r"conv_(glds|gemm)_kernel<0", nm(r))]
    dg = [(nm(r), dur(r)) for r in seg if re.search(r"conv_(glds|gemm)_kernel<1", nm(r))][::-1]
    tf = td = 0.0
    for i, (f, d) in enumerate(zip(fw[1:], dg)):
        tf += f[1]
        td += d[1]
        print(f"{i:2d} fwd {f[0][5:14]} {f[1]:7.1f}  dgrad {d[0][5:14]} {d[1]:7.1f} "
              f"{'<<' if d[1] > 1.3 * f[1] else ''}")
    print(f"total fwd {tf:.0f} us  dgrad {td:.0f} us")


if __name__ == "__main__":
    main(sys.argv[1])
