#!/usr/bin/env python3
"""Report scratch use and register spills of the conv kernels (hipcc kernel-resource-usage
remarks, and the scratch instructions actually present in the code) — a spill inside the LDS-DMA
kernel's K-step loop adds VMEM ops that force vmcnt drains of the operand ring, so the default
instantiations must execute none.  (A ScratchSize without any scratch instruction is a reserved
frame the optimiser emptied.)

  python tools/check_spills.py [--all]     (exit 1 if a default conv kernel executes scratch ops)"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the instantiations the default selection runs (mode, tile, waves, stages, STATS, BIAS, FK, FP8)
DEFAULT = [r"ILi0ELi256ELi128ELi4ELi2ELi3ELb[01]ELb[01]ELi1ELb0E", r"ILi1ELi256ELi128ELi4ELi2ELi3ELb0ELb0ELi1ELb0E", r"ILi1ELi128ELi128ELi4ELi2ELi4ELb1E", r"ILi1ELi256ELi128ELi4ELi2ELi3ELb1ELb0ELi1ELb0ELb1E",
           r"ILi2ELi256ELi128ELi4ELi2ELi3ELb0ELb0ELi1ELb0E", r"ILi[01]ELi256ELi64ELi8ELi1ELi3E",
           r"ILi[01]ELi256ELi128ELi4ELi2ELi3ELb[01]ELb0ELi1ELb1E"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--all", action="store_true", help="list every kernel with a spill")
    a = ap.parse_args()
    bad = False
    for src in ("conv_glds.hip", "conv_gemm.hip", "conv_pc.hip", "conv_halo.hip", "dwconv.hip"):
        with tempfile.TemporaryDirectory() as td:
            r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                                "-I" + os.path.join(ROOT, "csrc"), "-I" + os.path.join(ROOT, "csrc", "kernels"),
                                "-c", os.path.join(ROOT, "csrc", "kernels", src),
                                "-o", os.path.join(td, "k.o"), "-Rpass-analysis=kernel-resource-usage",
                                "--save-temps"], capture_output=True, text=True, cwd=td)
            asm = ""
            for f in os.listdir(td):
                if f.endswith("gfx950.s"):
                    asm = open(os.path.join(td, f)).read()

        def scratch_ops(kname):
            i = asm.find("\n" + kname + ":")
            if i < 0:
                return -1
            body = asm[i:asm.find(".Lfunc_end", i)]
            return sum(1 for l in body.splitlines() if "scratch_" in l or "s[0:3], 0 offen" in l)
        cur = None
        for line in r.stderr.splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = m.group(1)
                continue
            m = re.search(r"(ScratchSize \[bytes/lane\]|VGPRs Spill|SGPRs Spill): (\d+)", line)
            if m and cur and int(m.group(2)) > 0:
                default = "glds" in cur and any(re.search(p, cur) for p in DEFAULT)
                note = ""
                if m.group(1) == "ScratchSize [bytes/lane]":
                    n = scratch_ops(cur)
                    note = f" ({n} scratch instructions)"
                    if default and n != 0:
                        bad = True
                elif m.group(1) == "VGPRs Spill" and default:
                    bad = True
                if a.all or default:
                    print(f"{'DEFAULT ' if default else ''}{cur[:150]}: {m.group(1)} {m.group(2)}{note}")
    print("scratch in a default conv kernel" if bad else "default conv kernels: no scratch")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
