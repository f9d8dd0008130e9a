# halo kernel padded pitch + s&7 swizzle: numerics, then counters / durations of the 56x56x64 3x3
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "halo or dgrad_as_forward" tests/test_conv_route_gpu.py > gpurun_out/halo_tests.log 2>&1
bash dev/scripts/pmc_halo_narrow.sh
python3 - <<'PY' >> gpurun_out/pmch_summary.txt
import csv, glob
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for f in glob.glob("gpurun_out/pmch_c/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f)) if "conv_halo_kernel" in r["Kernel_Name"]]
print("conv_halo_kernel us (profiled):", [round(x / 1e3, 1) for x in d])
PY
