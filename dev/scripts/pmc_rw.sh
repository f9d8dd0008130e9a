# counters of the resident-filter 3x3 64->64 conv (ResNet-50 layer1 shape, b256): forward (BN sums
# in the epilogue) and the input gradient as a forward conv (mask + BN-backward sums)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S=256,56,64,64,3,1,1
P=$R/gpurun_out/pmcrw
for op in fwd dgrad_bnstat; do
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d ${P}_${op}_a -o run -- python3 $R/tools/conv_one.py --mode -1 --op $op --shape $S --iters 5 --flip > ${P}_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d ${P}_${op}_b -o run -- python3 $R/tools/conv_one.py --mode -1 --op $op --shape $S --iters 5 --flip > ${P}_b.log 2>&1 || exit $?
done
cd $R && python3 - <<'PY' > gpurun_out/pmcrw_summary.txt
import csv, glob, collections
for op in ("fwd", "dgrad_bnstat"):
    for x in "ab":
        c = collections.Counter(); n = collections.Counter(); d = []
        for f in glob.glob(f"gpurun_out/pmcrw_{op}_{x}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "conv_rw_kernel" in r["Kernel_Name"]:
                    c[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
        for f in glob.glob(f"gpurun_out/pmcrw_{op}_{x}/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "conv_rw_kernel" in r["Kernel_Name"]:
                    d.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k in sorted(c):
            print(f"{op} {x} {k:28s} {c[k] / max(n[k], 1):14.4g} per dispatch")
        if d:
            print(f"{op} {x} conv_rw_kernel us (profiled): {[round(v, 1) for v in d]}")
    g = None
PY
cat gpurun_out/pmcrw_summary.txt
