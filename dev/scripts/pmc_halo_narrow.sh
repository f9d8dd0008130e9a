# counters of the 56x56x64 3x3 forward on the halo kernel (ResNet-50 layer1, b256)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S=256,56,64,64,3,1,1
P=$R/gpurun_out/pmch
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d ${P}_a -o run -- python3 $R/tools/conv_one.py --mode -1 --op fwd --shape $S --iters 5 > ${P}_a.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d ${P}_b -o run -- python3 $R/tools/conv_one.py --mode -1 --op fwd --shape $S --iters 5 > ${P}_b.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d ${P}_c -o run -- python3 $R/tools/conv_one.py --mode -1 --op fwd --shape $S --iters 5 > ${P}_c.log 2>&1 || exit $?
cd $R && python3 - <<'PY' > gpurun_out/pmch_summary.txt
import csv, glob, collections
for x in "abc":
    c = collections.Counter(); n = collections.Counter()
    for f in glob.glob(f"gpurun_out/pmch_{x}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv_halo_kernel" in r["Kernel_Name"]:
                c[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    for k in sorted(c):
        print(f"{x} {k:28s} {c[k] / max(n[k], 1):14.4g} per dispatch")
PY
