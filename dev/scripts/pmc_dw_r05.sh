# LDS bank-conflict counters of the depthwise tile kernels (dev/tools/dw_micro.py), one pass
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_dw -o run -- python3 $R/dev/tools/dw_micro.py > $R/gpurun_out/pmc_dw.log 2>&1 || exit $?
cd $R && python3 - <<'PY' > gpurun_out/pmc_dw_summary.txt
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_dw/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.Counter())
for fn in f:
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"][:90]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        agg[k]["_n"] += 0
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_LDS_IDX_ACTIVE"]):
    act = c["SQ_LDS_IDX_ACTIVE"] or 1
    print(f"{c['SQ_LDS_BANK_CONFLICT'] / act * 100:6.1f}% conflict  idx_active {act:.3g}  lds_insts {c['SQ_INSTS_LDS']:.3g}  {k}")
PY
