# End-of-round check: full GPU suites, smoke, bench (ResNet-50 b1024), serial kernel profile
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash dev/scripts/r06_suite1.sh || exit 1
bash dev/scripts/r06_suite2.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r06_final_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_final_bench.log
cd /tmp && export TMPDIR=/tmp
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_final -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_final.log 2>&1 || exit $?
cd $R && python3 tools/prof_summary.py gpurun_out/prof_final/run_kernel_trace.csv --steps 3 --top 40 > gpurun_out/prof_final_summary.txt 2>&1
head -3 gpurun_out/prof_final_summary.txt
