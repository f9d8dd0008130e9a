# Serial kernel profiles, TDL_BNSTAT_FUSE=1 (joins fuse the BN-backward sums) vs 2 (default)
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for v in 1 2; do
TDL_BNSTAT_FUSE=$v TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_js$v -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_js$v.log 2>&1 || exit $?
(cd $R && python3 tools/prof_summary.py gpurun_out/prof_js$v/run_kernel_trace.csv --steps 3 --top 30 > gpurun_out/prof_js${v}_summary.txt 2>&1)
head -25 $R/gpurun_out/prof_js${v}_summary.txt
done
