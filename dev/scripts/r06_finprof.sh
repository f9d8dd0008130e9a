# Serial kernel profiles with / without the folded BN finalize
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu $GRAFT_REPO_ROOT/tests/test_kernels_gpu.py -k "finalize or max_pool" > $GRAFT_REPO_ROOT/gpurun_out/r06_fin2.log 2>&1; echo "tests rc=$?"; tail -1 $GRAFT_REPO_ROOT/gpurun_out/r06_fin2.log
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
TDL_BN_FIN_FOLD=$v TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_fin$v -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_fin$v.log 2>&1 || exit $?
(cd $R && python3 tools/prof_summary.py gpurun_out/prof_fin$v/run_kernel_trace.csv --steps 3 --top 12 > gpurun_out/prof_fin${v}_summary.txt 2>&1)
head -6 $R/gpurun_out/prof_fin${v}_summary.txt; grep -E "finalize|apply_vec" $R/gpurun_out/prof_fin${v}_summary.txt
done
cd $R
for v in 1 0 1 0; do
TDL_BN_FIN_FOLD=$v timeout -k 10 300 python bench.py --steps 40 > gpurun_out/r06_fin_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_fin_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fin_fold $v bench', d['value'], d['ms_per_step'])"
done
