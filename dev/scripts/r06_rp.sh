# LDS-staged row pack: exactness test + same-box A/B (TDL_ROWPACK_LDS)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "row_pack" > gpurun_out/r06_rp.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_rp.log | tail -3
for v in 1 0 1 0; do
TDL_ROWPACK_LDS=$v timeout -k 10 300 python bench.py > gpurun_out/r06_rp_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_rp_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rowpack_lds $v bench', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rp -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_rp.log 2>&1 || exit $?
grep -h "row_pack" $R/gpurun_out/prof_rp/*stats.csv $R/gpurun_out/prof_rp/*/*stats.csv 2>/dev/null | head -3
