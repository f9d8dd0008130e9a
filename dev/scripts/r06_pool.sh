# Stem pool kernels with all window loads issued up front: pool tests + bench + kernel profile
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "pool or row_pack" > gpurun_out/r06_pool.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_pool.log | tail -3
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/r06_pool_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_pool_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_pool -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_pool.log 2>&1 || exit $?
grep -h -E "pool|row_pack" $R/gpurun_out/prof_pool/*stats.csv $R/gpurun_out/prof_pool/*/*stats.csv 2>/dev/null | cut -c1-200
