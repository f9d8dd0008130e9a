R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py -k "wgrad" tests/test_kernels_gpu.py -k "halo or wgrad" > gpurun_out/r06_g.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_g.log | tail -5
timeout -k 10 200 python dev/tools/wgrad3_ab.py 1024 > gpurun_out/r06_wgrad3.txt 2>&1 || exit $?
grep -v amdgpu gpurun_out/r06_wgrad3.txt
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/r06_g_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_g_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])"
done
