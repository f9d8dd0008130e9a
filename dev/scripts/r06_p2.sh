# 2x2-block pool backward apply: exactness (tests + dx checksum vs the per-pixel kernel), timing, A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "pool" > gpurun_out/r06_p2.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/r06_p2.log
for v in 1 0; do
TDL_POOL_APPLY2X2=$v timeout -k 10 120 python dev/tools/pool_bench.py --n 1024 --iters 10 2>&1 | grep -v amdgpu.ids | sed "s/^/2x2=$v /"
done
for v in 1 0 1 0; do
TDL_POOL_APPLY2X2=$v timeout -k 10 300 python bench.py --steps 30 > gpurun_out/r06_p2_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_p2_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('apply2x2 $v bench', d['value'], d['ms_per_step'])"
done
