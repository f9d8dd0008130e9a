# fused stem max-pool + BN backward (two passes, g never written): oracle test + same-box A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "bn_relu_max_pool or maxpool" > gpurun_out/r06_i.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_i.log | tail -5
for v in 1 0 1 0; do
TDL_STEM_POOL_FUSED_BWD=$v timeout -k 10 300 python bench.py > gpurun_out/r06_i_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_i_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused_bwd $v bench', d['value'], d['ms_per_step'])"
done
