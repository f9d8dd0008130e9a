# Column-grouped tiling that fits the CU slots: route tests + Xception-41 b128 same-box A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py > gpurun_out/r06_gt.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/r06_gt.log
for v in 1 0 1 0; do
TDL_GROUPED_FIT=$v timeout -k 10 300 python bench.py --model xception41 --batch 128 --image-size 299 > gpurun_out/r06_gt_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_gt_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('grouped_fit $v xception41 b128', d['value'], d['ms_per_step'])"
done
