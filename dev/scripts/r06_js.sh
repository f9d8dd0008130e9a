# Residual-join BN-backward sums on the 256x128 tiles: route tests + same-box A/B of TDL_BNSTAT_FUSE
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py -k "join or every_route_row_runs" > gpurun_out/r06_js.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_js.log | tail -5
for v in 1 2 1 2; do
TDL_BNSTAT_FUSE=$v timeout -k 10 300 python bench.py > gpurun_out/r06_js_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_js_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bnstat_fuse $v bench', d['value'], d['ms_per_step'])"
done
