# resident-filter dgrad with its epilogue operands preloaded under the K loop; capture test after
# the deepcopy / no-decay fix; same-box bench
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_route_gpu.py -k "resident or rw64" tests/test_train_gpu.py::test_capture_after_one_warmup_matches_eager > gpurun_out/r06_d_tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|Error" gpurun_out/r06_d_tests.log | tail -5
timeout -k 10 120 python dev/tools/rw_ab.py 1024 56 > gpurun_out/r06_rw_ab2.txt 2>&1 || exit $?
cat gpurun_out/r06_rw_ab2.txt | grep -v amdgpu
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/r06_d_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_d_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])"
done
