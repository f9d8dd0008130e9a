# resident-filter 3x3 64->64 conv: oracle tests (new test + every route row), the capture / DP
# equality tests, the smoke, micro A/B vs the replaced rows, and a same-box ResNet-50 A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_route_gpu.py -k "resident or rw64 or halo" > gpurun_out/r06_rw_tests.log 2>&1
echo "route tests rc=$?"; tail -4 gpurun_out/r06_rw_tests.log
timeout -k 10 120 python dev/tools/rw_ab.py 1024 56 > gpurun_out/r06_rw_ab.txt 2>&1 || exit $?
cat gpurun_out/r06_rw_ab.txt
timeout -k 10 300 python bench.py > gpurun_out/r06_rw_bench_on.log 2>&1 || exit $?
TDL_ROUTE_OFF=fwd.halo.rw64,dgrad.asfwd.rw64 timeout -k 10 300 python bench.py > gpurun_out/r06_rw_bench_off.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r06_rw_bench_on2.log 2>&1 || exit $?
for f in on off on2; do tail -1 gpurun_out/r06_rw_bench_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_train_gpu.py::test_capture_after_one_warmup_matches_eager \
  tests/test_train_gpu.py::test_two_ranks_equal_single_process_average > gpurun_out/r06_misc_tests.log 2>&1
echo "misc tests rc=$?"; tail -4 gpurun_out/r06_misc_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r06_smoke.log
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for v in "TDL_WGRAD_EARLY=0" "TDL_COMPUTE_PRIO=-1" "TDL_SIDE_PRIO=1" "TDL_GLDS_WGRAD_TARGET=256"; do
  env $v timeout -k 10 300 python bench.py > gpurun_out/r06_ov_ab.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/r06_ov_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py > gpurun_out/r06_ov_ab.log 2>&1 || exit $?
echo "default $(tail -1 gpurun_out/r06_ov_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
