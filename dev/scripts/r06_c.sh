# graph-vs-eager diagnosis, DP equality + deterministic graph tests, fused stem BN+pool test and
# same-box A/B, resident-filter conv counters
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "bn_relu_max_pool or maxpool or batchnorm" > gpurun_out/r06_stem_tests.log 2>&1
echo "stem tests rc=$?"; grep -E "passed|failed|Error" gpurun_out/r06_stem_tests.log | tail -5
timeout -k 10 300 python bench.py > gpurun_out/r06_stem_on.log 2>&1 || exit $?
TDL_STEM_POOL_FUSE=0 timeout -k 10 300 python bench.py > gpurun_out/r06_stem_off.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r06_stem_on2.log 2>&1 || exit $?
for f in on off on2; do tail -1 gpurun_out/r06_stem_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stem fuse $f', d['value'], d['ms_per_step'])"; done
timeout -k 10 300 python dev/tools/graph_diag.py > gpurun_out/r06_gdiag.txt 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/r06_gdiag.txt
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_train_gpu.py::test_two_ranks_equal_single_process_average \
  tests/test_model_classifier.py::test_model_graph_training_tracks_eager > gpurun_out/r06_misc_tests.log 2>&1
echo "misc tests rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r06_misc_tests.log | head -20
bash dev/scripts/pmc_rw.sh
