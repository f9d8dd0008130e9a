R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python dev/tools/graph_diag.py > gpurun_out/r06_gdiag.txt 2>&1; echo rc=$?
cat gpurun_out/r06_gdiag.txt | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_train_gpu.py::test_two_ranks_equal_single_process_average \
  tests/test_model_classifier.py::test_model_graph_training_tracks_eager > gpurun_out/r06_misc_tests.log 2>&1
echo "misc tests rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r06_misc_tests.log | head -20
bash dev/scripts/pmc_rw.sh
