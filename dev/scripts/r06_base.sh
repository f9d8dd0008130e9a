# round-6 baseline on one box: smoke-oracle gap by shape, the new capture / graph tests, headline
# bench, hipBLASLt GEMM yardstick at the b1024 conv shapes, serial-stream kernel trace + per-conv
# efficiency of the current build
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python dev/tools/smoke_oracle_gap.py > gpurun_out/r06_gap.log 2>&1 || exit $?
grep "logits cos" gpurun_out/r06_gap.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_train_gpu.py::test_capture_after_one_warmup_matches_eager tests/test_model_classifier.py::test_model_graph_training_tracks_eager > gpurun_out/r06_tests.log 2>&1
echo "tests rc=$?"; tail -5 gpurun_out/r06_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r06_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_bench.log
timeout -k 10 300 python dev/tools/gemm_yardstick.py --batch 1024 > gpurun_out/r06_yardstick.txt 2>&1 || exit $?
cat gpurun_out/r06_yardstick.txt
bash dev/scripts/prof_r05g.sh || exit $?
head -3 gpurun_out/prof_g_summary.txt
