# side-stream overlap study: serial and concurrent kernel traces of the ResNet-50 b1024 bench on one
# box (tools/overlap_report.py), the capture / deterministic graph tests, the smoke, and the smoke
# shape's oracle gap at two learning rates, twice each
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_train_gpu.py::test_capture_after_one_warmup_matches_eager tests/test_model_classifier.py::test_model_graph_training_tracks_eager > gpurun_out/r06_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r06_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r06_smoke.log
timeout -k 10 400 python dev/tools/smoke_oracle_gap.py --configs 16x96 --lr 1e-3 --repeat 2 > gpurun_out/r06_gap2.log 2>&1 || exit $?
timeout -k 10 400 python dev/tools/smoke_oracle_gap.py --configs 16x96 --lr 3e-3 --repeat 2 >> gpurun_out/r06_gap2.log 2>&1 || exit $?
grep "logits cos" gpurun_out/r06_gap2.log
cd /tmp && export TMPDIR=/tmp
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ov_s -o run -- python3 $R/bench.py --steps 3 --warmup 3 > $R/gpurun_out/ov_s.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ov_c -o run -- python3 $R/bench.py --steps 3 --warmup 3 > $R/gpurun_out/ov_c.log 2>&1 || exit $?
cd $R && python3 tools/overlap_report.py $(ls gpurun_out/ov_s/*/run_kernel_trace.csv gpurun_out/ov_s/run_kernel_trace.csv 2>/dev/null | head -1) $(ls gpurun_out/ov_c/*/run_kernel_trace.csv gpurun_out/ov_c/run_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/ov_report.txt 2>&1
cat gpurun_out/ov_report.txt
