# Strided flipped filters rebuilt in place: strided dgrad / graph tests + profile check for copies
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_train_gpu.py tests/test_conv_route_gpu.py tests/test_model_classifier.py -k "capture or graph or strided or every_route or eager" > gpurun_out/r06_flipc.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR" gpurun_out/r06_flipc.log | head; tail -1 gpurun_out/r06_flipc.log
cd /tmp && export TMPDIR=/tmp
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_flipc -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_flipc.log 2>&1 || exit $?
cd $R && python3 tools/prof_summary.py gpurun_out/prof_flipc/run_kernel_trace.csv --steps 3 --top 60 > gpurun_out/prof_flipc_summary.txt 2>&1
head -1 gpurun_out/prof_flipc_summary.txt; grep -E "copyBuffer|at::native" gpurun_out/prof_flipc_summary.txt | cut -c1-100
cd $R
timeout -k 10 200 python dev/tools/dgrad_rows.py --shape 128,150,32,64,3,1,1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06_dgrad_rows.log
timeout -k 10 200 python dev/tools/dgrad_rows.py --shape 128,150,32,64,3,1,1 --stats 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_dgrad_rows.log
timeout -k 10 200 python dev/tools/dgrad_rows.py --op fwd --shape 128,150,32,64,3,1,1 --stats 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_dgrad_rows.log
