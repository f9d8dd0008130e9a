# serial-stream kernel trace of the ResNet-152 b256 fp8 bench step (default fp8 recipe)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_f8 -o run -- python3 $R/bench.py --model resnet152 --batch 256 --fp8 --steps 5 --warmup 3 > $R/gpurun_out/prof_f8.log 2>&1 || exit $?
cd $R && python3 tools/prof_summary.py $(ls gpurun_out/prof_f8/*/run_kernel_trace.csv gpurun_out/prof_f8/run_kernel_trace.csv 2>/dev/null | head -1) --steps 5 --top 40 > gpurun_out/prof_f8_summary.txt 2>&1
