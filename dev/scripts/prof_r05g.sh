# serial-stream kernel trace of the ResNet-50 b1024 bench (current build) + per-conv efficiency
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_g -o run -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/prof_g.log 2>&1 || exit $?
cd $R && python3 tools/prof_summary.py $(ls gpurun_out/prof_g/*/run_kernel_trace.csv gpurun_out/prof_g/run_kernel_trace.csv 2>/dev/null | head -1) --steps 5 --top 45 > gpurun_out/prof_g_summary.txt 2>&1 || exit $?
python3 tools/conv_eff.py $(ls gpurun_out/prof_g/*/run_kernel_trace.csv gpurun_out/prof_g/run_kernel_trace.csv 2>/dev/null | head -1) --model resnet50 --batch 1024 > gpurun_out/prof_g_conv.txt 2>&1
