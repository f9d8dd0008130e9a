# Xception-41 b128: concurrent trace + per-kernel summary; bench
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_x -o run -- python3 $R/bench.py --model xception41 --batch 128 --image-size 299 --steps 5 --warmup 3 > $R/gpurun_out/prof_x.log 2>&1 || exit $?
cd $R && python3 tools/prof_summary.py $(ls gpurun_out/prof_x/*/run_kernel_trace.csv gpurun_out/prof_x/run_kernel_trace.csv 2>/dev/null | head -1) --steps 5 --top 40 > gpurun_out/prof_x_summary.txt 2>&1
cd $R && timeout -k 10 200 python3 bench.py --model xception41 --batch 128 --image-size 299 > gpurun_out/x41.log 2>&1 && timeout -k 10 200 python3 bench.py --model xception41 --batch 128 --image-size 299 > gpurun_out/x41b.log 2>&1
