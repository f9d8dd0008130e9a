# Xception-41 b128 and the DeepLab preset on the current build: bench + serial kernel profile of Xception
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model xception41 --batch 128 --image-size 299 > gpurun_out/r06_x_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_x_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('xception41 b128', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --model deeplab_ref --batch 32 --graph > gpurun_out/r06_dl_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_dl_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('deeplab b32 graph', d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_x -o run -- python3 $R/bench.py --model xception41 --batch 128 --image-size 299 --steps 5 --warmup 3 > $R/gpurun_out/prof_x.log 2>&1 || exit $?
cd $R && python3 tools/prof_summary.py gpurun_out/prof_x/run_kernel_trace.csv --steps 5 --top 40 > gpurun_out/prof_x_summary.txt 2>&1
head -45 gpurun_out/prof_x_summary.txt
