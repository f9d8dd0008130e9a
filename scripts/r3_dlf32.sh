# round 3: the reference preset at the reference's precision (fp32): bench (eager, graph) + kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --steps 30 --warmup 5 > gpurun_out/dlf32_eager.log 2>&1 || exit $?
tail -1 gpurun_out/dlf32_eager.log
timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --batch 32 --steps 30 --warmup 5 > gpurun_out/dlf32_b32.log 2>&1 || exit $?
tail -1 gpurun_out/dlf32_b32.log
timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --graph --steps 30 --warmup 5 > gpurun_out/dlf32_graph.log 2>&1 || exit $?
tail -1 gpurun_out/dlf32_graph.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dlf32 -o run -- \
  python3 $R/bench.py --model deeplab_ref --dtype fp32 --steps 5 --warmup 3 > $R/gpurun_out/prof_dlf32.log 2>&1 || exit $?
cd $R
python3 tools/prof_summary.py gpurun_out/prof_dlf32/run_kernel_trace.csv --steps 5 --marker adam_kernel > gpurun_out/prof_dlf32_summary.txt 2>&1
echo done
