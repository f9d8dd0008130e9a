# round 3: fp32 reference preset kernel trace (b64) after the tile / launch-bound changes
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dlf32b -o run -- \
  python3 $R/bench.py --model deeplab_ref --dtype fp32 --steps 5 --warmup 3 > $R/gpurun_out/prof_dlf32b.log 2>&1 || exit $?
cd $R
python3 tools/prof_summary.py gpurun_out/prof_dlf32b/run_kernel_trace.csv --steps 5 --marker adam_kernel --top 40 > gpurun_out/prof_dlf32b_summary.txt 2>&1
python3 tools/stream_split.py gpurun_out/prof_dlf32b/run_kernel_trace.csv > gpurun_out/prof_dlf32b_streams.txt 2>&1 || true
echo done
