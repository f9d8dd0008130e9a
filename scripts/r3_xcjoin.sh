# round 3: GPU suite, fp32 preset bench, Xception join A/B + kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest.log 2>&1; echo "pytest rc=$?"
tail -2 gpurun_out/pytest.log
timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --steps 30 --warmup 5 > gpurun_out/dlf32_eager.log 2>&1 || exit $?
tail -1 gpurun_out/dlf32_eager.log
TDL_F32_BM64=0 timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --steps 30 --warmup 5 > gpurun_out/dlf32_nobm64.log 2>&1 || exit $?
tail -1 gpurun_out/dlf32_nobm64.log
for v in 1 0 1 0; do
  TDL_XC_JOIN=$v timeout -k 10 300 python bench.py --model xception41 --image-size 299 --batch 128 --steps 20 --warmup 5 > gpurun_out/xc_$v.log 2>&1 || exit $?
  echo "xc join=$v $(tail -1 gpurun_out/xc_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_xc -o run -- \
  python3 $R/bench.py --model xception41 --image-size 299 --batch 64 --steps 3 --warmup 3 > $R/gpurun_out/prof_xc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dlf32 -o run -- \
  python3 $R/bench.py --model deeplab_ref --dtype fp32 --steps 5 --warmup 3 > $R/gpurun_out/prof_dlf32.log 2>&1 || exit $?
cd $R
python3 tools/prof_summary.py gpurun_out/prof_xc/run_kernel_trace.csv --steps 3 > gpurun_out/prof_xc_summary.txt 2>&1
python3 tools/prof_summary.py gpurun_out/prof_dlf32/run_kernel_trace.csv --steps 5 --marker adam_kernel > gpurun_out/prof_dlf32_summary.txt 2>&1
echo done
