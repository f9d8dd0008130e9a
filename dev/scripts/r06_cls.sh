# Strided dgrad parity classes on concurrent streams (TDL_DGRAD_CLS_STREAMS=1): exactness + A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TDL_DGRAD_CLS_STREAMS=1 timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py tests/test_train_gpu.py -k "strided or every_route or capture or graph" > gpurun_out/r06_cls.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR" gpurun_out/r06_cls.log | head; tail -1 gpurun_out/r06_cls.log
for v in 1 0 1 0; do
TDL_DGRAD_CLS_STREAMS=$v timeout -k 10 300 python bench.py --steps 40 > gpurun_out/r06_cls_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_cls_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cls_streams $v bench', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
TDL_DGRAD_CLS_STREAMS=$v TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_cls$v -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_cls$v.log 2>&1 || exit $?
(cd $R && python3 tools/prof_summary.py gpurun_out/prof_cls$v/run_kernel_trace.csv --steps 3 --top 5 > gpurun_out/prof_cls${v}_summary.txt 2>&1; head -1 gpurun_out/prof_cls${v}_summary.txt)
done
