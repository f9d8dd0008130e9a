# Depthwise input-gradient row operands prefetched one row ahead: dw tests + Xception A/B + profile
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "dw or depthwise or separable" > gpurun_out/r06_dwpf.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/r06_dwpf.log
for v in 1 0 1 0; do
TDL_DW_PREFETCH=$v timeout -k 10 300 python bench.py --model xception41 --batch 128 --image-size 299 > gpurun_out/r06_dwpf_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_dwpf_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dw_prefetch $v xception41 b128', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
TDL_DW_PREFETCH=$v TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_xpf$v -o run -- python3 $R/bench.py --model xception41 --batch 128 --image-size 299 --steps 3 --warmup 2 > $R/gpurun_out/prof_xpf$v.log 2>&1 || exit $?
(cd $R && python3 tools/prof_summary.py gpurun_out/prof_xpf$v/run_kernel_trace.csv --steps 3 --top 40 > gpurun_out/prof_xpf${v}_summary.txt 2>&1)
grep -E "wall|dw_" $R/gpurun_out/prof_xpf${v}_summary.txt | head -12
done
