# BN finalize folded into the apply pass: BN / stem / training tests + ResNet-50 same-box A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py tests/test_train_gpu.py -k "bn or max_pool or train or finalize" > gpurun_out/r06_fin.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR" gpurun_out/r06_fin.log | head; tail -1 gpurun_out/r06_fin.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
for v in 1 0 1 0; do
TDL_BN_FIN_FOLD=$v timeout -k 10 300 python bench.py --steps 40 > gpurun_out/r06_fin_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_fin_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fin_fold $v bench', d['value'], d['ms_per_step'])"
done
