# fixes re-test, serial-stream profile of the current build, ResNet-152 fp8 vs bf16 at b512 (graph)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_train_gpu.py -k "large_batch" tests/test_kernels_gpu.py -k "bn_relu_max_pool or large_batch" > gpurun_out/r06_e.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_e.log | tail -5
bash dev/scripts/prof_r05g.sh || exit $?
head -40 gpurun_out/prof_g_summary.txt
cd $R
for m in "--fp8" ""; do
  timeout -k 10 400 python bench.py --model resnet152 --batch 512 --graph --steps 10 --warmup 3 $m > gpurun_out/r06_r152.log 2>&1 || exit $?
  tail -1 gpurun_out/r06_r152.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('r152 b512 $m', d['value'], d['ms_per_step'], d['dtype'])"
done
