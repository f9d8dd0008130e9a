# Row wgrad.halo.c64 (56x56x64 3x3 weight gradients on the halo kernel): route tests + same-box A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py > gpurun_out/r06_c64.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/r06_c64.log
for v in new old new old new old; do
if [ $v = old ]; then export TDL_ROUTE_OFF=wgrad.halo.c64; else unset TDL_ROUTE_OFF; fi
timeout -k 10 300 python bench.py --steps 30 > gpurun_out/r06_c64_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_c64_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c64 $v bench', d['value'], d['ms_per_step'])"
done
