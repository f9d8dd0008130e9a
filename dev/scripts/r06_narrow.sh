# Narrow 3x3 route rows (dgrad.asfwd.glds.n32, fwd.glds.narrow3x3): route tests + Xception A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py > gpurun_out/r06_narrow.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR" gpurun_out/r06_narrow.log | head; tail -1 gpurun_out/r06_narrow.log
timeout -k 10 200 python dev/tools/dgrad_rows.py --op fwd --shape 128,299,8,32,3,2,1 --stats 2>&1 | grep -v amdgpu.ids | grep -v " -  (" | tee gpurun_out/r06_narrow_rows.log
for v in new old new old; do
if [ $v = old ]; then export TDL_ROUTE_OFF=dgrad.asfwd.glds.n32,fwd.glds.narrow3x3; else unset TDL_ROUTE_OFF; fi
timeout -k 10 300 python bench.py --model xception41 --batch 128 --image-size 299 > gpurun_out/r06_narrow_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_narrow_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rows $v xception41 b128', d['value'], d['ms_per_step'])"
done
