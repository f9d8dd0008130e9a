# Xception-41 b128: 1x1 dgrads <= 128 wide from <= 128 channels on the GEMM (row dgrad.gemm.n128) A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for v in new old new old; do
if [ $v = old ]; then export TDL_ROUTE_OFF=dgrad.gemm.n128; else unset TDL_ROUTE_OFF; fi
timeout -k 10 300 python bench.py --model xception41 --batch 128 --image-size 299 --steps 30 > gpurun_out/r06_xg_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_xg_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gemm_n128 $v xception41 b128', d['value'], d['ms_per_step'])"
done
unset TDL_ROUTE_OFF
timeout -k 10 300 python bench.py --steps 30 > gpurun_out/r06_xg_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_xg_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('resnet50 with the row', d['value'], d['ms_per_step'])"
