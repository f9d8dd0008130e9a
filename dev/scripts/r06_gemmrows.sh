# 1x1 dgrads / wgrads on the register-staged GEMM: ResNet-50 same-box A/B (route overrides)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py -k "gemm" > gpurun_out/r06_gemmrows.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/r06_gemmrows.log
for rep in 1 2; do
for v in base dg dgwg wg; do
case $v in
base) export TDL_ROUTE_OFF=dgrad.gemm.k256;;
dg) unset TDL_ROUTE_OFF;;
dgwg) export TDL_ROUTE_OFF=wgrad.glds.1x1;;
wg) export TDL_ROUTE_OFF=dgrad.gemm.k256,wgrad.glds.1x1;;
esac
timeout -k 10 300 python bench.py --steps 40 > gpurun_out/r06_gemmrows_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_gemmrows_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])"
done; done
