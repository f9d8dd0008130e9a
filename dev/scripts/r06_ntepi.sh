# Conv output-tile stores non-temporal (dev/ntepi build, TDL_EPI_STORE_AUX=2) vs cached: same-box A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
NT=$R/dev/ntepi/_C.cpython-310-x86_64-linux-gnu.so
TDL_EXT_SO=$NT timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_conv_route_gpu.py -k "every_route" > gpurun_out/r06_ntepi.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/r06_ntepi.log
for v in nt base nt base; do
if [ $v = nt ]; then export TDL_EXT_SO=$NT; else unset TDL_EXT_SO; fi
timeout -k 10 300 python bench.py --steps 30 > gpurun_out/r06_ntepi_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_ntepi_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('epi $v resnet50', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --model xception41 --batch 128 --image-size 299 --steps 20 > gpurun_out/r06_ntepi_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_ntepi_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('epi $v xception41', d['value'], d['ms_per_step'])"
done
